"""GPU parity of the headline's timed region: the subproblems bench.py actually times.

bench.py (C3) runs 5 untimed + 20 timed steps of the warm-started Jacobi loop (scvx_hip.scvx.JacobiSCvx
with the bench's own settings, bench.py:516-523).  This test runs that loop for 25 steps and, at steps 6,
15 and 25 (1-based: the first, a middle and the last timed step), checks subproblems of that very step
against the reference-form oracle (oracle/qp_dense.py: Distributed_opt/dist_scvx_3d.py:51-111 as
written, with the C3 obstacles and SOC) on the exact inputs of that solve -- the FOH discretization the
step computed, the iterate (X, U) it linearised at, and the per-agent trust radius it was given.

Sample per step: the 8 agents with the most IPM iterations that step (the tail that sets the launch
time) and every 128th agent, at least 16 distinct agents; no skip escape.  Tolerances: status optimal,
objective 1e-8 relative (the stopping rule's gap tolerance, Clarabel's default), reference-form constraint
violation 1e-7."""
import numpy as np
import pytest

import scvx_hip
from oracle import problems as pb, qp_dense as qd

pytestmark = pytest.mark.gpu

CHECK_STEPS = (6, 15, 25)


def _pick(iters, n_top=8, stride=128, want=16):
    order = np.lexsort((np.arange(iters.size), -iters))   # most iterations first, ties by index
    pick = list(order[:n_top])
    for a in range(0, iters.size, stride):
        if a not in pick:
            pick.append(a)
    a = stride // 2
    while len(pick) < want:
        if a not in pick:
            pick.append(a)
        a += stride
    return np.array(sorted(int(v) for v in pick))


def test_timed_region_subproblems_match_dense_oracle(cuda):
    import torch
    import bench
    from scvx_hip.scvx import JacobiSCvx
    sc, w = bench.make_workload(bench.N_AGENTS, seed=1, device=cuda)
    spec = scvx_hip.QPSpec(model="di", K=bench.K, box=bench.BOX, obs=sc["obs"], w_obs=1e6, u_max=bench.U_MAX,
                           tol=1e-8, max_iter=60)
    drv = JacobiSCvx(spec, w["x_init"], w["x_final"], w["sigma"], bench.TR0, tr_rule="per_agent", tie_rtol=1e-9,
                     fused_update=True, warm_max_status=1)   # bench.py default (C3 ends every solve optimal)
    X, U = w["X"].clone(), w["U"].clone()
    caught = {}
    for step in range(1, max(CHECK_STEPS) + 1):
        tr = drv.tr.clone()
        warm = drv.warm is not None and bool(drv.warm.any().item())
        Xn, Un, out = drv.step(X, U)
        st = out["status"].cpu().numpy()
        assert (st == 0).mean() >= 0.99, (step, np.bincount(st, minlength=3))
        if step in CHECK_STEPS:
            caught[step] = dict(disc=drv.disc.cpu().numpy(), X=X.cpu().numpy(), U=U.cpu().numpy(),
                                tr=tr.cpu().numpy(), warm=warm, status=st, iters=out["iters"].cpu().numpy(),
                                Xs=out["X"].cpu().numpy(), Us=out["U"].cpu().numpy(), obj=out["obj"].cpu().numpy())
        X, U = Xn, Un
    x_final = sc["x_final"]
    report = []
    for step, c in caught.items():
        assert c["warm"], step          # the timed steps are warm-started solves
        pick = _pick(c["iters"])
        assert pick.size >= 16
        for a in pick:
            assert c["status"][a] == 0, (step, a, c["status"][a])
            A, B, C, S, z = pb.unpack_disc(c["disc"][a], 6, 3)
            prob = dict(A=A, B=B, C=C, c=S * sc["sigma"][a] + z, Xref=c["X"][a], Uref=c["U"][a], x_final=x_final[a],
                        tr=float(c["tr"][a]), box=bench.BOX, obs=sc["obs"], w_obs=1e6, umax=bench.U_MAX,
                        fix_last_input=True)
            with np.errstate(all="ignore"):
                Xd, Ud, objd, info = qd.solve_agent(prob, sparse=True, tol=1e-11, maxit=150)
            assert info["status"] == "optimal", (step, a, info["status"])
            rel = abs(c["obj"][a] - objd) / max(1.0, abs(objd))
            viol = max(qd.constraint_violation(prob, c["Xs"][a], c["Us"][a]).values())
            report.append((step, int(a), int(c["iters"][a]), rel, viol))
            assert rel <= 1e-8, (step, a, c["obj"][a], objd)
            assert viol < 1e-7, (step, a, viol)
    print("step agent iters rel_obj violation")
    for r in report:
        print("%4d %5d %3d %.2e %.2e" % r)

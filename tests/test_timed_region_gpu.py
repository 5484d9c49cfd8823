"""GPU parity of the headline's timed region: the subproblems bench.py actually times.

bench.py (C3) runs 5 untimed + 20 timed steps of the warm-started Jacobi loop (scvx_hip.scvx.JacobiSCvx
with the bench's own settings, bench.py main), once under the reference's global trust-region rule (the
headline `value`, Distributed_opt/dist_scvx_3d.py:248-252) and once under the per-agent rule (`other_rule`).
This test runs that loop for 25 steps under each rule and, at steps 6, 15 and 25 (1-based: the first, a
middle and the last timed step), checks subproblems of that very step against the reference-form oracle
(oracle/qp_dense.py: Distributed_opt/dist_scvx_3d.py:51-111 as written, with the C3 obstacles and SOC) on
the exact inputs of that solve -- the FOH discretization the step computed, the iterate (X, U) it
linearised at, and the trust radius it was given.  The C2 line (BASELINE.json configs[1]: N=128, no
obstacles, no SOC) gets the same check on its own loop.

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


def _loop_matches_dense_oracle(cuda, config, rule, check_steps=CHECK_STEPS):
    import bench
    from scvx_hip.scvx import JacobiSCvx
    c3 = config == "c3"
    N = bench.N_AGENTS if c3 else 128
    sc, w = bench.make_workload(N, seed=1 if c3 else 0, device=cuda, obstacles=bench.N_OBS if c3 else 0)
    umax = bench.U_MAX if c3 else None
    spec = scvx_hip.QPSpec(model="di", K=bench.K, box=bench.BOX, obs=sc["obs"], w_obs=1e6, u_max=umax,
                           tol=1e-8, max_iter=60)
    drv = JacobiSCvx(spec, w["x_init"], w["x_final"], w["sigma"], bench.TR0, tr_rule=rule, tie_rtol=1e-9,
                     fused_update=True, warm_max_status=1)   # bench.py defaults
    X, U = w["X"].clone(), w["U"].clone()
    caught = {}
    for step in range(1, max(check_steps) + 1):
        tr = drv.tr.clone()
        warm = drv.warm is not None and bool(drv.warm.any().item())
        Xn, Un, out = drv.step(X, U)
        st = out["status"].cpu().numpy()
        assert (st == 0).mean() >= 0.99, (step, np.bincount(st, minlength=3))
        if step in check_steps:
            caught[step] = dict(disc=drv.disc.cpu().numpy(), X=X.cpu().numpy(), U=U.cpu().numpy(),
                                tr=tr.cpu().numpy(), warm=warm, status=st, iters=out["iters"].cpu().numpy(),
                                Xs=out["X"].cpu().numpy(), Us=out["U"].cpu().numpy(), obj=out["obj"].cpu().numpy())
        X, U = Xn, Un
    x_final = sc["x_final"]
    report = []
    for step, c in caught.items():
        assert c["warm"], step          # the timed steps are warm-started solves
        pick = _pick(c["iters"], stride=N // 8)
        assert pick.size >= 16
        for a in pick:
            assert c["status"][a] == 0, (step, a, c["status"][a])
            A, B, C, S, z = pb.unpack_disc(c["disc"][a], 6, 3)
            prob = dict(A=A, B=B, C=C, c=S * sc["sigma"][a] + z, Xref=c["X"][a], Uref=c["U"][a], x_final=x_final[a],
                        tr=float(c["tr"][a]), box=bench.BOX, obs=sc["obs"], w_obs=1e6, umax=umax,
                        fix_last_input=True)
            with np.errstate(all="ignore"):
                Xd, Ud, objd, info = qd.solve_agent(prob, sparse=True, tol=1e-11, maxit=150)
            assert info["status"] == "optimal", (step, a, info["status"])
            rel = abs(c["obj"][a] - objd) / max(1.0, abs(objd))
            viol = max(qd.constraint_violation(prob, c["Xs"][a], c["Us"][a]).values())
            report.append((step, int(a), int(c["iters"][a]), rel, viol))
            assert rel <= 1e-8, (step, a, c["obj"][a], objd)
            assert viol < 1e-7, (step, a, viol)
    print(f"{config} {rule}: step agent iters rel_obj violation")
    for r in report:
        print("%4d %5d %3d %.2e %.2e" % r)


@pytest.mark.parametrize("rule", ["global", "per_agent"])
def test_timed_region_subproblems_match_dense_oracle(cuda, rule):
    _loop_matches_dense_oracle(cuda, "c3", rule)


def test_c2_loop_subproblems_match_dense_oracle(cuda):
    """bench.py --config c2 (N=128) under the headline's global rule."""
    _loop_matches_dense_oracle(cuda, "c2", "global")

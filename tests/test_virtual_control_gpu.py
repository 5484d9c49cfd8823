"""GPU parity of the virtual-control classes of the batched trust-region solve (QPSpec.w_nu > 0: nu_t in
every dynamics row priced w_nu sum_t ||nu_t||_1, the SCvx subproblem form of
SCvx/optimization/sc_problem.py:60-68; QPSpec.w_prox: a proximal state term), and of the C5 workload
built on them (12-state quadrotor, obstacles, Jacobi collision coupling of
Distributed_opt/dist_scvx_3d.py:93-107).

References: the kernel's CPU twin (oracle/scvx_cpu.cpp, the same Riccati elimination of nu) on every
agent, and the reference-form dense oracle (oracle/qp_dense.py with nu and its L1 epigraph as CVXPY
canonicalises them, solved by an independent sparse conic IPM) on samples.  Tolerances: objective 1e-8
relative against the twin and 1e-7 against the dense oracle (its gap test is on the problem scaled by
the 1e6 obstacle weight); inputs 1e-6 against the twin (unique: their cost is strictly convex; the states
and nu are unique only up to the degenerate, piecewise-linear nu penalty -- measured 1e-4 apart at equal
objective -- so they are held to feasibility of the reference form, 1e-7, instead)."""
import numpy as np
import pytest

import scvx_hip
from oracle import problems as pb, qp_cpu, qp_dense as qd

pytestmark = pytest.mark.gpu

BOX = [(0, -12, 12), (1, -12, 12)]
W_NU, W_PROX = 1e4, 10.0   # the C5 settings (bench.py make_coupled)


def _t(x, cuda, dtype=None):
    import torch
    return torch.tensor(np.ascontiguousarray(x), device=cuda, dtype=dtype or torch.float64)


@pytest.mark.parametrize("tr0,w_nu,w_prox", [(0.01, 1e3, 0.0), (0.01, 50.0, 1.0), (0.25, 1e3, 0.0)])
def test_di_virtual_control_matches_twin_and_dense(cuda, tr0, w_nu, w_prox):
    """C3 family with virtual control: tr = 0.01 puts the goal out of the inputs' reach, so nu is active."""
    N, K = 64, 50
    sc = pb.synthetic_di(N, K=K, seed=1, obstacles=8)
    X, U, sig = _t(sc["X"], cuda), _t(sc["U"], cuda), _t(sc["sigma"], cuda)
    disc = scvx_hip.foh_batched("di", X, U, sig)
    tr = np.full(N, tr0)
    spec = scvx_hip.QPSpec(model="di", K=K, box=BOX, obs=sc["obs"], w_obs=1e6, u_max=1.0, tol=1e-9, max_iter=80,
                           w_nu=w_nu, w_prox=w_prox)
    out = scvx_hip.qp_solve_batched(spec, disc, sig, X, U, _t(sc["x_init"], cuda), _t(sc["x_final"], cuda), _t(tr, cuda))
    st = out["status"].cpu().numpy()
    assert np.isin(st, (0, 1)).all() and (st == 0).mean() >= 0.95, np.bincount(st, minlength=3)
    dn = disc.cpu().numpy()
    tpl = qp_cpu.make_template(6, 3, K, box=BOX, obs=sc["obs"], w_obs=1e6, u_max=1.0, tol=1e-9, max_iter=80,
                               w_nu=w_nu, w_prox=w_prox)
    cpu = qp_cpu.solve_batched(tpl, dn, sc["sigma"], sc["X"], sc["U"], sc["x_init"], sc["x_final"], tr, nthreads=8)
    assert (st != cpu["status"]).sum() <= 2   # the same stopping rule (an agent at its threshold may differ)
    Xg, Ug, Ng, og = (out[k].cpu().numpy() for k in ("X", "U", "nu", "obj"))
    ok = (st == 0) & (cpu["status"] == 0)
    np.testing.assert_allclose(og[ok], cpu["obj"][ok], rtol=1e-8)
    # inputs: strong convexity (Hessian 2I) bounds ||U - U*||^2 by the gap, 1e-9 x the objective here
    assert np.abs(Ug[ok, :-1] - cpu["U"][ok, :-1]).max() < 3.0 * np.sqrt(1e-9 * max(1.0, np.abs(og).max()))
    if tr0 < 0.1:
        assert np.abs(Ng).max() > 1e-2    # nu carries the unreachable part of the transfer
    for a in [int(i) for i in np.nonzero(ok)[0][[0, -1]]]:
        A, B, C, S, z = pb.unpack_disc(dn[a], 6, 3)
        prob = dict(A=A, B=B, C=C, c=S * sc["sigma"][a] + z, Xref=sc["X"][a], Uref=sc["U"][a],
                    x_final=sc["x_final"][a], tr=tr0, box=BOX, obs=sc["obs"], w_obs=1e6, umax=1.0,
                    fix_last_input=True, w_nu=w_nu, w_prox=w_prox)
        with np.errstate(all="ignore"):
            Xd, Ud, objd, info = qd.solve_agent(prob, sparse=True, tol=1e-10)
        assert info["status"] == "optimal"
        assert abs(og[a] - objd) <= 1e-8 * max(1.0, abs(objd)), (a, og[a], objd)
        assert max(qd.constraint_violation(prob, Xg[a], Ug[a], nu=Ng[a]).values()) < 1e-7


def _quad_batch(N=64, seed=3):
    from scvx_hip import workloads
    sc = workloads.synthetic_quad(1024, K=50, seed=seed, sigma=30.0, obstacles=8)
    sub = {k: np.ascontiguousarray(sc[k][:N]) for k in ("X", "U", "x_init", "x_final", "sigma")}
    return sc["obs"], workloads.QUAD_BOX, sub


def test_quad_virtual_control_matches_twin_and_dense(cuda):
    """The C5 subproblem class (quadrotor n=12, m=4, QUAD_BOX, 8 obstacles, j_max = 8 collision rows with
    R = 0.5, w_nu 1e4, w_prox 10) at the first SCvx iteration: every agent against the twin, two against the
    reference-form oracle (one with collision rows)."""
    obs, box, sub = _quad_batch()
    N, K = sub["X"].shape[0], sub["X"].shape[1]
    X, U, sig = _t(sub["X"], cuda), _t(sub["U"], cuda), _t(sub["sigma"], cuda)
    disc = scvx_hip.foh_batched("quad", X, U, sig)
    rows, cnt = scvx_hip.collision_rows(X, 0, N, 0.5, 8)
    spec = scvx_hip.QPSpec(model="quad", K=K, box=box, obs=obs, w_obs=1e6, j_max=8, w_coll=1e4, tol=1e-8, max_iter=60,
                           w_nu=W_NU, w_prox=W_PROX)
    tr = np.full(N, 0.25)
    out = scvx_hip.qp_solve_batched(spec, disc, sig, X, U, _t(sub["x_init"], cuda), _t(sub["x_final"], cuda),
                                    _t(tr, cuda), rows, cnt)
    st = out["status"].cpu().numpy()
    assert (st == 0).all(), np.bincount(st, minlength=3)
    dn, rn, cn = disc.cpu().numpy(), rows.cpu().numpy(), cnt.cpu().numpy()
    tpl = qp_cpu.make_template(12, 4, K, box=box, obs=obs, w_obs=1e6, j_max=8, w_coll=1e4, tol=1e-8, max_iter=60,
                               model_id=3, w_nu=W_NU, w_prox=W_PROX)
    cpu = qp_cpu.solve_batched(tpl, dn, sub["sigma"], sub["X"], sub["U"], sub["x_init"], sub["x_final"], tr, rn, cn,
                               nthreads=8)
    assert (cpu["status"] == 0).all()
    Xg, Ug, Ng, Sg, og = (out[k].cpu().numpy() for k in ("X", "U", "nu", "slack_coll", "obj"))
    np.testing.assert_allclose(og, cpu["obj"], rtol=1e-8)
    assert np.abs(Ug[:, :-1] - cpu["U"][:, :-1]).max() < 1e-6
    busy = [a for a in range(N) if cn[a].max() > 0] or [0]
    for a in sorted({0, busy[0]}):
        A, B, C, S, z = pb.unpack_disc(dn[a], 12, 4)
        prob = pb.dense_prob_from_rows(A, B, sub["X"][a], sub["U"][a], sub["x_final"][a], 0.25,
                                       [rn[a, t, :cn[a, t]] for t in range(K)], box=box, obs=obs, w_obs=1e6,
                                       w_coll=1e4, fix_last_input=True, w_nu=W_NU, w_prox=W_PROX)
        prob.update(C=C, c=S * sub["sigma"][a] + z)
        with np.errstate(all="ignore"):
            Xd, Ud, objd, info = qd.solve_agent(prob, sparse=True, tol=1e-11)
        assert info["status"] in ("optimal", "optimal_inaccurate"), info["status"]
        assert abs(og[a] - objd) <= 1e-7 * max(1.0, abs(objd)), (a, og[a], objd)
        assert max(qd.constraint_violation(prob, Xg[a], Ug[a], S=Sg[a], nu=Ng[a]).values()) < 1e-7


def test_c5_jacobi_virtual_control_stays_feasible(cuda):
    """The C5 construction (first 64 quadrotors) through 10 Jacobi SCvx iterations of scvx_hip.scvx.JacobiSCvx:
    every subproblem solves (status 0 / 1: optimal / optimal_inaccurate) at every step and no reference
    collision row stays violated after the check + re-solve (coupling_check.overflow == 0); at the last step
    one agent is checked against the reference-form oracle on the rows its solve used."""
    from scvx_hip.scvx import CouplingSpec, JacobiSCvx
    obs, box, sub = _quad_batch()
    N, K = sub["X"].shape[0], sub["X"].shape[1]
    spec = scvx_hip.QPSpec(model="quad", K=K, box=box, obs=obs, w_obs=1e6, j_max=8, w_coll=1e4, tol=1e-8, max_iter=60,
                           w_nu=W_NU, w_prox=W_PROX)
    drv = JacobiSCvx(spec, _t(sub["x_init"], cuda), _t(sub["x_final"], cuda), _t(sub["sigma"], cuda), 0.25,
                     coupling=CouplingSpec(R=0.5), tr_rule="global")
    X, U = _t(sub["X"], cuda), _t(sub["U"], cuda)
    for step in range(10):
        Xr, Ur, tr_used = X.clone(), U.clone(), drv.tr.clone()
        X, U, out = drv.step(X, U)
        st = out["status"].cpu().numpy()
        assert np.isin(st, (0, 1)).all(), (step, np.bincount(st, minlength=3))
        assert drv.last_check["overflow"] == 0, (step, drv.last_check)
    assert np.isfinite(X.cpu().numpy()).all() and np.abs(X.cpu().numpy()[:, :, :2]).max() <= 12.0 + 1e-6
    # one agent of the last step against the reference form, on its solve's inputs
    a = 5
    dn = drv.disc.cpu().numpy()[a]
    rn, cn = drv.rows.cpu().numpy()[a], drv.count.cpu().numpy()[a]
    A, B, C, S, z = pb.unpack_disc(dn, 12, 4)
    Xa, Ua = Xr.cpu().numpy()[a], Ur.cpu().numpy()[a]
    prob = pb.dense_prob_from_rows(A, B, Xa, Ua, sub["x_final"][a], float(tr_used[a].item()),
                                   [rn[t, :cn[t]] for t in range(K)], box=box, obs=obs, w_obs=1e6, w_coll=1e4,
                                   fix_last_input=True, w_nu=W_NU, w_prox=W_PROX)
    prob.update(C=C, c=S * sub["sigma"][a] + z)
    if drv.last_check["resolved"] == 0:
        with np.errstate(all="ignore"):
            Xd, Ud, objd, info = qd.solve_agent(prob, sparse=True, tol=1e-11)
        og = out["obj"][a].item()
        assert abs(og - objd) <= 1e-7 * max(1.0, abs(objd)), (og, objd)

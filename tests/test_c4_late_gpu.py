"""GPU: the late steps of the C4 loop (bench.py --config c4: 4096 lattice agents, coupling R = 2.3, j_max = 8,
global trust-region rule, warm-started subproblems), where the trust region has shrunk to 1/64 of its start and a
few percent of the subproblems end at Clarabel's reduced tolerances (status 1, "optimal_inaccurate").

Why status 1 there: an active trust-region facet of ||w_t||_1 <= tr adds D g g' with
D = lambda / s ~ 1e12 to the node's input Hessian, whose sum with the O(1e-4) objective curvature cannot be
represented in float64; the normal-equation Riccati then clamps a pivot (kernel and CPU twin alike) and the dual
residual stalls near 1e-8.  The same subproblems solved cold end the same way, so it is not the warm start.
Round 5 keeps such facets out of the normal equations (explicit stage unknowns, Woodbury form: QPCfg::STF in
qp_ipm.hpp, Riccati::stiff in oracle/scvx_cpu.cpp): 444 -> 25-62 status-1 solves at the worst step.

Checked at step 18 (tr = 2^-4 x 0.25) of the loop, on the step's own inputs (discretisation, culled rows):
  * no solve fails (status 2) and >= 98 % end at the full tolerance (status 0) at every step (measured round 5:
    98.4-98.6 % at the worst step, >= 99.3 % at every other; round 4, before the stiff-facet stage system: 89 %);
  * status-1 solves against the dense reference-form oracle (oracle/qp_dense.py, dist_scvx_3d.py:51-111 as
    written): optimal value within 1e-7 relative, violation < 1e-5 (Clarabel's reduced feasibility, as
    tests/test_coupled_gpu.py); status-0 solves: value 1e-7, violation 1e-7;
  * the warm-started solve equals the cold solve of the same subproblem in value where both end optimal: 2e-8
    relative for 99 % of them (both within the 1e-8 gap test), 1e-6 for every one (the primal residual priced
    by the slack multipliers); 5e-5 where either ends at the reduced tolerances (measured 5.1e-6 at most)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

STEPS = 19


def test_c4_late_steps_match_dense_oracle(cuda):
    import torch
    import bench
    import scvx_hip
    from oracle import qp_dense as qd
    from scvx_hip.scvx import CouplingSpec, JacobiSCvx
    from test_coupled_gpu import _dense_prob
    sc, w, cfg = bench.make_coupled("c4", 1, 0, cuda)
    spec = scvx_hip.QPSpec(model="di", K=bench.K, box=cfg["box"], obs=cfg["obs"], w_obs=1e6, j_max=cfg["j_max"],
                           w_coll=1e4, tol=1e-8, max_iter=60)
    drv = JacobiSCvx(spec, w["x_init"], w["x_final"], w["sigma"], bench.TR0, coupling=CouplingSpec(R=cfg["R"]),
                     tr_rule="global", warm_max_status=1)   # bench.py's default
    X, U = w["X"].clone(), w["U"].clone()
    N = X.shape[0]
    fr0 = []
    for k in range(STEPS):
        trp = drv.tr.clone()
        Xn, Un, _ = drv.step(X, U)
        torch.cuda.synchronize()
        st = drv.solver.status.cpu().numpy()
        assert (st != 2).all(), (k, np.bincount(st, minlength=3))
        fr0.append(float((st == 0).mean()))
        if k == STEPS - 1:
            break
        X, U = Xn, Un
    print("status-0 fraction per step:", [round(f, 4) for f in fr0])
    # measured: round 4 >= 98 % at steps 0-14, 96 / 99 / 89 / 97 % at steps 15-18; round 5, with the stiff
    # trust-region facets kept out of the normal equations (QPCfg::STF), >= 99.4 % at every step but step 17
    # (98.4-98.5 %; pytest_r5e/r5f) -- the remaining status-1 solves lose accuracy in the state-side Riccati
    # (P = Qh - Sh' Rh^-1 Sh of collision-stiff nodes); every status-1 solve is checked below
    assert min(fr0) >= 0.98, fr0
    # the last step's subproblems: its inputs are still in the driver
    trn = trp.cpu().numpy()
    assert trn[0] <= 0.25 / 16      # the radius has halved four times by step 18 (profiles/round4_r4a_c4_drift.log)
    out = {k: getattr(drv.solver, a).clone() for k, a in (("status", "status"), ("obj", "obj"), ("X", "X"), ("U", "U"),
                                                         ("slack_coll", "slack"))}
    rows, cnt = drv.rows.clone(), drv.count.clone()
    cold = scvx_hip.QPSolver(spec, N, device=cuda).solve(drv.disc, drv.sigma, X, U, drv.x_init, drv.x_final, trp,
                                                         rows, cnt)
    st = out["status"].cpu().numpy()
    stc = cold["status"].cpu().numpy()
    ow, oc = out["obj"].cpu().numpy(), cold["obj"].cpu().numpy()
    # both optimal: the stopping rule bounds the gap by 1e-8 relative, but the objective also moves by the primal
    # residual (<= 1e-8 pnorm) times the multipliers, which reach the slack weights here (w_coll = 1e4 on the
    # objective's 1e6 scale) (measured round 4, before the stiff-facet stage system: 3 of 3964 agents above 2e-8,
    # max 4.4e-6, profiles/round4_r4n_pytest_gpu.log; round 5: max 5.7e-8 to 2.1e-7 over the builds of the round,
    # profiles/round5_r5o_pytest.log); a status-1 end on either side certifies only the reduced gap (5e-5)
    both = (st == 0) & (stc == 0)
    np.testing.assert_allclose(ow[both], oc[both], rtol=1e-6, atol=2e-8)
    assert np.mean(np.abs(ow[both] - oc[both]) <= 2e-8 * np.maximum(1.0, np.abs(oc[both]))) >= 0.99
    np.testing.assert_allclose(ow[~both], oc[~both], rtol=5e-5, atol=1e-8)
    print("warm vs cold: both optimal", int(both.sum()), "max rel diff there",
          float(np.max(np.abs(ow[both] - oc[both]) / np.maximum(1.0, np.abs(oc[both])), initial=0.0)),
          "max rel diff where either is status 1",
          float(np.max(np.abs(ow[~both] - oc[~both]) / np.maximum(1.0, np.abs(oc[~both])), initial=0.0)))
    dn, Xh, Uh = drv.disc.cpu().numpy(), X.cpu().numpy(), U.cpu().numpy()
    sig, xf = drv.sigma.cpu().numpy(), drv.x_final.cpu().numpy()
    rn, cn = rows.cpu().numpy(), cnt.cpu().numpy()
    Xg, Ug, Sg = (out[k].cpu().numpy() for k in ("X", "U", "slack_coll"))
    s1 = np.nonzero(st == 1)[0][:4]
    s0 = np.nonzero(st == 0)[0][::N // 4][:4]
    checked = 0
    for a in np.concatenate([s1, s0]):
        prob = _dense_prob("di", dn[a], sig[a], Xh[a], Uh[a], xf[a], trn[a], rn[a], cn[a], cfg["box"], [])
        with np.errstate(all="ignore"):
            Xd, Ud, objd, info = qd.solve_agent(prob, sparse=True, tol=1e-10, maxit=150)
        viol = max(qd.constraint_violation(prob, Xg[a], Ug[a], Sg[a]).values())
        print(f"agent {a}: status {st[a]} obj {ow[a]:.12e} dense {objd:.12e} ({info['status']}) viol {viol:.2e}")
        assert viol < (1e-5 if st[a] == 1 else 1e-7), (a, viol)
        if info["status"] != "optimal":
            continue
        assert abs(ow[a] - objd) <= 1e-7 * max(1.0, abs(objd)), (a, ow[a], objd)
        checked += 1
    assert checked >= 4

"""GPU: the drop-in surfaces run unmodified-style against the MI355X backend.

  * SCvx.discretization.first_order_hold.FirstOrderHold vs the reference goldens (LSODA) and the
    reference test_disc.py shape contract (SCvx/tests/test_disc.py:9-49);
  * Distributed_opt.dist_scvx_3d.x_traj_opt: one Jacobi sweep of the 3-robot scenario vs the dense
    reference-formulation oracle per robot, then several sweeps of the reference outer loop."""
import glob
import os

import numpy as np
import pytest

from oracle import qp_dense as qd

pytestmark = pytest.mark.gpu
GOLD = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "foh_*.npz")))


def _model(name):
    from SCvx.models.double_integrator_model import DoubleIntegratorModel
    from SCvx.models.quadrotor_model import QuadrotorModel
    from SCvx.models.single_integrator_model import SingleIntegratorModel
    from SCvx.models.unicycle_model import UnicycleModel
    return {"di": DoubleIntegratorModel, "unicycle": UnicycleModel, "si": SingleIntegratorModel,
            "quad": QuadrotorModel}[name]()


@pytest.mark.parametrize("name", ["unicycle", "quad"])
def test_first_order_hold_batched_helper(cuda, name):
    """calculate_discretization_batched (one launch for M agents) returns exactly what M single-agent
    calculate_discretization calls return (the kernel integrates every agent independently), as new
    arrays, and leaves the object's own output buffers alone; the device-resident form matches too."""
    import torch
    from SCvx.discretization.first_order_hold import FirstOrderHold
    import scvx_hip
    model = _model(name)
    K, M = 30, 5
    rng = np.random.default_rng(11)
    Xs = [0.1 * rng.standard_normal((model.n_x, K)) for _ in range(M)]
    Us = [0.1 * rng.standard_normal((model.n_u, K)) for _ in range(M)]
    sigmas = list(1.0 + rng.uniform(0, 2, M))
    foh = FirstOrderHold(model, K)
    single = [tuple(o.copy() for o in foh.calculate_discretization(X, U, s)) for X, U, s in zip(Xs, Us, sigmas)]
    keep = foh.A_bar.copy()
    batched = foh.calculate_discretization_batched(Xs, Us, sigmas)
    assert len(batched) == M
    for a in range(M):
        for got, want in zip(batched[a], single[a]):
            assert got.shape == want.shape
            np.testing.assert_array_equal(got, want)
        assert batched[a][0] is not foh.A_bar
    np.testing.assert_array_equal(foh.A_bar, keep)
    Xd = torch.tensor(np.ascontiguousarray(np.stack([x.T for x in Xs])), device=cuda)
    Ud = torch.tensor(np.ascontiguousarray(np.stack([u.T for u in Us])), device=cuda)
    disc = foh.calculate_discretization_device(Xd, Ud, torch.tensor(sigmas, dtype=torch.float64, device=cuda))
    A_dev = scvx_hip.unpack_disc(disc, name)[0].cpu().numpy()
    np.testing.assert_array_equal(A_dev[2], single[2][0])
    assert foh.calculate_discretization_batched([], [], []) == []


@pytest.mark.parametrize("path", GOLD, ids=[os.path.basename(p) for p in GOLD])
def test_first_order_hold_dropin(cuda, path):
    from SCvx.discretization.first_order_hold import FirstOrderHold
    d = np.load(path)
    model = _model(str(d["model"]))
    K = int(d["K"])
    foh = FirstOrderHold(model, K)
    outs = foh.calculate_discretization(d["X"], d["U"], float(d["sigma"]))
    shapes = [(model.n_x * model.n_x, K - 1), (model.n_x * model.n_u, K - 1), (model.n_x * model.n_u, K - 1),
              (model.n_x, K - 1), (model.n_x, K - 1)]
    for o, name, shp in zip(outs, ["A_bar", "B_bar", "C_bar", "S_bar", "z_bar"], shapes):
        assert o.shape == shp
        assert np.abs(o - d[name]).max() / max(1.0, np.abs(d[name]).max()) < 1e-7, name
    assert outs[0] is foh.A_bar  # reference aliasing: buffers owned by the object
    Xp = foh.integrate_nonlinear_piecewise(d["X"], d["U"], float(d["sigma_nl"]))
    Xf = foh.integrate_nonlinear_full(d["X"][:, 0], d["U"], float(d["sigma_nl"]))
    assert Xp.shape == (model.n_x, K) and Xf.shape == (model.n_x, K)
    assert np.abs(Xp - d["X_piecewise"]).max() / max(1, np.abs(d["X_piecewise"]).max()) < 1e-7
    assert np.abs(Xf - d["X_full"]).max() / max(1, np.abs(d["X_full"]).max()) < 1e-6


def _dense_reference_sweep(d, X_traj):
    """x_traj_opt restated with the dense oracle, robot by robot (dist_scvx_3d.py:51-118)."""
    names = d.robots_name
    new = {}
    for nm in names:
        Xr = X_traj[nm][:, 0:6]
        Ur = X_traj[nm][:, 6:9]
        coll = []
        for t in range(d.T - 1):
            rows = []
            for o in names:
                if o == nm:
                    continue
                diff = X_traj[nm][t, 0:3] - X_traj[o][t, 0:3]
                nr = np.linalg.norm(diff)
                rows.append(np.concatenate([diff / nr, [2 * d.R - nr]]))
            coll.append(np.array(rows))
        prob = dict(A=np.repeat(d.Ad[None], d.T - 1, 0), B=np.repeat(d.Bd[None], d.T - 1, 0), Xref=Xr, Uref=Ur,
                    x_final=d.x_des[nm][0:6], tr=d.trust_region, box=[(0, -1, 22), (1, -1, 20)], coll=coll,
                    w_coll=1e4, fix_last_input=True)
        Xn, Un, obj, info = qd.solve_agent(prob, tol=1e-10, maxit=150)
        assert info["status"] == "optimal"
        new[nm] = (Xn, Un, obj, prob)
    return new


def test_dist_scvx_3d_jacobi_sweep_matches_dense_oracle(cuda):
    from Distributed_opt import dist_scvx_3d as d
    X0 = d.x_initial(d.x_ini, d.x_des)
    ref = _dense_reference_sweep(d, X0)
    X1 = d.x_traj_opt({k: v.copy() for k, v in X0.items()}, d.trust_region)
    for nm in d.robots_name:
        Xn, Un, obj, prob = ref[nm]
        got_X, got_U = X1[nm][:, 0:6], X1[nm][:, 6:9]
        viol = qd.constraint_violation(prob, got_X, got_U, np.full(d.T, 1e9))
        # Clarabel's primal test is relative: 1e-8 x (||b|| + ||x|| + ||s||), positions here reach ~22
        assert max(v for k, v in viol.items() if k != "coll") < 2e-7, viol
        u_cost = np.sum(got_U[:-1] ** 2)
        # the reference objective at the drop-in's solution: the shared slack of node t is the smallest one
        # its rows allow, S_t = max(0, max_j (c_j - g_j' d_t)) (dist_scvx_3d.py:99-107)
        d_ = got_X - prob["Xref"]
        S = np.array([max(0.0, np.max(r[:, 3] - r[:, :3] @ d_[t, :3])) for t, r in enumerate(prob["coll"])])
        full = u_cost + prob["w_coll"] * S.sum()
        assert abs(full - obj) <= 1e-7 * max(1.0, obj), (nm, full, obj)   # slack-active robots included
        if obj < 1e3:  # no active collision slack: the minimum-energy trajectory is unique
            tol_obj = 1e-8 * max(1.0, obj)
            assert abs(u_cost - obj) <= tol_obj
            # sum ||u_t||^2 is 2-strongly convex, so on the feasible set f(U) - f(U*) >= ||U - U*||^2: the objective
            # tolerance (Clarabel's 1e-8, the solver dist_scvx_3d.py:110 calls) bounds the input error (factor 2:
            # the 2e-7 primal residual allowed above)
            dU = got_U - Un
            assert np.sum(dU[:-1] ** 2) <= 2.0 * tol_obj, (nm, np.sum(dU[:-1] ** 2), tol_obj)
            # and the states follow from the inputs through the dynamics (dX_0 = 0)
            dX = np.zeros_like(got_X)
            for t in range(d.T - 1):
                dX[t + 1] = d.Ad @ dX[t] + d.Bd @ dU[t]
            assert np.abs((got_X - Xn) - dX).max() < 1e-5
            # a direct bound on the state error: |dX_t| <= sum_s ||Ad^(t-1-s) Bd||_2 |dU_s| <= G ||dU||_F by
            # Cauchy-Schwarz, G^2 = max_t sum_{s<t} ||Ad^(t-1-s) Bd||_2^2 (the input-to-state gain over the horizon)
            gains, Phi = [], np.eye(6)
            for _ in range(d.T - 1):
                gains.append(np.linalg.norm(Phi @ d.Bd, 2) ** 2)
                Phi = d.Ad @ Phi
            G = np.sqrt(np.sum(gains))
            bound_x = G * np.sqrt(np.sum(dU[:-1] ** 2)) + 1e-6
            err_x = np.abs(got_X - Xn).max()
            print(f"{nm}: max |dU| {np.abs(dU[:-1]).max():.2e}  max |dX| {err_x:.2e}  bound {bound_x:.2e}")
            assert err_x <= bound_x, (nm, err_x, bound_x)
        np.testing.assert_array_equal(X1[nm][-1, 6:9], X0[nm][-1, 6:9])  # pinned unused row


def test_dist_scvx_3d_outer_loop_runs(cuda):
    from Distributed_opt import dist_scvx_3d as d
    X = d.x_initial(d.x_ini, d.x_des)
    tr = d.trust_region
    costs = []
    for it in range(6):
        X = d.x_traj_opt(X, tr)
        costs.append(d.cost_fcn(X))
        if it >= 1 and costs[-1] > costs[-2]:
            tr /= 2
    for nm in d.robots_name:
        np.testing.assert_allclose(X[nm][-1, 0:6], d.x_des[nm][0:6], atol=1e-7)
        np.testing.assert_allclose(X[nm][0, 0:6], d.x_ini[nm][0:6], atol=1e-12)
    assert all(np.isfinite(costs))


def test_dist_scvx_3d_failed_subproblem_aborts(cuda):
    """An infeasible sweep (trust region 1e-6 cannot absorb the straight-line start's dynamics defects)
    aborts, as the reference does (cvxpy SolverError, or `None.all()` at dist_scvx_3d.py:115)."""
    import pytest
    from Distributed_opt import dist_scvx_3d as d
    X0 = d.x_initial(d.x_ini, d.x_des)
    with pytest.raises(RuntimeError, match="solver_error"):
        d.x_traj_opt({k: v.copy() for k, v in X0.items()}, 1e-6)

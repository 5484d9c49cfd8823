"""GPU: the reference's SCvx solver surfaces on the MI355X backend.

Mirrors the reference tests SCvx/tests/test_sc_problem.py:10-52, SCvx/multi_agent_tests/
test_agent_solver.py:10-66 and SCvx/tests/test_scvx_solver.py:9-46 (shape / log / bounds contract),
and adds parity: the drop-in SCProblem's optimal value against oracle/scp_dense.py (the reference
formulation, sc_problem.py:15-83, solved by an independent conic IPM) on the same inputs (objective
relative 1e-7); the ADMM subproblem positions against the same oracle within the strong-convexity
bound; BatchedSCVXSolver against N independent SCVXSolver runs (bit-identical: one agent per
workgroup, so the batch does not change any agent's arithmetic)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _oracle_instance(model, Xref, Uref, sigma_ref, tr, x_init, x_final, **kw):
    from oracle import scp_problems as sp_
    return sp_.scp_instance(model, K=Xref.shape[1], Xref=Xref.T.copy(), Uref=Uref.T.copy(), sigma_ref=sigma_ref,
                            tr=tr, x_init=x_init, x_final=x_final, **kw)


def test_sc_problem_trivial_solve(cuda):
    """test_sc_problem.py:10-52 plus the optimal value against the reference formulation."""
    from oracle import scp_dense as sd
    from SCvx.discretization.first_order_hold import FirstOrderHold
    from SCvx.global_parameters import TRUST_RADIUS0, WEIGHT_NU, WEIGHT_SIGMA, WEIGHT_SLACK, K
    from SCvx.models.unicycle_model import UnicycleModel
    from SCvx.optimization.sc_problem import SCProblem
    model = UnicycleModel()
    X0, U0 = model.initialize_trajectory(np.zeros((model.n_x, K)), np.zeros((model.n_u, K)))
    foh = FirstOrderHold(model, K)
    A_bar, B_bar, C_bar, S_bar, z_bar = foh.calculate_discretization(X0, U0, 1.0)
    scp = SCProblem(model)
    scp.set_parameters(A_bar=A_bar, B_bar=B_bar, C_bar=C_bar, S_bar=S_bar, z_bar=z_bar, X_ref=X0, U_ref=U0,
                       sigma_ref=1.0, weight_nu=WEIGHT_NU, weight_slack=WEIGHT_SLACK, weight_sigma=WEIGHT_SIGMA,
                       tr_radius=TRUST_RADIUS0)
    assert not scp.solve(solver="ECOS", verbose=False)
    X, U, nu, sig = (scp.get_variable(k) for k in ("X", "U", "nu", "sigma"))
    assert X.shape == (3, K) and U.shape == (2, K) and nu.shape == (3, K - 1)
    assert np.isscalar(sig) or (isinstance(sig, np.ndarray) and sig.shape == ())
    assert scp.prob.status == "optimal"
    p = _oracle_instance("unicycle", X0, U0, 1.0, TRUST_RADIUS0, model.x_init, model.x_final)
    ref = sd.solve_scproblem(p, tol=1e-10)
    s_prime = np.stack([s.value[:, 0] for s in model.s_prime])
    obj = sd.scp_objective(p, X.T, U.T, nu.T, sig, s_prime=s_prime)
    assert abs(obj - ref["obj"]) <= 1e-7 * abs(ref["obj"]), (obj, ref["obj"])
    assert abs(scp.prob.value - ref["obj"]) <= 1e-7 * abs(ref["obj"])
    assert sd.scp_violation(p, X.T, U.T, nu.T, sig) < 1e-7


def test_agent_solver_basic_solve(cuda):
    """test_agent_solver.py:10-66 (with Y / Lambda assigned, which the reference test omits: an
    unassigned Parameter raises, as cvxpy does) plus positions against the reference formulation."""
    from oracle import scp_dense as sd, scp_problems as sp_
    from SCvx.discretization.first_order_hold import FirstOrderHold
    from SCvx.global_parameters import TRUST_RADIUS0, WEIGHT_NU, WEIGHT_SIGMA, K
    from SCvx.models.multi_agent_model import MultiAgentModel
    from SCvx.optimization.agent_solver import AgentSolver
    from SCvx.optimization.variables import ParameterError
    agent_params = [{"r_init": np.array([0.0, 0.0, 0.0]), "r_final": np.array([1.0, 1.0, 0.0])},
                    {"r_init": np.array([5.0, 5.0, 0.0]), "r_final": np.array([6.0, 6.0, 0.0])}]
    mam = MultiAgentModel(agent_params, d_min=1.0)
    solver = AgentSolver(agent_index=0, multi_agent_model=mam, rho_admm=1.0)
    a = np.linspace(0, 1, K)[None]
    X_ref_i = (1 - a) * agent_params[0]["r_init"][:, None] + a * agent_params[0]["r_final"][:, None]
    X_ref_j = (1 - a) * agent_params[1]["r_init"][:, None] + a * agent_params[1]["r_final"][:, None]
    U_ref_i = np.zeros((2, K))
    mats = FirstOrderHold(mam.models[0], K).calculate_discretization(X_ref_i, U_ref_i, sigma=1.0)
    mats = tuple(np.array(m_) for m_ in mats)
    solver.scp.par["weight_nu"].value = WEIGHT_NU
    solver.scp.par["weight_sigma"].value = WEIGHT_SIGMA
    solver.scp.par["tr_radius"].value = TRUST_RADIUS0
    solver.setup(X_ref_i, U_ref_i, sigma_ref_i=1.0, discretization_mats=mats, neighbor_refs={1: X_ref_j})
    with pytest.raises(ParameterError):
        solver.solve(solver="ECOS")
    rng = np.random.default_rng(7)
    Y = X_ref_j[0:2] + 0.1 * rng.standard_normal((2, K))
    Lam = 0.5 * rng.standard_normal((2, K))
    solver.Y[1].value, solver.Lambda[1].value = Y, Lam
    X_i, U_i, nu_i, slacks, p_i = solver.solve(solver="ECOS")
    assert X_i.shape == (3, K) and U_i.shape == (2, K) and nu_i.shape == (3, K - 1)
    assert isinstance(slacks, dict) and 1 in slacks and slacks[1].shape == (K, 1)
    assert p_i.shape == (2, K)
    p = _oracle_instance("unicycle", X_ref_i, U_ref_i, 1.0, TRUST_RADIUS0, agent_params[0]["r_init"],
                         agent_params[0]["r_final"])
    p = sp_.add_admm(p, [X_ref_j.T], Y=[Y.T], Lam=[Lam.T], rho=1.0, d_min=1.0)
    ref = sd.solve_scproblem(p, tol=1e-10)
    obj = sd.scp_objective(p, X_i.T, U_i.T, nu_i.T, float(solver.scp.get_variable("sigma")))
    assert abs(obj - ref["obj"]) <= 1e-7 * abs(ref["obj"]), (obj, ref["obj"])
    gap = abs(obj - ref["obj"]) + 1e-9 * abs(ref["obj"])
    assert np.abs(p_i.T - ref["X"][:, :2]).max() < np.sqrt(2.0 * gap) + 1e-6


def test_scvx_solver_runs_and_logs(cuda):
    """test_scvx_solver.py:9-46: shapes, record keys, finite non-negative norms, final position in the box;
    plus the loop's own rules: break-before-update and the trust-region schedule."""
    from SCvx.global_parameters import K
    from SCvx.models.unicycle_model import UnicycleModel
    from SCvx.optimization.scvx_solver import SCVXSolver
    model = UnicycleModel()
    solver = SCVXSolver(model)
    X, U, sigma, logger = solver.solve(verbose=False, initial_sigma=1.0)
    assert X.shape == (3, K) and U.shape == (2, K)
    assert np.isscalar(sigma)
    assert isinstance(logger.records, list) and len(logger.records) >= 1
    for rec in logger.records:
        assert set(rec) >= {"iter", "nu_norm", "slack_norm", "dx", "du", "ds", "sigma"}
        assert rec["nu_norm"] >= 0 and np.isfinite(rec["nu_norm"])
        assert rec["slack_norm"] >= 0 and np.isfinite(rec["slack_norm"])
    assert np.all(X[:2, -1] <= model.upper_bound + model.robot_radius)
    assert np.all(X[:2, -1] >= model.lower_bound - model.robot_radius)
    recs = logger.records
    tr = 100.0
    for rec in (recs[:-1] if _converged(recs[-1]) else recs):   # no update after the breaking iteration
        good = rec["nu_norm"] < 1e-2 and rec["slack_norm"] < 1e-2
        tr = max(min(tr * (1.5 if good else 1.2), 50.0), 1e-3)
    assert solver.tr_radius == pytest.approx(tr)


def _converged(rec, tol=1e-3):
    return rec["nu_norm"] < tol and rec["slack_norm"] < tol and rec["dx"] < tol and rec["ds"] < tol


def test_batched_scvx_matches_independent_runs(cuda):
    """N agents in lockstep == N single-agent SCVXSolver runs (per-agent trust radius, convergence)."""
    from SCvx.models.unicycle_model import UnicycleModel
    from SCvx.optimization.scvx_solver import BatchedSCVXSolver, SCVXSolver
    rng = np.random.default_rng(3)
    starts = [np.array([-8.0, -8.0, 0.0]) + np.r_[rng.uniform(-1, 1, 2), 0.0] for _ in range(4)]
    mk = lambda s: UnicycleModel(r_init=s, r_final=-s * np.array([1, 1, 0]))  # noqa: E731
    bat = BatchedSCVXSolver([mk(s) for s in starts])
    bat.max_iter = 6
    Xs, Us, ss, logs = bat.solve()
    for a, s in enumerate(starts):
        one = SCVXSolver(mk(s))
        one.max_iter = 6
        X1, U1, s1, lg = one.solve()
        assert np.array_equal(X1, Xs[a]) and np.array_equal(U1, Us[a]) and s1 == ss[a]
        assert [r["nu_norm"] for r in lg.records] == [r["nu_norm"] for r in logs[a].records]


def test_admm_coordinator_round_matches_oracle(cuda):
    """One Gauss-Seidel ADMM round (admm_coordinator.py:69-96) with 3 unicycle agents: every agent's
    positions against the reference formulation of its subproblem, built from the iterates the
    reference order feeds it; then the consensus / dual update arithmetic."""
    from oracle import scp_dense as sd, scp_problems as sp_
    from SCvx.global_parameters import K, TRUST_RADIUS0
    from SCvx.models.multi_agent_model import MultiAgentModel
    from SCvx.optimization.admm_coordinator import ADMMCoordinator
    params = [{"r_init": np.array([-8.0, -8.0, 0.0]), "r_final": np.array([8.0, 8.0, 0.0])},
              {"r_init": np.array([8.0, -8.0, np.pi / 2]), "r_final": np.array([-8.0, 8.0, np.pi / 2])},
              {"r_init": np.array([-8.0, 8.0, 0.0]), "r_final": np.array([8.0, -8.0, 0.0])}]
    mam = MultiAgentModel(params, d_min=1.0)
    coord = ADMMCoordinator(mam, rho_admm=1.0, max_iter=1)
    X_refs, U_refs = [], []
    for m in mam.models:
        X, U = m.initialize_trajectory(np.zeros((3, K)), np.zeros((2, K)))
        X_refs.append(X.copy())
        U_refs.append(U.copy())
    X_out, U_out, sig, ph, dh = coord.solve([x.copy() for x in X_refs], [u.copy() for u in U_refs], 1.0,
                                            verbose=False)
    assert len(ph) == 1 and len(dh) == 1 and sig == 1.0
    cur = [x.copy() for x in X_refs]
    for i, m in enumerate(mam.models):
        nb = [j for j in range(3) if j != i]
        p = _oracle_instance("unicycle", X_refs[i], U_refs[i], 1.0, TRUST_RADIUS0, m.x_init, m.x_final)
        p = sp_.add_admm(p, [cur[j].T for j in nb], Y=[X_refs[j][0:2].T for j in nb],
                         Lam=[np.zeros((K, 2)) for _ in nb], rho=1.0, d_min=1.0)
        ref = sd.solve_scproblem(p, tol=1e-10)
        solv = coord.agent_solvers[i]
        obj = sd.scp_objective(p, X_out[i].T, U_out[i].T, solv.scp.get_variable("nu").T,
                               float(solv.scp.get_variable("sigma")))
        assert abs(obj - ref["obj"]) <= 1e-7 * abs(ref["obj"]), (i, obj, ref["obj"])
        gap = abs(obj - ref["obj"]) + 1e-9 * abs(ref["obj"])
        assert np.abs(X_out[i][0:2].T - ref["X"][:, :2]).max() < np.sqrt(2.0 * gap / 2.0) + 1e-6
        cur[i] = X_out[i]
    pr = [np.linalg.norm(X_out[j][0:2] - 0.5 * (X_refs[j][0:2] + X_out[j][0:2])) for i in range(3) for j in range(3)
          if j != i]
    assert ph[0] == pytest.approx(np.mean(pr), rel=1e-12)
    s0 = coord.agent_solvers[0]
    assert np.allclose(s0.Lambda[1].value, 1.0 * (X_out[1][0:2] - s0.Y[1].value))


def test_si_admm_coordinator_jacobi_runs(cuda):
    """SI_ADMMCoordinator in the batched Jacobi schedule: one launch per round, finite residual history."""
    from SCvx.global_parameters import K
    from SCvx.models.SI_multi_agent_model import SI_MultiAgentModel
    from SCvx.optimization.si_admm_coordinator import SI_ADMMCoordinator
    params = [{"r_init": np.array([-8.0, -8.0, -8.0]), "r_final": np.array([8.0, 8.0, 8.0])},
              {"r_init": np.array([8.0, -8.0, -8.0]), "r_final": np.array([-8.0, 8.0, 8.0])}]
    mam = SI_MultiAgentModel(params, d_min=1.0)
    coord = SI_ADMMCoordinator(mam, rho_admm=1.0, max_iter=3, mode="jacobi")
    X_refs, U_refs = [], []
    for m in mam.models:
        X, U = m.initialize_trajectory(np.zeros((3, K)), np.zeros((3, K)))
        X_refs.append(X)
        U_refs.append(U)
    X_out, U_out, _, ph, dh = coord.solve(X_refs, U_refs, 1.0, verbose=False)
    assert len(ph) == 3 and all(np.isfinite(ph)) and all(np.isfinite(dh))
    for X, m in zip(X_out, mam.models):
        assert X.shape == (3, K) and np.allclose(X[:, 0], m.x_init) and np.allclose(X[:, -1], m.x_final)
        assert np.all(np.linalg.norm(np.diff(X, axis=1), axis=0) < 1e3)


def test_admm_consensus_kernel_matches_reference_update(cuda):
    """scvx_admm_consensus_batched vs the reference's host loop (admm_coordinator.py:80-91): the
    consensus and dual variables bit for bit, the residual norms (admm_utils.py) to rounding."""
    import torch
    import scvx_hip
    rng = np.random.default_rng(3)
    N, K, n, pd, rho = 5, 37, 6, 3, 0.7
    Xn = rng.normal(size=(N, K, n))
    nbr = np.array([[j for j in range(N) if j != i] for i in range(N)], np.int32)
    Y0 = rng.normal(size=(N, N - 1, K, pd))
    L0 = rng.normal(size=(N, N - 1, K, pd))
    T = lambda a, dt=torch.float64: torch.tensor(a, device=cuda, dtype=dt)  # noqa: E731
    Y, Lam = T(Y0), T(L0)
    pr, du = scvx_hip.admm_consensus(T(Xn), T(nbr, torch.int32), rho, Y, Lam, pd)
    Yh, Lh, prh, duh = Y.cpu().numpy(), Lam.cpu().numpy(), pr.cpu().numpy(), du.cpu().numpy()
    for i in range(N):
        for s, j in enumerate(nbr[i]):
            p_j = Xn[j][:, :pd].T                       # (pd, K), the reference's X_j[0:pd, :]
            Y_old = Y0[i, s].T
            Y_new = 0.5 * (Y_old + p_j)
            Lam_new = L0[i, s].T + rho * (p_j - Y_new)
            np.testing.assert_array_equal(Yh[i, s].T, Y_new)
            np.testing.assert_array_equal(Lh[i, s].T, Lam_new)
            assert prh[i, s] == pytest.approx(np.linalg.norm(p_j - Y_new), rel=1e-14)
            assert duh[i, s] == pytest.approx(np.linalg.norm(Y_new - Y_old), rel=1e-14)

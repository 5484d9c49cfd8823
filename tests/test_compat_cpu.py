"""CPU tests of the drop-in SCvx surface and the C-ABI (no GPU needed).

Known-answer tests restated from the reference suite:
  SCvx/multi_agent_tests/test_admm_utils.py:7-45, test_multi_agent_model.py:9-59,
  SCvx/tests/test_unicycle_model.py:10-64 (numpy parts)."""
import os
import re

import numpy as np
import pytest

from oracle import models_np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


# ---------------------------------------------------------------- admm_utils KATs
def test_primal_residual_zero():
    from SCvx.optimization.admm_utils import primal_residual
    assert primal_residual(np.zeros((2, 5)), np.zeros((2, 5))) == 0.0


def test_primal_residual_nonzero():
    from SCvx.optimization.admm_utils import primal_residual
    p = np.array([[1, 2, 3, 4, 5], [0, 0, 0, 0, 0]], dtype=float)
    assert primal_residual(p, np.zeros_like(p)) == pytest.approx(np.linalg.norm(p), rel=1e-6)


def test_dual_residual():
    from SCvx.optimization.admm_utils import dual_residual
    Y_new = np.array([[1, 1, 1, 1], [2, 2, 2, 2]], dtype=float)
    assert dual_residual(Y_new, np.zeros((2, 4))) == pytest.approx(np.linalg.norm(Y_new), rel=1e-6)


@pytest.mark.parametrize("rho0,pr,du,mu,ti,td,exp", [(1.0, 100.0, 1.0, 10.0, 3.0, 2.0, 3.0),
                                                     (10.0, 1.0, 100.0, 10.0, 3.0, 5.0, 2.0),
                                                     (2.0, 10.0, 1.0, 100.0, 4.0, 4.0, 2.0)])
def test_update_rho_admm(rho0, pr, du, mu, ti, td, exp):
    from SCvx.optimization.admm_utils import update_rho_admm
    assert update_rho_admm(rho0, primal_res=pr, dual_res=du, mu=mu, tau_inc=ti, tau_dec=td) == exp


# ---------------------------------------------------------------- multi-agent model KATs
def test_multi_agent_model_initialization():
    from SCvx.models.multi_agent_model import MultiAgentModel
    from SCvx.models.unicycle_model import UnicycleModel
    mam = MultiAgentModel([{"r_init": np.array([0.0, 0.0, 0.0]), "r_final": np.array([1.0, 1.0, 0.0])},
                           {"r_init": np.array([2.0, 2.0, 0.0]), "r_final": np.array([3.0, 3.0, 0.0])}], d_min=1.5)
    assert mam.N == 2 and mam.d_min == 1.5 and all(isinstance(m, UnicycleModel) for m in mam.models)


def test_linearize_collision_correctness():
    from SCvx.global_parameters import K
    from SCvx.models.multi_agent_model import MultiAgentModel
    d_min = 2.0
    mam = MultiAgentModel([{"r_init": np.array([0, d_min, 0]), "r_final": np.array([0, d_min, 0])},
                           {"r_init": np.array([0, 0, 0]), "r_final": np.array([0, 0, 0])}], d_min=d_min)
    X_i = np.tile(np.array([[0.0], [d_min], [0.0]]), (1, K))
    X_j = np.tile(np.array([[0.0], [0.0], [0.0]]), (1, K))
    A_ij, b_ij = mam.linearize_collision(0, 1, X_i, X_j)
    for k in range(K):
        assert np.allclose(A_ij[:, k], [0.0, 1.0], atol=1e-6)
        assert b_ij[k] == pytest.approx(d_min, rel=1e-6)


def test_si_linearize_matches_loop_form():
    from SCvx.models.SI_multi_agent_model import SI_MultiAgentModel
    rng = np.random.default_rng(0)
    mam = SI_MultiAgentModel([{}, {}], d_min=0.7)
    Xi, Xj = rng.normal(size=(3, 12)), rng.normal(size=(3, 12))
    A, b = mam.linearize_inter_agent_collision(0, 1, Xi, Xj)
    for k in range(12):  # SI_multi_agent_model.py:62-73 loop form
        diff = Xi[:, k] - Xj[:, k]
        a = diff / (np.linalg.norm(diff) + 1e-6)
        assert np.allclose(A[:, k], a) and b[k] == pytest.approx(0.7 + a @ Xj[:, k])


# ---------------------------------------------------------------- models
def test_unicycle_equation_shapes_and_values():
    from SCvx.global_parameters import K
    from SCvx.models.base_model import BaseModel
    from SCvx.models.unicycle_model import UnicycleModel
    model = UnicycleModel()
    assert isinstance(model, BaseModel)
    f, A, B = model.get_equations()
    x0, u0 = np.array([0.1, -0.2, 0.3]), np.array([0.5, -0.1])
    assert f(x0, u0).shape in [(3, 1), (3,)] and A(x0, u0).shape == (3, 3) and B(x0, u0).shape == (3, 2)
    fr, Ar, Br = models_np.unicycle_equations()
    assert np.allclose(f(x0, u0), fr(x0, u0)) and np.allclose(A(x0, u0), Ar(x0, u0)) and np.allclose(B(x0, u0), Br(x0, u0))
    X, U = model.initialize_trajectory(np.zeros((3, K)), np.zeros((2, K)))
    np.testing.assert_allclose(X[:, 0], model.x_init)
    np.testing.assert_allclose(X[:, -1], model.x_final)
    assert np.all(U == 0)


def test_quadrotor_jacobians_match_finite_differences():
    f, A, B = models_np.quad_equations()
    rng = np.random.default_rng(1)
    for _ in range(5):
        x = rng.normal(0, 0.3, 12)
        u = np.array([9.81, 0.01, -0.02, 0.005]) + rng.normal(0, 0.1, 4)
        Jx = np.stack([(f(x + e, u) - f(x - e, u)) / 2e-6 for e in np.eye(12) * 1e-6], axis=1)
        Ju = np.stack([(f(x, u + e) - f(x, u - e)) / 2e-6 for e in np.eye(4) * 1e-6], axis=1)
        assert np.abs(A(x, u) - Jx).max() < 1e-6 and np.abs(B(x, u) - Ju).max() < 1e-6
    from SCvx.models.quadrotor_model import QuadrotorModel
    q = QuadrotorModel()
    x = rng.normal(0, 0.3, 12)
    u = np.array([9.5, 0.01, 0.0, -0.01])
    assert np.allclose(q.f(x, u), f(x, u), atol=1e-12)


def test_dist_scvx_3d_zoh_matches_scipy():
    from scipy import signal
    from Distributed_opt import dist_scvx_3d as d
    A = np.zeros((6, 6)); A[0:3, 3:6] = np.eye(3)
    B = np.zeros((6, 3)); B[3:6] = np.eye(3)
    sysd = signal.StateSpace(A, B, np.eye(6), np.zeros((6, 3))).to_discrete(d.dt)
    assert np.abs(sysd.A - d.Ad).max() < 1e-12 and np.abs(sysd.B - d.Bd).max() < 1e-12
    assert d.T == 51 and d.R == 2.3 and d.trust_region == 0.25 and len(d.robots_name) == 3


# ---------------------------------------------------------------- C-ABI
def test_library_exports_every_header_symbol():
    import ctypes
    from scvx_hip import _lib
    hdr = open(os.path.join(REPO, "include", "scvx_hip.h")).read()
    declared = set(re.findall(r"^\w[\w\s\*]*?\b(scvx_\w+)\(", hdr, flags=re.M))
    assert {"scvx_foh_batched", "scvx_qp_solve_batched", "scvx_collision_rows_batched"} <= declared
    L = _lib.lib()
    for name in declared:
        assert hasattr(L, name), name
    assert set(_lib.EXPORTS) == declared
    assert L.scvx_version() >= 1
    # bad arguments are rejected without touching the GPU
    rc = L.scvx_foh_batched(0, None, 1, 4, None, None, None, 1, None, None)
    assert rc == -1 and b"bad args" in L.scvx_last_error()
    t = _lib.QPTemplate()
    t.K = 100
    assert L.scvx_qp_solve_batched(ctypes.byref(t), 1, *([None] * 17), None, 0, None) == -2
    assert L.scvx_version() >= 3   # v2: w_nu / w_prox template fields, the nu output; v3: scvx_rtc_*
    # the bindings' revision is the header's, and the loaded library's (lib() refuses any other)
    hv = int(re.search(r"#define SCVX_HIP_VERSION (\d+)", hdr).group(1))
    assert _lib.SCVX_HIP_VERSION == hv == L.scvx_version()


def test_first_order_hold_rejects_models_without_device_dynamics():
    """A model that neither names built-in device dynamics nor has traceable f/A/B (scvx_hip.rtc)."""
    from SCvx.discretization.first_order_hold import FirstOrderHold

    class Custom:
        n_x, n_u = 2, 1

        def get_equations(self):
            return None, None, None

    with pytest.raises(ValueError):
        FirstOrderHold(Custom(), 10)


# ---------------------------------------------------------------- SCProblem / AgentSolver host logic
def test_scproblem_surface_and_errors():
    """sc_problem.py:15-128 surface: var / par names and shapes, KeyError on unknown names,
    parameter shape validation, and the template data the kernel receives."""
    from SCvx.global_parameters import K
    from SCvx.models.unicycle_model import UnicycleModel
    from SCvx.optimization.sc_problem import SCProblem
    from SCvx.optimization.variables import ParameterError
    m = UnicycleModel()
    scp = SCProblem(m)
    assert set(scp.var) == {"X", "U", "nu", "sigma"}
    assert scp.var["X"].shape == (3, K) and scp.var["nu"].shape == (3, K - 1) and scp.var["sigma"].shape == ()
    assert set(scp.par) == {"A_bar", "B_bar", "C_bar", "S_bar", "z_bar", "X_ref", "U_ref", "sigma_ref", "weight_nu",
                            "weight_sigma", "tr_radius", "weight_slack"}
    assert scp.par["A_bar"].shape == (9, K - 1) and scp.par["B_bar"].shape == (6, K - 1)
    with pytest.raises(KeyError):
        scp.set_parameters(bogus=1.0)
    with pytest.raises(KeyError):
        scp.get_variable("Y")
    with pytest.raises(ValueError):
        scp.set_parameters(X_ref=np.zeros((2, K)))
    with pytest.raises(ValueError):
        scp.set_parameters(sigma_ref=-1.0)
    assert scp.get_variable("X") is None
    with pytest.raises(ParameterError):
        scp.spec()
    scp.set_parameters(weight_nu=1e4, weight_slack=1e6, weight_sigma=100.0)
    t = scp.spec().to_c()
    assert (t.n_x, t.n_u, t.K, t.pos_dim, t.n_obs, t.n_ubound, t.n_xbound) == (3, 2, K, 2, 3, 2, 2)
    assert t.obs_radius[0] == pytest.approx(3.5) and t.xb_lo[0] == pytest.approx(-9.5)
    assert (t.has_final, t.pin_u_first, t.pin_u_last, t.has_soc) == (1, 1, 1, 0)


def test_si_scproblem_template_has_soc():
    from SCvx.models.single_integrator_model import SingleIntegratorModel
    from SCvx.optimization.sc_problem import SCProblem
    scp = SCProblem(SingleIntegratorModel())
    scp.set_parameters(weight_nu=1e4, weight_slack=1e6, weight_sigma=100.0)
    t = scp.spec().to_c()
    assert (t.n_u, t.pos_dim, t.has_soc, t.n_obs, t.n_xbound) == (3, 3, 1, 2, 3)
    assert t.u_max == pytest.approx(1.0)


def test_agent_solver_surface():
    """agent_solver.py:10-41 / si_agent_solver.py:16-37: Y / Lambda / S per neighbour."""
    from SCvx.global_parameters import K
    from SCvx.models.SI_multi_agent_model import SI_MultiAgentModel
    from SCvx.models.multi_agent_model import MultiAgentModel
    from SCvx.optimization.agent_solver import AgentSolver
    from SCvx.optimization.si_agent_solver import SI_AgentSolver
    mam = MultiAgentModel([{"r_init": np.zeros(3), "r_final": np.ones(3)}] * 3, d_min=1.0)
    s = AgentSolver(1, mam, rho_admm=1.0)
    assert sorted(s.Y) == [0, 2] and s.Y[0].shape == (2, K) and s.S[2].shape == (K, 1)
    sim = SI_MultiAgentModel([{"r_init": np.zeros(3), "r_final": np.ones(3)}] * 2, d_min=1.0)
    s3 = SI_AgentSolver(0, sim, rho_admm=1.0)
    assert list(s3.Y) == [1] and s3.Lambda[1].shape == (3, K)
    with pytest.raises(RuntimeError):
        s3.solve()


def test_multi_agent_logging_format(capsys):
    from SCvx.utils.multi_agent_logging import print_iteration, print_summary
    print_iteration(3, 0.0, 0.0, 1.5, 0.25, 0.0, 0.0, 1.0, 1.0)
    print_summary(4, 1.0, runtime=2.5)
    out = capsys.readouterr().out
    assert out.startswith("Iter  3 | v=0.000e+00 | slack=0.000e+00 | p_res=1.500e+00 | d_res=2.500e-01 "
                          "| Δx=0.00e+00 | Δs=0.00e+00 | o= 1.000 | tr= 1.000\n")
    assert "\n=== SCvx+ADMM Summary ===\n  Total iterations: 4\n  Final time scale o: 1.000\n" in out
    assert "  Total runtime:    2.50s\n=========================\n" in out


# ---------------------------------------------------------------- bench workloads (host data)
def test_workload_constructions():
    """SURVEY §8d constructions: C4 lattice spacing exceeds 2R (no initial contact) and its goals are
    a permutation of the sites; C5 starts at hover thrust; C3 obstacles match the seeded spheres."""
    from scvx_hip import workloads
    c4 = workloads.synthetic_lattice(side=4, K=10, spacing=6.0)
    s, g = c4["x_init"][:, 0:3], c4["x_final"][:, 0:3]
    assert s.shape == (64, 6 // 2) and np.allclose(np.sort(s, 0), np.sort(g, 0))
    d = np.linalg.norm(s[:, None] - s[None], axis=-1) + np.eye(64) * 1e9
    assert d.min() > 2 * 2.3
    c5 = workloads.synthetic_quad(5, K=10, obstacles=3)
    assert c5["X"].shape == (5, 10, 12) and np.allclose(c5["U"][:, :, 0], 9.81) and len(c5["obs"]) == 3
    c3 = workloads.synthetic_di(7, K=10, obstacles=8)
    r = np.array([o[1] for o in c3["obs"]])
    assert c3["X"].shape == (7, 10, 6) and ((r >= 0.5) & (r <= 1.5)).all()


# ---------------------------------------------------------------- Parameter / Variable value shapes
def test_parameter_rejects_transposed_value():
    """cvxpy raises 'Invalid dimensions' for a value of the wrong shape; a transposed (K, n)
    trajectory for an (n, K) parameter must not be reshaped into a scrambled one."""
    from SCvx.optimization.variables import Parameter
    p = Parameter((3, 50))
    with pytest.raises(ValueError, match="Invalid dimensions"):
        p.value = np.zeros((50, 3))
    p.value = np.arange(150.0).reshape(3, 50)
    assert p.value.shape == (3, 50) and p.value[1, 0] == 50.0


def test_parameter_accepts_singleton_axes():
    from SCvx.optimization.variables import Parameter, Variable
    v = Variable((50, 1))
    v.value = np.ones(50)
    assert v.value.shape == (50, 1)
    s = Parameter(())
    s.value = np.array([2.5])
    assert s.value == 2.5


def test_initial_guess_matches_reference_goldens():
    """SCvx/utils/initial_guess.py restatement vs the reference's own outputs (tests/golden/
    make_initial_guess_goldens.py: the default 3-agent scenario + 21 seeded multi-obstacle cases)."""
    import os
    from SCvx.utils.initial_guess import initial_guess
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "initial_guess.npz"))
    for i in range(int(g["n"])):
        obs = [([o[0], o[1]], o[2]) for o in g[f"obs_{i}"]]
        X0, U0 = initial_guess(g[f"p0_{i}"], g[f"p1_{i}"], obs, float(g[f"clear_{i}"]), int(g[f"K_{i}"]))
        np.testing.assert_array_equal(X0, g[f"X0_{i}"])
        assert U0.shape == (2, int(g[f"K_{i}"])) and not U0.any()

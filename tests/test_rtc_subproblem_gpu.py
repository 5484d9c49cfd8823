"""GPU: the convex subproblems of a USER model (outside the built-in set), on kernels instantiated for its
dimensions at run time (csrc/subproblem_rtc.hip: csrc/qp_ipm.hpp and csrc/scp_kernel.hpp compiled by hipRTC
for (n_x, n_u) = (4, 2), model_id SCVX_MODEL_RUNTIME).

  * SCProblem (SCvx/optimization/sc_problem.py:15-83 drop-in) of the kinematic car of tests/custom_models.py,
    discretized by its runtime-compiled FOH, against the reference-form oracle (oracle/scp_dense.py):
    optimal value 1e-7 relative, constraint violation 1e-7 (the tolerances of tests/test_scp_gpu.py);
  * the trust-region QP (Distributed_opt/dist_scvx_3d.py:51-111 form, soft terminal) of the same car in
    JacobiSCvx's solver against the CPU twin (oracle/scvx_cpu.cpp, any (n, m)) on every agent (objective 1e-8
    relative) and the dense reference-form oracle (oracle/qp_dense.py) on a sample (objective 1e-7, violation
    1e-7)."""
import numpy as np
import pytest

import custom_models as cm

pytestmark = pytest.mark.gpu

X0, XF = np.array([-6.0, -2.0, 0.3, 0.0]), np.array([6.0, 3.0, 0.2, 0.0])
OBS = [(np.array([0.0, 1.2]), 1.5)]


class CarSCP(cm.KinematicCar):
    """The kinematic car with the constraint data SCProblem reads (the data of a reference model's
    get_constraints: boundary conditions, input bounds, a position box, one circular obstacle)."""

    def __init__(self, x_init=X0, x_final=XF):
        super().__init__()
        from SCvx.global_parameters import K
        from SCvx.optimization.variables import Variable
        self.x_init, self.x_final = np.asarray(x_init, float), np.asarray(x_final, float)
        self.s_prime = [Variable((K, 1), nonneg=True) for _ in OBS]

    def scp_constraints(self):
        return dict(pos_dim=2, x_init=self.x_init, x_final=self.x_final, u_bounds=[(0, -1.0, 1.0), (1, -0.5, 0.5)],
                    u_soc=None, x_bounds=[(0, -12.0, 12.0), (1, -12.0, 12.0)], obs=OBS)

    def initialize_trajectory(self, X, U):
        K = X.shape[1]
        a = np.linspace(0.0, 1.0, K)
        X = (1 - a)[None] * self.x_init[:, None] + a[None] * self.x_final[:, None]
        X[3] = np.linalg.norm(self.x_final[:2] - self.x_init[:2]) / 10.0
        return X, np.zeros((self.n_u, K))


def _ref_prob(A_bar, B_bar, C_bar, S_bar, z_bar, X, U, sigma, tr, n, m, cons):
    K = X.shape[1]
    F = lambda M, r, c: M.T.reshape(K - 1, c, r).transpose(0, 2, 1)  # noqa: E731  (order='F' columns)
    p = dict(cons, model="user", A=F(A_bar, n, n), B=F(B_bar, n, m), C=F(C_bar, n, m), S=S_bar.T.copy(), z=z_bar.T.copy(),
             Xref=X.T.copy(), Uref=U.T.copy(), sigma_ref=float(sigma), tr=float(tr), w_nu=1e4, w_slack=1e6, w_sigma=100.0)
    return p


def test_scproblem_of_a_user_model_matches_reference_formulation(cuda):
    from oracle import scp_dense as sd
    from SCvx.discretization.first_order_hold import FirstOrderHold
    from SCvx.global_parameters import K
    from SCvx.optimization.sc_problem import SCProblem
    from scvx_hip.rtc import DeviceModel
    car = CarSCP()
    foh = FirstOrderHold(car, K)
    assert isinstance(foh._name, DeviceModel) and foh._name.dims == (4, 2)
    X, U = car.initialize_trajectory(np.zeros((4, K)), np.zeros((2, K)))
    sigma = 10.0
    mats = [np.array(M) for M in foh.calculate_discretization(X, U, sigma)]
    scp = SCProblem(car)
    assert scp._dev_model is foh._name or scp._dev_model.source == foh._name.source
    scp.set_parameters(A_bar=mats[0], B_bar=mats[1], C_bar=mats[2], S_bar=mats[3], z_bar=mats[4], X_ref=X, U_ref=U,
                       sigma_ref=sigma, weight_nu=1e4, weight_sigma=100.0, weight_slack=1e6, tr_radius=5.0)
    assert scp.solve() is False
    assert scp.prob.status in ("optimal", "optimal_inaccurate"), scp.prob.status
    Xg, Ug, nug, sg = (np.asarray(scp.get_variable(k), float) for k in ("X", "U", "nu", "sigma"))
    assert Xg.shape == (4, K) and Ug.shape == (2, K) and nug.shape == (4, K - 1)
    p = _ref_prob(*mats, X, U, sigma, 5.0, 4, 2, car.scp_constraints())
    ref = sd.solve_scproblem(p, tol=1e-10)
    assert ref["status"] in ("optimal", "optimal_inaccurate") and ref["rel_gap"] <= 1e-8
    obj = sd.scp_objective(p, Xg.T, Ug.T, nug.T, float(sg))
    assert abs(obj - ref["obj"]) <= 1e-7 * abs(ref["obj"]), (obj, ref["obj"])
    assert abs(scp.prob.value - obj) <= 1e-7 * abs(obj)
    assert sd.scp_violation(p, Xg.T, Ug.T, nug.T, float(sg)) < 1e-7


def test_jacobi_qp_of_a_user_model_matches_twin_and_dense(cuda):
    import torch
    from oracle import problems as pb, qp_cpu, qp_dense as qd
    from scvx_hip import QPSolver, QPSpec
    from scvx_hip.rtc import DeviceModel
    car = cm.KinematicCar()
    dm = DeviceModel.from_callables(*car.get_equations(), 4, 2)
    N, K, sigma, tr = 16, 30, 10.0, 0.5
    rng = np.random.default_rng(7)
    a = np.linspace(0.0, 1.0, K)
    x0 = X0[None] + np.c_[rng.uniform(-1, 1, (N, 2)), np.zeros((N, 2))]
    xf = XF[None] + np.c_[rng.uniform(-1, 1, (N, 2)), np.zeros((N, 2))]
    X = (1 - a)[None, :, None] * x0[:, None] + a[None, :, None] * xf[:, None]
    X[:, 1:-1, 3] = 1.2                                     # X[:, 0] == x_init (the pinned first node)
    U = np.zeros((N, K, 2))
    T = lambda v: torch.tensor(np.ascontiguousarray(v), dtype=torch.float64, device=cuda)  # noqa: E731
    disc = dm.foh(T(X), T(U), T(np.full(N, sigma)))
    box = [(0, -12.0, 12.0), (1, -12.0, 12.0)]
    spec = QPSpec(model=dm, K=K, pos_dim=2, box=box, obs=OBS, w_obs=1e6, has_final=False, w_final=50.0, tol=1e-10,
                  max_iter=80)
    out = QPSolver(spec, N, device=cuda).solve(disc, T(np.full(N, sigma)), T(X), T(U), T(x0), T(xf), T(np.full(N, tr)))
    st = out["status"].cpu().numpy()
    assert (st == 0).all(), st
    dn = disc.cpu().numpy()
    tpl = qp_cpu.make_template(4, 2, K, pos_dim=2, box=box, obs=OBS, w_obs=1e6, has_final=False, w_final=50.0, tol=1e-10,
                               max_iter=80, model_id=255)
    cpu = qp_cpu.solve_batched(tpl, dn, np.full(N, sigma), X, U, x0, xf, np.full(N, tr))
    assert (cpu["status"] == 0).all()
    og, Xg, Ug = out["obj"].cpu().numpy(), out["X"].cpu().numpy(), out["U"].cpu().numpy()
    np.testing.assert_allclose(og, cpu["obj"], rtol=1e-8)
    for ag in (0, 5, 11):
        A, B, C, S, z = pb.unpack_disc(dn[ag], 4, 2)
        prob = dict(A=A, B=B, C=C, c=S * sigma + z, Xref=X[ag], Uref=U[ag], x_final=xf[ag], w_final=50.0, tr=tr,
                    box=box, obs=OBS, w_obs=1e6, fix_last_input=True, pos_dim=2)
        with np.errstate(all="ignore"):
            Xd, Ud, objd, info = qd.solve_agent(prob, sparse=True, tol=1e-11, maxit=150)
        assert info["status"] == "optimal", (ag, info["status"])
        # 1e-7 relative as the SCProblem parity (tests/test_scp_gpu.py): both solvers stop on gaps scaled by the
        # objective's largest weight (w_obs = 1e6), so their optimal values agree to ~1e-8 of it, not of obj
        assert abs(og[ag] - objd) <= 1e-7 * max(1.0, abs(objd)), (ag, og[ag], objd)
        assert max(qd.constraint_violation(prob, Xg[ag], Ug[ag]).values()) < 1e-7


@pytest.mark.parametrize("name,vc", [("unicycle_accel", True), ("triple_int", False), ("triple_int", True)])
def test_jacobi_qp_of_other_user_classes(cuda, name, vc):
    """The runtime QP classes the kernel builds for other (n_x, n_u): an odd n_x <= 8 with virtual control
    (UnicycleAccel, (5, 2)) and an n_x in 9..16 other than the built-in 12 (TripleInt3D, (9, 3): the dense packet /
    workspace row-state / descriptor-table path of the n > 8 classes), with and without virtual control.  Against
    the CPU twin on every agent (objective 1e-8 relative) and the dense reference-form oracle on a sample
    (objective 1e-7, violation 1e-7; virtual-control solutions are unique only up to the L1 penalty's
    degeneracy, so the value and feasibility are what is compared there, as tests/test_virtual_control_gpu.py)."""
    import torch
    from oracle import problems as pb, qp_cpu, qp_dense as qd
    from scvx_hip import QPSolver, QPSpec
    from scvx_hip.rtc import DeviceModel
    mdl = cm.UnicycleAccel() if name == "unicycle_accel" else cm.TripleInt3D()
    n, m = mdl.n_x, mdl.n_u
    dm = DeviceModel.from_callables(*mdl.get_equations(), n, m)
    N, K, sigma, tr = 12, 30, 8.0, 0.5
    rng = np.random.default_rng(11)
    pd = 2 if n == 5 else 3
    a = np.linspace(0.0, 1.0, K)
    x0 = np.zeros((N, n)); xf = np.zeros((N, n))
    lo, hi = (4, 6) if n == 5 else (2, 3)
    x0[:, :pd] = rng.uniform(-hi, -lo, (N, pd)); xf[:, :pd] = rng.uniform(lo, hi, (N, pd))
    if n == 5:
        xf[:, 2] = np.arctan2(xf[:, 1] - x0[:, 1], xf[:, 0] - x0[:, 0])
        x0[:, 2] = xf[:, 2]
    X = (1 - a)[None, :, None] * x0[:, None] + a[None, :, None] * xf[:, None]
    if n == 5:
        X[:, 1:-1, 3] = np.linalg.norm(xf[:, :2] - x0[:, :2], axis=1)[:, None] / sigma
    U = np.zeros((N, K, m))
    T = lambda v: torch.tensor(np.ascontiguousarray(v), dtype=torch.float64, device=cuda)  # noqa: E731
    disc = dm.foh(T(X), T(U), T(np.full(N, sigma)))
    box = [(0, -12.0, 12.0), (1, -12.0, 12.0)]
    obs = [(np.array([0.0, 0.5] + ([0.0] if pd == 3 else [])), 1.5 if n == 5 else 1.0)]
    extra = dict(w_nu=1e4, w_prox=1.0) if vc else {}
    tol = 1e-8 if vc else 1e-10   # virtual control: the bench's tolerance (tests/test_virtual_control_gpu.py: 1e-8/9)
    spec = QPSpec(model=dm, K=K, pos_dim=pd, box=box, obs=obs, w_obs=1e6, has_final=False, w_final=50.0, tol=tol,
                  max_iter=80, **extra)
    out = QPSolver(spec, N, device=cuda).solve(disc, T(np.full(N, sigma)), T(X), T(U), T(x0), T(xf), T(np.full(N, tr)))
    st = out["status"].cpu().numpy()
    # virtual control: an agent may end at Clarabel's reduced tolerances (measured: 1 of 12 on the (9, 3) class; as
    # tests/test_virtual_control_gpu.py, those are held to the reduced gap below)
    assert (st == 0).all() if not vc else ((st <= 1).all() and (st == 0).sum() >= N - 2), st
    dn = disc.cpu().numpy()
    tpl = qp_cpu.make_template(n, m, K, pos_dim=pd, box=box, obs=obs, w_obs=1e6, has_final=False, w_final=50.0,
                               tol=1e-8 if vc else 1e-10, max_iter=80, model_id=255, **extra)
    cpu = qp_cpu.solve_batched(tpl, dn, np.full(N, sigma), X, U, x0, xf, np.full(N, tr))
    assert (cpu["status"] == 0).all(), cpu["status"]
    og, Xg, Ug = out["obj"].cpu().numpy(), out["X"].cpu().numpy(), out["U"].cpu().numpy()
    print(name, vc, "status", st.tolist(), "max rel obj diff vs twin",
          np.max(np.abs(og - cpu["obj"]) / np.maximum(1.0, np.abs(cpu["obj"]))))
    np.testing.assert_allclose(og[st == 0], cpu["obj"][st == 0], rtol=1e-8)
    np.testing.assert_allclose(og[st == 1], cpu["obj"][st == 1], rtol=5e-5)   # Clarabel's reduced gap
    nug = out["nu"].cpu().numpy() if vc else None
    for ag in [a_ for a_ in range(N) if st[a_] == 0][:2]:
        A, B, C, S, z = pb.unpack_disc(dn[ag], n, m)
        prob = dict(A=A, B=B, C=C, c=S * sigma + z, Xref=X[ag], Uref=U[ag], x_final=xf[ag], w_final=50.0, tr=tr,
                    box=box, obs=obs, w_obs=1e6, fix_last_input=True, pos_dim=pd, **extra)
        with np.errstate(all="ignore"):
            Xd, Ud, objd, info = qd.solve_agent(prob, sparse=True, tol=1e-11, maxit=150)
        assert info["status"] == "optimal", (ag, info["status"])
        assert abs(og[ag] - objd) <= 1e-7 * max(1.0, abs(objd)), (ag, og[ag], objd)
        viol = qd.constraint_violation(prob, Xg[ag], Ug[ag], nu=nug[ag] if vc else None)
        assert max(viol.values()) < 1e-7, (ag, viol)

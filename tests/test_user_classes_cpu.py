"""CPU, no GPU: the kernel's CPU twin (oracle/scvx_cpu.cpp) on user-model QP classes beyond the built-in set --
an odd n_x <= 8 with virtual control (tests/custom_models.UnicycleAccel, (5, 2)) and an n_x in 9..16 other than 12
(TripleInt3D, (9, 3)), discretized by the generic FOH restatement (oracle/foh_generic.py) -- against the dense
reference-form oracle (oracle/qp_dense.py, Distributed_opt/dist_scvx_3d.py:51-111 with the soft terminal, box,
sphere and virtual-control rows): objective 1e-8 relative.  The same instances run through the runtime-compiled
kernel in tests/test_rtc_subproblem_gpu.py::test_jacobi_qp_of_other_user_classes."""
import numpy as np
import pytest

import custom_models as cm
from oracle import foh_generic as fg, problems as pb, qp_cpu, qp_dense as qd


def instance(name, vc):
    mdl = cm.UnicycleAccel() if name == "unicycle_accel" else cm.TripleInt3D()
    n, m = mdl.n_x, mdl.n_u
    N, K, sigma, tr = 12, 30, 8.0, 0.5
    rng = np.random.default_rng(11)
    pd = 2 if n == 5 else 3
    a = np.linspace(0.0, 1.0, K)
    x0, xf = np.zeros((N, n)), np.zeros((N, n))
    lo, hi = (4, 6) if n == 5 else (2, 3)
    x0[:, :pd] = rng.uniform(-hi, -lo, (N, pd))
    xf[:, :pd] = rng.uniform(lo, hi, (N, pd))
    if n == 5:
        xf[:, 2] = np.arctan2(xf[:, 1] - x0[:, 1], xf[:, 0] - x0[:, 0])
        x0[:, 2] = xf[:, 2]
    X = (1 - a)[None, :, None] * x0[:, None] + a[None, :, None] * xf[:, None]
    if n == 5:
        X[:, 1:-1, 3] = np.linalg.norm(xf[:, :2] - x0[:, :2], axis=1)[:, None] / sigma
    U = np.zeros((N, K, m))
    box = [(0, -12.0, 12.0), (1, -12.0, 12.0)]
    obs = [(np.array([0.0, 0.5] + ([0.0] if pd == 3 else [])), 1.5 if n == 5 else 1.0)]
    extra = dict(w_nu=1e4, w_prox=1.0) if vc else {}
    return mdl, n, m, N, K, sigma, tr, pd, X, U, x0, xf, box, obs, extra


@pytest.mark.parametrize("name,vc", [("unicycle_accel", True), ("triple_int", False), ("triple_int", True)])
def test_twin_user_classes_match_dense_oracle(name, vc):
    mdl, n, m, N, K, sigma, tr, pd, X, U, x0, xf, box, obs, extra = instance(name, vc)
    f, A_, B_ = mdl.get_equations()
    disc = np.stack([np.hstack([o.T for o in fg.foh(f, A_, B_, n, m, X[i].T, U[i].T, sigma)]) for i in range(N)])
    tpl = qp_cpu.make_template(n, m, K, pos_dim=pd, box=box, obs=obs, w_obs=1e6, has_final=False, w_final=50.0,
                               tol=1e-8 if vc else 1e-10, max_iter=80, model_id=255, **extra)
    cpu = qp_cpu.solve_batched(tpl, disc, np.full(N, sigma), X, U, x0, xf, np.full(N, tr))
    assert (cpu["status"] == 0).all(), cpu["status"]
    for ag in (0, 7):
        A, B, C, S, z = pb.unpack_disc(disc[ag], n, m)
        prob = dict(A=A, B=B, C=C, c=S * sigma + z, Xref=X[ag], Uref=U[ag], x_final=xf[ag], w_final=50.0, tr=tr,
                    box=box, obs=obs, w_obs=1e6, fix_last_input=True, pos_dim=pd, **extra)
        with np.errstate(all="ignore"):
            Xd, Ud, objd, info = qd.solve_agent(prob, sparse=True, tol=1e-11, maxit=150)
        assert info["status"] == "optimal", (ag, info["status"])
        assert abs(cpu["obj"][ag] - objd) <= 1e-8 * max(1.0, abs(objd)), (ag, cpu["obj"][ag], objd)

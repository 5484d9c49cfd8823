"""GPU parity of the runtime-compiled user-model FOH (scvx_hip.rtc.DeviceModel -> hipRTC ->
scvx_rtc_foh_batched / scvx_rtc_integrate_nonlinear_batched, include/scvx_hip.h), the model-agnostic
boundary of the reference's FirstOrderHold(model, K) (first_order_hold.py:13-50, 89-125):

  (1) golden vectors of the REFERENCE FirstOrderHold (LSODA) on three models outside the built-in set
      (tests/golden/make_rtc_foh_goldens.py): 1e-7 relative (the LSODA tolerance; roll-outs of the full
      trajectory 1e-6), as the built-in models are held (tests/test_foh_gpu.py);
  (2) the CPU restatement oracle/foh_generic.py (same RK4, pinned by (1)) on random batches: 1e-12;
  (3) a runtime-compiled unicycle against the built-in unicycle kernel: same integrator -> 1e-13;
  (4) the drop-in FirstOrderHold with a custom model class, end to end.
"""
import glob
import os

import numpy as np
import pytest

import custom_models as cm
import scvx_hip
from oracle import foh_generic

pytestmark = pytest.mark.gpu
GOLD = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "rtcfoh_*.npz")))


def rel(a, b):
    return np.max(np.abs(a - b)) / max(1.0, np.max(np.abs(b)))


def _t(x, cuda):
    import torch
    return torch.tensor(np.ascontiguousarray(x), dtype=torch.float64, device=cuda)


def _device_models(mdl):
    """Both construction routes: sympy with the parameters as launch params, and the re-traced callables
    (parameters inlined as constants)."""
    from scvx_hip.rtc import DeviceModel
    a = DeviceModel.from_sympy(mdl.x_sym, mdl.u_sym, mdl.f_param, p_syms=mdl.p_sym, params=list(mdl.params.values()))
    b = DeviceModel.from_callables(*mdl.get_equations(), mdl.n_x, mdl.n_u)
    return a, b


@pytest.mark.parametrize("path", GOLD, ids=[os.path.basename(p) for p in GOLD])
def test_rtc_foh_matches_reference_goldens(cuda, path):
    d = np.load(path)
    mdl = cm.MODELS[str(d["model"])]()
    X, U = _t(d["X"].T[None], cuda), _t(d["U"].T[None], cuda)
    for dm in _device_models(mdl):
        disc = dm.foh(X, U, _t([float(d["sigma"])], cuda))
        for name, o in zip(["A_bar", "B_bar", "C_bar", "S_bar", "z_bar"], dm.unpack_disc(disc)):
            o = o[0].cpu().numpy()
            assert o.shape == d[name].shape
            assert rel(o, d[name]) < 1e-7, name
        for pw, key in ((True, "X_piecewise"), (False, "X_full")):
            xo = dm.integrate_nonlinear(X, U, _t([float(d["sigma_nl"])], cuda), pw)[0].cpu().numpy().T
            assert rel(xo, d[key]) < (1e-7 if pw else 1e-6), key


@pytest.mark.parametrize("name", sorted(cm.MODELS))
def test_rtc_foh_matches_generic_oracle_batched(cuda, name):
    mdl = cm.MODELS[name]()
    n, m = mdl.n_x, mdl.n_u
    rng = np.random.default_rng(11)
    N, K = 37, 30
    X, U = rng.normal(0, 0.5, (N, K, n)), rng.normal(0, 0.5, (N, K, m))
    sig = rng.uniform(1.0, 4.0, N)
    f, A, B = mdl.get_equations()
    for dm in _device_models(mdl):
        disc = dm.foh(_t(X, cuda), _t(U, cuda), _t(sig, cuda))
        got = [o.cpu().numpy() for o in dm.unpack_disc(disc)]
        roll = dm.integrate_nonlinear(_t(X, cuda), _t(U, cuda), _t(sig, cuda), True).cpu().numpy()
        for a in (0, 18, 36):
            ref = foh_generic.foh(f, A, B, n, m, X[a].T, U[a].T, sig[a], nsub=16)
            for g, r in zip(got, ref):
                assert rel(g[a], r) < 1e-12
            xr = foh_generic.integrate_nonlinear(f, n, X[a].T, U[a].T, sig[a], True, nsub=16)
            assert rel(roll[a].T, xr) < 1e-12


def test_rtc_unicycle_equals_builtin_kernel(cuda):
    from scvx_hip.rtc import DeviceModel
    from SCvx.models.unicycle_model import UnicycleModel
    dm = DeviceModel.from_callables(*UnicycleModel().get_equations(), 3, 2)
    rng = np.random.default_rng(5)
    N, K = 64, 50
    X, U, sig = _t(rng.normal(0, 0.7, (N, K, 3)), cuda), _t(rng.normal(0, 0.5, (N, K, 2)), cuda), _t(rng.uniform(1, 5, N), cuda)
    a = dm.foh(X, U, sig, nsub=16).cpu().numpy()
    b = scvx_hip.foh_batched("unicycle", X, U, sig, nsub=16).cpu().numpy()
    assert rel(a, b) < 1e-13
    ra = dm.integrate_nonlinear(X, U, sig, False).cpu().numpy()
    rb = scvx_hip.integrate_nonlinear("unicycle", X, U, sig, False).cpu().numpy()
    assert rel(ra, rb) < 1e-13


def test_dropin_first_order_hold_with_custom_model(cuda):
    """A reference-style user model through the drop-in FirstOrderHold (no scvx_model attribute): the
    runtime path is taken automatically and reproduces the reference's own output (golden)."""
    from SCvx.discretization.first_order_hold import FirstOrderHold
    d = np.load([p for p in GOLD if "car" in p][0])
    foh = FirstOrderHold(cm.KinematicCar(), int(d["K"]))
    outs = foh.calculate_discretization(d["X"], d["U"], float(d["sigma"]))
    for name, o in zip(["A_bar", "B_bar", "C_bar", "S_bar", "z_bar"], outs):
        assert rel(o, d[name]) < 1e-7, name
    assert rel(foh.integrate_nonlinear_piecewise(d["X"], d["U"], float(d["sigma_nl"])), d["X_piecewise"]) < 1e-7
    assert rel(foh.integrate_nonlinear_full(d["X"][:, 0], d["U"], float(d["sigma_nl"])), d["X_full"]) < 1e-6


def test_rtc_params_change_without_recompile(cuda):
    """The launch params are runtime data: a different wheelbase gives the oracle's answer for it."""
    from scvx_hip.rtc import DeviceModel
    mdl = cm.KinematicCar()
    dm = DeviceModel.from_sympy(mdl.x_sym, mdl.u_sym, mdl.f_param, p_syms=mdl.p_sym, params=[2.5])
    rng = np.random.default_rng(2)
    X, U = rng.normal(0, 0.5, (1, 20, 4)), rng.normal(0, 0.3, (1, 20, 2))
    got = dm.unpack_disc(dm.foh(_t(X, cuda), _t(U, cuda), _t([3.0], cuda), params=[1.25]))
    import sympy as sp
    f1 = mdl.f_param.subs({mdl.p_sym[0]: 1.25})
    F, A, B = (sp.lambdify((sp.Matrix(mdl.x_sym), sp.Matrix(mdl.u_sym)), e, "numpy")
               for e in (f1, f1.jacobian(mdl.x_sym), f1.jacobian(mdl.u_sym)))
    ref = foh_generic.foh(F, A, B, 4, 2, X[0].T, U[0].T, 3.0, nsub=16)
    for g, r in zip(got, ref):
        assert rel(g[0].cpu().numpy(), r) < 1e-12

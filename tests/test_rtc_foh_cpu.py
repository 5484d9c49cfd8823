"""CPU, no GPU: the runtime-compiled user-model path (scvx_hip.rtc, include/scvx_hip.h scvx_rtc_*).

  * the CPU restatement oracle/foh_generic.py against golden vectors of the REFERENCE FirstOrderHold
    (first_order_hold.py:52-155, LSODA) on three models outside the built-in set
    (tests/golden/make_rtc_foh_goldens.py): pins the oracle the GPU tests use;
  * hipRTC compiles the generated kernels for gfx950 on a host without a GPU; structural zeros
    generate no code; a bad expression fails loudly with the compiler log;
  * symbolic re-tracing of numpy callables: reference-style sympy-lambdified models, the drop-in
    model classes (hand-written numpy), finite-difference Jacobians (differentiated from f);
  * the drop-in FirstOrderHold routes a custom model to the runtime path; SCProblem / BatchedSCVXSolver take
    it too (their kernels are instantiated for its dimensions at run time: tests/test_rtc_subproblem_gpu.py),
    the inter-sample search (built-in models only) rejects it loudly.
"""
import glob
import os

import numpy as np
import pytest
import sympy as sp

import custom_models as cm
from oracle import foh_generic

GOLD = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "rtcfoh_*.npz")))


def rel(a, b):
    return np.max(np.abs(a - b)) / max(1.0, np.max(np.abs(b)))


@pytest.mark.parametrize("path", GOLD, ids=[os.path.basename(p) for p in GOLD])
def test_generic_oracle_matches_reference_goldens(path):
    d = np.load(path)
    mdl = cm.MODELS[str(d["model"])]()
    f, A, B = mdl.get_equations()
    out = foh_generic.foh(f, A, B, mdl.n_x, mdl.n_u, d["X"], d["U"], float(d["sigma"]), nsub=16)
    for name, o in zip(["A_bar", "B_bar", "C_bar", "S_bar", "z_bar"], out):
        assert o.shape == d[name].shape
        assert rel(o, d[name]) < 1e-7, name
    for pw, key in ((True, "X_piecewise"), (False, "X_full")):
        xo = foh_generic.integrate_nonlinear(f, mdl.n_x, d["X"], d["U"], float(d["sigma_nl"]), pw, nsub=16)
        assert rel(xo, d[key]) < (1e-7 if pw else 1e-6), key


def test_generic_oracle_matches_builtin_c_oracle():
    """The numpy restatement and the C restatement (oracle/foh_ref.c) of the same integrator agree on a
    built-in model (unicycle), so the two oracles pin each other."""
    from oracle import foh_oracle
    x = sp.Matrix(sp.symbols("x y th", real=True))
    u = sp.Matrix(sp.symbols("v w", real=True))
    f = sp.Matrix([u[0] * sp.cos(x[2]), u[0] * sp.sin(x[2]), u[1]])
    F, A, B = (sp.lambdify((x, u), e, "numpy") for e in (f, f.jacobian(x), f.jacobian(u)))
    rng = np.random.default_rng(3)
    X, U = rng.normal(0, 0.7, (3, 20)), rng.normal(0, 0.5, (2, 20))
    a = foh_generic.foh(F, A, B, 3, 2, X, U, 4.0, nsub=16)
    b = foh_oracle.foh("unicycle", X, U, 4.0, nsub=16)
    for g, r in zip(a, b):
        assert rel(g, r) < 1e-13


def test_compile_without_gpu_and_structural_zeros():
    from scvx_hip.rtc import DeviceModel
    car = cm.KinematicCar()
    dm = DeviceModel.from_sympy(car.x_sym, car.u_sym, car.f_param, p_syms=car.p_sym, params=list(car.params.values()))
    assert dm.dims == (4, 2) and dm.params == (2.5,)
    src = dm.source
    assert 'extern "C" __global__' in src and "scvx_rtc_foh" in src and "scvx_rtc_nonlinear" in src
    # A has 5 nonzeros (d px/d th, d px/d v, d py/d th, d py/d v, d th/d v); the zero row is 0.0
    av = src[src.index("static void Av"):src.index("static void Bw")]
    assert av.count("* v_[") == 5 and "o_[3] = 0.0;" in av
    bw = src[src.index("static void Bw"):src.index("};")]
    assert bw.count("* w_[") == 2
    # one hipRTC compile per distinct model per process
    again = DeviceModel.from_sympy(car.x_sym, car.u_sym, car.f_param, p_syms=car.p_sym, params=[2.5])
    assert again._h is dm._h


def test_bad_expression_fails_with_compiler_log():
    from scvx_hip import ScvxError
    from scvx_hip.rtc import DeviceModel
    with pytest.raises(ScvxError) as e:
        DeviceModel(2, 1, ["x[1]", "u[0] + undefined_name"], A=[0, 1, 0, 0], B=[0, 1])
    assert "undefined_name" in str(e.value) and "generated source" in str(e.value)
    with pytest.raises(ValueError):
        DeviceModel(2, 1, ["x[1]"], A=[0, 1, 0, 0], B=[0, 1])          # wrong f length
    with pytest.raises(ValueError):
        DeviceModel(2, 1, ["x[1]", "u[0]"], A=[0, 1, 0], B=[0, 1])     # wrong A size
    with pytest.raises(ValueError):
        DeviceModel(17, 1, ["0"] * 17, A=["0"] * 289, B=["0"] * 17)    # beyond SCVX_RTC_MAX_NX


@pytest.mark.parametrize("name", sorted(cm.MODELS))
def test_retrace_of_lambdified_model_equals_its_expressions(name):
    """from_callables on a reference-style model (sympy-lambdified numpy f/A/B) recovers f and the
    model's own Jacobians (checked against the model's sympy expressions at random points)."""
    from scvx_hip.rtc import DeviceModel, _retrace
    mdl = cm.MODELS[name]()
    f, A, B = mdl.get_equations()
    xs = list(sp.symbols(f"xs0:{mdl.n_x}", real=True))
    us = list(sp.symbols(f"us0:{mdl.n_u}", real=True))
    sub = dict(zip(mdl.x_sym, xs))
    sub.update(zip(mdl.u_sym, us))
    fv = sp.Matrix(np.asarray(_retrace(f)(xs, us), dtype=object).reshape(mdl.n_x, 1).tolist())
    Av = sp.Matrix(np.asarray(_retrace(A)(xs, us), dtype=object).reshape(mdl.n_x, mdl.n_x).tolist())
    # equal as functions (lambdify prints the model's Float constants; compare at random points)
    rng = np.random.default_rng(0)
    for ref, got in ((mdl.f_expr, fv), (mdl.f_expr.jacobian(mdl.x_sym), Av)):
        diff = sp.lambdify((xs, us), got - ref.xreplace(sub), "numpy")
        for _ in range(5):
            assert np.abs(np.asarray(diff(rng.normal(size=mdl.n_x), rng.normal(size=mdl.n_u)), float)).max() < 1e-12
    dm = DeviceModel.from_callables(f, A, B, mdl.n_x, mdl.n_u)
    assert dm.dims == (mdl.n_x, mdl.n_u)


def test_retrace_of_dropin_models():
    """Hand-written numpy models (the drop-in unicycle: np.asarray(...).reshape, float(...)) and
    finite-difference Jacobians (the drop-in quadrotor: differentiated from the traced f)."""
    from scvx_hip.rtc import DeviceModel
    from SCvx.models.quadrotor_model import QuadrotorModel
    from SCvx.models.unicycle_model import UnicycleModel
    dm = DeviceModel.from_callables(*UnicycleModel().get_equations(), 3, 2)
    assert sum(e not in ("0", "0.0") for e in dm.A_exprs) == 2
    dq = DeviceModel.from_callables(*QuadrotorModel().get_equations(), 12, 4)
    assert dq.f_exprs[:3] == ["x[3]", "x[4]", "x[5]"]


def test_retrace_keeps_user_globals_that_share_a_math_name():
    """A model module's own constants named like a numpy / math object (a restitution `e = 0.8`, an exponent
    `power = 3.0`) stay the user's values; only numpy's and math's objects are re-bound to sympy."""
    import math
    from scvx_hip.rtc import _retrace
    g = {"np": np, "e": 0.8, "power": 3.0, "sin": np.sin, "pi": math.pi}
    exec("def f(x, u):\n    return np.array([x[1], -e * x[0] ** power + sin(pi * u[0])])", g)
    xs, us = sp.symbols("x0:2", real=True), sp.symbols("u0:1", real=True)
    got = np.asarray(_retrace(g["f"])(list(xs), list(us)), dtype=object)
    for x0, u0 in ((0.7, 0.3), (-1.3, 2.1)):
        want = -0.8 * x0 ** 3 + math.sin(math.pi * u0)
        assert abs(float(got[1].subs({xs[0]: x0, us[0]: u0})) - want) < 1e-12
    assert got[1].has(sp.sin) and got[1].has(sp.pi)


def test_untraceable_model_is_rejected():
    from scvx_hip.rtc import DeviceModel

    def f(x, u):
        if x[0] > 0:          # data-dependent branch: not a closed-form expression
            return np.array([x[1], u[0]])
        return np.array([-x[1], u[0]])
    with pytest.raises(ValueError, match="could not be traced"):
        DeviceModel.from_callables(f, f, f, 2, 1)


def test_first_order_hold_routes_custom_models():
    from scvx_hip.rtc import DeviceModel
    from SCvx.discretization.first_order_hold import builtin_model, device_model
    from SCvx.models.unicycle_model import UnicycleModel
    from SCvx.optimization.sc_problem import SCProblem
    assert device_model(UnicycleModel()) == "unicycle"
    car = cm.KinematicCar()
    dm = device_model(car)
    assert isinstance(dm, DeviceModel) and dm.dims == (4, 2)
    car.scvx_device_model = dm
    assert device_model(car) is dm
    with pytest.raises(NotImplementedError, match="runtime-compiled FOH path only"):
        builtin_model(car, "SCVXSolver")                # the kernels compiled per built-in model class
    from SCvx.discretization.first_order_hold import FirstOrderHold
    from SCvx.utils.intersample_collision import SegmentRollout
    seg = SegmentRollout(FirstOrderHold(car, 20), np.zeros(2), np.ones(2), 2.0)
    assert seg.model is dm                              # the inter-sample search: on the model's DeviceModel
    sp = SCProblem(car)                                 # the subproblem kernels take any (n_x, n_u) (hipRTC)
    assert sp._dev_model is dm
    from SCvx.discretization.first_order_hold import same_device_model
    assert same_device_model(dm, device_model(cm.KinematicCar())) and not same_device_model(dm, "unicycle")


@pytest.mark.parametrize("kind,cls", [(0, (4, 2, 2, 1, 0, 0)), (1, (4, 2, 0, 2))], ids=["qp_car", "scp_car"])
def test_runtime_subproblem_kernels_compile_without_gpu(kind, cls):
    """The subproblem kernels a user model's template is served by (model_id SCVX_MODEL_RUNTIME) compile
    through hipRTC from the headers embedded in the library (the classes tests/test_rtc_subproblem_gpu.py
    launches: the kinematic car's QP with 2 box rows + 1 obstacle, its SCProblem on 2 waves)."""
    import ctypes
    from scvx_hip import _lib
    L = _lib.lib()
    f = L.scvx_rtc_subproblem_compile
    f.restype = ctypes.c_int
    arr = (ctypes.c_int * len(cls))(*cls)
    nbytes = ctypes.c_size_t(0)
    rc = f(kind, arr, len(cls), ctypes.byref(nbytes))
    assert rc == 0, L.scvx_last_error().decode()
    assert nbytes.value > 10000
    assert f(0, arr, 3, None) != 0                     # wrong class length fails loudly

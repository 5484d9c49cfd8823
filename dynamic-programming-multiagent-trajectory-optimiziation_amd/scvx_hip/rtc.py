"""User dynamics models compiled for the MI355X at run time (hipRTC; include/scvx_hip.h scvx_rtc_*).

The reference's FirstOrderHold(model, K) discretizes ANY BaseModel through the numpy callables of
model.get_equations() (SCvx/discretization/first_order_hold.py:13-50, 89-125; SCvx/models/
base_model.py:16-24).  The library's built-in models (di, unicycle, si, quad) are compiled in; any
other model becomes a DeviceModel: its f, df/dx and df/du as HIP C expressions, compiled by hipRTC
into the same RK4 forward-sensitivity kernel (csrc/foh_body.hpp).  Three ways to build one:

  DeviceModel(n_x, n_u, f=[...], A=[...], B=[...], prelude="")   C expressions in x[i], u[j], p[k]
  DeviceModel.from_sympy(x_syms, u_syms, f_expr, p_syms=())      Jacobians derived, CSE'd, printed
  DeviceModel.from_callables(f, A, B, n_x, n_u)                  a reference-style model's own
                                                                 sympy-lambdified numpy callables,
                                                                 re-traced symbolically

There is no CPU path: compiling needs only the library, launching needs a ROCm device.
"""
import ctypes
import types

from . import _lib
from ._lib import ScvxError, check, lib

_CACHE = {}   # generated-source key -> compiled handle (one hipRTC compile per distinct model per process)


class _Handle:
    """Owns one scvx_rtc_model*."""

    def __init__(self, n_x, n_u, f, A, B, prelude):
        L = lib()
        arr = lambda xs: (ctypes.c_char_p * len(xs))(*[None if e is None else e.encode() for e in xs])  # noqa: E731
        self._keep = (arr(f), arr(A), arr(B))
        h = ctypes.c_void_p()
        rc = L.scvx_rtc_model_create(n_x, n_u, *self._keep, (prelude or "").encode(), ctypes.byref(h))
        self.ptr = h
        if rc != 0:
            log = L.scvx_rtc_model_log(h).decode(errors="replace") if h.value else ""
            src = L.scvx_rtc_model_source(h).decode(errors="replace") if h.value else ""
            if h.value:
                L.scvx_rtc_model_destroy(h)
                self.ptr = ctypes.c_void_p()
            raise ScvxError(f"hipRTC compile of the user model failed (code {rc}):\n{log}\n--- generated source ---\n{src}")
        self.source = L.scvx_rtc_model_source(h).decode()
        self.log = L.scvx_rtc_model_log(h).decode()

    def __del__(self):
        try:
            if self.ptr and self.ptr.value:
                lib().scvx_rtc_model_destroy(self.ptr)
        except Exception:
            pass


def _flat(M, rows, cols, what):
    """Nested (rows x cols) or flat row-major list of expression strings / numbers / None."""
    if M is None:
        raise ValueError(f"{what}: required (give C expressions, or use DeviceModel.from_sympy)")
    flat = [e for r in M for e in r] if len(M) == rows and rows and isinstance(M[0], (list, tuple)) else list(M)
    if len(flat) != rows * cols:
        raise ValueError(f"{what}: expected {rows}x{cols} entries, got {len(flat)}")
    return [None if e is None else str(e) for e in flat]


class DeviceModel:
    """A dynamics model x' = f(x, u; p) for the batched FOH / roll-out kernels, compiled with hipRTC.

    f: n_x C expressions; A: n_x x n_x, B: n_x x n_u (nested or flat row-major) C expressions of the
    Jacobians; structural zeros ("0" / None) generate no code.  Names: x[i], u[j], p[k] (p = the params
    of the launch, at most 16) and whatever `prelude` defines.  nsub: default RK4 substeps per FOH
    interval (16 holds the built-in nonlinear models within 1e-7 of the reference's LSODA)."""

    def __init__(self, n_x, n_u, f, A=None, B=None, prelude="", params=(), nsub=16, name="user"):
        n_x, n_u = int(n_x), int(n_u)
        if not (1 <= n_x <= _lib.SCVX_RTC_MAX_NX and 1 <= n_u <= _lib.SCVX_RTC_MAX_NU):
            raise ValueError(f"DeviceModel: need 1 <= n_x <= {_lib.SCVX_RTC_MAX_NX}, 1 <= n_u <= {_lib.SCVX_RTC_MAX_NU}")
        if len(params) > _lib.SCVX_MAX_MODEL_PARAMS:
            raise ValueError(f"DeviceModel: at most {_lib.SCVX_MAX_MODEL_PARAMS} params")
        self.n_x, self.n_u, self.name = n_x, n_u, name
        self.params = tuple(float(v) for v in params)
        self.nsub = int(nsub)
        fl = [str(e) for e in f]
        if len(fl) != n_x:
            raise ValueError(f"f: expected {n_x} expressions, got {len(fl)}")
        Al, Bl = _flat(A, n_x, n_x, "A"), _flat(B, n_x, n_u, "B")
        key = (n_x, n_u, tuple(fl), tuple(Al), tuple(Bl), prelude or "")
        h = _CACHE.get(key)
        if h is None:
            h = _CACHE[key] = _Handle(n_x, n_u, fl, Al, Bl, prelude)
        self._h = h
        self.f_exprs, self.A_exprs, self.B_exprs, self.prelude = fl, Al, Bl, prelude or ""

    @property
    def source(self):
        """The generated HIP source handed to hipRTC."""
        return self._h.source

    @property
    def dims(self):
        return self.n_x, self.n_u

    # ---- construction helpers -------------------------------------------------------------------
    @classmethod
    def from_sympy(cls, x_syms, u_syms, f_expr, p_syms=(), params=(), **kw):
        """f_expr: sympy column (or list) in x_syms / u_syms / p_syms; A = df/dx, B = df/du by sympy."""
        import sympy as sp
        xs, us = list(x_syms), list(u_syms)
        fm = sp.Matrix(f_expr).reshape(len(xs), 1)
        return cls._from_exprs(xs, us, list(p_syms), fm, fm.jacobian(xs), fm.jacobian(us), params=params, **kw)

    @classmethod
    def from_callables(cls, f, A, B, n_x, n_u, **kw):
        """Re-trace a model's numpy callables f(x, u), A(x, u), B(x, u) symbolically (the reference's
        models build them with sympy.lambdify(..., "numpy"), e.g. SCvx/models/unicycle_model.py:60-68):
        each function is re-bound to a namespace whose numpy names are sympy's and called on symbols.
        The model's own A and B are used when they trace; Jacobians that do not (finite differences,
        say) are the exact derivatives of the traced f.  Numeric constants are inlined as lambdify
        inlined them."""
        import sympy as sp
        xs = list(sp.symbols(f"xs0:{n_x}", real=True))
        us = list(sp.symbols(f"us0:{n_u}", real=True))
        import numpy as np
        mat = lambda v, r, c: sp.Matrix(np.asarray(v, dtype=object).reshape(r, c).tolist())  # noqa: E731
        try:
            fv = mat(_retrace(f)(xs, us), n_x, 1)
        except Exception as e:  # noqa: BLE001 -- any failure means: not symbolically traceable
            raise ValueError("the model's f callable could not be traced symbolically "
                             f"({type(e).__name__}: {e}); give DeviceModel C expressions or sympy expressions "
                             "(DeviceModel.from_sympy) and set model.scvx_device_model") from e
        try:
            Av = mat(_retrace(A)(xs, us), n_x, n_x)
            Bv = mat(_retrace(B)(xs, us), n_x, n_u)
        except Exception:  # noqa: BLE001 -- e.g. finite-difference Jacobians: differentiate the traced f
            Av, Bv = fv.jacobian(xs), fv.jacobian(us)
        return cls._from_exprs(xs, us, [], fv, Av, Bv, **kw)

    @classmethod
    def _from_exprs(cls, xs, us, ps, fm, Am, Bm, **kw):
        """Common subexpressions of f, A, B hoisted into the prelude (sympy.cse), printed with sympy.ccode
        in the kernel's names x[i], u[j], p[k]."""
        import sympy as sp
        sub = {s: sp.Symbol(f"x[{i}]", real=True) for i, s in enumerate(xs)}
        sub.update({s: sp.Symbol(f"u[{j}]", real=True) for j, s in enumerate(us)})
        sub.update({s: sp.Symbol(f"p[{k}]", real=True) for k, s in enumerate(ps)})
        exprs = [sp.sympify(e).xreplace(sub) for e in list(fm) + list(Am) + list(Bm)]
        reps, red = sp.cse(exprs, symbols=sp.numbered_symbols("c_"))
        pc = lambda e: sp.ccode(sp.sympify(e), standard="C99")  # noqa: E731
        prelude = "\n".join(f"const double {s} = {pc(e)};" for s, e in reps)
        n, m = len(xs), len(us)
        f = [pc(e) for e in red[:n]]
        A = ["0" if e == 0 else pc(e) for e in red[n:n + n * n]]
        B = ["0" if e == 0 else pc(e) for e in red[n + n * n:]]
        return cls(n, m, f, A, B, prelude=prelude, **kw)

    # ---- launches -------------------------------------------------------------------------------
    def _pp(self, params):
        import numpy as np
        p = self.params if params is None else tuple(float(v) for v in params)
        if len(p) > _lib.SCVX_MAX_MODEL_PARAMS:
            raise ValueError(f"at most {_lib.SCVX_MAX_MODEL_PARAMS} params")
        arr = np.ascontiguousarray(p if p else [0.0], dtype=np.float64)
        return arr, len(p)

    def foh(self, X, U, sigma, nsub=None, params=None, out=None, stream=None):
        """Batched FirstOrderHold.calculate_discretization: X (N,K,n), U (N,K,m), sigma (N,) float64
        device tensors -> disc (N, K-1, n(n+2m+2)) (layout of scvx_hip.foh_batched)."""
        from . import _dev, _stream, _torch
        torch = _torch()
        N, K, n = X.shape
        m = U.shape[2]
        if (n, m) != self.dims or tuple(U.shape[:2]) != (N, K) or tuple(sigma.shape) != (N,):
            raise ValueError(f"DeviceModel.foh: X (N,K,{self.n_x}), U (N,K,{self.n_u}), sigma (N,) expected; got "
                             f"{tuple(X.shape)}, {tuple(U.shape)}, {tuple(sigma.shape)}")
        if out is None:
            out = torch.empty((N, K - 1, n * (n + 2 * m + 2)), dtype=torch.float64, device=X.device)
        pa, npar = self._pp(params)
        rc = lib().scvx_rtc_foh_batched(self._h.ptr, pa.ctypes.data, npar, K, N, _dev(X, name="X"), _dev(U, name="U"),
                                        _dev(sigma, name="sigma"), int(nsub or self.nsub), _dev(out, name="out"),
                                        _stream(stream))
        check(rc, "scvx_rtc_foh_batched")
        return out

    def integrate_nonlinear(self, X, U, sigma, piecewise, nsub=16, params=None, out=None, stream=None):
        """Batched integrate_nonlinear_piecewise (piecewise=True) / integrate_nonlinear_full (False)."""
        from . import _dev, _stream, _torch
        torch = _torch()
        N, K, n = X.shape
        if (n, U.shape[2]) != self.dims or tuple(U.shape[:2]) != (N, K) or tuple(sigma.shape) != (N,):
            raise ValueError("DeviceModel.integrate_nonlinear: shapes do not match the model")
        if out is None:
            out = torch.empty((N, K, n), dtype=torch.float64, device=X.device)
        pa, npar = self._pp(params)
        rc = lib().scvx_rtc_integrate_nonlinear_batched(self._h.ptr, pa.ctypes.data, npar, K, N, _dev(X, name="X"),
                                                        _dev(U, name="U"), _dev(sigma, name="sigma"), int(nsub),
                                                        int(bool(piecewise)), _dev(out, name="out"), _stream(stream))
        check(rc, "scvx_rtc_integrate_nonlinear_batched")
        return out

    def unpack_disc(self, disc):
        """[..., K-1, n(n+2m+2)] -> (A_bar, B_bar, C_bar, S_bar, z_bar), as scvx_hip.unpack_disc."""
        n, m = self.dims
        o = [0, n * n, n * n + n * m, n * n + 2 * n * m, n * n + 2 * n * m + n, n * n + 2 * n * m + 2 * n]
        return tuple(disc[..., o[i]:o[i + 1]].transpose(-1, -2) for i in range(5))


# ---- symbolic re-tracing of numpy callables -------------------------------------------------------
# The callables are re-bound to a namespace in which numpy's elementwise math is sympy's and arrays are
# numpy OBJECT arrays of sympy expressions, so indexing, reshape, unpacking and stacking keep working.
def _sympy_math():
    import sympy as sp
    return dict(sin=sp.sin, cos=sp.cos, tan=sp.tan, arcsin=sp.asin, arccos=sp.acos, arctan=sp.atan,
                arctan2=sp.atan2, sinh=sp.sinh, cosh=sp.cosh, tanh=sp.tanh, exp=sp.exp, log=sp.log, sqrt=sp.sqrt,
                abs=sp.Abs, absolute=sp.Abs, fabs=sp.Abs, power=sp.Pow, sign=sp.sign, pi=sp.pi, e=sp.E,
                square=lambda a: a ** 2, hypot=lambda a, b: sp.sqrt(a ** 2 + b ** 2))


def _objarray(a, *_, **__):
    import numpy as np
    return np.array(a, dtype=object)


class _NumpyShim:
    """Stands in for the `numpy` / `np` module inside a re-traced function."""

    def __init__(self):
        import numpy as np
        self._np = np
        self._over = dict(_sympy_math(), array=_objarray, asarray=_objarray, asanyarray=_objarray,
                          zeros=lambda shape, *_, **__: np.zeros(shape, dtype=object),
                          ones=lambda shape, *_, **__: np.ones(shape, dtype=object),
                          eye=lambda k, *_, **__: np.eye(k, dtype=int).astype(object), float64=lambda a: a)

    def __getattr__(self, name):
        return self._over[name] if name in self._over else getattr(self._np, name)


def _is_math_name(k, v):
    """True when the global `k` holds numpy's or math's own object of that name (e.g. `from numpy import sin`,
    a lambdify namespace, `from math import e`); a user value that merely shares the name (a restitution
    coefficient `e = 0.8`, an exponent `power = 2.0`) is not re-bound."""
    import math
    import numpy as np
    for mod in (np, math):
        ref = getattr(mod, k, None)
        if ref is not None and v is ref:
            return True
    return False


def _retrace(fn):
    import numpy as np
    bound = getattr(fn, "__self__", None)
    fn = getattr(fn, "__func__", fn)
    shim = _NumpyShim()
    ns = dict(getattr(fn, "__globals__", {}))
    for k, v in list(ns.items()):
        if v is np:
            ns[k] = shim
        elif k in shim._over and _is_math_name(k, v):
            ns[k] = shim._over[k]
    ns["float"] = lambda a=0.0: a   # float(expr) of a traced scalar stays symbolic
    g = types.FunctionType(fn.__code__, ns, fn.__name__, fn.__defaults__, fn.__closure__)

    def call(X, U):
        args = (_objarray(list(X)), _objarray(list(U)))
        return g(bound, *args) if bound is not None else g(*args)
    return call

"""FirstOrderHold -- drop-in replacement of the reference SCvx/discretization/first_order_hold.py:5-162
whose integration runs in the batched HIP kernels (scvx_foh_batched / scvx_integrate_nonlinear_batched).

Same constructor, attributes (model, K, n_x, n_u, dt, f, A, B) and methods; same output layout
(A_bar (n*n, K-1), B_bar/C_bar (n*m, K-1), S_bar/z_bar (n, K-1), columns = order='F' vec of the
per-interval matrices, :75-85) and the same ownership rule: the returned arrays belong to the object
and are overwritten by the next call (:20-24, :87).  The reference integrates with LSODA; the kernels
use fixed-step RK4 on the equivalent forward-sensitivity system (agreement ~1e-8 relative, the
LSODA tolerance; tests/test_foh_gpu.py).  Models: the four built-in device models (attribute
`scvx_model`, or the drop-in model classes), or ANY other model -- its f/A/B are compiled for the GPU at
run time (scvx_hip.rtc.DeviceModel, hipRTC): `model.scvx_device_model` if the model provides one,
otherwise the model's own get_equations() callables re-traced symbolically (the reference's models are
sympy-lambdified numpy, which traces exactly).  There is no CPU fallback: a model that neither names
device dynamics nor traces is rejected.
"""
import numpy as np

import scvx_hip

_BY_CLASS = {"UnicycleModel": "unicycle", "SingleIntegratorModel": "si", "DoubleIntegratorModel": "di",
             "QuadrotorModel": "quad"}


def device_model(model):
    """Built-in model name ("di" | "unicycle" | "si" | "quad") or a runtime-compiled DeviceModel."""
    dm = getattr(model, "scvx_device_model", None)
    if dm is not None:
        if dm.dims != (model.n_x, model.n_u):
            raise ValueError(f"{type(model).__name__}: scvx_device_model dims {dm.dims} != (n_x, n_u)")
        return dm
    name = getattr(model, "scvx_model", "") or _BY_CLASS.get(type(model).__name__, "")
    if name:
        if name not in scvx_hip.MODEL_DIMS:
            raise ValueError(f"{type(model).__name__}: unknown device model {name!r} "
                             f"(built-in: {sorted(scvx_hip.MODEL_DIMS)})")
        if scvx_hip.MODEL_DIMS[name] != (model.n_x, model.n_u):
            raise ValueError(f"{type(model).__name__}: n_x/n_u do not match device model {name!r}")
        return name
    from scvx_hip.rtc import DeviceModel
    f, A, B = model.get_equations()
    return DeviceModel.from_callables(f, A, B, model.n_x, model.n_u)


def subproblem_model(model):
    """The device model the convex-subproblem kernels (QP / SCP) run: a built-in name, or for any other model
    its runtime-compiled DeviceModel -- those kernels depend only on (n_x, n_u) and are instantiated for them
    at the first solve (model_id SCVX_MODEL_RUNTIME, csrc/subproblem_rtc.hip)."""
    return device_model(model)


def same_device_model(a, b):
    """Two resolved device models describe one kernel class (built-in name, or equal generated source)."""
    if isinstance(a, str) or isinstance(b, str):
        return a == b
    return a is b or (a.dims == b.dims and a.source == b.source)


def builtin_model(model, what):
    """The built-in device model name of `model`, for the kernels that are compiled per model class
    (the SCP subproblem, the inter-sample search): any other model is rejected loudly, before anything is
    traced or compiled for it."""
    name = "" if getattr(model, "scvx_device_model", None) is not None else \
        (getattr(model, "scvx_model", "") or _BY_CLASS.get(type(model).__name__, ""))
    if not name:
        raise NotImplementedError(f"{what}: compiled for the built-in models {sorted(scvx_hip.MODEL_DIMS)}; "
                                  f"{type(model).__name__} runs on the runtime-compiled FOH path only")
    return device_model(model)   # validates the name and the dimensions


class FirstOrderHold:
    def __init__(self, model, K, device="cuda", nsub=None):
        self.model = model
        self.K = K
        self.n_x = model.n_x
        self.n_u = model.n_u
        self._name = device_model(model)
        self._params = getattr(model, "scvx_params", None)
        self._nsub = nsub
        self._device = device
        self.A_bar = np.zeros((self.n_x * self.n_x, K - 1))
        self.B_bar = np.zeros((self.n_x * self.n_u, K - 1))
        self.C_bar = np.zeros((self.n_x * self.n_u, K - 1))
        self.S_bar = np.zeros((self.n_x, K - 1))
        self.z_bar = np.zeros((self.n_x, K - 1))
        self.f, self.A, self.B = model.get_equations()
        self.dt = 1.0 / (K - 1)

    def nsub_for(self, sigma):
        """RK4 substeps of a call with this sigma: the constructor's nsub, else scvx_hip.default_nsub for the
        interval sigma / (K - 1) (the one count the FOH and the inter-sample roll-outs of this object share)."""
        return self._nsub or scvx_hip.default_nsub(self._name, float(sigma), self.K)

    def rollout_nsub(self, sigma):
        """RK4 substeps of the nonlinear roll-outs (integrate_nonlinear_*, the inter-sample segments): the
        constructor's nsub, else at least 16 (scvx_hip.integrate_nonlinear's default) and at least the FOH's count
        for this sigma."""
        if self._nsub:
            return self._nsub
        return max(16, self.nsub_for(sigma)) if isinstance(self._name, str) else self.nsub_for(sigma)

    def _to_dev(self, X, U, sigma):
        import torch
        Xd = torch.as_tensor(np.ascontiguousarray(np.asarray(X, float).T[None]), device=self._device)
        Ud = torch.as_tensor(np.ascontiguousarray(np.asarray(U, float).T[None]), device=self._device)
        sd = torch.full((1,), float(sigma), dtype=torch.float64, device=self._device)
        return Xd, Ud, sd

    def calculate_discretization(self, X, U, sigma):
        """X (n_x, K), U (n_u, K), sigma -> (A_bar, B_bar, C_bar, S_bar, z_bar)."""
        Xd, Ud, sd = self._to_dev(X, U, sigma)
        if isinstance(self._name, str):
            disc = scvx_hip.foh_batched(self._name, Xd, Ud, sd, nsub=self.nsub_for(sigma), params=self._params)
            outs = scvx_hip.unpack_disc(disc[0], self._name)
        else:
            disc = self._name.foh(Xd, Ud, sd, nsub=self._nsub, params=self._params)
            outs = self._name.unpack_disc(disc[0])
        for dst, src in zip((self.A_bar, self.B_bar, self.C_bar, self.S_bar, self.z_bar), outs):
            dst[...] = src.cpu().numpy()
        return self.A_bar, self.B_bar, self.C_bar, self.S_bar, self.z_bar

    # ---- caller-side batching (no reference counterpart; the reference integrates one agent per call)
    def calculate_discretization_device(self, Xd, Ud, sd, out=None):
        """Device-resident batch: Xd (M, K, n_x), Ud (M, K, n_u), sd (M,) float64 tensors on this object's
        device -> the packed per-interval matrices (M, K-1, n_x (n_x + 2 n_u + 2)) as a device tensor, one
        launch and no host transfer (unpack with self.unpack_disc); `out` is an optional buffer to reuse."""
        if isinstance(self._name, str):
            return scvx_hip.foh_batched(self._name, Xd, Ud, sd, nsub=self._nsub, params=self._params, out=out)
        return self._name.foh(Xd, Ud, sd, nsub=self._nsub, params=self._params, out=out)

    def unpack_disc(self, disc):
        """Packed device disc [..., K-1, n(n+2m+2)] -> (A_bar, B_bar, C_bar, S_bar, z_bar) views in the
        reference's F-order column layout."""
        if isinstance(self._name, str):
            return scvx_hip.unpack_disc(disc, self._name)
        return self._name.unpack_disc(disc)

    def calculate_discretization_batched(self, Xs, Us, sigmas):
        """calculate_discretization for M agents in one launch and one host round trip each way (a loop of
        M single-agent calls pays M of both).  Xs: M arrays (n_x, K), Us: M arrays (n_u, K), sigmas: M
        scalars.  Returns a list of M (A_bar, B_bar, C_bar, S_bar, z_bar) tuples of NEW arrays (the
        single-agent method's output buffers are not touched)."""
        import torch
        M = len(Xs)
        if len(Us) != M or len(sigmas) != M:
            raise ValueError("calculate_discretization_batched: Xs, Us and sigmas must have the same length")
        if M == 0:
            return []
        Xd = torch.as_tensor(np.ascontiguousarray(np.stack([np.asarray(x, float).T for x in Xs])), device=self._device)
        Ud = torch.as_tensor(np.ascontiguousarray(np.stack([np.asarray(u, float).T for u in Us])), device=self._device)
        sd = torch.as_tensor(np.asarray(sigmas, float).reshape(M), device=self._device)
        disc = self.calculate_discretization_device(Xd, Ud, sd)
        outs = [o.cpu().numpy() for o in self.unpack_disc(disc)]
        return [tuple(np.array(o[a]) for o in outs) for a in range(M)]

    def integrate_nonlinear_piecewise(self, X_lin, U, sigma):
        Xd, Ud, sd = self._to_dev(X_lin, U, sigma)
        out = self._roll(Xd, Ud, sd, True, self.rollout_nsub(sigma))
        return out[0].cpu().numpy().T.copy()

    def integrate_nonlinear_full(self, x0, U, sigma):
        X = np.zeros((self.n_x, self.K))
        X[:, 0] = np.asarray(x0, float).reshape(-1)
        Xd, Ud, sd = self._to_dev(X, U, sigma)
        out = self._roll(Xd, Ud, sd, False, self.rollout_nsub(sigma))
        return out[0].cpu().numpy().T.copy()

    def _roll(self, Xd, Ud, sd, piecewise, nsub):
        if isinstance(self._name, str):
            return scvx_hip.integrate_nonlinear(self._name, Xd, Ud, sd, piecewise, nsub=nsub, params=self._params)
        return self._name.integrate_nonlinear(Xd, Ud, sd, piecewise, nsub=nsub, params=self._params)

    def _dx(self, x, t, u0, u1, sigma):
        """Nonlinear dynamics in physical time with u interpolated by t/(dt*sigma) (:157-162); host-side,
        used by inter-sample utilities."""
        u = u0 + (t / (self.dt * sigma)) * (u1 - u0)
        return np.asarray(self.f(x, u), float).flatten()

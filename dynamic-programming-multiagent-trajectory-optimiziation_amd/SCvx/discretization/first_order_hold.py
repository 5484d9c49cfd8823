"""FirstOrderHold -- drop-in replacement of the reference SCvx/discretization/first_order_hold.py:5-162
whose integration runs in the batched HIP kernels (scvx_foh_batched / scvx_integrate_nonlinear_batched).

Same constructor, attributes (model, K, n_x, n_u, dt, f, A, B) and methods; same output layout
(A_bar (n*n, K-1), B_bar/C_bar (n*m, K-1), S_bar/z_bar (n, K-1), columns = order='F' vec of the
per-interval matrices, :75-85) and the same ownership rule: the returned arrays belong to the object
and are overwritten by the next call (:20-24, :87).  The reference integrates with LSODA; the kernels
use fixed-step RK4 on the equivalent forward-sensitivity system (agreement ~1e-8 relative, the
LSODA tolerance; tests/test_foh_gpu.py).  There is no CPU fallback: a model without device
dynamics (attribute `scvx_model`) is rejected.
"""
import numpy as np

import scvx_hip

_BY_CLASS = {"UnicycleModel": "unicycle", "SingleIntegratorModel": "si", "DoubleIntegratorModel": "di",
             "QuadrotorModel": "quad"}


def device_model(model):
    name = getattr(model, "scvx_model", "") or _BY_CLASS.get(type(model).__name__, "")
    if name not in scvx_hip.MODEL_DIMS:
        raise ValueError(f"{type(model).__name__}: no device dynamics for the MI355X FOH kernel "
                         f"(set model.scvx_model to one of {sorted(scvx_hip.MODEL_DIMS)})")
    if scvx_hip.MODEL_DIMS[name] != (model.n_x, model.n_u):
        raise ValueError(f"{type(model).__name__}: n_x/n_u do not match device model {name!r}")
    return name


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

    def _to_dev(self, X, U, sigma):
        import torch
        Xd = torch.as_tensor(np.ascontiguousarray(np.asarray(X, float).T[None]), device=self._device)
        Ud = torch.as_tensor(np.ascontiguousarray(np.asarray(U, float).T[None]), device=self._device)
        sd = torch.full((1,), float(sigma), dtype=torch.float64, device=self._device)
        return Xd, Ud, sd

    def calculate_discretization(self, X, U, sigma):
        """X (n_x, K), U (n_u, K), sigma -> (A_bar, B_bar, C_bar, S_bar, z_bar)."""
        Xd, Ud, sd = self._to_dev(X, U, sigma)
        disc = scvx_hip.foh_batched(self._name, Xd, Ud, sd, nsub=self._nsub, params=self._params)
        outs = scvx_hip.unpack_disc(disc[0], self._name)
        for dst, src in zip((self.A_bar, self.B_bar, self.C_bar, self.S_bar, self.z_bar), outs):
            dst[...] = src.cpu().numpy()
        return self.A_bar, self.B_bar, self.C_bar, self.S_bar, self.z_bar

    def integrate_nonlinear_piecewise(self, X_lin, U, sigma):
        Xd, Ud, sd = self._to_dev(X_lin, U, sigma)
        out = scvx_hip.integrate_nonlinear(self._name, Xd, Ud, sd, True, params=self._params)
        return out[0].cpu().numpy().T.copy()

    def integrate_nonlinear_full(self, x0, U, sigma):
        X = np.zeros((self.n_x, self.K))
        X[:, 0] = np.asarray(x0, float).reshape(-1)
        Xd, Ud, sd = self._to_dev(X, U, sigma)
        out = scvx_hip.integrate_nonlinear(self._name, Xd, Ud, sd, False, params=self._params)
        return out[0].cpu().numpy().T.copy()

    def _dx(self, x, t, u0, u1, sigma):
        """Nonlinear dynamics in physical time with u interpolated by t/(dt*sigma) (:157-162); host-side,
        used by inter-sample utilities."""
        u = u0 + (t / (self.dt * sigma)) * (u1 - u0)
        return np.asarray(self.f(x, u), float).flatten()

"""Inter-sample obstacle clearance -- drop-in for the reference SCvx/utils/intersample_collision.py.

Same functions and arguments: `h_i` (:7-26), `find_critical_times` (:29-67), `linearize_h`
(:70-101), `make_segment_f` (:104-126).  `make_segment_f` returns a `SegmentRollout`: callable as
`f(xk, u, t)` like the reference's closure, with its roll-out running on the GPU (fixed-step RK4
in scvx_integrate_nonlinear_batched instead of odeint).  When `find_critical_times` receives such a
segment, the whole scan (num_samples central differences, bisection, curvature test) runs as one
scvx_intersample_batched launch.

The batched entry point is `segment_minima(foh, X, U, obstacles, T, sigma)`: every segment x
obstacle of a trajectory in one launch, i.e. the data of the reference's per-segment loop in
SCvx/models/game_si_model.py:156-176 (`t*`, `h0`, `grad_x`, `grad_u` per minimum).

Any model the FirstOrderHold runs on the GPU is served: the built-in device models, and every other BaseModel
through its runtime-compiled DeviceModel (scvx_hip.rtc; the scan kernel is compiled next to the model's f,
scvx_rtc_intersample_batched) -- as the reference's scan integrates model.get_equations()'s f for any model.

A user-supplied Python callable `f` (not a `SegmentRollout`) can only run on the host.  For it, the
scan and the central differences are evaluated on the host by the same rules.
"""
from typing import Callable, List, Sequence, Tuple

import numpy as np

import scvx_hip



def _t(a, device):
    import torch
    return torch.as_tensor(np.ascontiguousarray(np.asarray(a, float)), dtype=torch.float64, device=device)


class SegmentRollout:
    """x(t) on segment [u0 -> u1] of a FirstOrderHold: dx/dtau = f(x, u0 + tau/dt_phys (u1 - u0)),
    tau in [0, t dt_phys], dt_phys = foh.dt * sigma (make_segment_f, :104-126)."""

    def __init__(self, foh, u0, u1, sigma):
        self.model = foh._name   # a built-in model name or the model's runtime-compiled DeviceModel
        self.params = getattr(foh.model, "scvx_params", None)
        self.device = getattr(foh, "_device", "cuda")
        self.u0 = np.asarray(u0, float).reshape(-1)
        self.u1 = np.asarray(u1, float).reshape(-1)
        self.sigma = float(sigma)
        self.foh_dt = float(foh.dt)
        self.dt_phys = self.foh_dt * self.sigma
        # one RK4 substep count for every roll-out of this segment: the critical-time scan (scvx_intersample_batched)
        # and the h0 / grad_x evaluations at t* (integrate_nonlinear) integrate the same discretisation
        self.nsub = foh.rollout_nsub(self.sigma)

    def __call__(self, xk, _u_dummy, t):
        # a one-interval roll-out whose interval is [0, t dt_phys] and whose end input is
        # u0 + t (u1 - u0): the interval's FOH interpolation is then exactly the segment's
        xk = np.asarray(xk, float).reshape(-1)
        X = _t(np.stack([xk, xk])[None], self.device)
        U = _t(np.stack([self.u0, self.u0 + t * (self.u1 - self.u0)])[None], self.device)
        s = _t([t * self.dt_phys], self.device)
        if isinstance(self.model, str):
            out = scvx_hip.integrate_nonlinear(self.model, X, U, s, True, nsub=self.nsub, params=self.params)
        else:
            out = self.model.integrate_nonlinear(X, U, s, True, nsub=self.nsub, params=self.params)
        return out[0, 1].cpu().numpy()


def make_segment_f(foh, U_ref_k: np.ndarray, U_ref_kp1: np.ndarray, sigma: float):
    """(f_seg, dt_phys) as the reference; f_seg(xk, _u, t) integrates from 0 to t * dt_phys."""
    seg = SegmentRollout(foh, U_ref_k, U_ref_kp1, sigma)
    return seg, seg.dt_phys


def h_i(xk, uk, t, f: Callable, T, obstacle) -> float:
    """Clearance ||T f(xk, uk, t) - p_c|| - r of the projected state."""
    p_c, r = obstacle
    return float(np.linalg.norm(np.asarray(T) @ np.asarray(f(xk, uk, t)) - np.asarray(p_c)) - r)


def _scan_device(seg: SegmentRollout, xk, T, obstacle, dt, num_samples, eps, tol):
    n = len(np.asarray(xk).reshape(-1))
    X = _t(np.stack([np.asarray(xk, float).reshape(-1)] * 2)[None], seg.device)
    U = _t(np.stack([seg.u0, seg.u1])[None], seg.device)
    sig = _t([seg.sigma], seg.device)
    out = scvx_hip.intersample_batched(seg.model, X, U, sig, [obstacle], proj=np.asarray(T, float).reshape(-1, n),
                                       dt=dt, seg_dt=seg.foh_dt, num_samples=num_samples, eps=eps, tol=tol,
                                       nsub=seg.nsub, params=seg.params)
    host = {k: v.cpu().numpy()[0, 0, 0] for k, v in out.items()}
    cnt = int(host["n_crit"])
    if cnt > host["t_crit"].shape[0]:
        raise RuntimeError(f"{cnt} interior minima on one segment exceed the kernel's max_crit")
    return host, cnt


def _scan_host(xk, uk, f, T, obstacle, dt, num_samples, eps, tol):
    """The reference's scan for an arbitrary host callable f (no device roll-out possible)."""
    def dphi(t):
        return (h_i(xk, uk, t + eps, f, T, obstacle) - h_i(xk, uk, t - eps, f, T, obstacle)) / (2 * eps)

    grid = np.linspace(eps, dt - eps, num_samples)
    d = np.array([dphi(t) for t in grid])
    roots = []
    for i in np.flatnonzero((d[:-1] == 0) | (d[:-1] * d[1:] < 0)):
        lo, hi = grid[i], grid[i + 1]
        for _ in range(30):
            mid = 0.5 * (lo + hi)
            lo, hi = (lo, mid) if dphi(lo) * dphi(mid) <= 0 else (mid, hi)
            if abs(hi - lo) < tol:
                break
        r = 0.5 * (lo + hi)
        if 0 < r < dt and (dphi(r + eps) - dphi(r - eps)) / (2 * eps) > 0:
            roots.append(r)
    return sorted(roots)


def find_critical_times(xk, uk, f: Callable, T, obstacle, dt: float, num_samples: int = 100, eps: float = 1e-4,
                        tol: float = 1e-6) -> List[float]:
    """Interior minima t* in (0, dt) of h_i (dh/dt = 0, d2h/dt2 > 0), ascending."""
    if isinstance(f, SegmentRollout):
        host, cnt = _scan_device(f, xk, T, obstacle, dt, num_samples, eps, tol)
        return [float(v) for v in host["t_crit"][:cnt]]
    return _scan_host(xk, uk, f, T, obstacle, dt, num_samples, eps, tol)


def linearize_h(xk, uk, t_star: float, f: Callable, T, obstacle, eps: float = 1e-4) -> Tuple[float, np.ndarray, np.ndarray]:
    """h0 = h_i(xk, uk, t*) and central-difference gradients w.r.t. xk and uk."""
    xk = np.asarray(xk, float).reshape(-1)
    uk = np.asarray(uk, float).reshape(-1)
    h0 = h_i(xk, uk, t_star, f, T, obstacle)
    gx = np.zeros_like(xk)
    for j in range(len(xk)):
        e = np.zeros_like(xk)
        e[j] = eps
        gx[j] = (h_i(xk + e, uk, t_star, f, T, obstacle) - h_i(xk - e, uk, t_star, f, T, obstacle)) / (2 * eps)
    gu = np.zeros_like(uk)
    if not isinstance(f, SegmentRollout):   # a SegmentRollout ignores its u argument: grad_u == 0
        for j in range(len(uk)):
            e = np.zeros_like(uk)
            e[j] = eps
            gu[j] = (h_i(xk, uk + e, t_star, f, T, obstacle) - h_i(xk, uk - e, t_star, f, T, obstacle)) / (2 * eps)
    return h0, gx, gu


def segment_minima(foh, X: np.ndarray, U: np.ndarray, obstacles: Sequence, T, sigma: float = 1.0, dt: float = 1.0,
                   num_samples: int = 100, eps: float = 1e-4, tol: float = 1e-6, max_crit: int = 8):
    """All segments x obstacles of one trajectory (X (n,K), U (m,K)) in one kernel launch:
    {(k, obstacle_index): [(t*, h0, grad_x, grad_u), ...]} -- what game_si_model.py:156-176
    computes with K-1 make_segment_f / find_critical_times / linearize_h rounds."""
    model = foh._name   # a built-in model name or the model's runtime-compiled DeviceModel
    dev = getattr(foh, "_device", "cuda")
    K = X.shape[1]
    out = scvx_hip.intersample_batched(model, _t(np.asarray(X, float).T[None], dev), _t(np.asarray(U, float).T[None], dev),
                                       _t([sigma], dev), list(obstacles), proj=T, dt=dt, seg_dt=foh.dt,
                                       num_samples=num_samples, eps=eps, tol=tol, max_crit=max_crit,
                                       nsub=foh.rollout_nsub(sigma), params=getattr(foh.model, "scvx_params", None))
    h = {k: v.cpu().numpy()[0] for k, v in out.items()}
    res = {}
    for k in range(K - 1):
        for o in range(len(obstacles)):
            c = int(h["n_crit"][k, o])
            if c > max_crit:
                raise RuntimeError(f"segment {k}, obstacle {o}: {c} minima exceed max_crit={max_crit}")
            res[(k, o)] = [(float(h["t_crit"][k, o, i]), float(h["h0"][k, o, i]), h["grad_x"][k, o, i].copy(),
                            h["grad_u"][k, o, i].copy()) for i in range(c)]
    return res

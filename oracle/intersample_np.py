"""ORACLE / TEST INFRASTRUCTURE ONLY -- CPU restatement of the inter-sample clearance scan
(SCvx/utils/intersample_collision.py: make_segment_f :104-126, h_i :7-26, find_critical_times
:29-67, linearize_h :70-101) with the kernel's fixed-step RK4 roll-outs in place of odeint.
Pinned to the reference itself by tests/golden/intersample_*.npz (made by importing the reference
module, tests/golden/make_intersample_goldens.py).  Never imported by the product path."""
import numpy as np

from . import models_np


def _rollout(f, x0, u0, u1, dtp, t, nsub):
    """x(t * dtp) of dx/dtau = f(x, u0 + tau/dtp (u1 - u0)) from x0 (FirstOrderHold._dx, :157-162)."""
    x = np.array(x0, float)
    hs = t * dtp / nsub

    def fx(tau, xs):
        return np.asarray(f(xs, u0 + (tau / dtp) * (u1 - u0)), float).reshape(-1)

    for s in range(nsub):
        tau = s * hs
        k1 = fx(tau, x)
        k2 = fx(tau + 0.5 * hs, x + 0.5 * hs * k1)
        k3 = fx(tau + 0.5 * hs, x + 0.5 * hs * k2)
        k4 = fx(tau + hs, x + hs * k3)
        x = x + (hs / 6.0) * (k1 + 2.0 * k2 + 2.0 * k3 + k4)
    return x


def segment(model, xk, u0, u1, dtp, T, center, radius, dt=1.0, num_samples=100, eps=1e-4, tol=1e-6, nsub=16):
    """Minima of one (segment, obstacle): list of (t*, h0, grad_x, grad_u)."""
    return segment_f(models_np.MODELS[model][2]()[0], xk, u0, u1, dtp, T, center, radius, dt, num_samples, eps, tol,
                     nsub)


def segment_f(f, xk, u0, u1, dtp, T, center, radius, dt=1.0, num_samples=100, eps=1e-4, tol=1e-6, nsub=16):
    """segment() for any model given as its numpy f(x, u) (a BaseModel's get_equations()[0])."""
    T = np.asarray(T, float)
    c = np.asarray(center, float)

    def h(x0, t):
        return float(np.linalg.norm(T @ _rollout(f, x0, u0, u1, dtp, t, nsub) - c) - radius)

    def phi(t):
        return (h(xk, t + eps) - h(xk, t - eps)) / (2.0 * eps)

    grid = np.linspace(eps, dt - eps, num_samples)
    vals = [phi(t) for t in grid]
    out = []
    for i in range(num_samples - 1):
        if not (vals[i] == 0.0 or vals[i] * vals[i + 1] < 0.0):
            continue
        lo, hi = grid[i], grid[i + 1]
        for _ in range(30):
            mid = 0.5 * (lo + hi)
            if phi(lo) * phi(mid) <= 0.0:
                hi = mid
            else:
                lo = mid
            if abs(hi - lo) < tol:
                break
        r = 0.5 * (lo + hi)
        if 0.0 < r < dt and (phi(r + eps) - phi(r - eps)) / (2.0 * eps) > 0.0:
            g = np.zeros(len(xk))
            for j in range(len(xk)):
                e = np.zeros(len(xk))
                e[j] = eps
                g[j] = (h(xk + e, r) - h(xk - e, r)) / (2.0 * eps)
            out.append((r, h(xk, r), g, np.zeros(len(u0))))
    return out

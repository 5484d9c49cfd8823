"""ORACLE / TEST INFRASTRUCTURE ONLY -- never imported by the product path.

CPU restatement, for ANY model given as numpy callables f(x,u), A(x,u), B(x,u) (the reference's
BaseModel.get_equations contract, SCvx/models/base_model.py:16-24), of the batched FOH and roll-out
kernels' algorithm (csrc/foh_body.hpp): classical RK4 with nsub fixed substeps on the
forward-sensitivity form of the reference's augmented ODE (first_order_hold.py:89-125):
    x'   = sigma f(x,u)
    col' = sigma A(x,u) (col - d_z x) + sigma B(x,u) w_c + d_S f(x,u)
with the columns [Phi | P_B | P_C | P_S | P_z] of one interval (w = alpha e_j for P_B, beta e_j for P_C,
-u for P_z).  At the end of the interval A_k = Phi, B_k = P_B, C_k = P_C, S_k = P_S, z_k = P_z, the
reference's Phi@B_mat ... (:75-85).  Roll-outs as first_order_hold.py:127-155 (physical time
[0, dt sigma], u interpolated by t/(dt sigma)).

Pinned against the reference FirstOrderHold itself: tests/golden/rtcfoh_*.npz
(tests/golden/make_rtc_foh_goldens.py, LSODA, 1e-7 relative; tests/test_rtc_foh_cpu.py).  Used by the
GPU tests of the runtime-compiled user-model path (scvx_hip.rtc) at the kernel's own accuracy (1e-12).
Pure numpy, one interval at a time: small sizes only.
"""
import numpy as np


def foh(f, A, B, n, m, X, U, sigma, nsub=16):
    """X (n,K), U (m,K) -> (A_bar (n*n,K-1), B_bar (n*m,K-1), C_bar, S_bar (n,K-1), z_bar), order='F'."""
    X, U = np.asarray(X, float), np.asarray(U, float)
    K = X.shape[1]
    dt = 1.0 / (K - 1)
    h = dt / nsub
    ncol = n + 2 * m + 2
    out = np.zeros((K - 1, n, ncol))
    fv = lambda x, u: np.asarray(f(x, u), float).reshape(n)  # noqa: E731
    Am = lambda x, u: np.asarray(A(x, u), float).reshape(n, n)  # noqa: E731
    Bm = lambda x, u: np.asarray(B(x, u), float).reshape(n, m)  # noqa: E731
    dS = np.zeros(ncol)
    dS[n + 2 * m] = 1.0
    dZ = np.zeros(ncol)
    dZ[n + 2 * m + 1] = 1.0
    for k in range(K - 1):
        u0, du = U[:, k], U[:, k + 1] - U[:, k]

        def rhs(t, x, C):
            beta = t / dt
            alpha = 1.0 - beta
            u = u0 + beta * du
            W = np.zeros((m, ncol))
            W[:, n:n + m] = alpha * np.eye(m)
            W[:, n + m:n + 2 * m] = beta * np.eye(m)
            W[:, n + 2 * m + 1] = -u
            fx = fv(x, u)
            dC = sigma * (Am(x, u) @ (C - np.outer(x, dZ)) + Bm(x, u) @ W) + np.outer(fx, dS)
            return sigma * fx, dC

        x = X[:, k].copy()
        C = np.zeros((n, ncol))
        C[:, :n] = np.eye(n)
        for s in range(nsub):
            t = s * h
            k1 = rhs(t, x, C)
            k2 = rhs(t + 0.5 * h, x + 0.5 * h * k1[0], C + 0.5 * h * k1[1])
            k3 = rhs(t + 0.5 * h, x + 0.5 * h * k2[0], C + 0.5 * h * k2[1])
            k4 = rhs(t + h, x + h * k3[0], C + h * k3[1])
            x = x + h / 6.0 * (k1[0] + 2 * k2[0] + 2 * k3[0] + k4[0])
            C = C + h / 6.0 * (k1[1] + 2 * k2[1] + 2 * k3[1] + k4[1])
        out[k] = C
    Ab = out[:, :, :n].transpose(0, 2, 1).reshape(K - 1, n * n).T          # vec_F(Phi)
    Bb = out[:, :, n:n + m].transpose(0, 2, 1).reshape(K - 1, n * m).T
    Cb = out[:, :, n + m:n + 2 * m].transpose(0, 2, 1).reshape(K - 1, n * m).T
    return (np.ascontiguousarray(Ab), np.ascontiguousarray(Bb), np.ascontiguousarray(Cb),
            np.ascontiguousarray(out[:, :, n + 2 * m].T), np.ascontiguousarray(out[:, :, n + 2 * m + 1].T))


def integrate_nonlinear(f, n, X, U, sigma, piecewise, nsub=16):
    """integrate_nonlinear_piecewise (piecewise=True, restart at X[:,k]) / _full (False): (n, K)."""
    X, U = np.asarray(X, float), np.asarray(U, float)
    K = X.shape[1]
    T = sigma / (K - 1)
    h = T / nsub
    out = np.zeros((n, K))
    out[:, 0] = X[:, 0]
    for k in range(K - 1):
        x = (X[:, k] if piecewise else out[:, k]).copy()
        u0, du = U[:, k], U[:, k + 1] - U[:, k]
        fx = lambda t, xs: np.asarray(f(xs, u0 + (t / T) * du), float).reshape(n)  # noqa: E731
        for s in range(nsub):
            t = s * h
            k1 = fx(t, x)
            k2 = fx(t + 0.5 * h, x + 0.5 * h * k1)
            k3 = fx(t + 0.5 * h, x + 0.5 * h * k2)
            k4 = fx(t + h, x + h * k3)
            x = x + h / 6.0 * (k1 + 2 * k2 + 2 * k3 + k4)
        out[:, k + 1] = x
    return out

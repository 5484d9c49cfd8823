"""ORACLE / TEST INFRASTRUCTURE ONLY: ctypes wrapper over oracle/foh_ref.c.

Mirrors the reference call surface FirstOrderHold(model, K).calculate_discretization(X, U, sigma)
(SCvx/discretization/first_order_hold.py:52-87) returning F-order (n*n, K-1) ... arrays.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "liboracle.so")
MODEL_IDS = {"di": 0, "unicycle": 1, "si": 2, "quad": 3}
MODEL_DIMS = {"di": (6, 3), "unicycle": (3, 2), "si": (3, 3), "quad": (12, 4)}
QUAD_PARAMS = np.array([1.0, 9.81, 0.02, 0.02, 0.04])

_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        _lib = ctypes.CDLL(LIB_PATH)
        dp = ctypes.POINTER(ctypes.c_double)
        _lib.oracle_foh.argtypes = [ctypes.c_int, dp, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                    dp, dp, ctypes.c_double, ctypes.c_int, dp]
        _lib.oracle_integrate_nonlinear.argtypes = [ctypes.c_int, dp, ctypes.c_int, ctypes.c_int,
                                                    ctypes.c_int, dp, dp, ctypes.c_double,
                                                    ctypes.c_int, ctypes.c_int, dp]
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


def foh(model, X, U, sigma, nsub=1, params=None):
    """X (n,K), U (m,K) -> A_bar (n^2,K-1), B_bar, C_bar (nm,K-1), S_bar, z_bar (n,K-1)."""
    n, m = MODEL_DIMS[model]
    K = X.shape[1]
    prm = np.ascontiguousarray(QUAD_PARAMS if params is None else params, dtype=np.float64)
    Xc = np.ascontiguousarray(X.T, dtype=np.float64)
    Uc = np.ascontiguousarray(U.T, dtype=np.float64)
    stride = n * n + 2 * n * m + 2 * n
    out = np.zeros((K - 1, stride))
    rc = lib().oracle_foh(MODEL_IDS[model], _p(prm), n, m, K, _p(Xc), _p(Uc), float(sigma), nsub, _p(out))
    if rc != 0:
        raise ValueError("oracle_foh failed")
    o = np.cumsum([0, n * n, n * m, n * m, n, n])
    return tuple(np.ascontiguousarray(out[:, o[i]:o[i + 1]].T) for i in range(5))


def foh_disc(model, X, U, sigma, nsub=1, params=None):
    """X (K,n), U (K,m) agent-major -> disc (K-1, n(n+2m+2)), per interval vec_F(A) | vec_F(B) | vec_F(C) | S | z
    (the layout of include/scvx_hip.h scvx_foh_batched)."""
    n, m = MODEL_DIMS[model]
    K = X.shape[0]
    prm = np.ascontiguousarray(QUAD_PARAMS if params is None else params, dtype=np.float64)
    Xc = np.ascontiguousarray(X, dtype=np.float64)
    Uc = np.ascontiguousarray(U, dtype=np.float64)
    out = np.zeros((K - 1, n * n + 2 * n * m + 2 * n))
    rc = lib().oracle_foh(MODEL_IDS[model], _p(prm), n, m, K, _p(Xc), _p(Uc), float(sigma), nsub, _p(out))
    if rc != 0:
        raise ValueError("oracle_foh failed")
    return out


def integrate_nonlinear(model, X, U, sigma, piecewise, nsub=16, params=None):
    n, m = MODEL_DIMS[model]
    K = X.shape[1]
    prm = np.ascontiguousarray(QUAD_PARAMS if params is None else params, dtype=np.float64)
    Xc = np.ascontiguousarray(X.T, dtype=np.float64)
    Uc = np.ascontiguousarray(U.T, dtype=np.float64)
    out = np.zeros((K, n))
    rc = lib().oracle_integrate_nonlinear(MODEL_IDS[model], _p(prm), n, m, K, _p(Xc), _p(Uc),
                                          float(sigma), nsub, int(piecewise), _p(out))
    if rc != 0:
        raise ValueError("oracle_integrate_nonlinear failed")
    return out.T.copy()

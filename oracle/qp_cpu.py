"""ORACLE / TEST INFRASTRUCTURE ONLY: ctypes wrapper of oracle/scvx_cpu.cpp (CPU restatement of the
batched trust-region subproblem, include/scvx_hip.h scvx_qp_solve_batched).  Used by tests/ and by
bench.py's cpu_baseline leg (kind "port")."""
import ctypes

import numpy as np

from . import foh_oracle

MAX_BOX, MAX_OBS = 4, 16


class QPTemplate(ctypes.Structure):
    _fields_ = [
        ("model_id", ctypes.c_int32), ("n_x", ctypes.c_int32), ("n_u", ctypes.c_int32), ("K", ctypes.c_int32),
        ("pos_dim", ctypes.c_int32), ("has_final", ctypes.c_int32), ("fix_last_input", ctypes.c_int32),
        ("ineq_last", ctypes.c_int32), ("w_last", ctypes.c_double), ("n_box", ctypes.c_int32),
        ("box_idx", ctypes.c_int32 * MAX_BOX), ("box_lo", ctypes.c_double * MAX_BOX),
        ("box_hi", ctypes.c_double * MAX_BOX), ("n_obs", ctypes.c_int32),
        ("obs_center", (ctypes.c_double * 3) * MAX_OBS), ("obs_radius", ctypes.c_double * MAX_OBS),
        ("w_obs", ctypes.c_double), ("j_max", ctypes.c_int32), ("w_coll", ctypes.c_double),
        ("has_soc", ctypes.c_int32), ("u_max", ctypes.c_double), ("max_iter", ctypes.c_int32),
        ("tol", ctypes.c_double), ("w_final", ctypes.c_double), ("w_nu", ctypes.c_double),
        ("w_prox", ctypes.c_double),
    ]


def make_template(n, m, K, pos_dim=3, has_final=True, fix_last_input=True, ineq_last=False, w_last=0.0,
                  box=(), obs=(), w_obs=1e6, j_max=0, w_coll=1e4, u_max=None, max_iter=60, tol=1e-9,
                  model_id=0, w_final=0.0, w_nu=0.0, w_prox=0.0):
    t = QPTemplate()
    t.model_id, t.n_x, t.n_u, t.K, t.pos_dim = model_id, n, m, K, pos_dim
    t.has_final, t.fix_last_input, t.ineq_last, t.w_last = int(has_final), int(fix_last_input), int(ineq_last), w_last
    t.n_box = len(box)
    for i, (bi, lo, hi) in enumerate(box):
        t.box_idx[i], t.box_lo[i], t.box_hi[i] = bi, lo, hi
    t.n_obs = len(obs)
    for o, (c, r) in enumerate(obs):
        for i in range(len(c)):
            t.obs_center[o][i] = c[i]
        t.obs_radius[o] = r
    t.w_obs, t.j_max, t.w_coll = w_obs, j_max, w_coll
    t.has_soc = int(u_max is not None)
    t.u_max = 0.0 if u_max is None else u_max
    t.max_iter, t.tol = max_iter, tol
    t.w_final = w_final
    t.w_nu = w_nu
    t.w_prox = w_prox
    return t


def _p(a, ty=ctypes.c_double):
    return a.ctypes.data_as(ctypes.POINTER(ty))


def warm_doubles(tpl):
    lib = foh_oracle.lib()
    lib.oracle_qp_warm_doubles.restype = ctypes.c_longlong
    return int(lib.oracle_qp_warm_doubles(ctypes.byref(tpl)))


def solve_batched(tpl, disc, sigma, Xref, Uref, x_init, x_final, tr, coll_rows=None, coll_count=None, nthreads=1,
                  warm=None, wstate=None):
    """warm (N,) int32 / wstate (N, warm_doubles(tpl)) float64 (experiment): agents with warm[a] != 0 start
    from the primal-dual state a previous call left in wstate[a]; every call writes its final state there."""
    """All arrays agent-major numpy float64 (see include/scvx_hip.h).  Returns dict of outputs."""
    lib = foh_oracle.lib()
    if not hasattr(lib, "_qp_ready"):
        lib.oracle_qp_solve_batched.restype = ctypes.c_int
        lib._qp_ready = True
    N, K, n = Xref.shape
    m = Uref.shape[2]
    c = np.ascontiguousarray
    disc, sigma, Xref, Uref = c(disc, np.float64), c(sigma, np.float64), c(Xref, np.float64), c(Uref, np.float64)
    x_init, x_final, tr = c(x_init, np.float64), c(x_final, np.float64), c(tr, np.float64)
    if coll_rows is None:
        coll_rows = np.zeros(1)
        coll_count = np.zeros(1, np.int32)
    coll_rows, coll_count = c(coll_rows, np.float64), c(coll_count, np.int32)
    X = np.zeros((N, K, n)); U = np.zeros((N, K, m)); S = np.zeros((N, K)); obj = np.zeros(N)
    nu = np.zeros((N, K - 1, n))
    st = np.zeros(N, np.int32); it = np.zeros(N, np.int32)
    rc = lib.oracle_qp_solve_batched(ctypes.byref(tpl), N, _p(disc), _p(sigma), _p(Xref), _p(Uref), _p(x_init),
                                     _p(x_final), _p(tr), _p(coll_rows), _p(coll_count, ctypes.c_int32), _p(X),
                                     _p(U), _p(S), _p(nu), _p(obj), _p(st, ctypes.c_int32), _p(it, ctypes.c_int32),
                                     int(nthreads),
                                     _p(warm, ctypes.c_int32) if warm is not None else None,
                                     _p(wstate) if wstate is not None else None)
    if rc != 0:
        raise ValueError("oracle_qp_solve_batched failed")
    return dict(X=X, U=U, slack_coll=S, nu=nu, obj=obj, status=st, iters=it)

"""ctypes binding of libscvx_hip.so (include/scvx_hip.h).

The library is the product: there is no CPU fallback.  Importing works without a GPU (so the
C-ABI can be checked on a build host); compute calls need a ROCm device and raise otherwise.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SCVX_HIP_LIB") or os.path.join(HERE, "libscvx_hip.so")  # override: diagnostics builds

# the C-ABI revision these bindings are written for (SCVX_HIP_VERSION of include/scvx_hip.h): a library of
# another revision would take these argument lists with shifted pointers, so lib() refuses it
SCVX_HIP_VERSION = 6
SCVX_MAX_BOX, SCVX_MAX_OBS, SCVX_MAX_NBR = 4, 16, 32
SCVX_IS_MAX_PROJ, SCVX_IS_MAX_STATE = 3, 12
MODEL_IDS = {"di": 0, "unicycle": 1, "si": 2, "quad": 3}
MODEL_DIMS = {"di": (6, 3), "unicycle": (3, 2), "si": (3, 3), "quad": (12, 4)}
SCVX_MODEL_RUNTIME = 255   # any other model: the subproblem kernels are compiled for its (n_x, n_u) at run time
STATUS = {0: "optimal", 1: "optimal_inaccurate", 2: "solver_error"}

# every symbol declared in include/scvx_hip.h
EXPORTS = ("scvx_version", "scvx_last_error", "scvx_foh_batched", "scvx_integrate_nonlinear_batched",
           "scvx_qp_solve_batched", "scvx_qp_solve_batched_ordered", "scvx_qp_workspace_bytes", "scvx_qp_set_trace",
           "scvx_collision_rows_batched", "scvx_collision_rows_indexed", "scvx_collision_check_batched", "scvx_scp_solve_batched", "scvx_scp_workspace_bytes",
           "scvx_intersample_batched", "scvx_admm_consensus_batched", "scvx_scp_game_solve_batched",
           "scvx_slab_update_batched", "scvx_jacobi_update_batched", "scvx_rtc_model_create",
           "scvx_rtc_model_source", "scvx_rtc_model_log", "scvx_rtc_model_destroy", "scvx_rtc_foh_batched",
           "scvx_rtc_integrate_nonlinear_batched", "scvx_rtc_subproblem_compile", "scvx_rtc_intersample_batched",
           "scvx_jacobi_update_costs_batched", "scvx_jacobi_global_rule")
SCVX_MAX_MODEL_PARAMS, SCVX_RTC_MAX_NX, SCVX_RTC_MAX_NU = 16, 16, 8


class ScvxError(RuntimeError):
    pass


class QPTemplate(ctypes.Structure):
    """Mirror of scvx_qp_template (include/scvx_hip.h)."""
    _fields_ = [
        ("model_id", ctypes.c_int32), ("n_x", ctypes.c_int32), ("n_u", ctypes.c_int32), ("K", ctypes.c_int32),
        ("pos_dim", ctypes.c_int32), ("has_final", ctypes.c_int32), ("fix_last_input", ctypes.c_int32),
        ("ineq_last", ctypes.c_int32), ("w_last", ctypes.c_double), ("n_box", ctypes.c_int32),
        ("box_idx", ctypes.c_int32 * SCVX_MAX_BOX), ("box_lo", ctypes.c_double * SCVX_MAX_BOX),
        ("box_hi", ctypes.c_double * SCVX_MAX_BOX), ("n_obs", ctypes.c_int32),
        ("obs_center", (ctypes.c_double * 3) * SCVX_MAX_OBS), ("obs_radius", ctypes.c_double * SCVX_MAX_OBS),
        ("w_obs", ctypes.c_double), ("j_max", ctypes.c_int32), ("w_coll", ctypes.c_double),
        ("has_soc", ctypes.c_int32), ("u_max", ctypes.c_double), ("max_iter", ctypes.c_int32),
        ("tol", ctypes.c_double), ("w_final", ctypes.c_double), ("w_nu", ctypes.c_double),
        ("w_prox", ctypes.c_double),
    ]


class SCPTemplate(ctypes.Structure):
    """Mirror of scvx_scp_template (include/scvx_hip.h)."""
    _fields_ = [
        ("model_id", ctypes.c_int32), ("n_x", ctypes.c_int32), ("n_u", ctypes.c_int32), ("K", ctypes.c_int32),
        ("pos_dim", ctypes.c_int32), ("has_final", ctypes.c_int32), ("pin_u_first", ctypes.c_int32),
        ("pin_u_last", ctypes.c_int32), ("n_ubound", ctypes.c_int32), ("ub_idx", ctypes.c_int32 * SCVX_MAX_BOX),
        ("ub_has_lo", ctypes.c_int32 * SCVX_MAX_BOX), ("ub_has_hi", ctypes.c_int32 * SCVX_MAX_BOX),
        ("ub_lo", ctypes.c_double * SCVX_MAX_BOX), ("ub_hi", ctypes.c_double * SCVX_MAX_BOX),
        ("has_soc", ctypes.c_int32), ("u_max", ctypes.c_double), ("n_xbound", ctypes.c_int32),
        ("xb_idx", ctypes.c_int32 * SCVX_MAX_BOX), ("xb_lo", ctypes.c_double * SCVX_MAX_BOX),
        ("xb_hi", ctypes.c_double * SCVX_MAX_BOX), ("n_obs", ctypes.c_int32),
        ("obs_center", (ctypes.c_double * 3) * SCVX_MAX_OBS), ("obs_radius", ctypes.c_double * SCVX_MAX_OBS),
        ("w_nu", ctypes.c_double), ("w_slack", ctypes.c_double), ("w_sigma", ctypes.c_double),
        ("n_nbr", ctypes.c_int32), ("rho", ctypes.c_double), ("d_min", ctypes.c_double), ("w_coll", ctypes.c_double),
        ("max_iter", ctypes.c_int32), ("tol", ctypes.c_double), ("reg", ctypes.c_double),
        ("game", ctypes.c_int32), ("sigma_fixed", ctypes.c_int32), ("w_u2", ctypes.c_double),
        ("w_du", ctypes.c_double), ("w_dth", ctypes.c_double), ("theta_idx", ctypes.c_int32),
        ("w_in", ctypes.c_double), ("n_slab", ctypes.c_int32), ("r_slab", ctypes.c_double),
        ("waves_per_agent", ctypes.c_int32),
    ]


class IntersampleTemplate(ctypes.Structure):
    """Mirror of scvx_intersample_template (include/scvx_hip.h)."""
    _fields_ = [
        ("model_id", ctypes.c_int32), ("n_obs", ctypes.c_int32),
        ("obs_center", (ctypes.c_double * SCVX_IS_MAX_PROJ) * SCVX_MAX_OBS), ("obs_radius", ctypes.c_double * SCVX_MAX_OBS),
        ("proj_rows", ctypes.c_int32), ("proj", ctypes.c_double * (SCVX_IS_MAX_PROJ * SCVX_IS_MAX_STATE)),
        ("dt", ctypes.c_double), ("seg_dt", ctypes.c_double), ("eps", ctypes.c_double), ("tol", ctypes.c_double),
        ("num_samples", ctypes.c_int32), ("max_crit", ctypes.c_int32), ("nsub", ctypes.c_int32),
    ]


_lib = None


def lib():
    """Load libscvx_hip.so once; raise loudly if it was not built (no fallback path exists)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} not built: run `make -C {os.path.dirname(HERE)}` "
                              "or __graft_entry__.build()")
        L = ctypes.CDLL(LIB_PATH)
        vp, i32, dbl, sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_double, ctypes.c_size_t
        L.scvx_version.restype = i32
        if L.scvx_version() != SCVX_HIP_VERSION:
            raise ImportError(f"{LIB_PATH} implements C-ABI revision {L.scvx_version()}, these bindings revision "
                              f"{SCVX_HIP_VERSION}: rebuild it (`make -C {os.path.dirname(HERE)}`)")
        L.scvx_last_error.restype = ctypes.c_char_p
        L.scvx_foh_batched.argtypes = [i32, vp, i32, i32, vp, vp, vp, i32, vp, vp]
        L.scvx_integrate_nonlinear_batched.argtypes = [i32, vp, i32, i32, vp, vp, vp, i32, i32, vp, vp]
        L.scvx_qp_workspace_bytes.argtypes = [ctypes.POINTER(QPTemplate), i32]
        L.scvx_qp_workspace_bytes.restype = sz
        L.scvx_qp_solve_batched.argtypes = [ctypes.POINTER(QPTemplate), i32] + [vp] * 17 + [vp, sz, vp]
        L.scvx_qp_solve_batched_ordered.argtypes = [ctypes.POINTER(QPTemplate), i32] + [vp] * 18 + [vp, sz, vp]
        L.scvx_qp_set_trace.argtypes = [vp, i32, i32]
        L.scvx_collision_rows_batched.argtypes = [i32, i32, i32, i32, vp, i32, i32, dbl, dbl, i32, vp, vp, vp]
        L.scvx_collision_rows_indexed.argtypes = [i32, i32, i32, i32, vp, vp, i32, dbl, dbl, i32, vp, vp, vp]
        L.scvx_collision_check_batched.argtypes = [i32, i32, i32, i32, vp, i32, i32, dbl, vp, vp, dbl, vp, vp, vp]
        L.scvx_rtc_subproblem_compile.argtypes = [i32, vp, i32, vp]
        L.scvx_scp_workspace_bytes.argtypes = [ctypes.POINTER(SCPTemplate), i32]
        L.scvx_scp_workspace_bytes.restype = sz
        L.scvx_scp_solve_batched.argtypes = [ctypes.POINTER(SCPTemplate), i32] + [vp] * 19 + [vp, sz, vp]
        L.scvx_intersample_batched.argtypes = [ctypes.POINTER(IntersampleTemplate), vp, i32, i32] + [vp] * 9
        L.scvx_admm_consensus_batched.argtypes = [i32, i32, i32, i32, i32, vp, vp, dbl, vp, vp, vp, vp, vp]
        L.scvx_scp_game_solve_batched.argtypes = [ctypes.POINTER(SCPTemplate), i32] + [vp] * 18 + [vp, sz, vp]
        L.scvx_slab_update_batched.argtypes = [i32, i32, i32, i32, i32, vp, vp, vp, vp]
        L.scvx_jacobi_update_batched.argtypes = [i32, i32, i32, i32] + [vp] * 9 + [i32, dbl, dbl, vp]
        L.scvx_jacobi_update_costs_batched.argtypes = [i32, i32, i32, i32] + [vp] * 8 + [vp]
        L.scvx_jacobi_global_rule.argtypes = [i32, i32] + [vp] * 6 + [i32, dbl, vp]
        cpp = ctypes.POINTER(ctypes.c_char_p)
        L.scvx_rtc_model_create.argtypes = [i32, i32, cpp, cpp, cpp, ctypes.c_char_p, ctypes.POINTER(vp)]
        L.scvx_rtc_model_source.argtypes = [vp]
        L.scvx_rtc_model_source.restype = ctypes.c_char_p
        L.scvx_rtc_model_log.argtypes = [vp]
        L.scvx_rtc_model_log.restype = ctypes.c_char_p
        L.scvx_rtc_model_destroy.argtypes = [vp]
        L.scvx_rtc_foh_batched.argtypes = [vp, vp, i32, i32, i32, vp, vp, vp, i32, vp, vp]
        L.scvx_rtc_integrate_nonlinear_batched.argtypes = [vp, vp, i32, i32, i32, vp, vp, vp, i32, i32, vp, vp]
        L.scvx_rtc_intersample_batched.argtypes = [vp, vp, i32, ctypes.POINTER(IntersampleTemplate), i32, i32] + [vp] * 9
        sized = ("scvx_last_error", "scvx_qp_workspace_bytes", "scvx_scp_workspace_bytes", "scvx_rtc_model_source",
                 "scvx_rtc_model_log")
        for fn in EXPORTS:
            getattr(L, fn).restype = getattr(L, fn).restype if fn in sized else i32
        _lib = L
    return _lib


def check(rc, what):
    if rc != 0:
        msg = lib().scvx_last_error().decode(errors="replace")
        raise ScvxError(f"{what} failed (code {rc}): {msg}")

"""scvx_hip -- MI355X-native batched SCvx inner loop (host side of libscvx_hip.so).

Thin PyTorch-ROCm layer over the C-ABI in include/scvx_hip.h: tensors are device buffers,
kernels run on torch's current HIP stream, nothing falls back to the CPU.

    foh_batched            FirstOrderHold.calculate_discretization for N agents
                           (SCvx/discretization/first_order_hold.py:52-87)
    integrate_nonlinear    FirstOrderHold.integrate_nonlinear_piecewise / _full (:127-155)
    collision_rows         linearized pairwise collision rows (Distributed_opt/dist_scvx_3d.py:93-107)
    collision_check        every reference collision row evaluated at a (culled) solution
    qp_solve_batched       the per-agent trust-region subproblem (dist_scvx_3d.py:51-111)
    QPSpec                 problem template of qp_solve_batched
    SCPSpec / SCPSolver    the SCvx convex subproblem SCProblem (+ AgentSolver ADMM terms)
                           (SCvx/optimization/sc_problem.py:15-83, agent_solver.py:78-102)
"""
import ctypes
import math
from dataclasses import dataclass, field
from typing import Optional, Sequence, Tuple

from . import _lib
from ._lib import MODEL_DIMS, MODEL_IDS, STATUS, QPTemplate, SCPTemplate, ScvxError, check, lib

# RK4 substeps per FOH interval: the smallest count that keeps each model within 1e-7 of the reference's LSODA
# goldens (tests/test_foh_gpu.py, tests/test_foh_oracle.py).  1 is exact for the (linear) integrators; the
# quadrotor holds at 10 (round 5, oracle/foh_ref.c on tests/golden/foh_quad_K50_s5.npz: max relative error 1.2e-7 at
# 8, 7.7e-8 at 9, 5.2e-8 at 10, 9e-10 at 16), the unicycle keeps 16.
DEFAULT_NSUB = {"di": 1, "si": 1, "unicycle": 16, "quad": 10}
# ... at the golden's interval T_pin = sigma / (K - 1).  The RK4 error grows with the interval (the quadrotor at
# sigma = 30, K = 50, six times the golden's interval: 3.8e-6 at 10 substeps, 5.7e-7 at 16, against 256 substeps), so
# for longer intervals the count scales as DEFAULT_NSUB * (T / T_pin)^0.75: the RK4 self-convergence test
# (tests/test_foh_oracle.py: K 30..100, sigma 2..45, attitudes to 0.6 rad) holds 1e-7 with it; C5 (sigma 30, K 50)
# runs 39.  (model: (T_pin, exponent))
NSUB_SCALE = {"quad": (5.0 / 49.0, 0.75)}
QUAD_PARAMS = (1.0, 9.81, 0.02, 0.02, 0.04)

__all__ = ["model_dims", "model_id", "default_nsub", "foh_batched", "jacobi_update", "jacobi_update_global", "integrate_nonlinear", "collision_rows", "collision_check", "qp_solve_batched", "QPSpec", "SCPSpec", "SCPSolver", "slab_update",
           "intersample_batched",
           "disc_stride", "unpack_disc", "ScvxError", "MODEL_DIMS", "DEFAULT_NSUB"]


def _torch():
    import torch
    return torch


def _stream(stream=None):
    torch = _torch()
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


def _dev(t, dtype=None, name="tensor"):
    torch = _torch()
    dtype = dtype or torch.float64
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name} must be a torch tensor on the ROCm device")
    if not t.is_cuda:
        raise ScvxError(f"{name} must live on the GPU (the HIP path has no CPU fallback)")
    if t.dtype != dtype:
        raise TypeError(f"{name} must be {dtype}, got {t.dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")
    return ctypes.c_void_p(t.data_ptr())


def model_dims(model):
    """(n_x, n_u) of a built-in model name or of a runtime-compiled model (scvx_hip.rtc.DeviceModel, `.dims`)."""
    if isinstance(model, str):
        return MODEL_DIMS[model]
    dims = getattr(model, "dims", None)
    if dims is None:
        raise TypeError(f"model must be a built-in name {sorted(MODEL_DIMS)} or a scvx_hip.rtc.DeviceModel")
    return tuple(dims)


def model_id(model):
    """The template's model_id: the built-in id, or SCVX_MODEL_RUNTIME for a runtime-compiled model (the QP and
    SCP kernels are then instantiated for its dimensions at the first solve)."""
    return MODEL_IDS[model] if isinstance(model, str) else _lib.SCVX_MODEL_RUNTIME


def default_nsub(model, sigma=None, K=None):
    """RK4 substeps of the FOH: the built-in table (a user model: its DeviceModel.nsub, 16 by default); with the
    interval known (sigma, K), a model in NSUB_SCALE gets DEFAULT_NSUB * (T / T_pin)^p for intervals T = sigma / (K-1)
    longer than its pinned T_pin (never fewer than the table)."""
    if not isinstance(model, str):
        return int(getattr(model, "nsub", 16))
    base = DEFAULT_NSUB[model]
    if sigma is None or K is None or model not in NSUB_SCALE:
        return base
    t_pin, p = NSUB_SCALE[model]
    T = float(sigma) / (int(K) - 1)
    return max(base, int(math.ceil(base * (T / t_pin) ** p - 1e-9)))


def _auto_nsub(model, sigma, K):
    """default_nsub for a device sigma batch: the longest interval of the batch (one host read of max(sigma), only
    for the models whose count depends on the interval)."""
    if isinstance(model, str) and model not in NSUB_SCALE:
        return DEFAULT_NSUB[model]
    if not isinstance(model, str):
        return default_nsub(model)
    return default_nsub(model, float(sigma.max().item()) if sigma.numel() else 0.0, K)


def disc_stride(model):
    n, m = model_dims(model)
    return n * (n + 2 * m + 2)


def unpack_disc(disc, model):
    """[..., K-1, n(n+2m+2)] -> (A_bar, B_bar, C_bar, S_bar, z_bar) in the reference's F-order
    column layout (..., n*n, K-1) etc. (first_order_hold.py:20-24, 75-85)."""
    n, m = model_dims(model)
    o = [0, n * n, n * n + n * m, n * n + 2 * n * m, n * n + 2 * n * m + n, n * n + 2 * n * m + 2 * n]
    return tuple(disc[..., o[i]:o[i + 1]].transpose(-1, -2) for i in range(5))


def _params(model, params):
    torch = _torch()
    if model != "quad":
        return None, ctypes.c_void_p(0)
    p = torch.tensor(params if params is not None else QUAD_PARAMS, dtype=torch.float64)
    buf = (ctypes.c_double * 5)(*p.tolist())
    return buf, ctypes.cast(buf, ctypes.c_void_p)


def foh_batched(model, X, U, sigma, nsub=None, params=None, out=None, stream=None):
    """X (N,K,n), U (N,K,m), sigma (N,) float64 device tensors -> disc (N,K-1,n(n+2m+2)).  nsub None: default_nsub
    for the batch's longest interval (for the quadrotor this reads max(sigma) on the host; pass nsub to avoid it)."""
    torch = _torch()
    N, K, n = X.shape
    m = U.shape[2]
    if (n, m) != MODEL_DIMS[model]:
        raise ValueError(f"{model}: expected n,m={MODEL_DIMS[model]}, got {(n, m)}")
    if tuple(U.shape[:2]) != (N, K) or tuple(sigma.shape) != (N,):
        raise ValueError(f"foh_batched: U (N,K,m) and sigma (N,) must match X (N,K,n); got "
                         f"{tuple(U.shape)}, {tuple(sigma.shape)}")
    if out is None:
        out = torch.empty((N, K - 1, disc_stride(model)), dtype=torch.float64, device=X.device)
    keep, pp = _params(model, params)
    rc = lib().scvx_foh_batched(MODEL_IDS[model], pp, K, N, _dev(X, name="X"), _dev(U, name="U"),
                                _dev(sigma, name="sigma"), int(nsub or _auto_nsub(model, sigma, K)),
                                _dev(out, name="out"), _stream(stream))
    check(rc, "scvx_foh_batched")
    return out


def integrate_nonlinear(model, X, U, sigma, piecewise, nsub=16, params=None, out=None, stream=None):
    """Batched FirstOrderHold.integrate_nonlinear_piecewise (piecewise=True) / _full (False)."""
    torch = _torch()
    N, K, n = X.shape
    m = U.shape[2] if U.dim() == 3 else -1
    if (n, m) != MODEL_DIMS[model]:
        raise ValueError(f"{model}: expected n,m={MODEL_DIMS[model]}, got {(n, m)}")
    if tuple(U.shape[:2]) != (N, K) or tuple(sigma.shape) != (N,):
        raise ValueError(f"integrate_nonlinear: U (N,K,m) and sigma (N,) must match X (N,K,n); got "
                         f"{tuple(U.shape)}, {tuple(sigma.shape)}")
    if out is None:
        out = torch.empty_like(X)
    keep, pp = _params(model, params)
    rc = lib().scvx_integrate_nonlinear_batched(MODEL_IDS[model], pp, K, N, _dev(X, name="X"), _dev(U, name="U"),
                                                _dev(sigma, name="sigma"), int(nsub), int(bool(piecewise)),
                                                _dev(out, name="out"), _stream(stream))
    check(rc, "scvx_integrate_nonlinear_batched")
    return out


def collision_rows(X_all, i0, n_local, R, j_max, pos_dim=3, cull_radius=0.0, rows=None, count=None, stream=None):
    """Rows (g, b) of dist_scvx_3d.py:93-107 for local agents [i0, i0+n_local) of X_all (N_total,K,n)."""
    torch = _torch()
    N_total, K, n = X_all.shape
    if rows is None:
        rows = torch.zeros((n_local, K, j_max, pos_dim + 1), dtype=torch.float64, device=X_all.device)
    if count is None:
        count = torch.zeros((n_local, K), dtype=torch.int32, device=X_all.device)
    rc = lib().scvx_collision_rows_batched(K, pos_dim, n, N_total, _dev(X_all, name="X_all"), int(i0), int(n_local),
                                           float(R), float(cull_radius), int(j_max), _dev(rows, name="rows"),
                                           _dev(count, torch.int32, "count"), _stream(stream))
    check(rc, "scvx_collision_rows_batched")
    return rows, count


def collision_rows_indexed(X_all, idx, R, j_max, pos_dim=3, cull_radius=0.0, rows=None, count=None, stream=None):
    """Rows of dist_scvx_3d.py:93-107 for the agents idx (device int32, distinct, in [0, N_total)) of X_all
    (scvx_collision_rows_indexed): rows [len(idx)][K][j_max][pos_dim+1], count [len(idx)][K]; rows / count
    may be larger buffers whose leading len(idx) entries are written."""
    torch = _torch()
    N_total, K, n = X_all.shape
    n_sel = int(idx.shape[0])
    if rows is None:
        rows = torch.zeros((n_sel, K, j_max, pos_dim + 1), dtype=torch.float64, device=X_all.device)
    if count is None:
        count = torch.zeros((n_sel, K), dtype=torch.int32, device=X_all.device)
    if rows.shape[0] < n_sel or tuple(rows.shape[1:]) != (K, j_max, pos_dim + 1) or count.shape[0] < n_sel:
        raise ValueError("collision_rows_indexed: rows / count too small")
    rc = lib().scvx_collision_rows_indexed(K, pos_dim, n, N_total, _dev(X_all, name="X_all"), _dev(idx, torch.int32, "idx"),
                                           n_sel, float(R), float(cull_radius), int(j_max), _dev(rows, name="rows"),
                                           _dev(count, torch.int32, "count"), _stream(stream))
    check(rc, "scvx_collision_rows_indexed")
    return rows, count


def collision_check(X_all, i0, X_new, slack, R, pos_dim=3, tol=1e-7, viol=None, vmax=None, stream=None):
    """Evaluate EVERY reference collision row (dist_scvx_3d.py:93-107) of local agents
    [i0, i0+N_local) at a solution X_new (N_local,K,n) with shared slacks slack (N_local,K), linearised
    at X_all (N_total,K,n).  Returns device tensors viol (N_local,K) int32 = rows violated by more
    than tol, vmax (N_local,K) = largest row value (scvx_collision_check_batched)."""
    torch = _torch()
    N_total, K, n = X_all.shape
    n_local = X_new.shape[0]
    if tuple(X_new.shape) != (n_local, K, n) or tuple(slack.shape) != (n_local, K):
        raise ValueError("collision_check: X_new (N_local,K,n) and slack (N_local,K) expected")
    if viol is None:
        viol = torch.empty((n_local, K), dtype=torch.int32, device=X_all.device)
    if vmax is None:
        vmax = torch.empty((n_local, K), dtype=torch.float64, device=X_all.device)
    rc = lib().scvx_collision_check_batched(K, pos_dim, n, N_total, _dev(X_all, name="X_all"), int(i0), int(n_local),
                                            float(R), _dev(X_new, name="X_new"), _dev(slack, name="slack"), float(tol),
                                            _dev(viol, torch.int32, "viol"), _dev(vmax, name="vmax"), _stream(stream))
    check(rc, "scvx_collision_check_batched")
    return viol, vmax


@dataclass
class QPSpec:
    """Template of the batched trust-region subproblem (include/scvx_hip.h scvx_qp_template)."""
    model: str = "di"
    K: int = 50
    pos_dim: int = 3
    has_final: bool = True
    fix_last_input: bool = True
    ineq_last: bool = False
    w_last: float = 0.0
    box: Sequence[Tuple[int, float, float]] = ()
    obs: Sequence[Tuple[Sequence[float], float]] = ()
    w_obs: float = 1e6
    j_max: int = 0
    w_coll: float = 1e4
    u_max: Optional[float] = None
    max_iter: int = 60
    # relative stopping tolerance (primal / dual residual and gap); 1e-8 is Clarabel's default
    # (tol_feas = tol_gap_rel = tol_gap_abs = 1e-8), the solver dist_scvx_3d.py:110 calls
    tol: float = 1e-8
    # soft terminal state (build-side option for nonlinear models; the reference's subproblem has the
    # hard row d_{T-1} + x_{T-1} == x_des): with has_final=False and w_final > 0 the objective gains
    # w_final ||x_{K-1} - x_final||^2, so the subproblem stays feasible whatever the linearisation
    w_final: float = 0.0
    # virtual control (the SCvx subproblem form of SCvx/optimization/sc_problem.py:60-68, build-side option for
    # nonlinear models under the Jacobi update): nu_t in every dynamics row, + w_nu sum_t ||nu_t||_1; the
    # subproblem is then feasible for any linearisation point.  Quadrotor (and one DI) classes only.
    w_nu: float = 0.0
    # proximal term w_prox sum_t ||x_t - xbar_t||^2: a soft trust region on the states (the hard trust region
    # of dist_scvx_3d.py:84 bounds the inputs only)
    w_prox: float = 0.0

    def to_c(self):
        n, m = model_dims(self.model)
        if self.w_final < 0 or (self.w_final > 0 and self.has_final):
            raise ValueError("QPSpec: w_final > 0 (soft terminal) needs has_final=False")
        t = QPTemplate()
        t.model_id, t.n_x, t.n_u, t.K, t.pos_dim = model_id(self.model), n, m, self.K, self.pos_dim
        t.has_final, t.fix_last_input, t.ineq_last = int(self.has_final), int(self.fix_last_input), int(self.ineq_last)
        t.w_last = self.w_last
        if len(self.box) > _lib.SCVX_MAX_BOX or len(self.obs) > _lib.SCVX_MAX_OBS:
            raise ValueError("too many box constraints / obstacles")
        t.n_box = len(self.box)
        for i, (bi, lo, hi) in enumerate(self.box):
            t.box_idx[i], t.box_lo[i], t.box_hi[i] = int(bi), float(lo), float(hi)
        t.n_obs = len(self.obs)
        for o, (c, r) in enumerate(self.obs):
            for i in range(len(c)):
                t.obs_center[o][i] = float(c[i])
            t.obs_radius[o] = float(r)
        t.w_obs, t.j_max, t.w_coll = float(self.w_obs), int(self.j_max), float(self.w_coll)
        t.has_soc = int(self.u_max is not None)
        t.u_max = 0.0 if self.u_max is None else float(self.u_max)
        t.max_iter, t.tol = int(self.max_iter), float(self.tol)
        t.w_final = float(self.w_final)
        if self.w_nu < 0 or self.w_prox < 0:
            raise ValueError("QPSpec: w_nu and w_prox must be >= 0")
        t.w_nu, t.w_prox = float(self.w_nu), float(self.w_prox)
        return t


class QPSolver:
    """Reusable batched solver: holds the C template and a device workspace for N agents."""

    def __init__(self, spec: QPSpec, N: int, device="cuda"):
        torch = _torch()
        self.spec, self.N = spec, N
        self.ctpl = spec.to_c()
        nbytes = lib().scvx_qp_workspace_bytes(ctypes.byref(self.ctpl), N)
        self.workspace = torch.empty(max(nbytes // 8, 1), dtype=torch.float64, device=device)
        n, m = model_dims(spec.model)
        K = spec.K
        self.X = torch.empty((N, K, n), dtype=torch.float64, device=device)
        self.U = torch.empty((N, K, m), dtype=torch.float64, device=device)
        self.slack = torch.empty((N, K), dtype=torch.float64, device=device)
        self.nu = torch.zeros((N, K - 1, n), dtype=torch.float64, device=device)   # zeros unless w_nu > 0
        self.obj = torch.empty(N, dtype=torch.float64, device=device)
        self.status = torch.empty(N, dtype=torch.int32, device=device)
        self.iters = torch.empty(N, dtype=torch.int32, device=device)
        self._dummy = torch.zeros(1, dtype=torch.float64, device=device)
        self._dummy_i = torch.zeros(1, dtype=torch.int32, device=device)
        # slots [0, _state_n) hold a solve's primal-dual state (solve(n=...) always fills a leading prefix):
        # a warm flag on any other slot would start the IPM from uninitialised workspace, so it is cleared
        self._state_n = 0

    def _check_shapes(self, disc, sigma, Xref, Uref, x_init, x_final, tr, coll_rows, coll_count, N=None):
        """Host-side shape checks: the kernel indexes every buffer with the template's compile-time
        dimensions, so a mis-shaped tensor would be read out of bounds on the device."""
        spec, N = self.spec, (self.N if N is None else N)
        n, m = model_dims(spec.model)
        K = spec.K
        want = {"disc": (disc, (N, K - 1, disc_stride(spec.model))), "sigma": (sigma, (N,)),
                "Xref": (Xref, (N, K, n)), "Uref": (Uref, (N, K, m)), "x_init": (x_init, (N, n)),
                "tr": (tr, (N,))}
        if spec.has_final or spec.w_final > 0:
            if x_final is None:
                raise ValueError("QPSolver.solve: the template has a terminal condition; x_final is required")
            want["x_final"] = (x_final, (N, n))
        if spec.j_max > 0:
            if coll_rows is None or coll_count is None:
                raise ValueError(f"QPSolver.solve: spec.j_max={spec.j_max} needs coll_rows and coll_count "
                                 "(scvx_hip.collision_rows)")
            want["coll_rows"] = (coll_rows, (N, K, spec.j_max, spec.pos_dim + 1))
            want["coll_count"] = (coll_count, (N, K))
        for name, (t, shp) in want.items():
            if tuple(t.shape) != shp:
                raise ValueError(f"QPSolver.solve: {name} has shape {tuple(t.shape)}, expected {shp}")

    supports_order = True

    def solve(self, disc, sigma, Xref, Uref, x_init, x_final, tr, coll_rows=None, coll_count=None, stream=None, n=None,
              warm=None, order=None):
        """n (<= N): solve only n agents (the inputs' leading dimension); the outputs are the leading n rows
        of the solver's buffers.  warm (N,) int32 device tensor or None: agents with warm != 0 start from the
        primal-dual point of their previous solve by THIS solver (the same agent slot), e.g. the previous
        SCvx iteration's status == 0.  order (n,) int32 device tensor or None: the dispatch order, a
        permutation of range(n) (scvx_qp_solve_batched_ordered; results do not depend on it).  Returns dict
        of device tensors (views of reused buffers)."""
        torch = _torch()
        n = self.N if n is None else int(n)
        if not 0 <= n <= self.N:
            raise ValueError(f"QPSolver.solve: n={n} outside [0, {self.N}]")
        self._check_shapes(disc, sigma, Xref, Uref, x_init, x_final, tr, coll_rows, coll_count, N=n)
        if self.spec.j_max == 0:
            coll_rows, coll_count = self._dummy, self._dummy_i
        xf = x_final if x_final is not None else self._dummy
        if n == 0:
            return {k: v[:0] for k, v in self._outputs().items()}
        if warm is not None and tuple(warm.shape) != (n,):
            raise ValueError(f"QPSolver.solve: warm has shape {tuple(warm.shape)}, expected ({n},)")
        if warm is not None and n > self._state_n:   # slots never solved by this solver start cold
            warm = warm.clone()
            warm[self._state_n:] = 0
        if order is not None and (tuple(order.shape) != (n,) or order.dtype != torch.int32):
            raise ValueError(f"QPSolver.solve: order must be an int32 ({n},) permutation, got "
                             f"{tuple(order.shape)} {order.dtype}")
        rc = lib().scvx_qp_solve_batched_ordered(
            ctypes.byref(self.ctpl), n, _dev(disc, name="disc"), _dev(sigma, name="sigma"),
            _dev(Xref, name="Xref"), _dev(Uref, name="Uref"), _dev(x_init, name="x_init"), _dev(xf, name="x_final"),
            _dev(tr, name="tr"), _dev(coll_rows, name="coll_rows"), _dev(coll_count, torch.int32, "coll_count"),
            _dev(self.X), _dev(self.U), _dev(self.slack), _dev(self.nu), _dev(self.obj), _dev(self.status, torch.int32),
            _dev(self.iters, torch.int32), _dev(warm, torch.int32, "warm") if warm is not None else None,
            _dev(order, torch.int32, "order") if order is not None else None,
            _dev(self.workspace), ctypes.c_size_t(self.workspace.numel() * 8), _stream(stream))
        check(rc, "scvx_qp_solve_batched_ordered")
        self._state_n = max(self._state_n, n)
        out = self._outputs()
        return out if n == self.N else {k: v[:n] for k, v in out.items()}

    def _outputs(self):
        return dict(X=self.X, U=self.U, slack_coll=self.slack, nu=self.nu, obj=self.obj, status=self.status,
                    iters=self.iters)


def qp_solve_batched(spec: QPSpec, disc, sigma, Xref, Uref, x_init, x_final, tr, coll_rows=None, coll_count=None):
    """One-shot batched solve (allocates a QPSolver); returns dict of device tensors (copies)."""
    s = QPSolver(spec, Xref.shape[0], device=Xref.device)
    out = s.solve(disc, sigma, Xref, Uref, x_init, x_final, tr, coll_rows, coll_count)
    return {k: v.clone() for k, v in out.items()}


@dataclass
class SCPSpec:
    """Template of the batched SCProblem solve (include/scvx_hip.h scvx_scp_template).  The
    constraint data come from the model (SCvx/models/*.scp_constraints())."""
    model: str = "unicycle"
    K: int = 100
    pos_dim: int = 2
    has_final: bool = True
    pin_u_first: bool = True
    pin_u_last: bool = True
    u_bounds: Sequence[Tuple[int, Optional[float], Optional[float]]] = ()
    u_soc: Optional[float] = None
    x_bounds: Sequence[Tuple[int, float, float]] = ()
    obs: Sequence[Tuple[Sequence[float], float]] = ()   # (center, total clearance r_o)
    w_nu: float = 1e4
    w_slack: float = 1e6
    w_sigma: float = 100.0
    n_nbr: int = 0
    rho: float = 0.0
    d_min: float = 1.0
    w_coll: float = 1e5
    max_iter: int = 100
    tol: float = 1e-9
    reg: float = 1e-10
    # Nash best-response terms (scvx_scp_game_solve_batched; game_model.py:68-126)
    game: bool = False
    sigma_fixed: bool = False
    w_u2: float = 0.0
    w_du: float = 0.0
    w_dth: float = 0.0
    theta_idx: int = -1
    w_in: float = 0.0
    n_slab: int = 0
    r_slab: float = 0.0
    # launch mapping of this template's solves: 0 = automatic (two waves per agent when K > 64 and the launch
    # leaves SIMDs idle), 1 or 2 forced -- per template, so concurrent callers never share it
    waves_per_agent: int = 0

    def to_c(self):
        n, m = model_dims(self.model)
        t = SCPTemplate()
        t.model_id, t.n_x, t.n_u, t.K, t.pos_dim = model_id(self.model), n, m, int(self.K), int(self.pos_dim)
        t.has_final, t.pin_u_first, t.pin_u_last = int(self.has_final), int(self.pin_u_first), int(self.pin_u_last)
        if len(self.u_bounds) > _lib.SCVX_MAX_BOX or len(self.x_bounds) > _lib.SCVX_MAX_BOX:
            raise ValueError("too many bound constraints")
        if len(self.obs) > _lib.SCVX_MAX_OBS or self.n_nbr > _lib.SCVX_MAX_NBR:
            raise ValueError("too many obstacles / neighbours")
        t.n_ubound = len(self.u_bounds)
        for b, (j, lo, hi) in enumerate(self.u_bounds):
            t.ub_idx[b] = int(j)
            t.ub_has_lo[b], t.ub_has_hi[b] = int(lo is not None), int(hi is not None)
            t.ub_lo[b] = 0.0 if lo is None else float(lo)
            t.ub_hi[b] = 0.0 if hi is None else float(hi)
        t.has_soc = int(self.u_soc is not None)
        t.u_max = 0.0 if self.u_soc is None else float(self.u_soc)
        t.n_xbound = len(self.x_bounds)
        for b, (i, lo, hi) in enumerate(self.x_bounds):
            t.xb_idx[b], t.xb_lo[b], t.xb_hi[b] = int(i), float(lo), float(hi)
        t.n_obs = len(self.obs)
        for o, (c, r) in enumerate(self.obs):
            for i in range(len(c)):
                t.obs_center[o][i] = float(c[i])
            t.obs_radius[o] = float(r)
        t.w_nu, t.w_slack, t.w_sigma = float(self.w_nu), float(self.w_slack), float(self.w_sigma)
        t.n_nbr, t.rho, t.d_min, t.w_coll = int(self.n_nbr), float(self.rho), float(self.d_min), float(self.w_coll)
        t.max_iter, t.tol, t.reg = int(self.max_iter), float(self.tol), float(self.reg)
        if self.game:
            if self.n_nbr:
                raise ValueError("game template: no ADMM neighbour terms")
            if self.n_slab > _lib.SCVX_MAX_NBR:
                raise ValueError("too many slab neighbours")
            t.game, t.sigma_fixed = 1, int(self.sigma_fixed)
            t.w_u2, t.w_du, t.w_dth, t.w_in = float(self.w_u2), float(self.w_du), float(self.w_dth), float(self.w_in)
            t.theta_idx, t.n_slab, t.r_slab = int(self.theta_idx), int(self.n_slab), float(self.r_slab)
        else:
            t.theta_idx = -1
        if self.waves_per_agent not in (0, 1, 2):
            raise ValueError("waves_per_agent must be 0, 1 or 2")
        t.waves_per_agent = int(self.waves_per_agent)
        return t


class SCPSolver:
    """Reusable batched SCProblem solver (scvx_scp_solve_batched): C template, device workspace and
    output buffers for N agents."""

    def __init__(self, spec: SCPSpec, N: int, device="cuda"):
        torch = _torch()
        self.spec, self.N = spec, N
        self.ctpl = spec.to_c()
        nbytes = lib().scvx_scp_workspace_bytes(ctypes.byref(self.ctpl), N)
        self.workspace = torch.empty(max(nbytes // 8, 1), dtype=torch.float64, device=device)
        n, m = model_dims(spec.model)
        K, f64 = spec.K, torch.float64
        self.X = torch.empty((N, K, n), dtype=f64, device=device)
        self.U = torch.empty((N, K, m), dtype=f64, device=device)
        self.nu = torch.empty((N, K - 1, n), dtype=f64, device=device)
        self.sigma = torch.empty(N, dtype=f64, device=device)
        self.s_obs = torch.empty((N, max(len(spec.obs), 1), K), dtype=f64, device=device)
        self.s_nbr = torch.empty((N, max(spec.n_nbr, 1), K), dtype=f64, device=device)
        self.obj = torch.empty(N, dtype=f64, device=device)
        self.status = torch.empty(N, dtype=torch.int32, device=device)
        self.iters = torch.empty(N, dtype=torch.int32, device=device)
        self._dummy = torch.zeros(1, dtype=f64, device=device)

    def solve(self, disc, Xref, Uref, sigma_ref, tr, x_init, x_final, nbr_pos=None, nbr_Y=None, nbr_Lam=None,
              stream=None):
        """disc (N,K-1,n(n+2m+2)), Xref (N,K,n), Uref (N,K,m), sigma_ref (N,), tr (N,), x_init/x_final (N,n);
        nbr_* (N,n_nbr,K,pos_dim) when spec.n_nbr > 0.  Returns dict of device tensors (reused buffers)."""
        if self.spec.n_nbr > 0 and (nbr_pos is None or nbr_Y is None or nbr_Lam is None):
            raise ValueError("ADMM terms need nbr_pos, nbr_Y and nbr_Lam")
        d = self._dummy
        rc = lib().scvx_scp_solve_batched(
            ctypes.byref(self.ctpl), self.N, _dev(disc, name="disc"), _dev(Xref, name="Xref"), _dev(Uref, name="Uref"),
            _dev(sigma_ref, name="sigma_ref"), _dev(tr, name="tr"), _dev(x_init, name="x_init"),
            _dev(x_final, name="x_final"), _dev(nbr_pos if nbr_pos is not None else d, name="nbr_pos"),
            _dev(nbr_Y if nbr_Y is not None else d, name="nbr_Y"),
            _dev(nbr_Lam if nbr_Lam is not None else d, name="nbr_Lam"), _dev(self.X), _dev(self.U), _dev(self.nu),
            _dev(self.sigma), _dev(self.s_obs), _dev(self.s_nbr), _dev(self.obj), _dev(self.status, _torch().int32),
            _dev(self.iters, _torch().int32), _dev(self.workspace), ctypes.c_size_t(self.workspace.numel() * 8),
            _stream(stream))
        check(rc, "scvx_scp_solve_batched")
        return dict(X=self.X, U=self.U, nu=self.nu, sigma=self.sigma, s_obs=self.s_obs[:, :len(self.spec.obs)],
                    s_nbr=self.s_nbr[:, :self.spec.n_nbr], obj=self.obj, status=self.status, iters=self.iters)

    def solve_game(self, disc, Xref, Uref, sigma_ref, tr, x_init, x_final, X_prev=None, slab_z=None, slab_P=None,
                   stream=None):
        """Nash best responses (scvx_scp_game_solve_batched; spec.game must be set): inputs as solve(),
        plus X_prev (N,K,n) when spec.w_in > 0 and slab_z / slab_P (N,n_slab,K,pos_dim) when
        spec.n_slab > 0.  Returns dict of device tensors (reused buffers)."""
        sp_ = self.spec
        if not sp_.game:
            raise ValueError("solve_game needs a game template (SCPSpec.game=True)")
        N, K, pd = self.N, sp_.K, sp_.pos_dim
        if sp_.w_in > 0 and (X_prev is None or tuple(X_prev.shape) != tuple(self.X.shape)):
            raise ValueError(f"X_prev {tuple(self.X.shape)} required (inertia_weight > 0)")
        if sp_.n_slab > 0:
            shp = (N, sp_.n_slab, K, pd)
            if slab_z is None or slab_P is None or tuple(slab_z.shape) != shp or tuple(slab_P.shape) != shp:
                raise ValueError(f"slab_z / slab_P {shp} required")
        d = self._dummy
        rc = lib().scvx_scp_game_solve_batched(
            ctypes.byref(self.ctpl), N, _dev(disc, name="disc"), _dev(Xref, name="Xref"), _dev(Uref, name="Uref"),
            _dev(sigma_ref, name="sigma_ref"), _dev(tr, name="tr"), _dev(x_init, name="x_init"),
            _dev(x_final, name="x_final"), _dev(X_prev if X_prev is not None else d, name="X_prev"),
            _dev(slab_z if slab_z is not None else d, name="slab_z"),
            _dev(slab_P if slab_P is not None else d, name="slab_P"), _dev(self.X), _dev(self.U), _dev(self.nu),
            _dev(self.sigma), _dev(self.s_obs), _dev(self.obj), _dev(self.status, _torch().int32),
            _dev(self.iters, _torch().int32), _dev(self.workspace), ctypes.c_size_t(self.workspace.numel() * 8),
            _stream(stream))
        check(rc, "scvx_scp_game_solve_batched")
        return dict(X=self.X, U=self.U, nu=self.nu, sigma=self.sigma, s_obs=self.s_obs[:, :len(sp_.obs)],
                    obj=self.obj, status=self.status, iters=self.iters)


def slab_update(p, P, pos_dim, z=None, stream=None):
    """ACS slab normals for every (agent, neighbour, node) in one launch (scvx_slab_update_batched;
    GameUnicycleModel.update_slabs, game_model.py:54-66): z = d/||d||, d = p[a,k,:pos_dim] - P[a,j,k],
    0 where ||d|| < 1e-6.  p (N,K,n) float64, P (N,n_slab,K,pos_dim); returns z like P."""
    torch = _torch()
    N, K, n = p.shape
    if P.dim() != 4 or P.shape[0] != N or P.shape[2] != K or P.shape[3] != pos_dim:
        raise ValueError(f"slab_update: P (N={N}, n_slab, K={K}, pos_dim={pos_dim}) expected")
    if z is None:
        z = torch.empty_like(P)
    elif tuple(z.shape) != tuple(P.shape):
        raise ValueError("slab_update: z must have P's shape")
    rc = lib().scvx_slab_update_batched(N, P.shape[1], K, pos_dim, n, _dev(p, name="p"), _dev(P, name="P"),
                                        _dev(z, name="z"), _stream(stream))
    check(rc, "scvx_slab_update_batched")
    return z


def admm_consensus(X_new, nbr, rho, Y, Lam, pos_dim, primal=None, dual=None, stream=None, check_index=True):
    """ADMM consensus / dual update of every (agent, neighbour slot) in one launch
    (scvx_admm_consensus_batched; the host loop of SCvx/optimization/admm_coordinator.py:80-96).
    X_new (N,K,n) float64, nbr (N,n_nbr) int32 neighbour indices, Y / Lam (N,n_nbr,K,pos_dim) updated in
    place.  Returns device tensors primal, dual (N,n_nbr): ||p_j - Y_new||_F, ||Y_new - Y_old||_F.
    check_index=False skips the range check of nbr (a device -> host read) for callers that built nbr
    themselves (the coordinators validate it once)."""
    torch = _torch()
    N, K, n = X_new.shape
    n_nbr = nbr.shape[1] if nbr.dim() == 2 else 0
    shp = (N, n_nbr, K, pos_dim)
    if tuple(nbr.shape) != (N, n_nbr) or tuple(Y.shape) != shp or tuple(Lam.shape) != shp:
        raise ValueError(f"admm_consensus: nbr (N,n_nbr), Y / Lam {shp} expected")
    if not 1 <= pos_dim <= n:
        raise ValueError("admm_consensus: pos_dim out of range")
    if check_index and n_nbr and (int(nbr.min()) < 0 or int(nbr.max()) >= N):
        raise ValueError("admm_consensus: neighbour index out of range")
    if primal is None:
        primal = torch.empty((N, n_nbr), dtype=torch.float64, device=X_new.device)
    if dual is None:
        dual = torch.empty((N, n_nbr), dtype=torch.float64, device=X_new.device)
    rc = lib().scvx_admm_consensus_batched(N, n_nbr, K, pos_dim, n, _dev(X_new, name="X_new"),
                                           _dev(nbr, torch.int32, "nbr"), float(rho), _dev(Y, name="Y"),
                                           _dev(Lam, name="Lam"), _dev(primal, name="primal"), _dev(dual, name="dual"),
                                           _stream(stream))
    check(rc, "scvx_admm_consensus_batched")
    return primal, dual


def jacobi_update(status, X_sol, U_sol, X, U, tr, prev_cost, grow=False, tr_max=float("inf"), X_out=None, U_out=None,
                  tie_rtol=0.0, stream=None):
    """Fused bookkeeping of one Jacobi SCvx iteration, per-agent trust-region rule
    (scvx_jacobi_update_batched): failed agents (status 2) keep (X, U), the others take (X_sol, U_sol);
    tr halves where sum_{t<K-1} ||u_t||^2 rose above prev_cost (1 + tie_rtol), then a failed agent's radius halves
    (or doubles up to tr_max with grow=True); prev_cost <- the new cost.  tr / prev_cost are updated in
    place; returns (X_out, U_out) (fresh tensors unless given)."""
    torch = _torch()
    N, K, n = X.shape
    m = U.shape[2]
    if (tuple(X_sol.shape) != (N, K, n) or tuple(U.shape) != (N, K, m) or tuple(U_sol.shape) != (N, K, m)
            or tuple(status.shape) != (N,) or tuple(tr.shape) != (N,) or tuple(prev_cost.shape) != (N,)):
        raise ValueError("jacobi_update: X / X_sol (N,K,n), U / U_sol (N,K,m), status / tr / prev_cost (N,)")
    X_out = torch.empty_like(X) if X_out is None else X_out
    U_out = torch.empty_like(U) if U_out is None else U_out
    if tuple(X_out.shape) != (N, K, n) or tuple(U_out.shape) != (N, K, m):
        raise ValueError("jacobi_update: X_out / U_out shapes")
    rc = lib().scvx_jacobi_update_batched(N, K, n, m, _dev(status, torch.int32, "status"), _dev(X_sol, name="X_sol"),
                                          _dev(U_sol, name="U_sol"), _dev(X, name="X"), _dev(U, name="U"),
                                          _dev(X_out, name="X_out"), _dev(U_out, name="U_out"), _dev(tr, name="tr"),
                                          _dev(prev_cost, name="prev_cost"), int(bool(grow)), float(tr_max),
                                          float(tie_rtol), _stream(stream))
    check(rc, "scvx_jacobi_update_batched")
    return X_out, U_out


def jacobi_update_global(status, X_sol, U_sol, X, U, tr, prev_total, grow=False, tr_max=float("inf"), X_out=None,
                         U_out=None, all_reduce=None, stream=None):
    """Fused bookkeeping of one Jacobi SCvx iteration under the reference's global trust-region rule
    (Distributed_opt/dist_scvx_3d.py:242-252; scvx_jacobi_update_costs_batched + scvx_jacobi_global_rule): failed agents
    (status 2) keep (X, U), the others take (X_sol, U_sol); every radius halves when the summed cost
    sum_i sum_{t<K-1} ||u_t||^2 exceeds prev_total (strict), then a failed agent's radius halves (or doubles up to
    tr_max with grow=True); prev_total (a (1,) device tensor) <- the total.  all_reduce: a callable that sums a (1,)
    device tensor over the ranks in place (torch.distributed.all_reduce), for agents sharded over ranks.  Returns
    (X_out, U_out)."""
    torch = _torch()
    N, K, n = X.shape
    m = U.shape[2]
    if (tuple(X_sol.shape) != (N, K, n) or tuple(U.shape) != (N, K, m) or tuple(U_sol.shape) != (N, K, m)
            or tuple(status.shape) != (N,) or tuple(tr.shape) != (N,) or tuple(prev_total.shape) != (1,)):
        raise ValueError("jacobi_update_global: X / X_sol (N,K,n), U / U_sol (N,K,m), status / tr (N,), prev_total (1,)")
    X_out = torch.empty_like(X) if X_out is None else X_out
    U_out = torch.empty_like(U) if U_out is None else U_out
    cost = torch.empty((N,), dtype=torch.float64, device=X.device)
    L, st = lib(), _stream(stream)
    rc = L.scvx_jacobi_update_costs_batched(N, K, n, m, _dev(status, torch.int32, "status"), _dev(X_sol, name="X_sol"),
                                            _dev(U_sol, name="U_sol"), _dev(X, name="X"), _dev(U, name="U"),
                                            _dev(X_out, name="X_out"), _dev(U_out, name="U_out"), _dev(cost, name="cost"),
                                            st)
    check(rc, "scvx_jacobi_update_costs_batched")
    s32, ptr = _dev(status, torch.int32, "status"), _dev(tr, name="tr")
    pt = _dev(prev_total, name="prev_total")
    if all_reduce is None:
        rc = L.scvx_jacobi_global_rule(N, 1, s32, _dev(cost, name="cost"), None, None, ptr, pt, int(bool(grow)),
                                       float(tr_max), st)
    else:
        total = torch.empty((1,), dtype=torch.float64, device=X.device)
        rc = L.scvx_jacobi_global_rule(N, 0, s32, _dev(cost, name="cost"), None, _dev(total, name="total"), None, None,
                                       0, 0.0, st)
        check(rc, "scvx_jacobi_global_rule")
        all_reduce(total)
        rc = L.scvx_jacobi_global_rule(N, 2, s32, None, _dev(total, name="total"), None, ptr, pt, int(bool(grow)),
                                       float(tr_max), st)
    check(rc, "scvx_jacobi_global_rule")
    return X_out, U_out


def intersample_batched(model, X, U, sigma, obstacles, proj=None, dt=1.0, seg_dt=None, num_samples=100, eps=1e-4,
                        tol=1e-6, max_crit=8, nsub=None, params=None, stream=None):
    """Inter-sample obstacle minima for every (agent, segment, obstacle) (scvx_intersample_batched;
    SCvx/utils/intersample_collision.py as called per segment by SCvx/models/game_si_model.py:156-176).

    model: a built-in model name, or a scvx_hip.rtc.DeviceModel (any user model: scvx_rtc_intersample_batched,
    the same scan on its runtime-compiled f).  X (N,K,n), U (N,K,m), sigma (N,) float64 device tensors;
    obstacles [(center (pd,), radius)]; proj (pd, n) projection T (default: the first pd state rows); dt as
    find_critical_times; seg_dt = FirstOrderHold.dt (default 1/(K-1)).  Returns device tensors n_crit (N,K-1,O)
    int32 and t_crit / h0 (N,K-1,O,max_crit), grad_x (...,n), grad_u (...,m); entries past n_crit are unset."""
    import numpy as np
    torch = _torch()
    rt = not isinstance(model, str)
    n, m = model.dims if rt else MODEL_DIMS[model]
    N, K = X.shape[0], X.shape[1]
    if X.shape != (N, K, n) or U.shape != (N, K, m) or sigma.shape != (N,):
        raise ValueError(f"intersample_batched: X (N,K,{n}), U (N,K,{m}), sigma (N,) expected")
    O = len(obstacles)
    if O > _lib.SCVX_MAX_OBS:
        raise ValueError("too many obstacles")
    if n > _lib.SCVX_IS_MAX_STATE:
        raise ValueError(f"intersample_batched: n_x {n} > {_lib.SCVX_IS_MAX_STATE}")
    pd = len(np.asarray(obstacles[0][0]).reshape(-1)) if O else 1
    Tm = np.eye(n)[:pd] if proj is None else np.asarray(proj, float).reshape(pd, n)
    t = _lib.IntersampleTemplate()
    t.model_id, t.n_obs, t.proj_rows = (_lib.SCVX_MODEL_RUNTIME if rt else MODEL_IDS[model]), O, pd
    for o, (c, r) in enumerate(obstacles):
        c = np.asarray(c, float).reshape(-1)
        if c.size != pd:
            raise ValueError("obstacle centres must match the projection rows")
        for i in range(pd):
            t.obs_center[o][i] = float(c[i])
        t.obs_radius[o] = float(r)
    for i in range(pd):
        for j in range(n):
            t.proj[i * _lib.SCVX_IS_MAX_STATE + j] = float(Tm[i, j])
    t.dt, t.seg_dt = float(dt), float(1.0 / (K - 1) if seg_dt is None else seg_dt)
    t.eps, t.tol, t.num_samples, t.max_crit = float(eps), float(tol), int(num_samples), int(max_crit)
    # default substeps: the FOH's for this segment length T = seg_dt * sigma (default_nsub; the quadrotor's count
    # grows with T, so max(sigma) is read on the host for it)
    t.nsub = int(nsub or (model.nsub if rt else
                          (default_nsub(model, t.seg_dt * float(sigma.max().item()), 2) if model in NSUB_SCALE and N
                           else DEFAULT_NSUB[model])))
    dev = X.device
    f64 = torch.float64
    shp = (N, K - 1, max(O, 1))
    out = dict(n_crit=torch.zeros(shp, dtype=torch.int32, device=dev),
               t_crit=torch.zeros(shp + (max_crit,), dtype=f64, device=dev),
               h0=torch.zeros(shp + (max_crit,), dtype=f64, device=dev),
               grad_x=torch.zeros(shp + (max_crit, n), dtype=f64, device=dev),
               grad_u=torch.zeros(shp + (max_crit, m), dtype=f64, device=dev))
    bufs = (_dev(X, name="X"), _dev(U, name="U"), _dev(sigma, name="sigma"), _dev(out["n_crit"], torch.int32),
            _dev(out["t_crit"]), _dev(out["h0"]), _dev(out["grad_x"]), _dev(out["grad_u"]), _stream(stream))
    if rt:
        pa, npar = model._pp(params)
        rc = lib().scvx_rtc_intersample_batched(model._h.ptr, pa.ctypes.data, npar, ctypes.byref(t), K, N, *bufs)
        check(rc, "scvx_rtc_intersample_batched")
    else:
        keep, pp = _params(model, params)
        rc = lib().scvx_intersample_batched(ctypes.byref(t), pp, K, N, *bufs)
        check(rc, "scvx_intersample_batched")
        del keep
    return {k: v[:, :, :O] for k, v in out.items()}

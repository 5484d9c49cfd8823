"""Batched Jacobi SCvx outer iteration over N agents, device-resident.

Semantics follow the reference's data-parallel SCvx driver Distributed_opt/dist_scvx_3d.py:
  * x_traj_opt (:31-118): every agent solves its trust-region subproblem against the PREVIOUS
    iterate of all other agents (Jacobi), and X_traj is updated only after all solves (:113-118);
  * cost_fcn (:131-138): cost = sum_t ||u_t||^2 over t < T-1;
  * outer loop (:242-252): if the cost increased, trust_region /= 2.
with the build's FOH discretization (SCvx/discretization/first_order_hold.py) in place of the
one-off ZOH (:9-28, :231), so one SCvx iteration = FOH -> [all-gather + collision rows] -> QP ->
update/bookkeeping.  Multi-GPU: agents are sharded contiguously over ranks; the only data-path
collective is one all_gather of the states per iteration (RCCL over xGMI), needed only when
collision coupling is on, plus one scalar all_reduce for the global trust-region rule.
"""
import dataclasses
from dataclasses import dataclass
from typing import Optional

from . import (QPSolver, QPSpec, collision_check, collision_rows, collision_rows_indexed, default_nsub, foh_batched,
               jacobi_update, jacobi_update_global, model_dims)


def balanced_order(iters, world):
    """An agent order for `world` contiguous shards (rank r owns order[r*n:(r+1)*n]) in which every shard gets
    the same mix of per-agent IPM iteration counts (e.g. the last step's `iters`): agents sorted by
    iterations (descending; ties by index) are dealt to the shards in serpentine order (0..W-1, W-1..0, ...),
    and each shard keeps its agents in ascending index order.  Under the Jacobi update every agent solves
    against the previous iterate of all others (Distributed_opt/dist_scvx_3d.py:93-118), so which rank solves
    which agent does not change any subproblem: the order only moves work between ranks.  A shard's QP launch
    lasts as long as its slowest SIMD's waves, so spreading the long solves evens out the ranks once a GPU holds
    more agents than SIMDs."""
    import numpy as np
    iters = np.asarray(iters)
    N = iters.size
    if N % world:
        raise ValueError(f"balanced_order: {N} agents do not shard over {world} ranks")
    idx = np.lexsort((np.arange(N), -iters))
    rank_of = np.empty(N, np.int64)
    for k, a in enumerate(idx):
        rd, ps = divmod(k, world)
        rank_of[a] = ps if rd % 2 == 0 else world - 1 - ps
    return np.concatenate([np.nonzero(rank_of == r)[0] for r in range(world)])


class HipBackend:
    """The product compute path: the libscvx_hip.so kernels (no CPU fallback)."""

    def foh(self, model, X, U, sigma, nsub, out):
        if isinstance(model, str):
            return foh_batched(model, X, U, sigma, nsub=nsub, out=out)
        return model.foh(X, U, sigma, nsub=nsub, out=out)   # a runtime-compiled model (scvx_hip.rtc.DeviceModel)

    def collision_rows(self, X_all, i0, n_local, R, j_max, pos_dim, cull, rows, count):
        return collision_rows(X_all, i0, n_local, R, j_max, pos_dim, cull, rows, count)

    def collision_rows_indexed(self, X_all, idx, R, j_max, pos_dim, cull, rows, count):
        return collision_rows_indexed(X_all, idx, R, j_max, pos_dim, cull, rows, count)

    def collision_check(self, X_all, i0, X_new, slack, R, pos_dim, tol):
        return collision_check(X_all, i0, X_new, slack, R, pos_dim, tol)

    def qp_solver(self, spec, N, device):
        return QPSolver(spec, N, device=device)

    def jacobi_update(self, status, X_sol, U_sol, X, U, tr, prev_cost, grow, tr_max, tie_rtol=0.0):
        return jacobi_update(status, X_sol, U_sol, X, U, tr, prev_cost, grow=grow, tr_max=tr_max, tie_rtol=tie_rtol)

    def jacobi_update_global(self, status, X_sol, U_sol, X, U, tr, prev_total, grow, tr_max, all_reduce=None):
        return jacobi_update_global(status, X_sol, U_sol, X, U, tr, prev_total, grow=grow, tr_max=tr_max,
                                    all_reduce=all_reduce)


@dataclass
class CouplingSpec:
    """Collision coupling of dist_scvx_3d.py:93-107.  The QP keeps the spec.j_max nearest rows per
    node; with check=True every dropped row is evaluated at the solution (collision_check) and the
    agents that violate one are re-solved with the j_max_hi nearest rows.  The culled problem is a
    relaxation of the reference's, so a solution that satisfies every row IS the reference's; agents
    still violating after the re-solve (more binding neighbours than j_max_hi) are counted in
    JacobiSCvx.last_check["overflow"]."""
    R: float = 2.3              # agent radius (dist_scvx_3d.py:211); rows use 2R
    cull_radius: float = 0.0    # <= 0: every neighbour (exact reference semantics)
    check: bool = True          # evaluate every reference row at the solution
    j_max_hi: int = 32          # nearest rows of the re-solve (the largest QP capacity class)
    check_tol: float = 1e-7     # row violation threshold (metres)


class JacobiSCvx:
    """Device-resident Jacobi SCvx for this rank's agents [i0, i0 + N_local) of N_total.

    on_fail: what a failed subproblem (status 2) does to its agent's trust radius -- "halve" (the
             default) or "grow" (x2, at most tr_max, default tr0: an infeasible trust-region subproblem is the trust
             region being too small to reach x_final, the usual SCP remedy; for nonlinear models).
    tr_rule: "global" -- one trust region for all agents, halved when the total cost rises
             (dist_scvx_3d.py:248-252); "per_agent" -- the same rule applied to each agent's own
             cost (independent agents, configs C2/C3).
    tie_rtol: per-agent rule only -- an agent's radius halves when its cost exceeds the previous one by
             more than this relative margin (default 1e-9).  A converged agent's successive costs agree
             only to rounding, so the reference's strict test would halve its radius on the rounding of
             the cost sum, differently for every summation order (the per-agent rule is this build's; the
             reference's global rule keeps the strict test).
    fused_update: the bookkeeping in csrc/jacobi.hip (default): the per-agent rule in one launch, the global rule in two
             (per-agent costs, then one workgroup sums them in a fixed order and applies the strict test; at world > 1
             the local total is all-reduced in between); False runs the same rules as tensor ops.
    warm_start: each agent's QP starts from the primal-dual point of its previous solve when that one was
             optimal (QPSolver.solve(warm=...), include/scvx_hip.h): the next subproblem is the same agent's
             re-linearised at that solution.  The optimum and the stopping rule are unchanged; C3 needs
             ~2.4x fewer IPM iterations.  False: every solve starts cold (CVXOPT-style).
    warm_max_status: the previous solve qualifies when its status is <= this (0: optimal only; 1: also
             optimal_inaccurate, whose iterate meets the reduced tolerances).
    dispatch_order: "lpt" (default) -- when the agents outnumber the resident waves (one per SIMD: 4 x the
             GPU's CUs; C4), each QP launch deals them longest-first by their previous solve's IPM iterations
             (QPSolver.solve(order=...)), so a slot that frees up takes the next-longest solve (C4 85 -> 93
             SCvx-it/s); with every agent resident at once (C3, C5) the agent order is kept (dealing the long
             solves first there only moves them onto shared CUs: C3 780 -> 764); "none" -- always agent order.
             Results do not depend on it.
    """

    def __init__(self, spec: QPSpec, x_init, x_final, sigma, tr0: float, coupling: Optional[CouplingSpec] = None,
                 tr_rule: str = "per_agent", group=None, nsub: Optional[int] = None, backend=None,
                 on_fail: str = "halve", tr_max: Optional[float] = None, fused_update: bool = True,
                 tie_rtol: float = 1e-9, warm_start: bool = True, warm_max_status: int = 0,
                 dispatch_order: str = "lpt"):
        import torch
        self.torch = torch
        self.backend = backend or HipBackend()
        self.spec = spec
        self.N = x_init.shape[0]
        self.device = x_init.device
        self.x_init, self.x_final, self.sigma = x_init, x_final, sigma
        self.coupling = coupling
        self.tr_rule = tr_rule
        if on_fail not in ("halve", "grow"):
            raise ValueError(f"on_fail must be 'halve' or 'grow', not {on_fail!r}")
        self.on_fail, self.tr_max = on_fail, float(tr0 if tr_max is None else tr_max)
        self.fused_update = fused_update
        self.tie_rtol = float(tie_rtol)
        self.warm_start = warm_start and spec.K >= 2 * model_dims(spec.model)[0]
        self.warm = None   # (N,) int32 device: the previous solve of the agent qualifies as a warm start
        self._warm_buf = None
        self.warm_max_status = int(warm_max_status)
        if dispatch_order not in ("lpt", "none"):
            raise ValueError(f"dispatch_order must be 'lpt' or 'none', not {dispatch_order!r}")
        self.dispatch_order = dispatch_order
        self.order = None  # (N,) int32 device: the next launch's dispatch order (longest previous solve first)
        resident = 4 * torch.cuda.get_device_properties(self.device).multi_processor_count \
            if self.device.type == "cuda" else self.N
        self._lpt = dispatch_order == "lpt" and self.N > resident
        self.group = group
        # RK4 substeps of the FOH: default_nsub for this run's longest interval (one host read of max(sigma) here,
        # none per step; the quadrotor's count grows with the interval)
        self.nsub = nsub or default_nsub(spec.model, float(sigma.max().item()) if self.N else None, spec.K)
        self.solver = self.backend.qp_solver(spec, self.N, self.device)
        self.tr = torch.full((self.N,), float(tr0), dtype=torch.float64, device=self.device)
        self.prev_cost = torch.full((self.N,), float("inf"), dtype=torch.float64, device=self.device)
        self.prev_total = torch.full((1,), float("inf"), dtype=torch.float64, device=self.device)
        self.disc = None
        self.last_check = None
        self.world = 1
        self.rank = 0
        if group is not None or (torch.distributed.is_available() and torch.distributed.is_initialized()):
            self.world = torch.distributed.get_world_size(group)
            self.rank = torch.distributed.get_rank(group)
        self.i0 = self.rank * self.N
        self.N_total = self.N * self.world
        if coupling is not None:
            n, _ = model_dims(spec.model)
            self.X_all = torch.empty((self.N_total, spec.K, n), dtype=torch.float64, device=self.device)
            self.rows = torch.zeros((self.N, spec.K, spec.j_max, spec.pos_dim + 1), dtype=torch.float64,
                                    device=self.device)
            self.count = torch.zeros((self.N, spec.K), dtype=torch.int32, device=self.device)
        self._hi = None   # re-solve buffers of the full-row check (allocated at the first violation)

    def _hi_buffers(self):
        """Rows, counts and a QPSolver at j_max_hi sized for all N local agents, allocated once: a re-solve
        uses their leading n_bad entries (QPSolver.solve(n=...))."""
        if self._hi is None:
            torch, spec, c = self.torch, self.spec, self.coupling
            spec_hi = dataclasses.replace(spec, j_max=c.j_max_hi)
            self._hi = dict(rows=torch.zeros((self.N, spec.K, c.j_max_hi, spec.pos_dim + 1), dtype=torch.float64,
                                             device=self.device),
                            count=torch.zeros((self.N, spec.K), dtype=torch.int32, device=self.device),
                            solver=self.backend.qp_solver(spec_hi, self.N, self.device))
        return self._hi

    def _enforce_all_rows(self, X_all, X, U, out):
        """Make the culled coupling exact: evaluate every reference row at the solution, re-solve the
        violating agents with the j_max_hi nearest rows (computed for those agents only), count what still
        violates (overflow)."""
        torch, spec, c = self.torch, self.spec, self.coupling
        ok = out["status"] != 2

        def violators():
            viol, _ = self.backend.collision_check(X_all, self.i0, out["X"], out["slack_coll"], c.R, spec.pos_dim,
                                                   c.check_tol)
            return (viol.sum(dim=1) > 0) & ok

        bad = violators()
        n_bad = int(bad.sum().item())   # one host read per SCvx iteration
        self.last_check = {"violated": n_bad, "resolved": 0, "overflow": n_bad}
        if n_bad == 0 or spec.j_max >= c.j_max_hi:
            return out
        idx = bad.nonzero().flatten()
        hi = self._hi_buffers()
        gidx = (idx + self.i0).to(torch.int32)
        self.backend.collision_rows_indexed(X_all, gidx, c.R, c.j_max_hi, spec.pos_dim, c.cull_radius, hi["rows"],
                                            hi["count"])
        g = lambda t: t.index_select(0, idx).contiguous()  # noqa: E731
        o2 = hi["solver"].solve(g(self.disc), g(self.sigma), g(X), g(U), g(self.x_init), g(self.x_final), g(self.tr),
                                hi["rows"][:n_bad], hi["count"][:n_bad], n=n_bad)
        out = {k: v.clone() for k, v in out.items()}
        for k in ("X", "U", "slack_coll", "nu", "obj", "status", "iters"):
            out[k].index_copy_(0, idx, o2[k])
        ok = out["status"] != 2
        still = int(violators().sum().item())
        self.last_check.update(resolved=n_bad - still, overflow=still)
        return out

    def gather_states(self, X, async_op=False):
        """All-gather the local states (N,K,n) into X_all (N_total,K,n) -- RCCL over xGMI.  async_op: return
        a handle whose wait() makes the current stream wait for the collective (overlap with the FOH)."""
        if self.world == 1:
            self.X_all.copy_(X)
            return None if async_op else self.X_all
        work = self.torch.distributed.all_gather_into_tensor(self.X_all, X.contiguous(), group=self.group,
                                                             async_op=async_op)
        return work if async_op else self.X_all

    def _mark(self, marks, name):
        """Record a timing event named `name` on the current (launch) stream (marks: list or None)."""
        if marks is not None:
            e = self.torch.cuda.Event(enable_timing=True)
            e.record(self.torch.cuda.current_stream())
            marks.append((name, e))

    def step(self, X, U, marks=None):
        """One SCvx iteration; returns the new (X, U) and the raw solver outputs.
        marks: optional list; (stage, event) pairs are appended on the launch stream -- "start", then
        the end of "foh", "gather" (all-gather), "rows" (collision rows), "qp" (the QP kernel),
        "check" (full-row check + re-solve) and "update" (bookkeeping); a stage's time is the
        difference to the previous mark."""
        torch = self.torch
        spec = self.spec
        self._mark(marks, "start")
        # the state all-gather (RCCL, its own stream) is issued first and overlaps the FOH launch
        work = self.gather_states(X, async_op=True) if self.coupling is not None else None
        self.disc = self.backend.foh(spec.model, X, U, self.sigma, self.nsub, self.disc)
        self._mark(marks, "foh")
        rows = count = X_all = None
        if self.coupling is not None:
            if work is not None:
                work.wait()
            X_all = self.X_all
            self._mark(marks, "gather")
            rows, count = self.backend.collision_rows(X_all, self.i0, self.N, self.coupling.R, spec.j_max,
                                                      spec.pos_dim, self.coupling.cull_radius, self.rows, self.count)
            self._mark(marks, "rows")
        kw = {"order": self.order} if self.order is not None else {}
        out = self.solver.solve(self.disc, self.sigma, X, U, self.x_init, self.x_final, self.tr, rows, count,
                                warm=self.warm, **kw)
        if self.warm_start:   # one launch: the comparison written straight into the int32 flag buffer
            if self._warm_buf is None:
                self._warm_buf = torch.empty((self.N,), dtype=torch.int32, device=self.device)
            self.warm = torch.le(out["status"], self.warm_max_status, out=self._warm_buf)
        if self._lpt and getattr(self.solver, "supports_order", False):
            self.order = torch.argsort(out["iters"], descending=True, stable=True).to(torch.int32)
        self._mark(marks, "qp")
        if self.coupling is not None and self.coupling.check:
            out = self._enforce_all_rows(X_all, X, U, out)
            self._mark(marks, "check")
        # an agent whose subproblem failed numerically (status 2) rejects the step: it keeps its
        # iterate (its output may be non-finite and would otherwise reach every other agent through
        # the collision all-gather) and halves its own trust radius so the next subproblem differs.
        # The reference aborts the whole run instead (cvxpy raises SolverError, dist_scvx_3d.py:110).
        fused = getattr(self.backend, "jacobi_update", None)
        if self.fused_update and self.tr_rule == "per_agent" and fused is not None:
            # one launch for the update, the cost rule and the failure rule (csrc/jacobi.hip)
            Xn, Un = fused(out["status"], out["X"], out["U"], X, U, self.tr, self.prev_cost, self.on_fail == "grow",
                           self.tr_max, self.tie_rtol)
            self._mark(marks, "update")
            return Xn, Un, out
        fused_g = getattr(self.backend, "jacobi_update_global", None)
        if self.fused_update and self.tr_rule == "global" and fused_g is not None:
            ar = None
            if self.world > 1:
                ar = lambda t: torch.distributed.all_reduce(t, group=self.group)  # noqa: E731
            Xn, Un = fused_g(out["status"], out["X"], out["U"], X, U, self.tr, self.prev_total, self.on_fail == "grow",
                             self.tr_max, all_reduce=ar)
            self._mark(marks, "update")
            return Xn, Un, out
        failed = out["status"] == 2
        ok = (~failed)[:, None, None]
        Xn, Un = torch.where(ok, out["X"], X), torch.where(ok, out["U"], U)
        # cost_fcn (dist_scvx_3d.py:131-138) and the trust-region halving rule (:250-252)
        cost = (Un[:, :-1, :] * Un[:, :-1, :]).sum(dim=(1, 2))
        if self.tr_rule == "global":
            total = cost.sum().reshape(1)
            if self.world > 1:
                torch.distributed.all_reduce(total, group=self.group)
            shrink = (total > self.prev_total).to(torch.float64)
            self.tr.mul_(1.0 - 0.5 * shrink)
            self.prev_total.copy_(total)
        else:
            shrink = (cost > self.prev_cost * (1.0 + self.tie_rtol)).to(torch.float64)
            self.tr.mul_(1.0 - 0.5 * shrink)
            self.prev_cost.copy_(cost)
        if self.on_fail == "grow":
            self.tr.mul_(1.0 + failed.to(torch.float64)).clamp_(max=self.tr_max)
        else:
            self.tr.mul_(1.0 - 0.5 * failed.to(torch.float64))
        self._mark(marks, "update")
        return Xn, Un, out

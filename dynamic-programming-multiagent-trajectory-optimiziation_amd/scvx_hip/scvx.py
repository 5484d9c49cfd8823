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
from dataclasses import dataclass
from typing import Optional

from . import (DEFAULT_NSUB, MODEL_DIMS, QPSolver, QPSpec, collision_rows, foh_batched)


class HipBackend:
    """The product compute path: the libscvx_hip.so kernels (no CPU fallback)."""

    def foh(self, model, X, U, sigma, nsub, out):
        return foh_batched(model, X, U, sigma, nsub=nsub, out=out)

    def collision_rows(self, X_all, i0, n_local, R, j_max, pos_dim, cull, rows, count):
        return collision_rows(X_all, i0, n_local, R, j_max, pos_dim, cull, rows, count)

    def qp_solver(self, spec, N, device):
        return QPSolver(spec, N, device=device)


@dataclass
class CouplingSpec:
    R: float = 2.3              # agent radius (dist_scvx_3d.py:211); rows use 2R
    cull_radius: float = 0.0    # <= 0: every neighbour (exact reference semantics)


class JacobiSCvx:
    """Device-resident Jacobi SCvx for this rank's agents [i0, i0 + N_local) of N_total.

    tr_rule: "global" -- one trust region for all agents, halved when the total cost rises
             (dist_scvx_3d.py:248-252); "per_agent" -- the same rule applied to each agent's own
             cost (independent agents, configs C2/C3).
    """

    def __init__(self, spec: QPSpec, x_init, x_final, sigma, tr0: float, coupling: Optional[CouplingSpec] = None,
                 tr_rule: str = "per_agent", group=None, nsub: Optional[int] = None, backend=None):
        import torch
        self.torch = torch
        self.backend = backend or HipBackend()
        self.spec = spec
        self.N = x_init.shape[0]
        self.device = x_init.device
        self.x_init, self.x_final, self.sigma = x_init, x_final, sigma
        self.coupling = coupling
        self.tr_rule = tr_rule
        self.group = group
        self.nsub = nsub or DEFAULT_NSUB[spec.model]
        self.solver = self.backend.qp_solver(spec, self.N, self.device)
        self.tr = torch.full((self.N,), float(tr0), dtype=torch.float64, device=self.device)
        self.prev_cost = torch.full((self.N,), float("inf"), dtype=torch.float64, device=self.device)
        self.prev_total = torch.full((1,), float("inf"), dtype=torch.float64, device=self.device)
        self.disc = None
        self.world = 1
        self.rank = 0
        if group is not None or (torch.distributed.is_available() and torch.distributed.is_initialized()):
            self.world = torch.distributed.get_world_size(group)
            self.rank = torch.distributed.get_rank(group)
        self.i0 = self.rank * self.N
        self.N_total = self.N * self.world
        if coupling is not None:
            n, _ = MODEL_DIMS[spec.model]
            self.X_all = torch.empty((self.N_total, spec.K, n), dtype=torch.float64, device=self.device)
            self.rows = torch.zeros((self.N, spec.K, spec.j_max, spec.pos_dim + 1), dtype=torch.float64,
                                    device=self.device)
            self.count = torch.zeros((self.N, spec.K), dtype=torch.int32, device=self.device)

    def gather_states(self, X):
        """All-gather the local states (N,K,n) into X_all (N_total,K,n) -- RCCL over xGMI."""
        if self.world == 1:
            self.X_all.copy_(X)
        else:
            self.torch.distributed.all_gather_into_tensor(self.X_all, X.contiguous(), group=self.group)
        return self.X_all

    def step(self, X, U, qp_events=None):
        """One SCvx iteration; returns the new (X, U) and the raw solver outputs.
        qp_events: optional list; a (start, end) pair of timing events recorded on the launch
        stream around the QP kernel is appended to it."""
        torch = self.torch
        spec = self.spec
        self.disc = self.backend.foh(spec.model, X, U, self.sigma, self.nsub, self.disc)
        rows = count = None
        if self.coupling is not None:
            X_all = self.gather_states(X)
            rows, count = self.backend.collision_rows(X_all, self.i0, self.N, self.coupling.R, spec.j_max,
                                                      spec.pos_dim, self.coupling.cull_radius, self.rows, self.count)
        if qp_events is not None:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(torch.cuda.current_stream())
        out = self.solver.solve(self.disc, self.sigma, X, U, self.x_init, self.x_final, self.tr, rows, count)
        if qp_events is not None:
            e1.record(torch.cuda.current_stream())
            qp_events.append((e0, e1))
        # an agent whose subproblem failed numerically (status 2) rejects the step: it keeps its
        # iterate (its output may be non-finite and would otherwise reach every other agent through
        # the collision all-gather) and halves its own trust radius so the next subproblem differs.
        # The reference aborts the whole run instead (cvxpy raises SolverError, dist_scvx_3d.py:110).
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
            shrink = (cost > self.prev_cost).to(torch.float64)
            self.tr.mul_(1.0 - 0.5 * shrink)
            self.prev_cost.copy_(cost)
        self.tr.mul_(1.0 - 0.5 * failed.to(torch.float64))
        return Xn, Un, out

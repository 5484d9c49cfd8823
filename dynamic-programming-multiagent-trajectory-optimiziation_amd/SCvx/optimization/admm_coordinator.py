"""ADMMCoordinator -- drop-in replacement of the reference SCvx/optimization/admm_coordinator.py:13-118
(2-D unicycle agents; the 3-D SI_ADMMCoordinator in si_admm_coordinator.py shares this code).

Same surface: `ADMMCoordinator(multi_agent_model, rho_admm=1.0, max_iter=10)`, `.agent_solvers`,
`.discretizers`, `solve(X_refs, U_refs, sigma_ref, verbose=True) -> (X_list, U_list, sigma_ref,
primal_hist, dual_hist)`, with the reference's round structure:

  1. local solves (:70-78): agent i discretizes at its current iterate, linearizes collisions at its
     neighbours' CURRENT iterates and solves its AgentSolver subproblem;
  2. consensus / dual updates (:80-91): Y_ij <- (Y_ij + p_j)/2, Lambda_ij += rho (p_j - Y_ij), with
     the mean primal / dual residuals logged.

Two schedules for step 1:
  * mode="gauss_seidel" (default, the reference's order): agent i sees the iterates agents j < i
    produced earlier in the same round.  All N discretizations still run as ONE FOH launch (agent i's
    own iterate does not change before its turn); the subproblems are N single-agent launches.
  * mode="jacobi": every agent sees the iterates of the previous round; the N subproblems are ONE
    batched launch.  Results differ from the reference's ordering (flagged, not a parity mode).
"""
import time

import numpy as np

import scvx_hip

from ..discretization.first_order_hold import FirstOrderHold
from ..global_parameters import K
from ..utils.multi_agent_logging import print_iteration, print_summary
from .admm_utils import dual_residual, primal_residual
from .agent_solver import AgentSolver, solve_agents_batched


def discretize_batched(discretizers, X_list, U_list, sigma):
    """All agents' FirstOrderHold.calculate_discretization in one scvx_foh_batched launch; returns
    per-agent (A_bar, B_bar, C_bar, S_bar, z_bar) host arrays."""
    import torch
    d0 = discretizers[0]
    dev = d0._device
    X = torch.as_tensor(np.stack([np.asarray(x, float).T for x in X_list]), device=dev)
    U = torch.as_tensor(np.stack([np.asarray(u, float).T for u in U_list]), device=dev)
    s = torch.full((len(X_list),), float(sigma), dtype=torch.float64, device=dev)
    disc = scvx_hip.foh_batched(d0._name, X.contiguous(), U.contiguous(), s, nsub=d0._nsub, params=d0._params)
    host = [t.cpu().numpy() for t in scvx_hip.unpack_disc(disc, d0._name)]
    return [tuple(np.ascontiguousarray(h[a]) for h in host) for a in range(len(X_list))]


class ADMMCoordinator:
    agent_cls = AgentSolver
    pos_dim = 2
    trust_ref_is_initial = False   # SI_ADMMCoordinator passes X_refs[i] to setup (si_admm_coordinator.py:83-86)

    def __init__(self, multi_agent_model, rho_admm: float = 1.0, max_iter: int = 10, mode: str = "gauss_seidel"):
        if mode not in ("gauss_seidel", "jacobi"):
            raise ValueError("mode must be 'gauss_seidel' or 'jacobi'")
        self.model = multi_agent_model
        self.N = multi_agent_model.N
        self.rho_admm = rho_admm
        self.max_iter = max_iter
        self.mode = mode
        self.agent_solvers = [self.agent_cls(i, multi_agent_model, rho_admm) for i in range(self.N)]
        self.discretizers = [FirstOrderHold(multi_agent_model.models[i], K) for i in range(self.N)]

    def solve(self, X_refs: list, U_refs: list, sigma_ref: float, verbose: bool = True):
        pd = self.pos_dim
        for solver in self.agent_solvers:
            for j in solver.Y:
                solver.Y[j].value = np.asarray(X_refs[j])[0:pd, :]
                solver.Lambda[j].value = np.zeros((pd, K))
        X_curr, U_curr = list(X_refs), list(U_refs)
        primal_hist, dual_hist = [], []
        t0 = time.time()
        for it in range(self.max_iter):
            mats = discretize_batched(self.discretizers, X_curr, U_curr, sigma_ref)
            new_positions = [None] * self.N
            if self.mode == "jacobi":
                snap = list(X_curr)
                for i, solver in enumerate(self.agent_solvers):
                    solver.setup(self._tr_ref(i, X_refs, X_curr), self._tr_ref(i, U_refs, U_curr), sigma_ref,
                                 mats[i], {j: snap[j] for j in range(self.N) if j != i})
                res = solve_agents_batched(self.agent_solvers)
                for i, (X_i, U_i, _, _, p_i) in enumerate(res):
                    X_curr[i], U_curr[i], new_positions[i] = X_i, U_i, p_i
            else:
                for i, solver in enumerate(self.agent_solvers):
                    solver.setup(self._tr_ref(i, X_refs, X_curr), self._tr_ref(i, U_refs, U_curr), sigma_ref,
                                 mats[i], {j: X_curr[j] for j in range(self.N) if j != i})
                    X_i, U_i, _, _, p_i = solver.solve(solver="ECOS")
                    X_curr[i], U_curr[i], new_positions[i] = X_i, U_i, p_i
            pr_vals, du_vals = [], []
            for solver in self.agent_solvers:
                for j in solver.Y:
                    p_j = new_positions[j]
                    Y_old = solver.Y[j].value
                    Y_new = 0.5 * (Y_old + p_j)
                    solver.Y[j].value = Y_new
                    solver.Lambda[j].value = solver.Lambda[j].value + self.rho_admm * (p_j - Y_new)
                    pr_vals.append(primal_residual(p_j, Y_new))
                    du_vals.append(dual_residual(Y_new, Y_old))
            pr_avg, du_avg = float(np.mean(pr_vals)), float(np.mean(du_vals))
            primal_hist.append(pr_avg)
            dual_hist.append(du_avg)
            if verbose:
                print_iteration(it, nu_norm=0.0, slack_norm=0.0, primal_res=pr_avg, dual_res=du_avg, dx=0.0, ds=0.0,
                                sigma=sigma_ref, tr_radius=self.rho_admm)
        runtime = time.time() - t0
        if verbose:
            print_summary(len(primal_hist), sigma_ref, runtime)
        return X_curr, U_curr, sigma_ref, primal_hist, dual_hist

    def _tr_ref(self, i, refs, curr):
        return refs[i] if self.trust_ref_is_initial else curr[i]

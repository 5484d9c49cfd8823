"""NashSolver -- drop-in replacement of the reference SCvx/optimization/nash_solver.py:15-149: Iterative
Best Response with the ACS (alternating primal solve / slab dual update) inner loop.

Same surface: `NashSolver(multi_agent_model, max_iter=20, tol=1e-3, max_acs_iters=5, acs_tol=1e-3)`,
`.br_solvers`, `.fohs`, `solve(X_refs, U_refs, sigma_ref=1.0, verbose=False) -> (X_curr, U_curr,
change_hist)`, with the reference's iteration:

  outer it:  snapshot X_prev_all = X_curr
    agent i:  discretize at (X_curr[i], U_curr[i], sigma_ref); slab normals z from X_prev_all
              (update_slabs in setup); slab rows against the neighbours' CURRENT positions
      ACS:    best response -> X_new;  z <- normals of (X_new, X_curr[j]);  stop when
              ||X_new - X_curr[i]||_F < acs_tol (at most max_acs_iters solves)
    accept X_curr[i] = X_new; change = max_i ||X_new - X_curr[i]||_F; stop when change < tol.

Everything stays on the device: per outer iteration one FOH launch for all agents (agent i's own
iterate does not change before its turn), per ACS step one best-response launch
(scvx_scp_game_solve_batched) and one slab launch (scvx_slab_update_batched); the host reads one
(status, delta) pair per ACS step -- the loop's own stopping test.

mode="gauss_seidel" (default) is the reference's order (agent i sees agents j < i of the same
iteration).  mode="jacobi" solves all agents in one launch per ACS step against the previous
iteration's trajectories (a different iteration, flagged, not a parity mode)."""
import time
from typing import List, Tuple

import numpy as np

import scvx_hip

from ..discretization.first_order_hold import FirstOrderHold
from ..global_parameters import TRUST_RADIUS0, K
from ..utils.reporting import print_iteration, print_summary
from .agent_best_response import AgentBestResponse
from .sc_problem import _solver


class NashSolver:
    """Non-cooperative Nash via Iterative Best Response with ACS-based collision handling."""

    br_cls = AgentBestResponse

    def __init__(self, multi_agent_model, max_iter: int = 20, tol: float = 1e-3, max_acs_iters: int = 5,
                 acs_tol: float = 1e-3, mode: str = "gauss_seidel") -> None:
        if mode not in ("gauss_seidel", "jacobi"):
            raise ValueError("mode must be 'gauss_seidel' or 'jacobi'")
        self.mam = multi_agent_model
        self.N = multi_agent_model.N
        self.max_iter = max_iter
        self.tol = tol
        self.br_solvers = [self.br_cls(i, multi_agent_model) for i in range(self.N)]
        self.fohs = [FirstOrderHold(m, K) for m in multi_agent_model.models]
        self.max_acs_iters = max_acs_iters
        self.acs_tol = acs_tol
        self.mode = mode
        self.trace = None    # set to a list to record every best-response solve (host copies; tests)
        self.solves = 0      # best-response solves of the last solve() (agents x ACS steps)

    # ---------------------------------------------------------------------------------------------
    def _specs(self, X_h, U_h, sigma_ref):
        """Per-agent kernel templates: each best response set up once on the warm start (the template
        does not depend on the iterate), as the reference's setup() would build it."""
        specs = []
        for i, br in enumerate(self.br_solvers):
            refs = {j: X_h[j] for j in range(self.N) if j != i}
            disc = tuple(np.zeros_like(a) for a in (br.foh.A_bar, br.foh.B_bar, br.foh.C_bar, br.foh.S_bar, br.foh.z_bar))
            br.setup(X_h[i], U_h[i], sigma_ref, disc, refs, X_h[i], refs, tr_radius=TRUST_RADIUS0)
            specs.append(br.spec())
        return specs

    def solve(self, X_refs: List[np.ndarray], U_refs: List[np.ndarray], sigma_ref: float = 1.0,
              verbose: bool = False) -> Tuple[List[np.ndarray], List[np.ndarray], List[float]]:
        import torch
        N = self.N
        dev = self.fohs[0]._device
        br0 = self.br_solvers[0]
        pd = br0.pos_dim
        Th = lambda a: torch.as_tensor(np.ascontiguousarray(a, dtype=float), dtype=torch.float64, device=dev)  # noqa: E731
        X_h = [np.asarray(x, float).copy() for x in X_refs]
        U_h = [np.asarray(u, float).copy() for u in U_refs]
        specs = self._specs(X_h, U_h, sigma_ref)
        X = Th(np.stack([x.T for x in X_h]))                       # (N, K, n)
        U = Th(np.stack([u.T for u in U_h]))
        cons = [m.scp_constraints() for m in self.mam.models]
        x_init = Th(np.stack([np.asarray(c["x_init"], float).reshape(-1) for c in cons]))
        x_final = Th(np.stack([np.asarray(c["x_final"], float).reshape(-1) for c in cons]))
        sig = torch.full((N,), float(sigma_ref), dtype=torch.float64, device=dev)
        tr = torch.full((N,), float(TRUST_RADIUS0), dtype=torch.float64, device=dev)
        nbr = torch.as_tensor(np.array([[j for j in range(N) if j != i] for i in range(N)], dtype=np.int64).reshape(N, N - 1),
                              device=dev)
        d0 = self.fohs[0]
        disc = None
        change_hist: List[float] = []
        last = [None] * N
        slabs = [None] * N
        t0 = time.time()
        self.solves = 0
        for it in range(self.max_iter):
            if verbose:
                print(f"\n--- Outer iteration {it} ---")
            self._it = it
            Xp = X.clone()                                          # X_prev_all
            disc = d0.calculate_discretization_device(X, U, sig, out=disc)
            if self.mode == "jacobi":
                max_change = self._jacobi_round(specs, disc, X, U, Xp, sig, tr, x_init, x_final, nbr, pd, last, slabs)
            else:
                max_change = 0.0
                for i in range(N):
                    delta, Xn, Un = self._agent(i, specs[i], disc, X, U, Xp, sig, tr, x_init, x_final, nbr, pd, last,
                                                slabs)
                    max_change = max(max_change, delta)
                    if verbose:
                        print(f"  Agent {i}: cost={float(last[i]['obj'][0]):8.3f}, ΔX={delta:6.2e}")
                    X[i], U[i] = Xn, Un
            change_hist.append(max_change)
            if verbose:
                print_iteration(it, nu_norm=0.0, slack_norm=0.0, primal_res=max_change, dual_res=0.0, dx=max_change,
                                ds=0.0, sigma=sigma_ref, tr_radius=0.0)
            if max_change < self.tol:
                if verbose:
                    print("Converged.")
                break
        if verbose:
            print_summary(len(change_hist), sigma_ref, time.time() - t0)
        self._publish(last, slabs, Xp, pd)
        Xh, Uh = X.cpu().numpy(), U.cpu().numpy()
        return [Xh[i].T.copy() for i in range(N)], [Uh[i].T.copy() for i in range(N)], change_hist

    def _agent(self, i, spec, disc, X, U, Xp, sig, tr, x_init, x_final, nbr, pd, last, slabs):
        """Agent i's ACS loop (nash_solver.py:96-112) on the device; returns (delta, X_new, U_new)."""
        import torch
        s_ = slice(i, i + 1)
        P = X[nbr[i]][..., :pd].unsqueeze(0).contiguous()           # neighbours' current positions
        Pprev = Xp[nbr[i]][..., :pd].unsqueeze(0).contiguous()
        z = scvx_hip.slab_update(Xp[s_].contiguous(), Pprev, pd)     # setup(): update_slabs(X_prev, neighbour_prev)
        solver = _solver(spec, 1, X.device)
        Xr, Ur = X[s_].contiguous(), U[s_].contiguous()
        for acs in range(self.max_acs_iters):
            zin = z.clone()
            out = solver.solve_game(disc[s_], Xr, Ur, sig[s_], tr[s_], x_init[s_], x_final[s_], X_prev=Xp[s_].contiguous(),
                                    slab_z=zin, slab_P=P)
            self.solves += 1
            if self.trace is not None:
                self.trace.append(dict(it=self._it, agent=i, acs=acs, disc=disc[i].cpu().numpy(), Xref=Xr[0].cpu().numpy(),
                                       Uref=Ur[0].cpu().numpy(), X_prev=Xp[i].cpu().numpy(), z=zin[0].cpu().numpy(),
                                       P=P[0].cpu().numpy(), **{k: v[0].cpu().numpy() for k, v in out.items()}))
            Xn, Un = out["X"].clone(), out["U"].clone()
            scvx_hip.slab_update(Xn, P, pd, z=z)
            probe = torch.stack([out["status"][0].double(), torch.linalg.vector_norm(Xn[0] - X[i])]).cpu().numpy()
            last[i] = {k: v.clone() for k, v in out.items()}
            slabs[i] = (zin, P)
            if probe[0] >= 2:
                self.br_solvers[i].scp.prob.status = "solver_error"
                raise self.br_solvers[i]._failed()
            delta = float(probe[1])
            if delta < self.acs_tol:
                break
        slabs[i] = (z, P)
        return delta, Xn[0], Un[0]

    def _jacobi_round(self, specs, disc, X, U, Xp, sig, tr, x_init, x_final, nbr, pd, last, slabs):
        import torch
        N = self.N
        if any(bytes(s.to_c()) != bytes(specs[0].to_c()) for s in specs[1:]):
            raise ValueError("NashSolver(mode='jacobi'): agents must share one best-response template")
        P = Xp[nbr][..., :pd].contiguous()                          # (N, N-1, K, pd): previous iteration
        z = scvx_hip.slab_update(Xp, P, pd)
        solver = _solver(specs[0], N, X.device)
        active = torch.ones(N, dtype=torch.bool, device=X.device)
        Xn, Un = X.clone(), U.clone()
        delta = torch.zeros(N, dtype=torch.float64, device=X.device)
        out = None
        for _ in range(self.max_acs_iters):
            out = solver.solve_game(disc, X.clone(), U.clone(), sig, tr, x_init, x_final, X_prev=Xp, slab_z=z.clone(),
                                    slab_P=P)
            self.solves += int(active.sum())
            if bool((out["status"][active] >= 2).any()):
                i = int((active & (out["status"] >= 2)).nonzero()[0, 0])
                raise self.br_solvers[i]._failed()
            Xn[active], Un[active] = out["X"][active], out["U"][active]
            z_new = scvx_hip.slab_update(out["X"], P, pd)
            z[active] = z_new[active]
            delta[active] = torch.linalg.vector_norm((out["X"] - X).reshape(N, -1), dim=1)[active]
            active &= delta >= self.acs_tol
            if not bool(active.any()):
                break
        for i in range(N):
            last[i] = {k: v[i:i + 1].clone() for k, v in out.items()}
            slabs[i] = (z[i:i + 1], P[i:i + 1])
        X.copy_(Xn)
        U.copy_(Un)
        return float(delta.max())

    def _publish(self, last, slabs, Xp, pd):
        """The reference's host-visible state after solve(): every best response's last subproblem
        (.scp .var / .prob), its X_prev / neighbour-position parameters, and the models' slab normals."""
        Xph = Xp.cpu().numpy()
        for i, br in enumerate(self.br_solvers):
            if last[i] is None:
                continue
            br.scp.store({k: v.cpu().numpy() for k, v in last[i].items()}, 0)
            br.X_prev_param.value = Xph[i].T.copy()
            z, P = (t[0].cpu().numpy() for t in slabs[i])
            for slot, j in enumerate(sorted(br.Y_params)):
                br.Y_params[j].value = P[slot].T.copy()
                for k in range(K):
                    br.model.z_params[slot][k].value = z[slot, k]

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
from ..global_parameters import TRUST_RADIUS0, WEIGHT_NU, WEIGHT_SIGMA, WEIGHT_SLACK, K
from ..utils.multi_agent_logging import print_iteration, print_summary
from .admm_utils import WEIGHT_COLLISION_SLACK
from .agent_solver import AgentSolver
from .sc_problem import _solver
from .variables import ProblemResult, SolverError


def discretize_batched(discretizers, X_list, U_list, sigma):
    """All agents' FirstOrderHold.calculate_discretization in one scvx_foh_batched launch; returns
    per-agent (A_bar, B_bar, C_bar, S_bar, z_bar) host arrays."""
    import torch
    d0 = discretizers[0]
    dev = d0._device
    X = torch.as_tensor(np.stack([np.asarray(x, float).T for x in X_list]), device=dev)
    U = torch.as_tensor(np.stack([np.asarray(u, float).T for u in U_list]), device=dev)
    s = torch.full((len(X_list),), float(sigma), dtype=torch.float64, device=dev)
    disc = d0.calculate_discretization_device(X.contiguous(), U.contiguous(), s)
    host = [t.cpu().numpy() for t in d0.unpack_disc(disc)]
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
        """The reference's rounds (admm_coordinator.py:53-118) with every iterate device-resident:
        per round one FOH launch, the subproblems (one batched launch in Jacobi mode, N single-agent
        launches in the reference's Gauss-Seidel order), one consensus / dual-update launch
        (scvx_admm_consensus_batched) for all (i, j) pairs.  The host reads one status word per round
        (a failed subproblem raises SolverError, where cvxpy would) and the residual history at the end."""
        import torch
        pd, N, Kn = self.pos_dim, self.N, K
        d0 = self.discretizers[0]
        dev = d0._device
        T = lambda a: torch.as_tensor(np.ascontiguousarray(a, dtype=float), dtype=torch.float64, device=dev)  # noqa: E731
        X = T(np.stack([np.asarray(x, float).T for x in X_refs]))          # (N, K, n)
        U = T(np.stack([np.asarray(u, float).T for u in U_refs]))          # (N, K, m)
        X0, U0 = X.clone(), U.clone()
        nbr_h = np.array([[j for j in range(N) if j != i] for i in range(N)], dtype=np.int32).reshape(N, N - 1)
        nbr = torch.as_tensor(nbr_h, device=dev)
        nbr_l = nbr.long()
        # Y_ij <- X_refs[j] positions, Lambda_ij <- 0 (:64-68); layout (N, N-1, K, pos_dim)
        Y = X[nbr_l][..., :pd].contiguous()
        Lam = torch.zeros_like(Y)
        pr = torch.zeros((self.max_iter, N, N - 1), dtype=torch.float64, device=dev)
        du = torch.zeros_like(pr)
        probs = [s.scp for s in self.agent_solvers]
        for p in probs:
            p.set_parameters(weight_nu=WEIGHT_NU, weight_slack=WEIGHT_SLACK, weight_sigma=WEIGHT_SIGMA,
                             tr_radius=TRUST_RADIUS0, sigma_ref=float(sigma_ref))
        spec = probs[0].spec(n_nbr=N - 1, rho=float(self.rho_admm), d_min=float(self.model.d_min),
                             w_coll=WEIGHT_COLLISION_SLACK, max_iter=100, tol=1e-9)
        key = bytes(spec.to_c())
        for p in probs[1:]:
            if bytes(p.spec(n_nbr=N - 1, rho=float(self.rho_admm), d_min=float(self.model.d_min),
                            w_coll=WEIGHT_COLLISION_SLACK, max_iter=100, tol=1e-9).to_c()) != key:
                raise ValueError("ADMMCoordinator: agents must share one subproblem template")
        cons = [p.model.scp_constraints() for p in probs]
        x_init = T(np.stack([np.asarray(c["x_init"], float).reshape(-1) for c in cons]))
        x_final = T(np.stack([np.asarray(c["x_final"], float).reshape(-1) for c in cons]))
        sig = torch.full((N,), float(sigma_ref), dtype=torch.float64, device=dev)
        tr = torch.full((N,), float(TRUST_RADIUS0), dtype=torch.float64, device=dev)
        batch = _solver(spec, N, dev) if self.mode == "jacobi" else _solver(spec, 1, dev)
        disc = None
        out = None
        t0 = time.time()
        for it in range(self.max_iter):
            disc = d0.calculate_discretization_device(X, U, sig, out=disc)
            Xr, Ur = (X0, U0) if self.trust_ref_is_initial else (X, U)
            if self.mode == "jacobi":
                pos = X[nbr_l][..., :pd].contiguous()                # every agent sees the previous round
                out = batch.solve(disc, Xr.clone(), Ur.clone(), sig, tr, x_init, x_final, nbr_pos=pos, nbr_Y=Y,
                                  nbr_Lam=Lam)
                bad = out["status"] >= 2
                X, U = out["X"].clone(), out["U"].clone()
            else:
                bad = torch.zeros(N, dtype=torch.bool, device=dev)
                outs = []
                for i in range(N):                                    # agent i sees agents j < i of this round
                    s_ = slice(i, i + 1)
                    pos = X[nbr_l[i]][..., :pd].unsqueeze(0).contiguous()
                    o = batch.solve(disc[s_], Xr[s_].clone(), Ur[s_].clone(), sig[s_], tr[s_], x_init[s_], x_final[s_],
                                    nbr_pos=pos, nbr_Y=Y[s_], nbr_Lam=Lam[s_])
                    bad[i] = o["status"][0] >= 2
                    # a failed agent keeps its previous (finite) iterate, so the agents after it in this
                    # round never see a non-finite X[i]; the round then raises on the first failed agent,
                    # as the reference aborts at the failing solve (cvxpy raises) -- without a host sync
                    # per agent
                    X[i] = torch.where(bad[i], X[i], o["X"][0])
                    U[i] = torch.where(bad[i], U[i], o["U"][0])
                    outs.append({k: v.clone() for k, v in o.items()})
                out = {k: torch.cat([o[k] for o in outs]) for k in outs[0]}
            if bool(bad.any()):                                       # one host read per round
                i = int(bad.nonzero()[0, 0])
                raise SolverError(f"ADMM round {it}: subproblem of agent {i} failed (status "
                                  f"{int(out['status'][i])})")
            scvx_hip.admm_consensus(X, nbr, self.rho_admm, Y, Lam, pd, primal=pr[it], dual=du[it], check_index=False)
            if verbose:
                print_iteration(it, nu_norm=0.0, slack_norm=0.0, primal_res=float(pr[it].mean()),
                                dual_res=float(du[it].mean()), dx=0.0, ds=0.0, sigma=sigma_ref, tr_radius=self.rho_admm)
        runtime = time.time() - t0
        primal_hist = [float(v) for v in pr.mean(dim=(1, 2)).cpu().numpy()]
        dual_hist = [float(v) for v in du.mean(dim=(1, 2)).cpu().numpy()]
        self._publish(X, U, Y, Lam, out)
        if verbose:
            print_summary(len(primal_hist), sigma_ref, runtime)
        Xh, Uh = X.cpu().numpy(), U.cpu().numpy()
        return [Xh[i].T.copy() for i in range(N)], [Uh[i].T.copy() for i in range(N)], sigma_ref, primal_hist, dual_hist

    def _publish(self, X, U, Y, Lam, out):
        """The reference's host-visible state after solve(): Y / Lambda parameters, every AgentSolver's
        last subproblem solution (.scp .var / .prob) and collision slacks."""
        host = {k: v.cpu().numpy() for k, v in out.items()}
        Yh, Lh = Y.cpu().numpy(), Lam.cpu().numpy()
        for i, solver in enumerate(self.agent_solvers):
            js = sorted(solver.Y)
            solver.scp.store(host, i)
            solver.prob = ProblemResult()
            solver.prob.status, solver.prob.value = solver.scp.prob.status, solver.scp.prob.value
            for slot, j in enumerate(js):
                solver.Y[j].value = Yh[i, slot].T.copy()
                solver.Lambda[j].value = Lh[i, slot].T.copy()
                solver.S[j].value = np.maximum(host["s_nbr"][i][slot], 0.0).reshape(-1, 1)

    def _tr_ref(self, i, refs, curr):
        return refs[i] if self.trust_ref_is_initial else curr[i]

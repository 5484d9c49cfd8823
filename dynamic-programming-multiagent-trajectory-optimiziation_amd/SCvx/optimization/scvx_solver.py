"""SCVXSolver -- drop-in replacement of the reference SCvx/optimization/scvx_solver.py:10-133, with the
whole SCvx loop device-resident.

Same surface: `SCVXSolver(model)`, attributes max_iter / conv_tol / tr_radius / weight_* /
discretizer / problem / logger, `solve(verbose=False, initial_sigma=1.0) -> (X, U, sigma, logger)`
with the reference's record keys (iter, nu_norm, slack_norm, dx, du, ds, sigma), its
break-before-update convergence test (:103-111, du ignored) and trust-region rule (:125-133).

Per iteration the trajectory never leaves HBM: FOH (scvx_foh_batched) -> SCProblem solve
(scvx_scp_solve_batched) -> metrics as device reductions; the one host synchronisation is the
read-back of the handful of scalars the convergence test and the logger need.

`BatchedSCVXSolver(models)` runs N independent SCvx loops in lockstep (one FOH launch and one
SCProblem launch per iteration for all agents), each with its own trust radius, log and
convergence flag; a converged agent is frozen at the iterate the reference would return.
"""
from typing import List, Sequence

import numpy as np

import scvx_hip

from ..discretization.first_order_hold import FirstOrderHold, same_device_model, subproblem_model
from ..global_parameters import CONV_TOL, MAX_ITER, TRUST_RADIUS0, WEIGHT_NU, WEIGHT_SIGMA, WEIGHT_SLACK, K
from ..utils.logging import Logger
from .sc_problem import SCProblem, _solver
from .variables import SolverError


class BatchedSCVXSolver:
    def __init__(self, models: Sequence, device="cuda"):
        if not models:
            raise ValueError("BatchedSCVXSolver needs at least one model")
        self.models = list(models)
        self.N = len(self.models)
        self.K = K
        self.device = device
        self.max_iter = MAX_ITER
        self.conv_tol = CONV_TOL
        self.tr_radius = TRUST_RADIUS0
        self.weight_nu = WEIGHT_NU
        self.weight_slack = WEIGHT_SLACK
        self.weight_sigma = WEIGHT_SIGMA
        self._name = subproblem_model(self.models[0])
        for m in self.models[1:]:
            if not same_device_model(subproblem_model(m), self._name):
                raise ValueError("BatchedSCVXSolver: all agents must share one model class")
        self.problems = [SCProblem(m, device=device) for m in self.models]
        self.loggers = [Logger() for _ in self.models]
        self.ipm_iters = []

    def _spec(self):
        for p in self.problems:
            p.set_parameters(weight_nu=self.weight_nu, weight_slack=self.weight_slack, weight_sigma=self.weight_sigma)
        spec = self.problems[0].spec()
        key = bytes(spec.to_c())
        for p in self.problems[1:]:
            if bytes(p.spec().to_c()) != key:
                raise ValueError("BatchedSCVXSolver: agents must share constraint data (bounds, obstacles)")
        return spec

    def solve(self, verbose=False, initial_sigma=1.0):
        """Returns lists (X_i (n,K), U_i (m,K), sigma_i) and the per-agent loggers."""
        import torch
        dev, f64, N, Kn = self.device, torch.float64, self.N, self.K
        n, m = self.models[0].n_x, self.models[0].n_u
        spec = self._spec()
        X0, U0, xi, xf = [], [], [], []
        for mdl in self.models:
            X, U = mdl.initialize_trajectory(np.zeros((n, Kn)), np.zeros((m, Kn)))
            X0.append(np.asarray(X, float).T)
            U0.append(np.asarray(U, float).T)
            c = mdl.scp_constraints()
            xi.append(np.asarray(c["x_init"], float).reshape(-1))
            xf.append(np.asarray(c["x_final"], float).reshape(-1))
        T = lambda a: torch.as_tensor(np.ascontiguousarray(np.asarray(a, float)), dtype=f64, device=dev)  # noqa: E731
        X, U = T(np.stack(X0)), T(np.stack(U0))
        sigma = torch.full((N,), float(initial_sigma), dtype=f64, device=dev)
        x_init, x_final = T(np.stack(xi)), T(np.stack(xf))
        tr = torch.full((N,), float(self.tr_radius), dtype=f64, device=dev)
        active = torch.ones(N, dtype=torch.bool, device=dev)
        solver = _solver(spec, N, dev)
        disc = None
        for lg in self.loggers:
            lg.clear()
        self.ipm_iters = []
        for it in range(self.max_iter):
            disc = (scvx_hip.foh_batched(self._name, X, U, sigma, out=disc) if isinstance(self._name, str)
                    else self._name.foh(X, U, sigma, out=disc))
            out = solver.solve(disc, X, U, sigma, tr, x_init, x_final)
            Xn, Un, nun, sgn = out["X"], out["U"], out["nu"], out["sigma"].clamp_min(0.0)
            nu_norm = nun.abs().sum(-1).amax(-1)                       # induced 1-norm (scvx_solver.py:82)
            slack = out["s_obs"].clamp_min(0.0).sum((-1, -2)) if spec.obs else torch.zeros_like(nu_norm)
            dx = (Xn - X).flatten(1).norm(dim=1)
            du = (Un - U).flatten(1).norm(dim=1)
            ds = (sgn - sigma).abs()
            met = torch.stack([nu_norm, slack, dx, du, ds, sgn, out["status"].to(f64), out["iters"].to(f64),
                               active.to(f64)], 1).cpu().numpy()
            if (met[:, 6][met[:, 8] > 0] >= 2).any():
                bad = int(np.flatnonzero((met[:, 6] >= 2) & (met[:, 8] > 0))[0])
                raise RuntimeError(f"SCvx iteration {it}: convex subproblem infeasible (agent {bad})")
            self.ipm_iters.append(met[:, 7][met[:, 8] > 0].copy())
            for a in np.flatnonzero(met[:, 8] > 0):
                r = met[a]
                self.loggers[a].log({"iter": it, "nu_norm": float(r[0]), "slack_norm": float(r[1]), "dx": float(r[2]),
                                     "du": float(r[3]), "ds": float(r[4]), "sigma": float(r[5])})
                if verbose:
                    pre = f"[agent {a}] " if N > 1 else ""
                    print(f"{pre}Iter {it}: nu={r[0]:.3e}, slack={r[1]:.3e}, dx={r[2]:.3e}, ds={r[4]:.3e}")
            tol = self.conv_tol
            conv = (nu_norm < tol) & (slack < tol) & (dx < tol) & (ds < tol)
            upd = active & ~conv
            # trust-region rule (scvx_solver.py:125-133), per agent
            good = (nu_norm < 1e-2) & (slack < 1e-2)
            tr_new = torch.where(good, (tr * 1.5).clamp_max(50.0), (tr * 1.2).clamp_max(50.0)).clamp_min(1e-3)
            tr = torch.where(upd, tr_new, tr)
            # break-before-update: converged agents keep the iterate they were linearised at
            X = torch.where(upd[:, None, None], Xn, X)
            U = torch.where(upd[:, None, None], Un, U)
            sigma = torch.where(upd, sgn, sigma)
            active = upd
            conv_h = (met[:, 0] < tol) & (met[:, 1] < tol) & (met[:, 2] < tol) & (met[:, 4] < tol)
            if not np.any((met[:, 8] > 0) & ~conv_h):
                break
        self._last = out
        self.tr_final = tr.cpu().numpy()
        Xh, Uh, sh = X.cpu().numpy(), U.cpu().numpy(), sigma.cpu().numpy()
        host = {k: v.cpu().numpy() for k, v in out.items()}
        for a, p in enumerate(self.problems):
            p.prob.status = {0: "optimal", 1: "optimal_inaccurate"}.get(int(host["status"][a]), "solver_error")
            p.prob.value = float(host["obj"][a])
            p.var["X"].value, p.var["U"].value = host["X"][a].T, host["U"][a].T
            p.var["nu"].value, p.var["sigma"].value = host["nu"][a].T, max(float(host["sigma"][a]), 0.0)
            for o, s in enumerate(self.models[a].s_prime):
                s.value = np.maximum(host["s_obs"][a][o], 0.0).reshape(-1, 1)
        Xs = [self.models[a].x_redim(Xh[a].T.copy()) for a in range(N)]
        Us = [self.models[a].u_redim(Uh[a].T.copy()) for a in range(N)]
        return Xs, Us, [float(s) for s in sh], self.loggers


class SCVXSolver:
    """Single-agent SCvx (scvx_solver.py:10-133) on the batched device loop with N = 1."""

    def __init__(self, model, device="cuda"):
        self.model = model
        self.K = K
        self.max_iter = MAX_ITER
        self.conv_tol = CONV_TOL
        self.tr_radius = TRUST_RADIUS0
        self.weight_nu = WEIGHT_NU
        self.weight_slack = WEIGHT_SLACK
        self.weight_sigma = WEIGHT_SIGMA
        self.discretizer = FirstOrderHold(model, self.K, device=device)
        self._batch = BatchedSCVXSolver([model], device=device)
        self.problem = self._batch.problems[0]
        self.logger = self._batch.loggers[0]

    def solve(self, verbose=False, initial_sigma=1.0):
        b = self._batch
        b.max_iter, b.conv_tol, b.tr_radius = self.max_iter, self.conv_tol, self.tr_radius
        b.weight_nu, b.weight_slack, b.weight_sigma = self.weight_nu, self.weight_slack, self.weight_sigma
        Xs, Us, ss, _ = b.solve(verbose=verbose, initial_sigma=initial_sigma)
        self.tr_radius = float(b.tr_final[0])
        return Xs[0], Us[0], ss[0], self.logger

    def _compute_slack_norm(self):
        return float(sum(np.sum(s.value) for s in self.model.s_prime if s.value is not None))

    def _update_trust_region(self, nu_norm, slack_norm):
        if nu_norm < 1e-2 and slack_norm < 1e-2:
            self.tr_radius = min(self.tr_radius * 1.5, 50.0)
        else:
            self.tr_radius = min(self.tr_radius * 1.2, 50.0)
        self.tr_radius = max(self.tr_radius, 1e-3)


__all__: List[str] = ["SCVXSolver", "BatchedSCVXSolver", "SolverError"]

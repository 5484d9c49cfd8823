"""SCProblem -- drop-in replacement of the reference SCvx/optimization/sc_problem.py:6-128.

Same surface: `SCProblem(model)`, `.var` (X (n,K), U (m,K), nu (n,K-1), sigma), `.par` (A_bar ..
z_bar, X_ref, U_ref, sigma_ref, weight_nu / weight_sigma / weight_slack, tr_radius), `.prob`
(`.status`, `.value`), `set_parameters(**kw)` (KeyError on an unknown key), `solve(**kw) -> bool`
(True only on a solver error, :93-103) and `get_variable(name)` (KeyError on an unknown name).

The problem -- the model constraints (model.scp_constraints(), the data of get_constraints), the
F-order dynamics with virtual control nu, the induced-1-norm trust region and the objective
w_nu ||nu||_1 + w_slack sum s' + w_sigma sigma (:48-83) -- is solved by the batched HIP kernel
scvx_scp_solve_batched (csrc/scp_ipm.hip); no expression tree is built and nothing runs on the CPU.
`solve_batched` solves many SCProblems with the same template in one launch.
"""
from typing import Dict, List, Optional, Sequence

import numpy as np

import scvx_hip

from ..discretization.first_order_hold import subproblem_model
from ..global_parameters import K as GLOBAL_K
from .variables import Parameter, ParameterError, ProblemResult, SolverError, Variable

_PAR_SHAPES = ("A_bar", "B_bar", "C_bar", "S_bar", "z_bar", "X_ref", "U_ref")
_SOLVERS: Dict[tuple, "scvx_hip.SCPSolver"] = {}


def _solver(spec: "scvx_hip.SCPSpec", N: int, device):
    """SCPSolver cache keyed by the C template bytes (workspace and output buffers are reused)."""
    key = (bytes(spec.to_c()), N, str(device))
    s = _SOLVERS.get(key)
    if s is None:
        if len(_SOLVERS) > 64:
            _SOLVERS.clear()
        s = _SOLVERS[key] = scvx_hip.SCPSolver(spec, N, device=device)
    return s


def _status_name(code: int) -> str:
    return {0: "optimal", 1: "optimal_inaccurate"}.get(int(code), "solver_error")


class SCProblem:
    """One agent's convex SCvx subproblem (sc_problem.py:15-83)."""

    def __init__(self, model, device="cuda"):
        self.model = model
        self.n_x = model.n_x
        self.n_u = model.n_u
        self.K = GLOBAL_K
        self.device = device
        # a built-in model name, or a user model's runtime-compiled DeviceModel: its constraint data come from
        # model.scp_constraints() (the data of the reference's get_constraints, sc_problem.py:50)
        self._dev_model = subproblem_model(model)
        n, m, K = self.n_x, self.n_u, self.K
        self.var = {"X": Variable((n, K), name="X"), "U": Variable((m, K), name="U"),
                    "nu": Variable((n, K - 1), name="nu"), "sigma": Variable((), name="sigma", nonneg=True)}
        self.par = {"A_bar": Parameter((n * n, K - 1), name="A_bar"), "B_bar": Parameter((n * m, K - 1), name="B_bar"),
                    "C_bar": Parameter((n * m, K - 1), name="C_bar"), "S_bar": Parameter((n, K - 1), name="S_bar"),
                    "z_bar": Parameter((n, K - 1), name="z_bar"), "X_ref": Parameter((n, K), name="X_ref"),
                    "U_ref": Parameter((m, K), name="U_ref"),
                    "sigma_ref": Parameter((), name="sigma_ref", nonneg=True),
                    "weight_nu": Parameter((), name="weight_nu", nonneg=True),
                    "weight_sigma": Parameter((), name="weight_sigma", nonneg=True),
                    "tr_radius": Parameter((), name="tr_radius", nonneg=True),
                    "weight_slack": Parameter((), name="weight_slack", nonneg=True)}
        self.prob = ProblemResult()

    # --- reference API ---------------------------------------------------------------------------
    def set_parameters(self, **kwargs):
        for key, val in kwargs.items():
            if key in self.par:
                self.par[key].value = val
            else:
                raise KeyError(f"Parameter '{key}' not found in SCProblem.")

    def solve(self, **kwargs) -> bool:
        """Solve on the GPU.  kwargs (solver=, verbose=, warm_start=, ...) are accepted for call
        compatibility; `max_iters` / `abstol` map onto the IPM's iteration cap and tolerance."""
        try:
            solve_batched([self], **_opts(kwargs))
            return False
        except SolverError:
            return True

    def get_variable(self, name):
        if name in self.var:
            return self.var[name].value
        raise KeyError(f"Variable '{name}' not found.")

    def print_available_parameters(self):
        print("Available parameters:")
        for k in self.par:
            print(f"  {k}")

    def print_available_variables(self):
        print("Available variables:")
        for k in self.var:
            print(f"  {k}")

    # --- batched-solver plumbing ------------------------------------------------------------------
    def spec(self, n_nbr=0, rho=0.0, d_min=1.0, w_coll=1e5, max_iter=100, tol=1e-9) -> "scvx_hip.SCPSpec":
        c = self.model.scp_constraints()
        p = self.par
        return scvx_hip.SCPSpec(model=self._dev_model, K=self.K, pos_dim=c["pos_dim"], u_bounds=c["u_bounds"],
                                u_soc=c["u_soc"], x_bounds=c["x_bounds"], obs=c["obs"],
                                w_nu=float(p["weight_nu"].require()), w_slack=float(p["weight_slack"].require()),
                                w_sigma=float(p["weight_sigma"].require()), n_nbr=n_nbr, rho=rho, d_min=d_min,
                                w_coll=w_coll, max_iter=max_iter, tol=tol)

    def host_inputs(self):
        """Per-agent kernel inputs in the device layout (agent-major, node-major rows)."""
        p = self.par
        mats = [np.asarray(p[k].require(), float) for k in _PAR_SHAPES[:5]]
        disc = np.concatenate(mats, axis=0).T                      # (K-1, n(n+2m+2)); columns are F-order vecs
        c = self.model.scp_constraints()
        return dict(disc=disc, Xref=np.asarray(p["X_ref"].require(), float).T,
                    Uref=np.asarray(p["U_ref"].require(), float).T, sigma_ref=float(p["sigma_ref"].require()),
                    tr=float(p["tr_radius"].require()), x_init=np.asarray(c["x_init"], float).reshape(-1),
                    x_final=np.asarray(c["x_final"], float).reshape(-1))

    def store(self, out: Dict[str, np.ndarray], a: int):
        """Write agent a's solution into .var, model.s_prime and .prob."""
        st = int(out["status"][a])
        self.prob.status = _status_name(st)
        self.prob.solver_stats = {"num_iters": int(out["iters"][a]), "solver_name": "scvx_hip.scp_ipm"}
        if st not in (0, 1):
            for v in self.var.values():
                v.value = None
            self.prob.value = None
            raise SolverError(f"Solver 'scvx_hip.scp_ipm' failed (status {st}). Try another solver, or solve "
                              "with verbose=True for more information.")
        self.var["X"].value = out["X"][a].T
        self.var["U"].value = out["U"][a].T
        self.var["nu"].value = out["nu"][a].T
        self.var["sigma"].value = max(float(out["sigma"][a]), 0.0)
        for o, s in enumerate(self.model.s_prime):
            s.value = np.maximum(out["s_obs"][a][o], 0.0).reshape(-1, 1)
        self.prob.value = float(out["obj"][a])


def _opts(kwargs) -> dict:
    o = {}
    if "max_iters" in kwargs:
        o["max_iter"] = int(kwargs["max_iters"])
    if "abstol" in kwargs:
        o["tol"] = float(kwargs["abstol"])
    return o


def solve_batched(problems: Sequence[SCProblem], nbr: Optional[List[dict]] = None, max_iter=100, tol=1e-9):
    """Solve many SCProblems that share one template (same model class, constraint data and weights)
    in ONE kernel launch.  `nbr` (AgentSolver ADMM terms): per problem a dict with `pos`, `Y`, `Lam`
    (n_nbr, pos_dim, K) arrays and scalars `rho`, `d_min`, `w_coll`.  Returns the raw output dict
    (numpy) and fills each problem's .var / .prob; raises SolverError if any agent failed."""
    import torch
    if not problems:
        return {}
    p0 = problems[0]
    nn = 0 if nbr is None else int(nbr[0]["pos"].shape[0])
    kw = dict(n_nbr=nn, max_iter=max_iter, tol=tol)
    if nn:
        kw.update(rho=float(nbr[0]["rho"]), d_min=float(nbr[0]["d_min"]), w_coll=float(nbr[0]["w_coll"]))
    spec = p0.spec(**kw)
    key = bytes(spec.to_c())
    for p in problems[1:]:
        if bytes(p.spec(**kw).to_c()) != key:
            raise ValueError("solve_batched: problems do not share one template (model constraints / weights)")
    ins = [p.host_inputs() for p in problems]
    dev = p0.device
    T = lambda a: torch.as_tensor(np.ascontiguousarray(a), dtype=torch.float64, device=dev)  # noqa: E731
    args = {k: T(np.stack([i[k] for i in ins]) if np.ndim(ins[0][k]) else [i[k] for i in ins]) for k in ins[0]}
    if nn:
        pd = spec.pos_dim
        for name in ("pos", "Y", "Lam"):
            arr = np.stack([np.asarray(d[name], float).reshape(nn, pd, -1).transpose(0, 2, 1) for d in nbr])
            args["nbr_" + name] = T(arr)                            # (N, n_nbr, K, pos_dim)
    out = _solver(spec, len(problems), dev).solve(**args)
    host = {k: v.cpu().numpy() for k, v in out.items()}
    failed = None
    for a, p in enumerate(problems):
        try:
            p.store(host, a)
        except SolverError as e:
            failed = failed or e
    if failed is not None:
        raise failed
    return host

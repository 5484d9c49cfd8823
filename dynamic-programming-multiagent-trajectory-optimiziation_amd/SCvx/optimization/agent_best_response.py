"""AgentBestResponse -- drop-in replacement of the reference SCvx/optimization/agent_best_response.py:15-113
(2-D unicycle agents; SI_AgentBestResponse in si_agent_best_response.py shares this code).

Same surface: `AgentBestResponse(i, multi_agent_model)`, `.model`, `.foh`, `.Y_params[j]` (neighbour
positions, Parameter (pos_dim, K)), `.X_prev_param`, `.scp`, `setup(X_ref, U_ref, sigma_ref,
discr_mats, neighbour_refs, X_prev, neighbour_prev_refs, tr_radius=TRUST_RADIUS0)` and
`solve(solver="ECOS", **kw) -> (X_i, U_i, nu_i, slack_i, p_i)` (RuntimeError when the solve fails, :104-105).

setup() follows the reference step by step (:46-98): a fresh SCProblem, the previous-trajectory and
neighbour parameters, the model's cost record and slab constraints (get_cost_function), the slab
normals from X_prev (update_slabs), sigma == sigma_ref, the global weights and the trust radius.  The
problem -- SCProblem + game cost + slab rows + fixed sigma -- is solved by the batched HIP kernel
scvx_scp_game_solve_batched; `solve_best_responses` solves several agents in one launch."""
from dataclasses import replace
from typing import Sequence

import numpy as np

from ..discretization.first_order_hold import FirstOrderHold
from ..global_parameters import TRUST_RADIUS0, WEIGHT_NU, WEIGHT_SIGMA, WEIGHT_SLACK, K
from ..models.game_model import SlabConstraint
from .sc_problem import SCProblem, _opts, _solver
from .variables import Parameter, SolverError


def game_spec(scp: SCProblem, cost, slabs, max_iter=100, tol=1e-9):
    """The kernel template of one best response: SCProblem.spec() + the game terms."""
    if cost.path_weight > 0:
        raise NotImplementedError("path_weight > 0 (path-length SOC term) has no kernel form in scvx_hip")
    js = sorted({c.j for c in slabs})
    radii = {c.radius for c in slabs}
    if len(radii) > 1:
        raise ValueError("slab constraints with different radii")
    if len(slabs) != len(js) * scp.K or any(sorted(c.k for c in slabs if c.j == j) != list(range(scp.K)) for j in js):
        raise ValueError("slab constraints must cover every node for each neighbour")
    theta = cost.theta_idx if cost.theta_idx is not None else -1
    return replace(scp.spec(max_iter=max_iter, tol=tol), game=True, sigma_fixed=True, w_u2=cost.control_weight,
                   w_du=cost.control_rate_weight, w_dth=cost.curvature_weight if theta >= 0 else 0.0,
                   theta_idx=theta, w_in=cost.inertia_weight, n_slab=len(js), r_slab=radii.pop() if radii else 0.0)


def slab_arrays(slabs, n_slab, pos_dim):
    """(n_slab, K, pos_dim) normals z and neighbour positions P from the slab constraint records."""
    z = np.zeros((n_slab, K, pos_dim))
    P = np.zeros((n_slab, K, pos_dim))
    slot = {j: s for s, j in enumerate(sorted({c.j for c in slabs}))}
    for c in slabs:
        z[slot[c.j], c.k] = np.asarray(c.z.require(), float)[:pos_dim]
        P[slot[c.j], c.k] = np.asarray(c.P.require(), float)[:pos_dim, c.k]
    return z, P


class AgentBestResponse:
    """Solve one agent's best-response (pure Nash, fixed time-scale)."""

    pos_dim = 2

    def __init__(self, i: int, multi_agent_model):
        self.i = i
        self.multi_model = multi_agent_model
        self.model = multi_agent_model.models[i]
        self.foh = FirstOrderHold(self.model, K)
        self.Y_params = {j: Parameter((self.pos_dim, K)) for j in range(self.multi_model.N) if j != i}
        self.X_prev_param = Parameter((self.model.n_x, K))
        self.scp = None
        self._cost = None
        self._sigma_ref = None

    def _extra_constraints_hook(self, X_ref, U_ref, sigma_ref):
        """Model rows added after the slabs (the SI variant's inter-sample rows)."""

    def setup(self, X_ref: np.ndarray, U_ref: np.ndarray, sigma_ref: float, discr_mats: tuple, neighbour_refs: dict,
              X_prev: np.ndarray, neighbour_prev_refs: dict, tr_radius: float = TRUST_RADIUS0) -> None:
        pd = self.pos_dim
        self.scp = SCProblem(self.model)
        self.X_prev_param.value = X_prev
        for j, P in self.Y_params.items():
            P.value = np.asarray(neighbour_refs[j], float)[0:pd, :]
        neighbour_prev_pos = [np.asarray(neighbour_prev_refs[j], float)[0:pd, :] for j in self.Y_params]
        self._cost = self.model.get_cost_function(X_v=self.scp.var["X"], U_v=self.scp.var["U"],
                                                  neighbour_pos=list(self.Y_params.values()), X_prev=self.X_prev_param,
                                                  neighbour_prev_pos=neighbour_prev_pos)
        # one dual update with the initial guess (z along X_prev -> neighbour_prev, :66-71)
        self.model.update_slabs(np.asarray(X_prev, float)[0:pd, :], neighbour_prev_pos)
        self._extra_constraints_hook(X_ref, U_ref, sigma_ref)
        self._sigma_ref = float(sigma_ref)
        A_bar, B_bar, C_bar, S_bar, z_bar = discr_mats
        self.scp.set_parameters(A_bar=A_bar, B_bar=B_bar, C_bar=C_bar, S_bar=S_bar, z_bar=z_bar, X_ref=X_ref,
                                U_ref=U_ref, sigma_ref=sigma_ref, weight_nu=WEIGHT_NU, weight_slack=WEIGHT_SLACK,
                                weight_sigma=WEIGHT_SIGMA, tr_radius=tr_radius)

    def slab_constraints(self):
        return [c for c in self.model.extra_constraints if isinstance(c, SlabConstraint)]

    def spec(self, max_iter=100, tol=1e-9):
        return game_spec(self.scp, self._cost, self.slab_constraints(), max_iter=max_iter, tol=tol)

    def _failed(self):
        return RuntimeError("SCProblem error inside AgentBestResponse")

    def solve(self, solver: str = "ECOS", **solver_kwargs):  # noqa: ARG002
        if self.scp is None:
            raise RuntimeError("call setup() before solve()")
        try:
            solve_best_responses([self], **_opts(solver_kwargs))
        except SolverError:
            raise self._failed() from None
        X_i = self.scp.get_variable("X")
        U_i = self.scp.get_variable("U")
        nu_i = self.scp.get_variable("nu")
        slack_i = getattr(self.model, "get_linear_cost", lambda: 0.0)()
        return X_i, U_i, nu_i, slack_i, X_i[0:self.pos_dim, :]


def solve_best_responses(brs: Sequence[AgentBestResponse], max_iter=100, tol=1e-9):
    """Best responses of several agents (same template: model class, weights, obstacles, neighbour
    count) in ONE kernel launch; fills each agent's .scp and returns the raw output dict (numpy)."""
    import torch
    specs = [b.spec(max_iter=max_iter, tol=tol) for b in brs]
    key = bytes(specs[0].to_c())
    if any(bytes(s.to_c()) != key for s in specs[1:]):
        raise ValueError("solve_best_responses: agents do not share one template")
    spec = specs[0]
    dev = brs[0].scp.device
    T = lambda a: torch.as_tensor(np.ascontiguousarray(a, dtype=float), dtype=torch.float64, device=dev)  # noqa: E731
    ins = [b.scp.host_inputs() for b in brs]
    args = {k: T(np.stack([i[k] for i in ins]) if np.ndim(ins[0][k]) else [i[k] for i in ins]) for k in ins[0]}
    if spec.w_in > 0:
        args["X_prev"] = T(np.stack([np.asarray(b.X_prev_param.require(), float).T for b in brs]))
    if spec.n_slab:
        zs, Ps = zip(*(slab_arrays(b.slab_constraints(), spec.n_slab, spec.pos_dim) for b in brs))
        args["slab_z"], args["slab_P"] = T(np.stack(zs)), T(np.stack(Ps))
    out = _solver(spec, len(brs), dev).solve_game(**args)
    host = {k: v.cpu().numpy() for k, v in out.items()}
    failed = None
    for a, b in enumerate(brs):
        try:
            b.scp.store(host, a)
        except SolverError as e:
            failed = failed or e
    if failed is not None:
        raise failed
    return host

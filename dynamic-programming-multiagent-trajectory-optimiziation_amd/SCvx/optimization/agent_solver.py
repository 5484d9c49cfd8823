"""AgentSolver -- drop-in replacement of the reference SCvx/optimization/agent_solver.py:10-117 (2-D
unicycle agents) and, via `pos_dim`, of si_agent_solver.py:10-105 (3-D single integrators).

Same surface: `AgentSolver(agent_index, multi_agent_model, rho_admm)`, `.scp` (the agent's
SCProblem), `.Y[j]` / `.Lambda[j]` (Parameters, (pos_dim, K)), `.S[j]` (Variable (K, 1) >= 0),
`setup(X_ref_i, U_ref_i, sigma_ref_i, discretization_mats, neighbor_refs)` and
`solve(**kw) -> (X_i, U_i, nu_i, slacks, p_i)`.

setup() fixes the SCProblem parameters exactly as the reference (global weights, tr_radius =
TRUST_RADIUS0, :63-76) and records the neighbour reference positions; the collision rows
a_kᵀ(p_i,k - Y_j,k) + S_j,k >= d_min with a_k from MultiAgentModel.linearize_collision (:80-90) and
the augmented-Lagrangian terms (:92-95) are built inside the HIP kernel (scvx_scp_solve_batched with
n_nbr > 0).  `solve_agents_batched` solves many agents' subproblems in one launch."""
from typing import Dict, Sequence

import numpy as np

from ..global_parameters import TRUST_RADIUS0, WEIGHT_NU, WEIGHT_SIGMA, WEIGHT_SLACK, K
from .admm_utils import WEIGHT_COLLISION_SLACK
from .sc_problem import SCProblem, _opts, solve_batched
from .variables import Parameter, ProblemResult, Variable


class AgentSolver:
    pos_dim = 2

    def __init__(self, agent_index: int, multi_agent_model, rho_admm: float):
        self.i = agent_index
        self.multi_agent_model = multi_agent_model
        self.model_i = multi_agent_model.models[self.i]
        self.K = K
        self.d_min = multi_agent_model.d_min
        self.scp = SCProblem(self.model_i)
        self.rho_admm = rho_admm
        self.Y: Dict[int, Parameter] = {}
        self.Lambda: Dict[int, Parameter] = {}
        self.S: Dict[int, Variable] = {}
        for j in range(multi_agent_model.N):
            if j == self.i:
                continue
            self.Y[j] = Parameter((self.pos_dim, self.K), name=f"Y_{j}")
            self.Lambda[j] = Parameter((self.pos_dim, self.K), name=f"Lambda_{j}")
            self.S[j] = Variable((self.K, 1), name=f"S_{j}", nonneg=True)
        self.prob = None
        self._nbr_refs = {}

    def setup(self, X_ref_i: np.ndarray, U_ref_i: np.ndarray, sigma_ref_i: float, discretization_mats: tuple,
              neighbor_refs: dict):
        A_bar, B_bar, C_bar, S_bar, z_bar = discretization_mats
        self.scp.set_parameters(A_bar=A_bar, B_bar=B_bar, C_bar=C_bar, S_bar=S_bar, z_bar=z_bar, X_ref=X_ref_i,
                                U_ref=U_ref_i, sigma_ref=sigma_ref_i, weight_nu=WEIGHT_NU, weight_slack=WEIGHT_SLACK,
                                weight_sigma=WEIGHT_SIGMA, tr_radius=TRUST_RADIUS0)
        for j in neighbor_refs:
            if j not in self.Y:
                raise KeyError(j)
        # positions the collision normals are linearized at (linearize_collision(i, j, X_ref_i, X_ref_j))
        self._nbr_refs = {j: np.array(np.asarray(X, float)[0:self.pos_dim, :]) for j, X in neighbor_refs.items()}
        self.prob = ProblemResult()

    def _nbr_block(self):
        js = sorted(self._nbr_refs)
        pos = np.stack([self._nbr_refs[j] for j in js]) if js else np.zeros((0, self.pos_dim, self.K))
        Y = np.stack([self.Y[j].require() for j in js]) if js else pos
        Lam = np.stack([self.Lambda[j].require() for j in js]) if js else pos
        return js, dict(pos=pos, Y=Y, Lam=Lam, rho=self.rho_admm, d_min=self.d_min, w_coll=WEIGHT_COLLISION_SLACK)

    def _store(self, js, out, a):
        self.prob.status, self.prob.value = self.scp.prob.status, self.scp.prob.value
        for slot, j in enumerate(js):
            self.S[j].value = np.maximum(out["s_nbr"][a][slot], 0.0).reshape(-1, 1)

    def _result(self):
        X_i = self.scp.get_variable("X")
        slacks = {j: self.S[j].value for j in self.S}
        return X_i, self.scp.get_variable("U"), self.scp.get_variable("nu"), slacks, X_i[0:self.pos_dim, :]

    def solve(self, **kwargs):
        if self.prob is None:
            raise RuntimeError("AgentSolver.solve() before setup()")
        solve_agents_batched([self], **_opts(kwargs))
        return self._result()


def solve_agents_batched(solvers: Sequence[AgentSolver], max_iter=100, tol=1e-9):
    """One kernel launch for the ADMM subproblems of several agents (same template, same neighbour
    count); returns [(X_i, U_i, nu_i, slacks, p_i)] in order."""
    blocks = [s._nbr_block() for s in solvers]
    if len({len(js) for js, _ in blocks}) > 1:
        raise ValueError("solve_agents_batched: agents have different neighbour counts")
    nbr = [b for _, b in blocks] if blocks[0][0] else None
    out = solve_batched([s.scp for s in solvers], nbr=nbr, max_iter=max_iter, tol=tol)
    for a, (s, (js, _)) in enumerate(zip(solvers, blocks)):
        s._store(js, out, a)
    return [s._result() for s in solvers]

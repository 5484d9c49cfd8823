"""GameUnicycleModel -- drop-in replacement of the reference SCvx/models/game_model.py:11-126: the
unicycle with per-agent Nash cost weights and the primal-dual "slab" collision constraints.

Same surface: the keyword-only constructor (control / collision / control-rate / curvature / inertia
/ path weights, collision_radius), `.z_params[j][k]` (slab normals, Parameter (2,)),
`.extra_constraints`, `update_slabs(p_i, neighbour_prev_pos)` and
`get_cost_function(X_v, U_v, neighbour_pos, X_prev, neighbour_prev_pos)`.

Nothing here builds an expression tree: get_cost_function returns a `GameCost` record of the terms
(control effort, control-rate and curvature smoothing, inertia) and fills `extra_constraints` with
`SlabConstraint` records z_jk'(p_i,k - P_j,k) >= collision_radius; AgentBestResponse hands both to the
batched HIP kernel (scvx_scp_game_solve_batched), which carries u_{k-1} and th_{k-1} as augmented
Riccati states.  The path-length term (path_weight > 0, an SOC epigraph per segment) has no kernel
form: it is rejected when the best response is set up (no reference scenario sets it)."""
from typing import List, Optional

import numpy as np

from ..global_parameters import K
from ..optimization.variables import Parameter
from .unicycle_model import UnicycleModel

_COST_KEYS = ("control_weight", "collision_weight", "collision_radius", "control_rate_weight", "curvature_weight",
              "inertia_weight", "path_weight")


def slab_normals(p_i: np.ndarray, P_j: np.ndarray) -> np.ndarray:
    """z*_k = argmax_{|z| <= 1} z'(p_i,k - P_j,k) = d_k/|d_k| (0 where |d_k| < 1e-6), p (d, K) -> (K, d)."""
    out = np.zeros((p_i.shape[1], p_i.shape[0]))
    for k in range(p_i.shape[1]):
        d = p_i[:, k] - P_j[:, k]
        nd = np.linalg.norm(d)
        if not nd < 1e-6:
            out[k] = d / nd
    return out


class GameCost:
    """Record of the per-agent Nash cost (game_model.py:84-106); `value(X, U)` evaluates it."""

    def __init__(self, control_weight, control_rate_weight, curvature_weight, inertia_weight, path_weight,
                 theta_idx: Optional[int], X_prev: Parameter, pos_dim: int):
        self.control_weight = float(control_weight)
        self.control_rate_weight = float(control_rate_weight)
        self.curvature_weight = float(curvature_weight)
        self.inertia_weight = float(inertia_weight)
        self.path_weight = float(path_weight)
        self.theta_idx = theta_idx
        self.X_prev = X_prev
        self.pos_dim = pos_dim

    def value(self, X: np.ndarray, U: np.ndarray) -> float:
        """X (n, K), U (m, K): the cost the reference's expression evaluates to."""
        c = self.control_weight * float(np.sum(U ** 2))
        if self.control_rate_weight > 0:
            c += self.control_rate_weight * float(np.sum(np.diff(U, axis=1) ** 2))
        if self.curvature_weight > 0 and self.theta_idx is not None:
            c += self.curvature_weight * float(np.sum(np.diff(X[self.theta_idx]) ** 2))
        if self.inertia_weight > 0:
            c += self.inertia_weight * float(np.sum((X - self.X_prev.require()) ** 2))
        if self.path_weight > 0:
            c += self.path_weight * float(np.linalg.norm(np.diff(X[:self.pos_dim], axis=1), axis=0).sum())
        return c


class SlabConstraint:
    """z'(p_i[:, k] - P[:, k]) >= radius (game_model.py:121-124); z and P are the model's / the best
    response's Parameters, read when the problem is solved."""

    def __init__(self, j: int, k: int, z: Parameter, P: Parameter, radius: float, pos_dim: int):
        self.j, self.k, self.z, self.P, self.radius, self.pos_dim = j, k, z, P, float(radius), pos_dim

    def violation(self, X: np.ndarray) -> float:
        p = X[:self.pos_dim, self.k] - self.P.require()[:self.pos_dim, self.k]
        return max(0.0, self.radius - float(self.z.require() @ p))


class GameUnicycleModel(UnicycleModel):
    """Unicycle model with per-agent cost parameters for Nash games."""

    pos_dim = 2
    theta_idx = 2

    def __init__(self, *, r_init: np.ndarray, r_final: np.ndarray, obstacles: Optional[List] = None,
                 control_weight: float = 1.0, collision_weight: float = 10.0, collision_radius: float = 0.50,
                 control_rate_weight: float = 5.0, curvature_weight: float = 100.0, inertia_weight: float = 0.0,
                 path_weight: float = 0.0, **kwargs):
        for key in _COST_KEYS:
            kwargs.pop(key, None)
        super().__init__(r_init=r_init, r_final=r_final, obstacles=obstacles, **kwargs)
        self.control_weight = control_weight
        self.collision_weight = collision_weight      # stored, unused by the cost (as in the reference)
        self.collision_radius = collision_radius
        self.control_rate_weight = control_rate_weight
        self.curvature_weight = curvature_weight
        self.inertia_weight = inertia_weight
        self.path_weight = path_weight
        self.extra_constraints: list = []
        self.z_params: List[List[Parameter]] = []

    def update_slabs(self, p_i: np.ndarray, neighbour_prev_pos: List[np.ndarray]):
        """z*_jk = d/|d| with d = p_i[:, k] - P_j[:, k] (0 if |d| < 1e-6) into z_params[j][k]
        (game_model.py:54-66; an IndexError before get_cost_function created z_params, as there)."""
        for j, P_j in enumerate(neighbour_prev_pos):
            z = slab_normals(np.asarray(p_i, float), np.asarray(P_j, float))
            for k in range(K):
                self.z_params[j][k].value = z[k]

    def _cost_record(self, X_prev) -> GameCost:
        return GameCost(self.control_weight, self.control_rate_weight, self.curvature_weight, self.inertia_weight,
                        getattr(self, "path_weight", 0.0), self.theta_idx, X_prev, self.pos_dim)

    def get_cost_function(self, X_v, U_v, neighbour_pos: List[Parameter], X_prev: Parameter,
                          neighbour_prev_pos: List[np.ndarray]) -> GameCost:  # noqa: ARG002
        """The cost record; slab constraints for every neighbour and node into extra_constraints
        (z_params created at zero on first use or when the neighbour count changes, :110-118)."""
        self.extra_constraints.clear()
        if not self.z_params or len(self.z_params) != len(neighbour_pos):
            self.z_params = [[Parameter((self.pos_dim,), name=f"slab_z_{j}_{k}") for k in range(K)]
                             for j in range(len(neighbour_pos))]
            for row in self.z_params:
                for z in row:
                    z.value = np.zeros(self.pos_dim)
        for j, P_j in enumerate(neighbour_pos):
            for k in range(K):
                self.extra_constraints.append(SlabConstraint(j, k, self.z_params[j][k], P_j, self.collision_radius,
                                                             self.pos_dim))
        return self._cost_record(X_prev)

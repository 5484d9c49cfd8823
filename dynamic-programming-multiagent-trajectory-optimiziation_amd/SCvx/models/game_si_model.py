"""GameSIModel -- drop-in replacement of the reference SCvx/models/game_si_model.py:7-188: the 3-D
single integrator with Nash cost weights, slab normals and inter-sample obstacle rows.

Reference behaviour kept as is:
  * cost (:104-125): control effort + control-rate smoothing + inertia + path length; the
    collision slacks s_coll_j (nonneg, weight collision_weight) appear in no constraint, so they are
    0 at any optimum and are not modelled; curvature_weight is stored but not used;
  * get_cost_function refreshes the slab normals from X_prev (:127-128) and lists one slab row per
    neighbour and node; update_intersample_constraints (:138-188) then REPLACES extra_constraints
    by the inter-sample rows h0 + grad_x'(x_k - xbar_k) + grad_u'(u_k - ubar_k) + s >= 0 -- so the
    SI best response solves without slab rows, as the reference does;
  * every inter-sample row has its own nonneg slack that enters no cost: each such row is satisfiable
    for any (x, u) and cannot move the optimum; the rows are computed (batched HIP kernel,
    SCvx/utils/intersample_collision.segment_minima) and recorded, and the best-response kernel
    skips them."""
from typing import List, Optional, Tuple

import numpy as np

from ..config.SI_default_game import AGT_COLL_RAD
from ..global_parameters import K as GLOBAL_K
from ..optimization.variables import Parameter, Variable
from .game_model import GameCost, SlabConstraint, slab_normals
from .single_integrator_model import SingleIntegratorModel


class IntersampleConstraint:
    """h0 + grad_x'(x_k - x_nom_k) + grad_u'(u_k - u_nom_k) + s >= 0 with s >= 0 free (:160-188)."""

    def __init__(self, k, obstacle, t_star, h0, grad_x, grad_u, x_nom, u_nom, slack: Variable):
        self.k, self.obstacle, self.t_star, self.h0 = k, obstacle, t_star, h0
        self.grad_x, self.grad_u, self.x_nom, self.u_nom, self.slack = grad_x, grad_u, x_nom, u_nom, slack

    def value(self, X: np.ndarray, U: np.ndarray) -> float:
        return float(self.h0 + self.grad_x @ (X[:, self.k] - self.x_nom) + self.grad_u @ (U[:, self.k] - self.u_nom))


class GameSIModel(SingleIntegratorModel):
    """Single-integrator model with per-agent cost parameters for Nash games (x = [x, y, z], u = v)."""

    pos_dim = 3
    theta_idx = None
    _COST_KEYS = {"control_weight", "collision_weight", "control_rate_weight", "curvature_weight", "inertia_weight",
                  "path_weight"}

    def __init__(self, r_init: np.ndarray, r_final: np.ndarray, robot_radius: float = 0.5,
                 collision_radius: Optional[float] = None,
                 obstacles: Optional[List[Tuple[List[float], float]]] = None, **kwargs):
        self.robot_radius = robot_radius
        self.agent_coll_rad = collision_radius if collision_radius is not None else AGT_COLL_RAD
        self.control_weight = kwargs.pop("control_weight", 1.0)
        self.collision_weight = kwargs.pop("collision_weight", 80.0)
        self.control_rate_weight = kwargs.pop("control_rate_weight", 5.0)
        self.curvature_weight = kwargs.pop("curvature_weight", 0.0)
        self.inertia_weight = kwargs.pop("inertia_weight", 0.0)
        self.path_weight = kwargs.pop("path_weight", 0.0)
        super().__init__(r_init=r_init, r_final=r_final, robot_radius=self.robot_radius, obstacles=obstacles)
        self.coll_slacks: List[Variable] = []
        self.z_params: List[List[Parameter]] = []
        self.inter_slacks: List[Variable] = []
        self.extra_constraints: list = []

    def update_slabs(self, p_i: np.ndarray, neighbour_prev_pos: List[np.ndarray]) -> None:
        """z*_jk = (x_i - x_j)/|x_i - x_j| (0 if < 1e-6); z_params created on first use (:69-88)."""
        if not self.z_params:
            self.z_params = [[Parameter((self.n_x,), name=f"z_{j}_{k}") for k in range(GLOBAL_K)]
                             for j in range(len(neighbour_prev_pos))]
        for j, P_j in enumerate(neighbour_prev_pos):
            z = slab_normals(np.asarray(p_i, float), np.asarray(P_j, float))
            for k in range(GLOBAL_K):
                self.z_params[j][k].value = z[k]

    def get_cost_function(self, X_v, U_v, neighbour_pos: List[Parameter], X_prev: Parameter,
                          neighbour_prev_pos: List[np.ndarray]) -> GameCost:
        self.extra_constraints.clear()
        self.coll_slacks = [Variable((GLOBAL_K,), name=f"s_coll_{j}", nonneg=True) for j in range(len(neighbour_pos))]
        for s in self.coll_slacks:
            s.value = np.zeros(GLOBAL_K)
        self.update_slabs(X_prev.require(), neighbour_prev_pos)
        for j, P in enumerate(neighbour_pos):
            for k in range(GLOBAL_K):
                self.extra_constraints.append(SlabConstraint(j, k, self.z_params[j][k], P, self.agent_coll_rad,
                                                             self.pos_dim))
        return GameCost(self.control_weight, self.control_rate_weight, 0.0, self.inertia_weight, self.path_weight,
                        None, X_prev, self.pos_dim)

    def update_intersample_constraints(self, X_v, U_v, X_nom: np.ndarray, U_nom: np.ndarray, foh,
                                       sigma_ref: float) -> None:  # noqa: ARG002
        """Replace extra_constraints by the linearized inter-sample rows of every segment minimum
        (segment roll-out at sigma = 1, T = I, dt = 1, as :156-176)."""
        from ..utils.intersample_collision import segment_minima
        self.extra_constraints = []
        self.inter_slacks = []
        if not self.obstacles:
            return
        X_nom, U_nom = np.asarray(X_nom, float), np.asarray(U_nom, float)
        rows = segment_minima(foh, X_nom, U_nom, self.obstacles, np.eye(self.n_x), sigma=1.0, dt=1.0)
        for k in range(X_nom.shape[1] - 1):
            for o, obstacle in enumerate(self.obstacles):
                for t_star, h0, gx, gu in rows[(k, o)]:
                    s = Variable((), name=f"s_intersample_k{k}_obs{o}_t{int(t_star * 1e3)}", nonneg=True)
                    self.inter_slacks.append(s)
                    self.extra_constraints.append(IntersampleConstraint(k, obstacle, t_star, h0, gx, gu, X_nom[:, k],
                                                                        U_nom[:, k], s))

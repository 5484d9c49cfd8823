"""3-D single integrator (n=m=3), the reference's SCvx/models/single_integrator_model.py:12-141:
f = u, per-node SOC ||u_k|| <= v_max, linearized sphere obstacles with r + robot_radius + MARGIN_OBS."""
from typing import List, Optional, Tuple

import numpy as np

from ..global_parameters import K
from ..optimization.variables import Variable
from .base_model import BaseModel, straight_line

MARGIN_OBS = 0.0  # SCvx/config/SI_default_game.py:9 (extra clearance around static obstacles)


class SingleIntegratorModel(BaseModel):
    n_x = 3
    n_u = 3
    scvx_model = "si"

    def __init__(self, r_init: np.ndarray = np.array([-8.0, -8.0, -8.0]),
                 r_final: np.ndarray = np.array([8.0, 8.0, 8.0]), v_max: float = 1.0,
                 bounds: Tuple[float, float] = (-10.0, 10.0), robot_radius: float = 0.5,
                 obstacles: Optional[List[Tuple[List[float], float]]] = None):
        self.x_init = np.asarray(r_init, dtype=float).reshape(-1)
        self.x_final = np.asarray(r_final, dtype=float).reshape(-1)
        self.v_max = v_max
        self.lower_bound, self.upper_bound = bounds
        self.robot_radius = robot_radius
        self.obstacles = obstacles if obstacles is not None else [([-5.0, -4.0, -5.0], 2.0), ([0.0, 0.0, 4.0], 2.0)]
        self.s_prime = [Variable((K, 1), nonneg=True) for _ in self.obstacles]  # :51
        self.f = lambda x, u: np.asarray(u, float).reshape(-1).copy()
        self.A = lambda x, u: np.zeros((self.n_x, self.n_x))
        self.B = lambda x, u: np.eye(self.n_x)

    def get_equations(self):
        return self.f, self.A, self.B

    def initialize_trajectory(self, X: np.ndarray, U: np.ndarray):
        straight_line(X, self.x_init, self.x_final)
        U[:] = 0
        return X, U

    def scp_constraints(self):
        """get_constraints (single_integrator_model.py:80-126) as solver template data: BCs, per-node
        SOC ||u_k|| <= v_max, box X[0:3] within [lb + r, ub - r], linearized spheres with clearance
        r + robot_radius + MARGIN_OBS and slack s_prime."""
        lb, ub, r = self.lower_bound, self.upper_bound, self.robot_radius
        return dict(pos_dim=3, x_init=self.x_init, x_final=self.x_final, u_bounds=[], u_soc=self.v_max,
                    x_bounds=[(i, lb + r, ub - r) for i in range(3)],
                    obs=[(np.asarray(c, float)[:3], rad + r + MARGIN_OBS) for c, rad in self.obstacles])

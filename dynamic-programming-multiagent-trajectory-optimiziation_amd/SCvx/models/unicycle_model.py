"""Unicycle (n=3, m=2), the reference's SCvx/models/unicycle_model.py:12-122: f=[v cos th, v sin th, w],
linearized circular obstacles, |w| <= w_max, 0 <= v <= v_max.  Dynamics are hand-written numpy
(the reference lambdifies the same expressions with sympy, :54-63) and run on device as
csrc/models.hpp::Unicycle."""
from typing import List, Optional, Tuple

import numpy as np

from ..global_parameters import K
from ..optimization.variables import Variable
from .base_model import BaseModel, straight_line


class UnicycleModel(BaseModel):
    n_x = 3
    n_u = 2
    scvx_model = "unicycle"

    def __init__(self, r_init: np.ndarray = np.array([-8.0, -8.0, 0.0]),
                 r_final: np.ndarray = np.array([8.0, 8.0, 0.0]), v_max: float = 1.0, w_max: float = np.pi / 6,
                 bounds: Tuple[float, float] = (-10.0, 10.0), robot_radius: float = 0.5,
                 obstacles: Optional[List[Tuple[List[float], float]]] = None):
        self.x_init = np.asarray(r_init, dtype=float).reshape(-1)
        self.x_final = np.asarray(r_final, dtype=float).reshape(-1)
        self.v_max, self.w_max = v_max, w_max
        self.lower_bound, self.upper_bound = bounds
        self.robot_radius = robot_radius
        self.obstacles = obstacles if obstacles is not None else [([5.0, 4.0], 3.0), ([-5.0, -4.0], 3.0),
                                                                  ([0.0, 0.0], 2.0)]
        # obstacle slacks (unicycle_model.py:51); values are filled in by the batched solve
        self.s_prime = [Variable((K, 1), nonneg=True) for _ in self.obstacles]

    @staticmethod
    def _f(x, u):
        x = np.asarray(x, float).reshape(-1)
        u = np.asarray(u, float).reshape(-1)
        return np.array([[u[0] * np.cos(x[2])], [u[0] * np.sin(x[2])], [u[1]]])

    @staticmethod
    def _A(x, u):
        x = np.asarray(x, float).reshape(-1)
        u = np.asarray(u, float).reshape(-1)
        return np.array([[0.0, 0.0, -u[0] * np.sin(x[2])], [0.0, 0.0, u[0] * np.cos(x[2])], [0.0, 0.0, 0.0]])

    @staticmethod
    def _B(x, u):
        th = float(np.asarray(x, float).reshape(-1)[2])
        return np.array([[np.cos(th), 0.0], [np.sin(th), 0.0], [0.0, 1.0]])

    def get_equations(self):
        return self._f, self._A, self._B

    def initialize_trajectory(self, X: np.ndarray, U: np.ndarray):
        straight_line(X, self.x_init, self.x_final)
        U[:] = 0
        return X, U

    def scp_constraints(self):
        """The constraint set of get_constraints (unicycle_model.py:88-114) as solver template data:
        BCs, 0 <= v <= v_max, |w| <= w_max, box X[0:2] within [lb + r, ub - r], linearized obstacles
        with total clearance r + robot_radius and slack s_prime."""
        lb, ub, r = self.lower_bound, self.upper_bound, self.robot_radius
        return dict(pos_dim=2, x_init=self.x_init, x_final=self.x_final,
                    u_bounds=[(0, 0.0, self.v_max), (1, -self.w_max, self.w_max)], u_soc=None,
                    x_bounds=[(i, lb + r, ub - r) for i in range(2)],
                    obs=[(np.asarray(c, float)[:2], rad + r) for c, rad in self.obstacles])

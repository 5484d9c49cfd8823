"""3-D double integrator (n=6: p, v; m=3: a) -- the model of Distributed_opt/dist_scvx_3d.py:10-21 as
an SCvx BaseModel (the reference has no BaseModel for it).  Device dynamics:
csrc/models.hpp::DoubleIntegrator3D."""
import numpy as np

from .base_model import BaseModel, straight_line


class DoubleIntegratorModel(BaseModel):
    n_x = 6
    n_u = 3
    scvx_model = "di"

    def __init__(self, r_init=np.zeros(6), r_final=np.array([10.0, 5.0, 8.0, 0.0, 0.0, 0.0]), u_max=None,
                 bounds=None, robot_radius=0.0, obstacles=None):
        self.x_init = np.asarray(r_init, dtype=float).reshape(-1)
        self.x_final = np.asarray(r_final, dtype=float).reshape(-1)
        self.u_max = u_max
        self.bounds = bounds
        self.robot_radius = robot_radius
        self.obstacles = obstacles or []
        self.s_prime = []
        A = np.zeros((6, 6))
        A[0:3, 3:6] = np.eye(3)
        B = np.zeros((6, 3))
        B[3:6] = np.eye(3)
        self._Ac, self._Bc = A, B

    def get_equations(self):
        f = lambda x, u: np.concatenate([np.asarray(x, float).reshape(-1)[3:6], np.asarray(u, float).reshape(-1)])
        return f, (lambda x, u: self._Ac.copy()), (lambda x, u: self._Bc.copy())

    def initialize_trajectory(self, X, U):
        straight_line(X, self.x_init, self.x_final)
        U[:] = 0
        return X, U

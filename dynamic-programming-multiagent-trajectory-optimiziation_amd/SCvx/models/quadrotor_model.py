"""12-state quadrotor (build-defined; the reference has meshes only):
x = [p(3), v(3), euler (phi, theta, psi), body rates (p, q, r)], u = [thrust, tau_x, tau_y, tau_z],
    p' = v,  v' = (T/m) R(euler) e3 - g e3,  euler' = W(euler) omega,  omega' = J^-1 (tau - omega x J omega)
with diagonal inertia J.  Device dynamics: csrc/models.hpp::Quadrotor12 (same expressions)."""
import numpy as np

from .base_model import BaseModel, straight_line


class QuadrotorModel(BaseModel):
    n_x = 12
    n_u = 4
    scvx_model = "quad"

    def __init__(self, r_init=np.zeros(12), r_final=np.zeros(12), mass=1.0, g=9.81, Jx=0.02, Jy=0.02, Jz=0.04,
                 obstacles=None, robot_radius=0.5):
        self.x_init = np.asarray(r_init, dtype=float).reshape(-1)
        self.x_final = np.asarray(r_final, dtype=float).reshape(-1)
        self.mass, self.g, self.J = mass, g, (Jx, Jy, Jz)
        self.scvx_params = (mass, g, Jx, Jy, Jz)
        self.obstacles = obstacles or []
        self.robot_radius = robot_radius
        self.s_prime = []

    def f(self, x, u):
        x = np.asarray(x, float).reshape(-1)
        u = np.asarray(u, float).reshape(-1)
        Jx, Jy, Jz = self.J
        cf, sf = np.cos(x[6]), np.sin(x[6])
        ct, st = np.cos(x[7]), np.sin(x[7])
        cp, sp = np.cos(x[8]), np.sin(x[8])
        p, q, r = x[9:12]
        a = u[0] / self.mass
        w = q * sf + r * cf
        return np.array([x[3], x[4], x[5],
                         a * (cf * st * cp + sf * sp), a * (cf * st * sp - sf * cp), a * cf * ct - self.g,
                         p + w * st / ct, q * cf - r * sf, w / ct,
                         (u[1] + (Jy - Jz) * q * r) / Jx, (u[2] + (Jz - Jx) * p * r) / Jy,
                         (u[3] + (Jx - Jy) * p * q) / Jz])

    def A(self, x, u, eps=1e-7):
        """Central-difference Jacobian (host-side reference only; the kernels use the analytic one)."""
        x = np.asarray(x, float).reshape(-1)
        J = np.zeros((12, 12))
        for j in range(12):
            d = np.zeros(12)
            d[j] = eps
            J[:, j] = (self.f(x + d, u) - self.f(x - d, u)) / (2 * eps)
        return J

    def B(self, x, u, eps=1e-7):
        u = np.asarray(u, float).reshape(-1)
        J = np.zeros((12, 4))
        for j in range(4):
            d = np.zeros(4)
            d[j] = eps
            J[:, j] = (self.f(x, u + d) - self.f(x, u - d)) / (2 * eps)
        return J

    def get_equations(self):
        return self.f, self.A, self.B

    def initialize_trajectory(self, X, U):
        straight_line(X, self.x_init, self.x_final)
        U[:] = 0
        U[0, :] = self.mass * self.g
        return X, U

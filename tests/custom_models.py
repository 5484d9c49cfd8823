"""User models outside the four built-in device models, written the way the reference writes its models
(sympy expressions lambdified to numpy f/A/B callables, SCvx/models/unicycle_model.py:54-68; the
BaseModel.get_equations contract of SCvx/models/base_model.py:16-24).  They exercise the
runtime-compiled FOH path (scvx_hip.rtc.DeviceModel, hipRTC) against golden vectors of the reference
FirstOrderHold (tests/golden/make_rtc_foh_goldens.py).

  KinematicCar     x = [px, py, theta, v], u = [a, delta]:  f = [v cos th, v sin th, v tan(delta)/L, a]
  DampedDI2D       x = [p (2), v (2)], u = a (2):           f = [v, a - c v]
  CartPole         x = [s, phi, ds, dphi], u = [F]:         the frictionless cart-pole (rational in cos)
  UnicycleAccel    x = [px, py, th, v, w], u = [a, alpha]:  f = [v cos th, v sin th, w, a, alpha] (odd n_x = 5)
  TripleInt3D      x = [p (3), v (3), a (3)], u = jerk (3): f = [v, a - c v, u]  (n_x = 9: the kernel's n > 8 path)
"""
import sympy as sp


class _SympyModel:
    """f, A, B lambdified from sympy, as the reference's models build them."""
    params = {}

    def __init__(self):
        xs = sp.Matrix(sp.symbols(self.x_names, real=True, seq=True))
        us = sp.Matrix(sp.symbols(self.u_names, real=True, seq=True))
        self.n_x, self.n_u = len(xs), len(us)
        self.x_sym, self.u_sym = list(xs), list(us)
        self.p_sym = [sp.Symbol(k, real=True) for k in self.params]
        self.f_param = sp.Matrix(self.dynamics(xs, us, *self.p_sym))      # with the parameters as symbols
        f_expr = self.f_param.subs({s: v for s, v in zip(self.p_sym, self.params.values())})
        self.f_expr = f_expr
        self.f = sp.lambdify((xs, us), f_expr, "numpy")
        self.A = sp.lambdify((xs, us), f_expr.jacobian(xs), "numpy")
        self.B = sp.lambdify((xs, us), f_expr.jacobian(us), "numpy")

    def get_equations(self):
        return self.f, self.A, self.B


class KinematicCar(_SympyModel):
    x_names, u_names = "px py theta v", "a delta"
    params = {"L": 2.5}

    @staticmethod
    def dynamics(x, u, L):
        return [x[3] * sp.cos(x[2]), x[3] * sp.sin(x[2]), x[3] * sp.tan(u[1]) / L, u[0]]


class DampedDI2D(_SympyModel):
    x_names, u_names = "px py vx vy", "ax ay"
    params = {"c": 0.3}

    @staticmethod
    def dynamics(x, u, c):
        return [x[2], x[3], u[0] - c * x[2], u[1] - c * x[3]]


class CartPole(_SympyModel):
    x_names, u_names = "s phi ds dphi", "F"
    params = {"mc": 1.0, "mp": 0.2, "l": 0.5, "g": 9.81}

    @staticmethod
    def dynamics(x, u, mc, mp, l, g):
        s, c = sp.sin(x[1]), sp.cos(x[1])
        den = mc + mp * s ** 2
        dds = (u[0] + mp * s * (l * x[3] ** 2 + g * c)) / den
        ddphi = (-u[0] * c - mp * l * x[3] ** 2 * c * s - (mc + mp) * g * s) / (l * den)
        return [x[2], x[3], dds, ddphi]


class UnicycleAccel(_SympyModel):
    x_names, u_names = "px py th v w", "a alpha"

    @staticmethod
    def dynamics(x, u):
        return [x[3] * sp.cos(x[2]), x[3] * sp.sin(x[2]), x[4], u[0], u[1]]


class TripleInt3D(_SympyModel):
    x_names, u_names = "px py pz vx vy vz ax ay az", "jx jy jz"
    params = {"c": 0.2}

    @staticmethod
    def dynamics(x, u, c):
        return [x[3], x[4], x[5], x[6] - c * x[3], x[7] - c * x[4], x[8] - c * x[5], u[0], u[1], u[2]]


MODELS = {"car": KinematicCar, "damped_di": DampedDI2D, "cartpole": CartPole}

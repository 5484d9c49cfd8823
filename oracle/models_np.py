"""ORACLE / TEST INFRASTRUCTURE ONLY -- never imported by the product path.

Plain-numpy dynamics f(x,u), A=df/dx, B=df/du for the four models the batched
SCvx path supports.  They follow the reference model contract
`BaseModel.get_equations() -> (f, A, B)` (SCvx/models/base_model.py:16-24):

* unicycle  -- SCvx/models/unicycle_model.py:54-63 (sympy lambdify of
               f=[v cos th, v sin th, w]); re-derived by hand here.
* single integrator -- SCvx/models/single_integrator_model.py:54-57 (f=u).
* 3-D double integrator -- the continuous A,B of Distributed_opt/dist_scvx_3d.py:10-21
  (x=[p;v], u=a).  The reference has no SCvx BaseModel for it.
* 12-state quadrotor -- build-defined (absent in the reference):
  x=[p(3), v(3), euler(phi,theta,psi), body rates(p,q,r)], u=[thrust, tau_x, tau_y, tau_z].

These callables are fed to the *reference* FirstOrderHold to make the FOH golden
vectors (tests/golden/make_foh_goldens.py), so the reference's integrator is
what pins the outputs; this file only supplies the model.
"""
import numpy as np

QUAD_DEFAULT = dict(mass=1.0, g=9.81, Jx=0.02, Jy=0.02, Jz=0.04)


def di_equations():
    n, m = 6, 3
    A = np.zeros((n, n))
    A[0:3, 3:6] = np.eye(3)
    B = np.zeros((n, m))
    B[3:6, :] = np.eye(3)

    def f(x, u):
        x = np.asarray(x, float).reshape(-1)
        u = np.asarray(u, float).reshape(-1)
        return np.concatenate([x[3:6], u])

    return f, (lambda x, u: A.copy()), (lambda x, u: B.copy())


def unicycle_equations():
    def f(x, u):
        x = np.asarray(x, float).reshape(-1)
        u = np.asarray(u, float).reshape(-1)
        return np.array([[u[0] * np.cos(x[2])], [u[0] * np.sin(x[2])], [u[1]]])

    def A(x, u):
        x = np.asarray(x, float).reshape(-1)
        u = np.asarray(u, float).reshape(-1)
        return np.array([[0.0, 0.0, -u[0] * np.sin(x[2])],
                         [0.0, 0.0, u[0] * np.cos(x[2])],
                         [0.0, 0.0, 0.0]])

    def B(x, u):
        x = np.asarray(x, float).reshape(-1)
        return np.array([[np.cos(x[2]), 0.0], [np.sin(x[2]), 0.0], [0.0, 1.0]])

    return f, A, B


def si_equations():
    def f(x, u):
        return np.asarray(u, float).reshape(-1).copy()

    return f, (lambda x, u: np.zeros((3, 3))), (lambda x, u: np.eye(3))


def quad_equations(mass=1.0, g=9.81, Jx=0.02, Jy=0.02, Jz=0.04):
    def f(x, u):
        x = np.asarray(x, float).reshape(-1)
        u = np.asarray(u, float).reshape(-1)
        ph, th, ps = x[6:9]
        p, q, r = x[9:12]
        cf, sf, ct, st, cp, sp = np.cos(ph), np.sin(ph), np.cos(th), np.sin(th), np.cos(ps), np.sin(ps)
        a = u[0] / mass
        out = np.zeros(12)
        out[0:3] = x[3:6]
        out[3] = a * (cf * st * cp + sf * sp)
        out[4] = a * (cf * st * sp - sf * cp)
        out[5] = a * (cf * ct) - g
        out[6] = p + (q * sf + r * cf) * st / ct
        out[7] = q * cf - r * sf
        out[8] = (q * sf + r * cf) / ct
        out[9] = (u[1] + (Jy - Jz) * q * r) / Jx
        out[10] = (u[2] + (Jz - Jx) * p * r) / Jy
        out[11] = (u[3] + (Jx - Jy) * p * q) / Jz
        return out

    def A(x, u):
        x = np.asarray(x, float).reshape(-1)
        u = np.asarray(u, float).reshape(-1)
        ph, th, ps = x[6:9]
        p, q, r = x[9:12]
        cf, sf, ct, st, cp, sp = np.cos(ph), np.sin(ph), np.cos(th), np.sin(th), np.cos(ps), np.sin(ps)
        a = u[0] / mass
        J = np.zeros((12, 12))
        J[0, 3] = J[1, 4] = J[2, 5] = 1.0
        J[3, 6] = a * (-sf * st * cp + cf * sp)
        J[3, 7] = a * (cf * ct * cp)
        J[3, 8] = a * (-cf * st * sp + sf * cp)
        J[4, 6] = a * (-sf * st * sp - cf * cp)
        J[4, 7] = a * (cf * ct * sp)
        J[4, 8] = a * (cf * st * cp + sf * sp)
        J[5, 6] = a * (-sf * ct)
        J[5, 7] = a * (-cf * st)
        tt = st / ct
        J[6, 6] = (q * cf - r * sf) * tt
        J[6, 7] = (q * sf + r * cf) / (ct * ct)
        J[6, 9] = 1.0
        J[6, 10] = sf * tt
        J[6, 11] = cf * tt
        J[7, 6] = -q * sf - r * cf
        J[7, 10] = cf
        J[7, 11] = -sf
        J[8, 6] = (q * cf - r * sf) / ct
        J[8, 7] = (q * sf + r * cf) * st / (ct * ct)
        J[8, 10] = sf / ct
        J[8, 11] = cf / ct
        J[9, 10] = (Jy - Jz) * r / Jx
        J[9, 11] = (Jy - Jz) * q / Jx
        J[10, 9] = (Jz - Jx) * r / Jy
        J[10, 11] = (Jz - Jx) * p / Jy
        J[11, 9] = (Jx - Jy) * q / Jz
        J[11, 10] = (Jx - Jy) * p / Jz
        return J

    def B(x, u):
        x = np.asarray(x, float).reshape(-1)
        ph, th, ps = x[6:9]
        cf, sf, ct, st, cp, sp = np.cos(ph), np.sin(ph), np.cos(th), np.sin(th), np.cos(ps), np.sin(ps)
        Bm = np.zeros((12, 4))
        Bm[3, 0] = (cf * st * cp + sf * sp) / mass
        Bm[4, 0] = (cf * st * sp - sf * cp) / mass
        Bm[5, 0] = (cf * ct) / mass
        Bm[9, 1] = 1.0 / Jx
        Bm[10, 2] = 1.0 / Jy
        Bm[11, 3] = 1.0 / Jz
        return Bm

    return f, A, B


MODELS = {
    "di": (6, 3, di_equations),
    "unicycle": (3, 2, unicycle_equations),
    "si": (3, 3, si_equations),
    "quad": (12, 4, quad_equations),
}


class DuckModel:
    """Duck-typed model accepted by the reference FirstOrderHold (n_x, n_u, get_equations)."""

    def __init__(self, name, **kw):
        n, m, eq = MODELS[name]
        self.n_x, self.n_u = n, m
        self._eq = eq(**kw) if kw else eq()

    def get_equations(self):
        return self._eq

"""Generate FOH golden vectors by running the REFERENCE FirstOrderHold in this container.

Run (container only; /root/reference never travels to the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_foh_goldens.py

The reference discretizer SCvx/discretization/first_order_hold.py:52-87 (LSODA via
scipy.integrate.odeint, default rtol=atol=1.49e-8) and its nonlinear roll-outs
(:127-155) are imported unmodified; only the model callables come from
oracle/models_np.py.  Outputs are written as small .npz fixtures next to this
script (inputs + expected outputs, nothing else).
"""
import importlib.util
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, "/root/reference")
from SCvx.discretization.first_order_hold import FirstOrderHold  # noqa: E402  (reference)

spec = importlib.util.spec_from_file_location("models_np", os.path.join(REPO, "oracle", "models_np.py"))
models_np = importlib.util.module_from_spec(spec)
spec.loader.exec_module(models_np)


def straight(x0, x1, K):
    a = np.linspace(0.0, 1.0, K)
    return np.outer(x0, 1 - a) + np.outer(x1, a)


def cases():
    rng = np.random.default_rng(1234)
    out = []
    # 3-D double integrator, K=30 (C1) and K=50 (C2/C3), sigma = Tf = 30 as dist_scvx_3d.py:200-204
    for K, sigma in ((30, 30.0), (50, 30.0), (50, 2.5)):
        X = straight(np.zeros(6), np.array([10.0, 5.0, 8.0, 0, 0, 0]), K) + rng.normal(0, 0.5, (6, K))
        U = rng.normal(0, 0.3, (3, K))
        out.append((f"di_K{K}_s{sigma:g}", "di", K, sigma, X, U))
    # unicycle K=50 (config K), K=100 (global_parameters.K)
    for K, sigma in ((50, 24.141896627765153), (100, 1.0)):
        X = straight(np.array([-8.0, -8.0, 0.0]), np.array([8.0, 8.0, 0.0]), K)
        X[2] += rng.normal(0, 0.4, K)
        U = np.vstack([rng.uniform(0, 1.0, K), rng.uniform(-0.5, 0.5, K)])
        out.append((f"unicycle_K{K}_s{sigma:.4g}", "unicycle", K, sigma, X, U))
    # single integrator K=30
    K = 30
    X = straight(np.array([-8.0, -8.0, -8.0]), np.array([8.0, 8.0, 8.0]), K) + rng.normal(0, 0.2, (3, K))
    U = rng.normal(0, 0.5, (3, K))
    out.append(("si_K30_s12", "si", K, 12.0, X, U))
    # 12-state quadrotor K=50, near hover
    K = 50
    X = np.zeros((12, K))
    X[0:3] = straight(np.zeros(3), np.array([5.0, -3.0, 2.0]), K)
    X[3:6] = rng.normal(0, 0.5, (3, K))
    X[6:9] = rng.normal(0, 0.2, (3, K))
    X[9:12] = rng.normal(0, 0.5, (3, K))
    U = np.vstack([9.81 + rng.normal(0, 1.0, K), rng.normal(0, 0.01, (3, K))])
    out.append(("quad_K50_s5", "quad", K, 5.0, X, U))
    return out


def main():
    for name, model_name, K, sigma, X, U in cases():
        model = models_np.DuckModel(model_name)
        foh = FirstOrderHold(model, K)
        A, B, C, S, z = (a.copy() for a in foh.calculate_discretization(X, U, sigma))
        # nonlinear roll-outs (first_order_hold.py:127-155); sigma kept small so the physical
        # horizon stays sane for the unstable quadrotor
        sig_nl = sigma if model_name != "quad" else 1.0
        Xp = foh.integrate_nonlinear_piecewise(X, U, sig_nl)
        Xf = foh.integrate_nonlinear_full(X[:, 0].copy(), U, sig_nl)
        path = os.path.join(HERE, f"foh_{name}.npz")
        np.savez_compressed(path, model=model_name, K=K, sigma=sigma, X=X, U=U,
                            A_bar=A, B_bar=B, C_bar=C, S_bar=S, z_bar=z,
                            sigma_nl=sig_nl, X_piecewise=Xp, X_full=Xf)
        print(path, A.shape, os.path.getsize(path))


if __name__ == "__main__":
    main()

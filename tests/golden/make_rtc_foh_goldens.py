"""Generate FOH golden vectors for USER models (the runtime-compiled path, scvx_hip.rtc) by running the
REFERENCE FirstOrderHold in this container.

Run (container only; /root/reference never travels to the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_rtc_foh_goldens.py

The reference discretizer SCvx/discretization/first_order_hold.py:52-87 (LSODA via
scipy.integrate.odeint) and its roll-outs (:127-155) are imported unmodified; the models are
tests/custom_models.py (sympy-lambdified numpy f/A/B, the reference's own model idiom).  Outputs are
small .npz fixtures next to this script (inputs + expected outputs).
"""
import importlib.util
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, "/root/reference")
from SCvx.discretization.first_order_hold import FirstOrderHold  # noqa: E402  (reference)

spec = importlib.util.spec_from_file_location("custom_models", os.path.join(os.path.dirname(HERE), "custom_models.py"))
custom_models = importlib.util.module_from_spec(spec)
spec.loader.exec_module(custom_models)


def straight(x0, x1, K):
    a = np.linspace(0.0, 1.0, K)
    return np.outer(x0, 1 - a) + np.outer(x1, a)


def cases():
    rng = np.random.default_rng(4321)
    out = []
    K = 40
    X = straight(np.array([0.0, 0.0, 0.0, 1.0]), np.array([20.0, 8.0, 0.6, 3.0]), K)
    X[2] += rng.normal(0, 0.2, K)
    U = np.vstack([rng.normal(0, 0.5, K), rng.uniform(-0.4, 0.4, K)])
    out.append(("car_K40_s8", "car", K, 8.0, X, U, 1.0))
    K = 30
    X = straight(np.array([-5.0, 2.0, 0.0, 0.0]), np.array([6.0, -3.0, 0.0, 0.0]), K) + rng.normal(0, 0.3, (4, K))
    U = rng.normal(0, 0.6, (2, K))
    out.append(("damped_di_K30_s12", "damped_di", K, 12.0, X, U, 4.0))
    K = 50
    X = np.zeros((4, K))
    X[0] = np.linspace(0.0, 1.0, K)
    X[1] = np.linspace(np.pi, 0.2, K) + rng.normal(0, 0.1, K)
    X[2:] = rng.normal(0, 0.5, (2, K))
    U = rng.normal(0, 2.0, (1, K))
    out.append(("cartpole_K50_s3", "cartpole", K, 3.0, X, U, 1.0))
    return out


def main():
    for name, model_name, K, sigma, X, U, sig_nl in cases():
        model = custom_models.MODELS[model_name]()
        foh = FirstOrderHold(model, K)
        A, B, C, S, z = (a.copy() for a in foh.calculate_discretization(X, U, sigma))
        Xp = foh.integrate_nonlinear_piecewise(X, U, sig_nl)
        Xf = foh.integrate_nonlinear_full(X[:, 0].copy(), U, sig_nl)
        path = os.path.join(HERE, f"rtcfoh_{name}.npz")
        np.savez_compressed(path, model=model_name, K=K, sigma=sigma, X=X, U=U, A_bar=A, B_bar=B, C_bar=C,
                            S_bar=S, z_bar=z, sigma_nl=sig_nl, X_piecewise=Xp, X_full=Xf)
        print(path, A.shape, os.path.getsize(path))


if __name__ == "__main__":
    main()

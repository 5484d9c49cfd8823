"""Generate inter-sample collision golden vectors by running the REFERENCE implementation here.

Run (container only; /root/reference never travels to the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_intersample_goldens.py

Imported unmodified from the reference: SCvx/utils/intersample_collision.py (make_segment_f,
find_critical_times, linearize_h: odeint roll-outs, central differences, 100-sample scan +
bisection) and SCvx/discretization/first_order_hold.py (FirstOrderHold._dx, .dt).  Only the model
callables come from oracle/models_np.py.  The scenario follows the reference's own call site,
SCvx/models/game_si_model.py:156-176 (per segment k: make_segment_f(foh, U[:,k], U[:,k+1],
sigma=1.0); per obstacle: find_critical_times(..., dt=1.0) then linearize_h at every t*).
Outputs: small .npz fixtures (inputs + expected outputs) next to this script.
"""
import importlib.util
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, "/root/reference")
from SCvx.discretization.first_order_hold import FirstOrderHold  # noqa: E402  (reference)
from SCvx.utils.intersample_collision import find_critical_times, linearize_h, make_segment_f  # noqa: E402

spec = importlib.util.spec_from_file_location("models_np", os.path.join(REPO, "oracle", "models_np.py"))
models_np = importlib.util.module_from_spec(spec)
spec.loader.exec_module(models_np)

MAXC = 4


def run_case(name, model, K, sigma, X, U, T, obstacles):
    foh = FirstOrderHold(models_np.DuckModel(model), K)
    n, m = X.shape[0], U.shape[0]
    O = len(obstacles)
    cnt = np.zeros((K - 1, O), np.int32)
    tc = np.zeros((K - 1, O, MAXC))
    h0 = np.zeros((K - 1, O, MAXC))
    gx = np.zeros((K - 1, O, MAXC, n))
    gu = np.zeros((K - 1, O, MAXC, m))
    for k in range(K - 1):
        f_seg, _ = make_segment_f(foh, U[:, k], U[:, k + 1], sigma=sigma)
        for o, obs in enumerate(obstacles):
            ts = find_critical_times(xk=X[:, k], uk=U[:, k], f=f_seg, T=T, obstacle=obs, dt=1.0)
            assert len(ts) <= MAXC
            cnt[k, o] = len(ts)
            for c, t in enumerate(ts):
                tc[k, o, c] = t
                h0[k, o, c], gx[k, o, c], gu[k, o, c] = linearize_h(xk=X[:, k], uk=U[:, k], t_star=t, f=f_seg, T=T,
                                                                     obstacle=obs)
    oc = np.array([np.asarray(c, float) for c, _ in obstacles])
    orad = np.array([r for _, r in obstacles], float)
    np.savez(os.path.join(HERE, f"intersample_{name}.npz"), model=model, K=K, sigma=sigma, X=X, U=U, T=T,
             obs_center=oc, obs_radius=orad, count=cnt, t_crit=tc, h0=h0, grad_x=gx, grad_u=gu)
    print(name, "segments with minima:", int((cnt > 0).sum()), "total minima:", int(cnt.sum()))


def main():
    rng = np.random.default_rng(77)
    # 3-D single integrator (the reference's own intersample user, game_si_model.py), K = 20, sigma 1
    K = 20
    a = np.linspace(0, 1, K)
    X = np.outer([-8.0, -8.0, -8.0], 1 - a) + np.outer([8.0, 7.0, 9.0], a) + rng.normal(0, 0.05, (3, K))
    U = np.tile(np.array([[16.0], [15.0], [17.0]]), (1, K)) + rng.normal(0, 1.0, (3, K))
    obstacles = [(np.array([0.3, -0.4, 0.2]), 2.0), (np.array([-4.0, -3.0, -5.0]), 1.5),
                 (np.array([5.0, 5.5, 4.0]), 1.0)]
    run_case("si_K20", "si", K, 1.0, X, U, np.eye(3), obstacles)
    # unicycle (nonlinear), planar projection T = [I2 0], K = 16, sigma 1
    K = 16
    a = np.linspace(0, 1, K)
    X = np.outer([-8.0, -8.0, np.pi / 4], 1 - a) + np.outer([8.0, 8.0, np.pi / 4], a)
    X[2] += rng.normal(0, 0.1, K)
    U = np.vstack([np.full(K, 22.6) + rng.normal(0, 1.0, K), rng.normal(0, 0.8, K)])
    T = np.array([[1.0, 0.0, 0.0], [0.0, 1.0, 0.0]])
    obstacles = [(np.array([0.5, -0.5]), 2.0), (np.array([-5.0, -4.0]), 3.0), (np.array([5.0, 4.0]), 3.0)]
    run_case("unicycle_K16", "unicycle", K, 1.0, X, U, T, obstacles)


if __name__ == "__main__":
    main()

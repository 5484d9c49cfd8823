"""GPU parity of the inter-sample clearance scan (scvx_intersample_batched; SCvx/utils/
intersample_collision.py as called by SCvx/models/game_si_model.py:156-176).

  * against the reference itself: tests/golden/intersample_*.npz were produced by importing the
    reference's find_critical_times / linearize_h / make_segment_f with odeint roll-outs
    (tests/golden/make_intersample_goldens.py).  Same minima; t* within 1e-5, h0 within 1e-6,
    grad_x within 1e-4 (the reference's own central differences of an ODE solved to 1.49e-8 carry
    ~1e-4 noise), grad_u identically 0;
  * against oracle/intersample_np.py (the same RK4 arithmetic on the CPU) on a random batch:
    t* within 1e-8, h0 within 1e-10, grad_x within 1e-6."""
import glob
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
GOLD = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "intersample_*.npz")))


def _foh(model, K):
    from SCvx.discretization.first_order_hold import FirstOrderHold
    from SCvx.models.single_integrator_model import SingleIntegratorModel
    from SCvx.models.unicycle_model import UnicycleModel
    return FirstOrderHold({"si": SingleIntegratorModel, "unicycle": UnicycleModel}[model](), K)


def _obstacles(d):
    return [(d["obs_center"][o], float(d["obs_radius"][o])) for o in range(d["obs_center"].shape[0])]


@pytest.mark.parametrize("path", GOLD, ids=[os.path.basename(p) for p in GOLD])
def test_batched_scan_matches_reference_goldens(cuda, path):
    from SCvx.utils.intersample_collision import segment_minima
    d = np.load(path)
    K, model = int(d["K"]), str(d["model"])
    res = segment_minima(_foh(model, K), d["X"], d["U"], _obstacles(d), d["T"], sigma=float(d["sigma"]))
    for k in range(K - 1):
        for o in range(d["obs_center"].shape[0]):
            got = res[(k, o)]
            assert len(got) == d["count"][k, o], (k, o)
            for c, (t, h0, gx, gu) in enumerate(got):
                assert abs(t - d["t_crit"][k, o, c]) < 1e-5
                assert abs(h0 - d["h0"][k, o, c]) < 1e-6
                assert np.abs(gx - d["grad_x"][k, o, c]).max() < 1e-4
                assert np.all(gu == 0.0)


@pytest.mark.parametrize("path", GOLD, ids=[os.path.basename(p) for p in GOLD])
def test_reference_api_on_device_segments(cuda, path):
    """make_segment_f -> find_critical_times -> linearize_h, the reference's call sequence."""
    from SCvx.utils.intersample_collision import find_critical_times, h_i, linearize_h, make_segment_f
    d = np.load(path)
    K, model = int(d["K"]), str(d["model"])
    foh = _foh(model, K)
    obs = _obstacles(d)
    for k, o in zip(*np.nonzero(d["count"])):
        f_seg, dtp = make_segment_f(foh, d["U"][:, k], d["U"][:, k + 1], sigma=float(d["sigma"]))
        assert dtp == pytest.approx(float(d["sigma"]) / (K - 1))
        ts = find_critical_times(xk=d["X"][:, k], uk=d["U"][:, k], f=f_seg, T=d["T"], obstacle=obs[o], dt=1.0)
        assert len(ts) == d["count"][k, o]
        for c, t in enumerate(ts):
            assert abs(t - d["t_crit"][k, o, c]) < 1e-5
            h0, gx, gu = linearize_h(xk=d["X"][:, k], uk=d["U"][:, k], t_star=t, f=f_seg, T=d["T"], obstacle=obs[o])
            assert abs(h0 - d["h0"][k, o, c]) < 1e-6
            assert np.abs(gx - d["grad_x"][k, o, c]).max() < 1e-4
            assert np.all(gu == 0.0)
            assert h_i(d["X"][:, k], d["U"][:, k], t, f_seg, d["T"], obs[o]) == pytest.approx(h0, abs=1e-12)


def test_random_batch_matches_cpu_restatement(cuda):
    import torch
    import scvx_hip
    from oracle import intersample_np
    rng = np.random.default_rng(5)
    N, K = 3, 12
    a = np.linspace(0, 1, K)
    X = np.zeros((N, K, 3))
    U = np.zeros((N, K, 3))
    for i in range(N):
        p0, p1 = rng.uniform(-8, -6, 3), rng.uniform(6, 8, 3)
        X[i] = np.outer(1 - a, p0) + np.outer(a, p1) + rng.normal(0, 0.1, (K, 3))
        U[i] = (p1 - p0)[None] / 1.0 + rng.normal(0, 2.0, (K, 3))
    sig = np.ones(N)
    obs = [(rng.uniform(-2, 2, 3), 1.5), (rng.uniform(-5, 5, 3), 1.0)]
    T = lambda x: torch.tensor(x, dtype=torch.float64, device=cuda)  # noqa: E731
    out = scvx_hip.intersample_batched("si", T(X), T(U), T(sig), obs, max_crit=4)
    h = {k: v.cpu().numpy() for k, v in out.items()}
    total = 0
    for i in range(N):
        for k in range(K - 1):
            for o, (c, r) in enumerate(obs):
                ref = intersample_np.segment("si", X[i, k], U[i, k], U[i, k + 1], 1.0 / (K - 1), np.eye(3), c, r, nsub=1)
                assert h["n_crit"][i, k, o] == len(ref)
                total += len(ref)
                for q, (t, h0, gx, _) in enumerate(ref):
                    assert abs(h["t_crit"][i, k, o, q] - t) < 1e-8
                    assert abs(h["h0"][i, k, o, q] - h0) < 1e-10
                    assert np.abs(h["grad_x"][i, k, o, q] - gx).max() < 1e-6
    assert total >= 3

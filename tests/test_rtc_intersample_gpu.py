"""GPU: the inter-sample clearance scan of a USER model (tests/custom_models.KinematicCar, outside the built-in
device models), on the scan kernel compiled next to the model's own f (csrc/intersample_body.hpp through hipRTC,
scvx_rtc_intersample_batched) -- the reference's scan is model-agnostic (SCvx/utils/intersample_collision.py:104-126
integrates model.get_equations()'s f with odeint).

  * segment_minima (every segment x obstacle in one launch) against oracle/intersample_np.segment_f (the same RK4
    arithmetic on the CPU, with the car's own numpy f): the same minima, t* within 1e-8, h0 within 1e-10, grad_x
    within 1e-6 (the tolerances of tests/test_intersample_gpu.py's random batch), grad_u identically 0;
  * the reference's call sequence make_segment_f -> find_critical_times -> linearize_h on the device segments."""
import numpy as np
import pytest

import custom_models as cm

pytestmark = pytest.mark.gpu

K, SIGMA = 16, 6.0
OBS = [(np.array([-2.0, 0.9]), 0.6), (np.array([2.5, 0.0]), 0.8), (np.array([0.0, 3.0]), 0.5)]
T = np.eye(4)[:2]


def _traj():
    x0, xf = np.array([-6.0, -1.0, 0.2, 1.5]), np.array([6.0, 2.0, 0.3, 1.5])
    a = np.linspace(0.0, 1.0, K)
    X = (1 - a)[None] * x0[:, None] + a[None] * xf[:, None]
    U = np.zeros((2, K))
    U[0] = 0.3 * np.sin(np.linspace(0, 3, K))
    U[1] = 0.05 * np.cos(np.linspace(0, 2, K))
    return X, U


def test_user_model_segment_minima_matches_oracle(cuda):
    from oracle import intersample_np
    from SCvx.discretization.first_order_hold import FirstOrderHold
    from SCvx.utils.intersample_collision import segment_minima
    from scvx_hip.rtc import DeviceModel
    car = cm.KinematicCar()
    foh = FirstOrderHold(car, K)
    assert isinstance(foh._name, DeviceModel)
    X, U = _traj()
    res = segment_minima(foh, X, U, OBS, T, sigma=SIGMA)
    f = car.get_equations()[0]
    dtp = SIGMA / (K - 1)
    found = 0
    for k in range(K - 1):
        for o, (c, r) in enumerate(OBS):
            ref = intersample_np.segment_f(f, X[:, k], U[:, k], U[:, k + 1], dtp, T, c, r, nsub=foh._name.nsub)
            got = res[(k, o)]
            assert len(got) == len(ref), (k, o, len(got), len(ref))
            for (t, h0, gx, gu), (tr, hr, gxr, _) in zip(got, ref):
                assert abs(t - tr) < 1e-8 and abs(h0 - hr) < 1e-10, (k, o, t, tr, h0, hr)
                assert np.abs(gx - gxr).max() < 1e-6 and np.all(gu == 0.0)
            found += len(got)
    assert found >= 3, found   # the construction passes every obstacle: interior minima exist


def test_user_model_reference_api_on_device_segments(cuda):
    from oracle import intersample_np
    from SCvx.discretization.first_order_hold import FirstOrderHold
    from SCvx.utils.intersample_collision import find_critical_times, linearize_h, make_segment_f
    car = cm.KinematicCar()
    foh = FirstOrderHold(car, K)
    X, U = _traj()
    f = car.get_equations()[0]
    checked = 0
    for k in range(K - 1):
        f_seg, dtp = make_segment_f(foh, U[:, k], U[:, k + 1], sigma=SIGMA)
        assert dtp == pytest.approx(SIGMA / (K - 1))
        for o, obs in enumerate(OBS):
            ts = find_critical_times(xk=X[:, k], uk=U[:, k], f=f_seg, T=T, obstacle=obs, dt=1.0)
            ref = intersample_np.segment_f(f, X[:, k], U[:, k], U[:, k + 1], dtp, T, obs[0], obs[1],
                                           nsub=foh._name.nsub)
            assert len(ts) == len(ref)
            for t, (tr, hr, gxr, _) in zip(ts, ref):
                assert abs(t - tr) < 1e-8
                h0, gx, gu = linearize_h(X[:, k], U[:, k], t, f_seg, T, obs)
                assert abs(h0 - hr) < 1e-9 and np.abs(gx - gxr).max() < 1e-5 and np.all(gu == 0.0)
                checked += 1
    assert checked >= 3

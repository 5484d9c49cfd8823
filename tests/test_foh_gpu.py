"""GPU parity: the HIP batched FOH (scvx_foh_batched, through the C-ABI) against
  (1) golden vectors of the reference FirstOrderHold (LSODA, first_order_hold.py:52-155) and
  (2) the C restatement oracle/foh_ref.c on random batches (same RK4 algorithm -> ~1e-13)."""
import glob
import os

import numpy as np
import pytest

import scvx_hip
from oracle import foh_oracle

pytestmark = pytest.mark.gpu
GOLD = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "foh_*.npz")))


def rel(a, b):
    return np.max(np.abs(a - b)) / max(1.0, np.max(np.abs(b)))


@pytest.mark.parametrize("path", GOLD, ids=[os.path.basename(p) for p in GOLD])
def test_hip_foh_matches_reference_goldens(cuda, path):
    import torch
    d = np.load(path)
    model = str(d["model"])
    X = torch.tensor(d["X"].T[None].copy(), device=cuda)
    U = torch.tensor(d["U"].T[None].copy(), device=cuda)
    sig = torch.tensor([float(d["sigma"])], dtype=torch.float64, device=cuda)
    disc = scvx_hip.foh_batched(model, X, U, sig)
    outs = scvx_hip.unpack_disc(disc, model)
    for name, o in zip(["A_bar", "B_bar", "C_bar", "S_bar", "z_bar"], outs):
        o = o[0].cpu().numpy()
        assert o.shape == d[name].shape
        assert rel(o, d[name]) < 1e-7, name
    for pw, key in ((True, "X_piecewise"), (False, "X_full")):
        sgn = torch.tensor([float(d["sigma_nl"])], dtype=torch.float64, device=cuda)
        xo = scvx_hip.integrate_nonlinear(model, X, U, sgn, pw)[0].cpu().numpy().T
        assert rel(xo, d[key]) < (1e-7 if pw else 1e-6), key


@pytest.mark.parametrize("model", ["di", "unicycle", "si", "quad"])
def test_hip_foh_matches_oracle_batched(cuda, model):
    import torch
    n, m = scvx_hip.MODEL_DIMS[model]
    rng = np.random.default_rng(7)
    N, K = 33, 50
    X = rng.normal(0, 0.5, (N, K, n))
    U = rng.normal(0, 0.3, (N, K, m))
    if model == "quad":
        U[:, :, 0] += 9.81
    sig = rng.uniform(1.0, 5.0, N)
    disc = scvx_hip.foh_batched(model, torch.tensor(X, device=cuda), torch.tensor(U, device=cuda),
                                torch.tensor(sig, device=cuda)).cpu().numpy()
    nsub = scvx_hip.DEFAULT_NSUB[model]
    for a in (0, 17, 32):
        ref = foh_oracle.foh(model, X[a].T, U[a].T, sig[a], nsub=nsub)
        got = [o.numpy() for o in scvx_hip.unpack_disc(__import__("torch").tensor(disc[a]), model)]
        for g, r in zip(got, ref):
            assert rel(g, r) < 1e-12

"""GPU: the HIP trust-region kernel (scvx_qp_solve_batched through the C-ABI) against the 48 HiGHS-certified Q1
subproblems of tests/golden/highs_qp_{c3,c4}.npz (see tests/test_highs_qp_cpu.py for what they are).

One launch per family at the bench's tolerance (1e-8): every agent status 0, optimal value within 1e-8 relative
of the certified optimum, inputs within the strong-convexity bound of that gap (tests/highs_fixtures.U_BOUND)."""
import numpy as np
import pytest

from highs_fixtures import FAMILIES, K, U_BOUND, load, rel, u_dist

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", FAMILIES)
def test_kernel_matches_highs(cuda, name):
    import torch
    import scvx_hip
    f = load(name)
    t = lambda x, dt=torch.float64: torch.tensor(np.ascontiguousarray(x), device=cuda, dtype=dt)   # noqa: E731
    spec = scvx_hip.QPSpec(model="di", K=K, box=f["box_list"], obs=f["obs_list"], w_obs=1e6, j_max=f["jm"],
                           w_coll=1e4, tol=1e-8, max_iter=80)
    rows = (t(f["rows"]), t(f["cnt"], torch.int32)) if f["jm"] else (None, None)
    out = scvx_hip.qp_solve_batched(spec, t(f["disc"]), t(f["sigma"]), t(f["Xref"]), t(f["Uref"]), t(f["x_init"]),
                                    t(f["x_final"]), t(f["tr"]), *rows)
    st = out["status"].cpu().numpy()
    assert (st == 0).all(), st
    og = out["obj"].cpu().numpy()
    r = rel(og, f["obj"])
    print(name, "kernel max rel obj diff", r.max())
    assert (r <= 1e-8).all(), r
    ud = u_dist(out["U"].cpu().numpy(), f)
    assert (ud <= U_BOUND * np.maximum(1.0, np.abs(f["obj"]))).all(), ud

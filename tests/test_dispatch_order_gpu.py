"""GPU: the QP launch's dispatch order (scvx_qp_solve_batched_ordered, include/scvx_hip.h; QPSolver.solve(order=...);
JacobiSCvx(dispatch_order="lpt")).  Workgroup b solves agent order[b]: the order only decides which solves start
first when the agents outnumber the resident waves, so every output must be bit-identical to the agent-order
launch -- cold and warm-started, and through the coupled Jacobi loop that deals the agents longest-first."""
import numpy as np
import pytest

import scvx_hip

pytestmark = pytest.mark.gpu

BOX = [(0, -12, 12), (1, -12, 12)]
KEYS = ("X", "U", "slack_coll", "obj", "status", "iters")


def _t(x, cuda, dtype=None):
    import torch
    return torch.tensor(np.ascontiguousarray(x), device=cuda, dtype=dtype or torch.float64)


def test_ordered_launch_is_bit_identical(cuda):
    import torch
    from scvx_hip import workloads
    N, K = 1536, 50            # more agents than one wave per SIMD holds at once (1024): later starts follow the order
    sc = workloads.synthetic_di(N, K=K, seed=5, obstacles=8)
    spec = scvx_hip.QPSpec(model="di", K=K, box=BOX, obs=sc["obs"], w_obs=1e6, u_max=1.0, tol=1e-8, max_iter=60)
    X, U, sig = _t(sc["X"], cuda), _t(sc["U"], cuda), _t(sc["sigma"], cuda)
    xi, xf, tr = _t(sc["x_init"], cuda), _t(sc["x_final"], cuda), _t(np.full(N, 0.25), cuda)
    disc = scvx_hip.foh_batched("di", X, U, sig)
    rng = np.random.default_rng(0)
    orders = [None, torch.arange(N - 1, -1, -1, dtype=torch.int32, device=cuda),
              _t(rng.permutation(N), cuda, torch.int32)]
    solvers = [scvx_hip.QPSolver(spec, N, device=cuda) for _ in orders]
    outs = [{k: v.clone() for k, v in s.solve(disc, sig, X, U, xi, xf, tr, order=o).items()}
            for s, o in zip(solvers, orders)]
    assert (outs[0]["status"] != 2).all() and (outs[0]["status"] == 0).float().mean() > 0.9
    for o in outs[1:]:
        for k in KEYS:
            assert torch.equal(o[k], outs[0][k]), k
    # warm-started re-solve at the solution (each solver's own workspace), orders swapped
    X2, U2 = outs[0]["X"], outs[0]["U"]
    disc2 = scvx_hip.foh_batched("di", X2, U2, sig)
    warm = torch.ones(N, dtype=torch.int32, device=cuda)
    outs2 = [{k: v.clone() for k, v in s.solve(disc2, sig, X2, U2, xi, xf, tr, warm=warm, order=o).items()}
             for s, o in zip(solvers, orders[::-1])]
    for o in outs2[1:]:
        for k in KEYS:
            assert torch.equal(o[k], outs2[0][k]), k
    with pytest.raises(ValueError):
        solvers[0].solve(disc, sig, X, U, xi, xf, tr, order=torch.arange(N, device=cuda))   # int64: rejected


def test_jacobi_lpt_dispatch_matches_agent_order(cuda):
    """The coupled Jacobi loop (the C4 construction) with the longest-first dispatch reproduces the
    agent-order run exactly, step by step."""
    import bench
    import torch
    from scvx_hip.scvx import CouplingSpec, JacobiSCvx
    sc, w, cfg = bench.make_coupled("c4", 1, 0, cuda)      # 4096 agents: four rounds of resident waves
    spec = scvx_hip.QPSpec(model=cfg["model"], K=bench.K, box=cfg["box"], obs=cfg["obs"], w_obs=1e6, j_max=cfg["j_max"],
                           w_coll=1e4, tol=1e-8, max_iter=60, **cfg["vc"])
    runs = []
    for mode in ("none", "lpt"):
        drv = JacobiSCvx(spec, w["x_init"], w["x_final"], w["sigma"], bench.TR0, coupling=CouplingSpec(R=cfg["R"]),
                         tr_rule="global", warm_max_status=1, dispatch_order=mode)
        X, U = w["X"].clone(), w["U"].clone()
        hist = []
        for _ in range(4):
            X, U, out = drv.step(X, U)
            hist.append((X.clone(), out["iters"].clone()))
        assert (mode == "none") == (drv.order is None)   # 4096 agents > the resident waves: lpt applies
        runs.append(hist)
    for (xa, ia), (xb, ib) in zip(*runs):
        assert torch.equal(xa, xb) and torch.equal(ia, ib)

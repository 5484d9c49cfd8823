"""GPU: the QP kernel's warm start (scvx_qp_solve_batched(warm=...), include/scvx_hip.h) on the Jacobi SCvx
loop of the bench workload (C3): each step re-solves every agent's subproblem re-linearised at its own
previous solution, starting from that solve's primal-dual point.

The warm-started solve must reach the same optimum as a cold solve of the same subproblem (objective 1e-8
relative -- the stopping rule's gap tolerance -- and the inputs within the strong-convexity bound of that
gap), as the CPU twin's warm start does (oracle/scvx_cpu.cpp warm_point, the same rule), with fewer IPM
iterations."""
import numpy as np
import pytest

import scvx_hip
from oracle import qp_cpu

pytestmark = pytest.mark.gpu

BOX = [(0, -12, 12), (1, -12, 12)]


def _t(x, cuda, dtype=None):
    import torch
    return torch.tensor(np.ascontiguousarray(x), device=cuda, dtype=dtype or torch.float64)


def test_warm_start_reaches_the_cold_optimum(cuda):
    import torch
    from scvx_hip import workloads
    N, K = 512, 50
    sc = workloads.synthetic_di(1024, K=K, seed=1, obstacles=8)
    sub = {k: np.ascontiguousarray(sc[k][::2]) for k in ("X", "U", "x_init", "x_final", "sigma")}
    spec = scvx_hip.QPSpec(model="di", K=K, box=BOX, obs=sc["obs"], w_obs=1e6, u_max=1.0, tol=1e-8, max_iter=60)
    tpl = qp_cpu.make_template(6, 3, K, box=BOX, obs=sc["obs"], w_obs=1e6, u_max=1.0, tol=1e-8, max_iter=60)
    warm_solver, cold_solver = scvx_hip.QPSolver(spec, N, device=cuda), scvx_hip.QPSolver(spec, N, device=cuda)
    ws = np.zeros((N, qp_cpu.warm_doubles(tpl)))
    X, U, sig = _t(sub["X"], cuda), _t(sub["U"], cuda), _t(sub["sigma"], cuda)
    xi, xf, tr = _t(sub["x_init"], cuda), _t(sub["x_final"], cuda), _t(np.full(N, 0.25), cuda)
    warm = None
    its_cold, its_warm = [], []
    for step in range(4):
        disc = scvx_hip.foh_batched("di", X, U, sig)
        ow = {k: v.clone() for k, v in warm_solver.solve(disc, sig, X, U, xi, xf, tr, warm=warm).items()}
        oc = cold_solver.solve(disc, sig, X, U, xi, xf, tr)
        sw, sc_ = ow["status"].cpu().numpy(), oc["status"].cpu().numpy()
        assert (sw == 0).all() and (sc_ == 0).all(), (step, np.bincount(sw, minlength=3), np.bincount(sc_, minlength=3))
        ow_, oc_ = ow["obj"].cpu().numpy(), oc["obj"].cpu().numpy()
        assert np.all(np.abs(ow_ - oc_) <= 1e-8 * np.maximum(1.0, np.abs(oc_))), step
        du = np.abs(ow["U"].cpu().numpy()[:, :-1] - oc["U"].cpu().numpy()[:, :-1]).max(axis=(1, 2))
        assert np.all(du <= 3.0 * np.sqrt(1e-8 * np.maximum(1.0, np.abs(oc_)))), step
        # the CPU twin's warm start on the same subproblems
        wn = None if warm is None else warm.cpu().numpy()
        cpu = qp_cpu.solve_batched(tpl, disc.cpu().numpy(), sub["sigma"], X.cpu().numpy(), U.cpu().numpy(),
                                   sub["x_init"], sub["x_final"], np.full(N, 0.25), nthreads=8, warm=wn, wstate=ws)
        assert (cpu["status"] == 0).all()
        assert np.all(np.abs(ow_ - cpu["obj"]) <= 1e-8 * np.maximum(1.0, np.abs(cpu["obj"]))), step
        if step:
            its_cold.append(oc["iters"].float().mean().item())
            its_warm.append(ow["iters"].float().mean().item())
            # the twin's warm iteration counts track the kernel's (same rule, rounding-level differences)
            assert abs(cpu["iters"].mean() - its_warm[-1]) < 0.5, (cpu["iters"].mean(), its_warm[-1])
        X, U = ow["X"], ow["U"]      # the Jacobi update (every agent solved)
        warm = (ow["status"] == 0).to(torch.int32)
    assert np.mean(its_warm) < 0.6 * np.mean(its_cold), (its_warm, its_cold)


def test_warm_flag_on_a_never_solved_slot_starts_cold(cuda):
    """QPSolver.solve(warm=...) on slots this solver has not solved yet: their workspace holds no primal-dual
    state, so they start cold (the same result as warm=None), bit for bit."""
    import torch
    from scvx_hip import workloads
    N, K = 64, 50
    sc = workloads.synthetic_di(N, K=K, seed=1, obstacles=8)
    spec = scvx_hip.QPSpec(model="di", K=K, box=BOX, obs=sc["obs"], w_obs=1e6, u_max=1.0, tol=1e-8, max_iter=60)
    X, U, sig = _t(sc["X"], cuda), _t(sc["U"], cuda), _t(sc["sigma"], cuda)
    xi, xf, tr = _t(sc["x_init"], cuda), _t(sc["x_final"], cuda), _t(np.full(N, 0.25), cuda)
    disc = scvx_hip.foh_batched("di", X, U, sig)
    ref = {k: v.clone() for k, v in scvx_hip.QPSolver(spec, N, device=cuda).solve(disc, sig, X, U, xi, xf, tr).items()}
    s = scvx_hip.QPSolver(spec, N, device=cuda)
    s.workspace.fill_(float("nan"))                      # what an uninitialised slot could hold
    half = s.solve(disc[:N // 2], sig[:N // 2], X[:N // 2], U[:N // 2], xi[:N // 2], xf[:N // 2], tr[:N // 2],
                   n=N // 2, warm=torch.ones(N // 2, dtype=torch.int32, device=cuda))
    assert torch.equal(half["X"], ref["X"][:N // 2]) and torch.equal(half["status"], ref["status"][:N // 2])
    out = s.solve(disc, sig, X, U, xi, xf, tr, warm=torch.zeros(N, dtype=torch.int32, device=cuda) + 1)
    # slots >= N/2 were never solved: cold; slots < N/2 warm-start from the identical subproblem's optimum
    assert torch.equal(out["X"][N // 2:], ref["X"][N // 2:])
    assert (out["status"] == 0).all()
    assert out["iters"][:N // 2].float().mean() < ref["iters"][:N // 2].float().mean()

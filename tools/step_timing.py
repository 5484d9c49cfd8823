"""Diagnostics: wall-clock breakdown of one bench step (FOH, QP launch, bookkeeping) with syncs."""
import os, sys, time
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "dynamic-programming-multiagent-trajectory-optimiziation_amd"))
sys.path.insert(0, REPO)
import torch
import bench
import scvx_hip
from scvx_hip.scvx import JacobiSCvx

dev = torch.device("cuda")
sc, w = bench.make_workload(1024, 1, dev)
spec = scvx_hip.QPSpec(model="di", K=50, box=bench.BOX, obs=sc["obs"], w_obs=1e6, u_max=1.0, tol=1e-9, max_iter=60)
drv = JacobiSCvx(spec, w["x_init"], w["x_final"], w["sigma"], 0.25)
X, U = w["X"].clone(), w["U"].clone()
for rep in range(4):
    torch.cuda.synchronize(); t0 = time.perf_counter()
    drv.disc = scvx_hip.foh_batched("di", X, U, w["sigma"], out=drv.disc)
    torch.cuda.synchronize(); t1 = time.perf_counter()
    out = drv.solver.solve(drv.disc, w["sigma"], X, U, w["x_init"], w["x_final"], drv.tr)
    t2 = time.perf_counter()
    torch.cuda.synchronize(); t3 = time.perf_counter()
    Xn, Un, o2 = drv.step(X, U)
    torch.cuda.synchronize(); t4 = time.perf_counter()
    print(f"foh {1e3*(t1-t0):.3f} ms | qp launch (host) {1e3*(t2-t1):.3f} ms, qp total {1e3*(t3-t1):.3f} ms | full drv.step {1e3*(t4-t3):.3f} ms", flush=True)

# bench.py's timed loop, instrumented
stream = torch.cuda.current_stream()
for rep in range(3):
    torch.cuda.synchronize(); t0 = time.perf_counter()
    for _ in range(5):
        drv.disc = scvx_hip.foh_batched("di", X, U, w["sigma"], out=drv.disc)
        e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        out = drv.solver.solve(drv.disc, w["sigma"], X, U, w["x_init"], w["x_final"], drv.tr)
        e1.record(stream)
        cost = (out["U"][:, :-1, :] ** 2).sum(dim=(1, 2))
        shrink = (cost > drv.prev_cost).to(torch.float64)
        drv.tr.mul_(1.0 - 0.5 * shrink)
        drv.prev_cost.copy_(cost)
        X.copy_(out["X"]); U.copy_(out["U"])
    torch.cuda.synchronize(); t1 = time.perf_counter()
    print(f"bench-like loop: {1e3*(t1-t0)/5:.3f} ms/step, last qp event {e0.elapsed_time(e1):.3f} ms, iters max {int(out['iters'].max())}", flush=True)

"""C3 dispatch-order experiment (GPU diagnostic): the bench's C3 Jacobi loop with every agent resident, its QP
launches dealt in different orders by the previous step's IPM iterations -- agent order, longest first,
shortest first, longest spread over CUs (rank r -> workgroup (r % 256) * 4 + r // 256), random -- alternating
per step.  The order decides only which CU / SIMD an agent's wave lands on (results are bit-identical,
tests/test_dispatch_order_gpu.py).  Prints the median QP launch time per order.
usage: python tools/dispatch_ab.py [steps]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "dynamic-programming-multiagent-trajectory-optimiziation_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import scvx_hip  # noqa: E402
from scvx_hip.scvx import JacobiSCvx  # noqa: E402


def main(steps=40):
    steps = int(steps)
    dev = torch.device("cuda:0")
    N = 1024
    sc, w = bench.make_workload(N, seed=1, device=dev)
    spec = scvx_hip.QPSpec(model="di", K=bench.K, box=bench.BOX, obs=sc["obs"], w_obs=1e6, u_max=bench.U_MAX, tol=1e-8,
                           max_iter=60)
    drv = JacobiSCvx(spec, w["x_init"], w["x_final"], w["sigma"], bench.TR0, tr_rule="per_agent", warm_max_status=1,
                     dispatch_order="none")
    X, U = w["X"].clone(), w["U"].clone()
    for _ in range(5):
        X, U, out = drv.step(X, U)
    rng = np.random.default_rng(0)
    n_cu = torch.cuda.get_device_properties(dev).multi_processor_count

    def orders(iters):
        desc = torch.argsort(iters, descending=True, stable=True)
        spread = torch.empty_like(desc)
        r = torch.arange(N, device=dev)
        spread[(r % n_cu) * (N // n_cu) + r // n_cu] = desc
        return {"agent": None, "longest_first": desc, "shortest_first": desc.flip(0), "spread": spread,
                "random": torch.as_tensor(rng.permutation(N), device=dev)}

    times = {}
    solver = drv.solver
    orig = solver.solve
    for k in range(steps):
        ords = orders(out["iters"].clone())
        name = list(ords)[k % len(ords)]
        o = ords[name]
        o = None if o is None else o.to(torch.int32)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]

        def timed(*a, **kw):
            kw["order"] = o
            ev[0].record()
            r = orig(*a, **kw)
            ev[1].record()
            return r
        solver.solve = timed
        X, U, out = drv.step(X, U)
        torch.cuda.synchronize()
        times.setdefault(name, []).append(ev[0].elapsed_time(ev[1]))
    solver.solve = orig
    for name, t in times.items():
        print(f"{name:15s} QP median {np.median(t):.4f} ms  min {np.min(t):.4f}  ({len(t)} launches)", flush=True)


if __name__ == "__main__":
    main(*sys.argv[1:])

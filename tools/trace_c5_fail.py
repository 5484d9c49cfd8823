"""Diagnostics: re-solve the dumped failing C5 subproblems (tools/dump_c5_failures.py) on the GPU with
the IPM trace of one agent enabled (scvx_qp_set_trace)."""
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "dynamic-programming-multiagent-trajectory-optimiziation_amd"))
sys.path.insert(0, REPO)


def main(path="gpurun_out/c5_fail.npz", cap=100):
    import torch
    import bench
    import scvx_hip
    from scvx_hip import workloads
    dev = torch.device("cuda:0")
    d = dict(np.load(path))
    sc = workloads.synthetic_quad(1024, K=bench.K, seed=3, obstacles=bench.N_OBS)
    T = lambda x, dt=torch.float64: torch.tensor(np.ascontiguousarray(x), device=dev, dtype=dt)  # noqa: E731
    spec = scvx_hip.QPSpec(model="quad", K=bench.K, box=bench.BOX, obs=sc["obs"], w_obs=1e6, j_max=8, w_coll=1e4,
                           tol=1e-9, max_iter=80)
    n = d["X"].shape[0]
    solver = scvx_hip.QPSolver(spec, n, device=dev)
    for agent in range(min(n, 3)):
        buf = torch.zeros(8 * cap + 32, dtype=torch.float64, device=dev)
        scvx_hip.lib().scvx_qp_set_trace(ctypes.c_void_p(buf.data_ptr()), agent, cap)
        out = solver.solve(T(d["disc"]), T(d["sigma"]), T(d["X"]), T(d["U"]), T(d["x_init"]), T(d["x_final"]),
                           T(d["tr"]), T(d["rows"]), T(d["count"], torch.int32))
        torch.cuda.synchronize()
        scvx_hip.lib().scvx_qp_set_trace(None, 0, 0)
        bb = buf.cpu().numpy()
        print(f"agent {agent}: status {out['status'][agent].item()} iters {out['iters'][agent].item()} "
              f"fail_code {bb[8 * cap + 3]} obj {out['obj'][agent].item():.9e}")
        b = bb[:8 * cap].reshape(cap, 8)
        for i in range(min(int(out["iters"][agent].item()) + 1, cap)):
            print("  it %2d pres %.2e dres %.2e gap %.2e pobj %.9e aa %.3f al %.3f sg %.2e mu %.2e" % ((i,) + tuple(b[i])))


if __name__ == "__main__":
    main(*sys.argv[1:2])

"""Region trace of the QP kernel on a coupled config's warm-started subproblems (GPU diagnostic).

Runs `W` steps of bench.py's c4 / c5 loop, then replays the last step's solve (same workspace snapshot, same
warm flags) with the in-kernel region timers on one agent (s_memtime stamps: cycles per IPM iteration per
region, tools/gpurun_quick.py's layout).  usage: python tools/trace_coupled.py c5 [W] [agent]"""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "dynamic-programming-multiagent-trajectory-optimiziation_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import scvx_hip  # noqa: E402
from scvx_hip.scvx import CouplingSpec, JacobiSCvx  # noqa: E402

NAMES = ["node+assemble", "factor", "newton rhs", "post-solve/step", "bwd pre", "bwd chain", "bwd post+mu",
         "fwd pre", "fwd chain", "fwd post", "update", "f-ph1 (-DQP_PHASE_TRACE)", "f-ph2", "f-ph3", "f-ph4",
         "f-ph5+0 (VC)"]


def main(config="c5", W=4, agent=None):
    W = int(W)
    dev = torch.device("cuda:0")
    sc, w, cfg = bench.make_coupled(config, 1, 0, dev)
    spec = scvx_hip.QPSpec(model=cfg["model"], K=bench.K, box=cfg["box"], obs=cfg["obs"], w_obs=1e6, j_max=cfg["j_max"],
                           w_coll=1e4, tol=1e-8, max_iter=60, **cfg["vc"])
    drv = JacobiSCvx(spec, w["x_init"], w["x_final"], w["sigma"], bench.TR0, coupling=CouplingSpec(R=cfg["R"]),
                     tr_rule="global")
    X, U = w["X"].clone(), w["U"].clone()
    for _ in range(W):
        X, U, _ = drv.step(X, U)
    trp, warm = drv.tr.clone(), drv.warm.clone()
    snap = drv.solver.workspace.clone()
    X0, U0 = X.clone(), U.clone()
    drv.step(X, U)
    torch.cuda.synchronize()
    it = drv.solver.iters.cpu().numpy()
    a = int(np.argsort(it)[len(it) // 2]) if agent is None else int(agent)
    print(f"{config}: step {W}: iters mean {it.mean():.2f} max {it.max()}; tracing agent {a} ({it[a]} iterations)")
    cap = 80
    buf = torch.zeros(8 * cap + 32, dtype=torch.float64, device=dev)
    drv.solver.workspace.copy_(snap)
    lib = scvx_hip.lib()
    lib.scvx_qp_set_trace(ctypes.c_void_p(buf.data_ptr()), a, cap)
    o = drv.solver.solve(drv.disc, drv.sigma, X0, U0, drv.x_init, drv.x_final, trp, drv.rows, drv.count, warm=warm)
    torch.cuda.synchronize()
    lib.scvx_qp_set_trace(None, 0, 0)
    cyc = buf[8 * cap:8 * cap + 20].cpu().numpy()
    n_it = max(int(o["iters"][a].item()), 1)
    print(f"total {cyc[2]:.3e} cycles, {cyc[2] / n_it:.3e}/it over {n_it} iterations")
    for k, nm in enumerate(NAMES):
        print(f"  {nm:16s} {cyc[4 + k] / n_it:10.0f} cycles/it  ({100 * cyc[4 + k] / cyc[2]:.1f}%)")


if __name__ == "__main__":
    main(*sys.argv[1:])

"""Diagnostics: run the C5 workload for a few SCvx iterations and dump the subproblems of agents whose
QP ended with status 2, so they can be re-solved by the CPU oracles (infeasible vs kernel failure)."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "dynamic-programming-multiagent-trajectory-optimiziation_amd"))
sys.path.insert(0, REPO)


def main(iters=4, out="gpurun_out/c5_fail.npz"):
    import torch
    import bench
    import scvx_hip
    from scvx_hip.scvx import CouplingSpec, JacobiSCvx
    dev = torch.device("cuda:0")
    sc, w, cfg = bench.make_coupled("c5", 1, 0, dev)
    spec = scvx_hip.QPSpec(model="quad", K=bench.K, box=cfg["box"], obs=cfg["obs"], w_obs=1e6, j_max=cfg["j_max"],
                           w_coll=1e4, tol=1e-9, max_iter=60)
    drv = JacobiSCvx(spec, w["x_init"], w["x_final"], w["sigma"], bench.TR0, coupling=CouplingSpec(R=cfg["R"]),
                     tr_rule="global")
    X, U = w["X"].clone(), w["U"].clone()
    for it in range(iters):
        Xp, Up, trp = X.clone(), U.clone(), drv.tr.clone()
        Xn, Un, o = drv.step(X, U)
        st = o["status"].cpu().numpy()
        print(f"iter {it}: status counts {np.bincount(st, minlength=3)}, tr {trp[0].item():.4g}", flush=True)
        bad = np.flatnonzero(st == 2)[:6]
        if bad.size:
            np.savez(out, agents=bad, disc=drv.disc[bad].cpu().numpy(), X=Xp[bad].cpu().numpy(),
                     U=Up[bad].cpu().numpy(), tr=trp[bad].cpu().numpy(), rows=drv.rows[bad].cpu().numpy(),
                     count=drv.count[bad].cpu().numpy(), x_init=w["x_init"][bad].cpu().numpy(),
                     x_final=w["x_final"][bad].cpu().numpy(), sigma=w["sigma"][bad].cpu().numpy(),
                     iters=o["iters"][bad].cpu().numpy(), it=it)
            print("dumped", bad.tolist(), flush=True)
            return
        X.copy_(Xn)
        U.copy_(Un)


if __name__ == "__main__":
    main()

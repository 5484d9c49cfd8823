"""Diagnostic: fused Jacobi update vs tensor path, per-step radii / costs of the agents that differ."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "dynamic-programming-multiagent-trajectory-optimiziation_amd"))
import torch
import scvx_hip
from scvx_hip import workloads
from scvx_hip.scvx import HipBackend, JacobiSCvx


class TensorPath(HipBackend):
    jacobi_update = None


dev = torch.device("cuda:0")
sc = workloads.synthetic_di(128, K=50, seed=3, sigma=30.0, obstacles=8)
w = {k: torch.tensor(sc[k], device=dev) for k in ("X", "U", "x_init", "x_final", "sigma")}
spec = scvx_hip.QPSpec(model="di", K=50, box=[(0, -12, 12), (1, -12, 12)], obs=sc["obs"], w_obs=1e6, u_max=1.0, max_iter=60)
drvs = [JacobiSCvx(spec, w["x_init"], w["x_final"], w["sigma"], 0.25, backend=b, fused_update=True)
        for b in (HipBackend(), TensorPath())]
st = [[w["X"].clone(), w["U"].clone()] for _ in drvs]
for k in range(3):
    outs = []
    for d, s in zip(drvs, st):
        s[0], s[1], o = d.step(s[0], s[1])
        outs.append(o)
    dX = (st[0][0] - st[1][0]).abs().max().item()
    dsol = (outs[0]["U"] - outs[1]["U"]).abs().max().item()
    diff = (drvs[0].tr != drvs[1].tr).nonzero().flatten().tolist()
    print(f"step {k}: max|dX| {dX:.3e} max|dUsol| {dsol:.3e} tr differ at {diff[:10]}")
    for a in diff[:5]:
        print("   agent", a, "tr", drvs[0].tr[a].item(), drvs[1].tr[a].item(), "prev_cost", drvs[0].prev_cost[a].item(), drvs[1].prev_cost[a].item())

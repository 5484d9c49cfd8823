"""Diagnostic (GPU, QP_BYTE_TRACE build): where the QP kernel's workspace traffic comes from, per region of an IPM
iteration.  Build: tools/build_variant.sh bytetrace -DQP_BYTE_TRACE; run with SCVX_HIP_LIB=variants/bytetrace/
libscvx_hip.so.  The headline loop (C3, bench.py's settings and its global trust-region rule) runs STEP warm steps;
at the last one the traced agent (WHO=tail: the one with the most IPM iterations the step before, the default;
WHO=bulk: the first agent that took the minimum; or an agent index) records per region the cycles (s_memtime) and the workspace bytes every lane of the wave requested (buffer loads
and stores that address a node; interface reads of disc / X / U and the outputs are not workspace traffic).
Prints bytes per IPM iteration per region and the launch's requested-bytes estimate
(sum over agents of iterations x the bulk agent's bytes per iteration + its setup), to set beside the PMC traffic
(FETCH_SIZE x2 + WRITE_SIZE) of the same launch.
usage: SCVX_HIP_LIB=... [WHO=tail|bulk|i] python tools/qp_bytes_trace.py [STEP=10] [out.json]"""
import ctypes
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "dynamic-programming-multiagent-trajectory-optimiziation_amd"))
import torch  # noqa: E402

import bench  # noqa: E402
import scvx_hip  # noqa: E402
from scvx_hip.scvx import JacobiSCvx  # noqa: E402

STEP = int(sys.argv[1]) if len(sys.argv) > 1 else 10
dev = torch.device("cuda", 0)
sc, w = bench.make_workload(bench.N_AGENTS, seed=1, device=dev)
spec = scvx_hip.QPSpec(model="di", K=bench.K, box=bench.BOX, obs=sc["obs"], w_obs=1e6, u_max=bench.U_MAX, tol=1e-8,
                       max_iter=60)
drv = JacobiSCvx(spec, w["x_init"], w["x_final"], w["sigma"], bench.TR0, tr_rule="global", warm_max_status=1)
X, U = w["X"].clone(), w["U"].clone()
it_prev = None
for s in range(STEP - 1):
    X, U, out = drv.step(X, U)
    it_prev = out["iters"].cpu().numpy()
names = ["node+assemble", "factor", "newton rhs", "post-solve/step", "bwd pre", "bwd chain", "bwd post+mu", "fwd pre",
         "fwd chain", "fwd post", "update", "r11", "r12", "r13", "r14", "r15"]
CAP = 80
res = {}
who = os.environ.get("WHO", "tail")
agent = int(np.argmax(it_prev)) if who == "tail" else (int(np.argmin(it_prev)) if who == "bulk" else int(who))
buf = torch.zeros(8 * CAP + 36, dtype=torch.float64, device=dev)
scvx_hip.lib().scvx_qp_set_trace(ctypes.c_void_p(buf.data_ptr()), agent, CAP)
X, U, out = drv.step(X, U)
torch.cuda.synchronize()
scvx_hip.lib().scvx_qp_set_trace(None, 0, 0)
b = buf.cpu().numpy()
n_it = max(int(out["iters"][agent].item()), 1)
cyc, byt = b[8 * CAP + 4: 8 * CAP + 20], b[8 * CAP + 20: 8 * CAP + 36]
res = dict(who=who, agent=agent, step=STEP, iters=n_it, cycles_per_iter={nm: float(c) / n_it for nm, c in zip(names, cyc)},
           bytes_per_iter={nm: float(v) / n_it for nm, v in zip(names, byt)}, bytes_total=float(byt.sum()))
print(f"{who} agent {agent}: {n_it} IPM iterations, {byt.sum() / n_it / 1e3:.1f} KB requested per iteration "
      f"(setup and exit included in the regions they fall in)")
for nm, c, v in zip(names, cyc, byt):
    if c or v:
        print(f"  {nm:16s} {c / n_it:9.0f} cycles/it  {v / n_it / 1e3:8.1f} KB/it  ({100 * v / max(byt.sum(), 1):.1f}%)")
iters = out["iters"].cpu().numpy().astype(float)
per_it = res["bytes_total"] / n_it
est = float(iters.sum() * per_it)
res["launch"] = dict(agents=int(iters.size), ipm_iters_sum=float(iters.sum()), requested_bytes_estimate=est)
print(f"launch: {iters.size} agents, {iters.sum():.0f} IPM iterations -> ~{est / 1e9:.2f} GB requested "
      f"(at this agent's {per_it / 1e3:.1f} KB per iteration)")
if len(sys.argv) > 2:
    json.dump(res, open(sys.argv[2], "w"), indent=1)

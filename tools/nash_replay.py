"""Diagnostic: re-solve one recorded NashSolver step (dbg/nash_trace.npz from tools/nash_trace_dump.py)
with SCPSolver.solve_game and compare with the oracle (an instrumented build can be loaded with
SCVX_HIP_LIB=..., see tools/build_variant.sh).
usage: python tools/nash_replay.py <step> [max_iter] [tol]"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "dynamic-programming-multiagent-trajectory-optimiziation_amd"))

import torch  # noqa: E402

import scvx_hip  # noqa: E402
from tests.test_nash_gpu import GAME, OBS_G, WTS, _disc_stacks  # noqa: E402

n = int(sys.argv[1])
max_iter = int(sys.argv[2]) if len(sys.argv) > 2 else 100
tol = float(sys.argv[3]) if len(sys.argv) > 3 else 1e-9
d = np.load(os.path.join(REPO, "dbg", "nash_trace.npz"))
e = {k.split("_", 1)[1]: d[k] for k in d.files if k.startswith(f"{n}_")}
i = int(e["agent"])
from oracle import nash_ref, scp_dense as sd, scp_problems as sp_  # noqa: E402
c = sp_.model_constraints("unicycle", GAME[i][0], GAME[i][1], obstacles=OBS_G)
K = e["Xref"].shape[0]
spec = scvx_hip.SCPSpec(model="unicycle", K=K, pos_dim=2, u_bounds=c["u_bounds"], x_bounds=c["x_bounds"], obs=c["obs"],
                        w_nu=1e4, w_slack=1e6, w_sigma=100.0, max_iter=max_iter, tol=tol, game=True, sigma_fixed=True,
                        w_u2=5.0, w_du=5.0, w_dth=100.0, theta_idx=2, n_slab=2, r_slab=0.5)
T = lambda a: torch.tensor(np.ascontiguousarray(a), dtype=torch.float64, device="cuda")  # noqa: E731
out = scvx_hip.SCPSolver(spec, 1).solve_game(T(e["disc"][None]), T(e["Xref"][None]), T(e["Uref"][None]), T([1.0]),
                                              T([100.0]), T(np.array(GAME[i][0])[None]), T(np.array(GAME[i][1])[None]),
                                              slab_z=T(e["z"][None]), slab_P=T(e["P"][None]))
torch.cuda.synchronize()
g = {k: v.cpu().numpy()[0] for k, v in out.items()}
print("kernel status", int(g["status"]), "iters", int(g["iters"]), "obj %.12e" % float(g["obj"]),
      "recorded obj %.12e" % float(e["obj"]))
p = nash_ref.game_problem("unicycle", e["Xref"], e["Uref"], 1.0, c, WTS, e["X_prev"], list(zip(e["z"], e["P"])), 0.5,
                          disc=_disc_stacks(e["disc"], 3, 2))
ref = nash_ref.best_response(p)
print("oracle", ref["status"], ref["iters"], "obj %.12e" % ref["obj"], "kernel point obj %.12e" %
      sd.scp_objective(p, g["X"], g["U"], g["nu"], 1.0), "viol", sd.scp_violation(p, g["X"], g["U"], g["nu"], 1.0))

"""Diagnostic: the batched game-kernel workload of `bench.py --config nash` (the last Gauss-Seidel
best responses, neighbour positions jittered); status / iteration histograms at several jitters and
iteration caps, and the oracle on a few failing instances.
usage: python tools/nash_batch_diag.py"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "dynamic-programming-multiagent-trajectory-optimiziation_amd"))
import torch  # noqa: E402

import scvx_hip  # noqa: E402
from SCvx.config import default_game as G  # noqa: E402
from SCvx.global_parameters import K as KG  # noqa: E402
from SCvx.models.game_model import GameUnicycleModel  # noqa: E402
from SCvx.models.multi_agent_model import MultiAgentModel  # noqa: E402
from SCvx.optimization.nash_solver import NashSolver  # noqa: E402
from SCvx.utils.initial_guess import initial_guess  # noqa: E402
from dataclasses import replace  # noqa: E402

dev = torch.device("cuda")
X0, U0 = (list(v) for v in zip(*(initial_guess(p["r_init"], p["r_final"], G.OBSTACLES, G.CLEARANCE, KG)
                                 for p in G.AGENT_PARAMS)))
mam = MultiAgentModel(G.AGENT_PARAMS)
for i, p in enumerate(G.AGENT_PARAMS):
    mam.models[i] = GameUnicycleModel(**{k: p[k] for k in ("r_init", "r_final", "obstacles", "control_weight",
                                                           "collision_weight", "collision_radius",
                                                           "control_rate_weight", "curvature_weight")})
ns = NashSolver(mam, max_iter=2, tol=-1.0)
ns.solve(X0, U0, 1.0)
br = ns.br_solvers
T = lambda a: torch.as_tensor(np.ascontiguousarray(a), dtype=torch.float64, device=dev)  # noqa: E731
N = 384
pick = [a % 3 for a in range(N)]
ins = [b.scp.host_inputs() for b in br]
args_b = {k: T(np.stack([ins[i][k] for i in pick]) if np.ndim(ins[0][k]) else [ins[i][k] for i in pick]) for k in ins[0]}
X_prev = T(np.stack([np.asarray(br[i].X_prev_param.require(), float).T for i in pick]))
P0 = np.stack([np.stack([np.asarray(br[i].Y_params[j].require(), float).T for j in sorted(br[i].Y_params)]) for i in pick])
rng = np.random.default_rng(5)
noise = rng.uniform(-1, 1, P0.shape)
for jit in (0.0, 0.01, 0.05):
    for cap, tol in ((100, 1e-9), (300, 1e-9), (100, 1e-8)):
        spec = replace(br[0].spec(), max_iter=cap, tol=tol)
        P = T(P0 + jit * noise)
        z = scvx_hip.slab_update(X_prev, P, spec.pos_dim)
        out = scvx_hip.SCPSolver(spec, N, device=dev).solve_game(X_prev=X_prev, slab_z=z, slab_P=P, **args_b)
        st, it = out["status"].cpu().numpy(), out["iters"].cpu().numpy()
        print(f"jitter {jit} cap {cap} tol {tol}: status {np.bincount(st, minlength=3)} iters mean {it.mean():.1f} "
              f"max {it.max()}  by agent kind: " +
              " ".join(f"{k}:{np.bincount(st[np.array(pick) == k], minlength=3).tolist()}" for k in range(3)), flush=True)

# one agent-2 instance (jitter 0) for an offline oracle / feasibility check
spec = br[2].spec()
z = scvx_hip.slab_update(X_prev[2:3], T(P0[2:3]), spec.pos_dim)
np.savez(os.path.join(REPO, "gpurun_out", "nash_fail.npz"), disc=ins[2]["disc"], Xref=ins[2]["Xref"], Uref=ins[2]["Uref"],
         X_prev=X_prev[2].cpu().numpy(), z=z[0].cpu().numpy(), P=P0[2])

"""Diagnostic: run NashSolver (default game, global K) with its solve trace on and dump every step to
gpurun_out/nash_trace.npz for offline comparison with oracle/nash_ref.py.
usage: python tools/nash_trace_dump.py [max_iter] [max_acs_iters]"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "dynamic-programming-multiagent-trajectory-optimiziation_amd"))

from tests.test_nash_gpu import _mam, _warm  # noqa: E402
from SCvx.global_parameters import K  # noqa: E402
from SCvx.optimization.nash_solver import NashSolver  # noqa: E402

its = int(sys.argv[1]) if len(sys.argv) > 1 else 2
acs = int(sys.argv[2]) if len(sys.argv) > 2 else 3
X0, U0 = (list(v) for v in _warm(K))
ns = NashSolver(_mam(), max_iter=its, max_acs_iters=acs)
ns.trace = []
X, U, hist = ns.solve(X0, U0, sigma_ref=1.0)
print("hist", hist)
out = {}
for n, e in enumerate(ns.trace):
    for k, v in e.items():
        out[f"{n}_{k}"] = np.asarray(v)
    print(n, e["it"], e["agent"], e["acs"], "status", int(e["status"]), "iters", int(e["iters"]), "obj", float(e["obj"]))
os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
np.savez(os.path.join(REPO, "gpurun_out", "nash_trace.npz"), n=len(ns.trace), **out)

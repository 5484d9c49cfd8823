"""Generate warm-start golden vectors by running the REFERENCE SCvx/utils/initial_guess.py here.

Run (container only; /root/reference never travels to the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_initial_guess_goldens.py

Cases: the three agents of SCvx/config/default_scenario.py at K = 50 (the scenario of
SCvx/examples/compare_admm_vs_nash.py:104-110) and seeded random start/goal pairs across 1-3 random
circles at K in {30, 50, 100}.  Output: initial_guess.npz (inputs + expected X0) next to this script."""
import importlib.util
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
spec = importlib.util.spec_from_file_location("ref_initial_guess", "/root/reference/SCvx/utils/initial_guess.py")
ref = importlib.util.module_from_spec(spec)
spec.loader.exec_module(ref)

cases = []
obst = [([1.0, 1.0], 0.25)]
off = 0.25 + 0.05 + 0.6
for a, b in (((0, 0, 0), (2, 2, 0)), ((2, 0, 0), (0, 2, 0)), ((1, 1 - off, 0), (1, 1 + off, 0))):
    cases.append((np.array(a, float), np.array(b, float), obst, 0.05, 50))
rng = np.random.default_rng(7)
while len(cases) < 24:
    n_obs = int(rng.integers(1, 4))
    obs = [(list(rng.uniform(-1, 1, 2)), float(rng.uniform(0.1, 0.4))) for _ in range(n_obs)]
    a = np.r_[rng.uniform(-4, -2, 2), 0.0]
    b = np.r_[rng.uniform(2, 4, 2), 0.0]
    try:
        ref.initial_guess(a, b, obs, 0.05, 50)
    except ValueError:
        continue
    cases.append((a, b, obs, 0.05, int(rng.choice([30, 50, 100]))))
out = {"n": len(cases)}
for i, (a, b, obs, cl, K) in enumerate(cases):
    X0, U0 = ref.initial_guess(a, b, obs, cl, K)
    out[f"p0_{i}"], out[f"p1_{i}"] = a, b
    out[f"obs_{i}"] = np.array([[c[0], c[1], r] for c, r in obs])
    out[f"clear_{i}"], out[f"K_{i}"] = cl, K
    out[f"X0_{i}"] = X0
np.savez_compressed(os.path.join(HERE, "initial_guess.npz"), **out)
print("wrote", len(cases), "cases")

"""3-agent unicycle ADMM scenario (reference SCvx/config/default_scenario.py): agents 0 and 1 cross
diagonally, agent 2 passes the obstacle from below to above with clearance + margin."""
import numpy as np

K = 50
D_MIN = 0.5
CLEARANCE = 0.05
MARGIN = 0.6
OBSTACLES = [([1.0, 1.0], 0.25)]

_c, _r = OBSTACLES[0]
_off = _r + CLEARANCE + MARGIN
AGENT_PARAMS = [
    {"r_init": np.array([0.0, 0.0, 0.0]), "r_final": np.array([2.0, 2.0, 0.0]), "obstacles": OBSTACLES},
    {"r_init": np.array([2.0, 0.0, 0.0]), "r_final": np.array([0.0, 2.0, 0.0]), "obstacles": OBSTACLES},
    {"r_init": np.array([_c[0], _c[1] - _off, 0.0]), "r_final": np.array([_c[0], _c[1] + _off, 0.0]),
     "obstacles": OBSTACLES},
]

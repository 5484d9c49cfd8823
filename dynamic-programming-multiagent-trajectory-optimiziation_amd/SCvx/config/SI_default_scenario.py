"""3-agent single-integrator ADMM scenario (reference SCvx/config/SI_default_scenario.py): three agents
crossing along the x, y and z axes through one sphere."""
import numpy as np

K = 100
D_MIN = 0.5
CLEARANCE = 0.05
MARGIN = 0.6
OBSTACLES = [([0.0, 0.0, 0.0], 1)]

AGENT_PARAMS = [{"r_init": -4.0 * e + 0.0, "r_final": 4.0 * e, "obstacles": OBSTACLES} for e in np.eye(3)]

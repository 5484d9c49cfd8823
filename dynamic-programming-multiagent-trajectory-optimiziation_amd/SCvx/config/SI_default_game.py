"""3-agent single-integrator Nash-game scenario (reference SCvx/config/SI_default_game.py)."""
import numpy as np

K = 100
D_MIN = 0.0
CLEARANCE = 0.1
MARGIN_OBS = 0.0
MARGIN_AGT = 0.0
ROBOT_RADIUS = 0.5
OBSTACLES = [([0.0, 0.0, 0.0], 0.8)]
CTRL_W = 5.0
COLL_W = 200.0
AGT_COLL_RAD = 2 * ROBOT_RADIUS + MARGIN_AGT
CTRL_RATE_W = 5.0
CURVATURE_W = 100.0

AGENT_PARAMS = [dict(r_init=-4.0 * e + 0.0, r_final=4.0 * e, obstacles=OBSTACLES, robot_radius=ROBOT_RADIUS,
                     control_weight=CTRL_W, collision_weight=COLL_W, collision_radius=AGT_COLL_RAD,
                     control_rate_weight=CTRL_RATE_W, curvature_weight=CURVATURE_W) for e in np.eye(3)]

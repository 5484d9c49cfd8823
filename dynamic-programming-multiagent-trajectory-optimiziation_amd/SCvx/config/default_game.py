"""3-agent unicycle Nash-game scenario (reference SCvx/config/default_game.py): two obstacles, the
game cost weights of every agent."""
import numpy as np

K = 50
D_MIN = 0.5
CLEARANCE = 0.05
MARGIN = 0.6
OBSTACLES = [([1.0, 1.0], 0.25), ([1.0, -0.3], 0.02)]
CTRL_W, COLL_W, COLL_RAD = 5, 10.0, 0.5
CTRL_RATE_W, CURVATURE_W = 5.0, 100.0

_WEIGHTS = {"control_weight": CTRL_W, "collision_weight": COLL_W, "collision_radius": COLL_RAD,
            "control_rate_weight": CTRL_RATE_W, "curvature_weight": CURVATURE_W}
_ENDS = [((0.0, -1.0), (2.0, 3.0)), ((2.0, -1.0), (0.0, 3.0)), ((1.0, -1.5), (OBSTACLES[0][0][0], 3.0))]
AGENT_PARAMS = [dict(r_init=np.array([a[0], a[1], 0.0]), r_final=np.array([b[0], b[1], 0.0]), obstacles=OBSTACLES,
                     **_WEIGHTS) for a, b in _ENDS]

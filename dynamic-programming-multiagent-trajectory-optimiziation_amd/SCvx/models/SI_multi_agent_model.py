"""Multi-agent 3-D single-integrator wrapper -- reference SCvx/models/SI_multi_agent_model.py:8-74."""
import numpy as np

from .multi_agent_model import linearize_pairwise
from .single_integrator_model import SingleIntegratorModel


class SI_MultiAgentModel:  # noqa: N801  (reference name)
    _ALLOWED_KEYS = {"r_init", "r_final", "v_max", "bounds", "robot_radius", "obstacles"}

    def __init__(self, agent_params: list, d_min: float = 1.0):
        self.N = len(agent_params)
        self.models = [SingleIntegratorModel(**{k: v for k, v in p.items() if k in self._ALLOWED_KEYS})
                       for p in agent_params]
        self.d_min = d_min

    def get_local_dynamics(self, i: int):
        return self.models[i].get_equations()

    def linearize_inter_agent_collision(self, i: int, j: int, X_ref_i, X_ref_j):
        """3-D version of MultiAgentModel.linearize_collision."""
        return linearize_pairwise(np.asarray(X_ref_i)[0:3, :], np.asarray(X_ref_j)[0:3, :], self.d_min)

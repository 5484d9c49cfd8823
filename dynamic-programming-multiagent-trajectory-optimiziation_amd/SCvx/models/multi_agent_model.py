"""Multi-agent unicycle wrapper -- reference SCvx/models/multi_agent_model.py:8-79: per-agent models,
d_min, and the linearized pairwise collision normal a_k = (p_i - p_j)/(|p_i - p_j| + 1e-6),
b_k = d_min + a_k' p_j (KAT: SCvx/multi_agent_tests/test_multi_agent_model.py:42-59)."""
import numpy as np

from ..global_parameters import K as GLOBAL_K
from ..optimization.variables import Variable
from .unicycle_model import UnicycleModel


def linearize_pairwise(p_i: np.ndarray, p_j: np.ndarray, d_min: float):
    """Vectorized over the K columns: p_i, p_j (d, K) -> A_ij (d, K), b_ij (K,)."""
    diff = p_i - p_j
    nrm = np.linalg.norm(diff, axis=0) + 1e-6
    A = diff / nrm
    b = d_min + np.sum(A * p_j, axis=0)
    return A, b


class MultiAgentModel:
    def __init__(self, agent_params, d_min=1.0):
        self.N = len(agent_params)
        self.models = []
        for params in agent_params:
            kw = {k: params[k] for k in ("r_init", "r_final") if k in params}
            kw.update({k: params[k] for k in ("v_max", "w_max", "bounds", "robot_radius")
                       if params.get(k) is not None})
            m = UnicycleModel(**kw)
            if params.get("obstacles") is not None:
                m.obstacles = params["obstacles"]
                m.s_prime = [Variable((GLOBAL_K, 1), nonneg=True) for _ in m.obstacles]  # :40-41
            self.models.append(m)
        self.d_min = d_min

    def get_local_dynamics(self, i):
        return self.models[i].get_equations()

    def get_static_constraints(self, i, X, U, X_ref, U_ref):
        return self.models[i].get_constraints(X, U, X_ref, U_ref)

    def linearize_collision(self, i, j, X_ref_i, X_ref_j):
        """||p_i - p_j|| >= d_min linearized at the reference positions (2-D)."""
        return linearize_pairwise(np.asarray(X_ref_i)[0:2, :], np.asarray(X_ref_j)[0:2, :], self.d_min)

"""ADMM residual helpers -- same contract as the reference SCvx/optimization/admm_utils.py:5-58
(pinned by its KATs, SCvx/multi_agent_tests/test_admm_utils.py)."""
import numpy as np

WEIGHT_COLLISION_SLACK = 1e5


def primal_residual(p_j: np.ndarray, Y_ij: np.ndarray) -> float:
    """||p_j - Y_ij|| (Frobenius)."""
    return np.linalg.norm(p_j - Y_ij)


def dual_residual(Y_new: np.ndarray, Y_old: np.ndarray) -> float:
    """||Y_new - Y_old|| (Frobenius)."""
    return np.linalg.norm(Y_new - Y_old)


def update_rho_admm(rho: float, primal_res: float, dual_res: float, mu: float = 10.0, tau_inc: float = 2.0,
                    tau_dec: float = 2.0) -> float:
    """Residual-balancing rho update: x tau_inc if primal > mu*dual, / tau_dec if dual > mu*primal."""
    if primal_res > mu * dual_res:
        return rho * tau_inc
    if dual_res > mu * primal_res:
        return rho / tau_dec
    return rho

"""Model contract of the reference SCvx/models/base_model.py:7-88: get_equations() -> (f, A, B),
initialize_trajectory, optional (non)dimensionalisation hooks.  The MI355X path adds one attribute,
`scvx_model`, naming the device dynamics (csrc/models.hpp) that stand in for the numpy callables
inside the batched kernels."""
from abc import ABC, abstractmethod

import numpy as np


class BaseModel(ABC):
    scvx_model: str = ""   # "di" | "unicycle" | "si" | "quad"
    scvx_params = None     # device model parameters (quadrotor)

    @abstractmethod
    def get_equations(self):
        """(f, A, B) numpy callables of (x, u)."""

    def get_constraints(self, X, U, X_ref, U_ref):
        raise NotImplementedError(
            "CVXPY constraint objects are not built by the MI355X backend; the batched solver takes "
            "the constraint set through scvx_hip.QPSpec (see qp_spec())")

    def get_objective(self, X, U, X_ref, U_ref):
        raise NotImplementedError("see get_constraints")

    @abstractmethod
    def initialize_trajectory(self, X: np.ndarray, U: np.ndarray):
        """Fill X (n_x, K), U (n_u, K) with the initial guess and return them."""

    def nondimensionalize(self):
        return

    def redimensionalize(self):
        return

    def x_nondim(self, x):
        return x

    def u_nondim(self, u):
        return u

    def x_redim(self, X):
        return X

    def u_redim(self, U):
        return U


def straight_line(X: np.ndarray, x0: np.ndarray, x1: np.ndarray) -> np.ndarray:
    """Row-wise linear interpolation between x0 and x1 over the K columns of X (in place)."""
    K = X.shape[1]
    for k in range(K):
        a = k / (K - 1)
        X[:, k] = (1.0 - a) * x0 + a * x1
    return X

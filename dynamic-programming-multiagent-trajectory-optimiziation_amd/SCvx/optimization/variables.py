"""Value holders standing in for the CVXPY objects the reference's SCvx call surface exposes
(SCProblem.var / .par / .prob, model.s_prime, AgentSolver.Y / .Lambda / .S;
SCvx/optimization/sc_problem.py:22-44, agent_solver.py:33-41).  Callers read and assign `.value`
exactly as they do on cvxpy.Variable / cvxpy.Parameter; the solve itself runs in the batched HIP
kernel (scvx_hip.SCPSolver), so no expression trees are built."""
import numpy as np


class SolverError(Exception):
    """Raised where cvxpy raises cvxpy.SolverError (the kernel reported a numerical failure)."""


class ParameterError(ValueError):
    """Raised where cvxpy raises cvxpy.error.ParameterError (a Parameter without a value at solve)."""


class _Leaf:
    _count = 0

    def __init__(self, shape=(), name=None, nonneg=False):
        if isinstance(shape, int):
            shape = (shape,)
        self.shape = tuple(shape)
        _Leaf._count += 1
        self._name = name or f"{type(self).__name__.lower()}{_Leaf._count}"
        self.nonneg = nonneg
        self._value = None

    def name(self):
        return self._name

    @property
    def value(self):
        return self._value

    @value.setter
    def value(self, v):
        if v is None:
            self._value = None
            return
        a = np.asarray(v, dtype=float)
        # only singleton axes may differ ((K,) vs (K, 1), a 1-element array for a scalar): any other
        # mismatch -- a transposed (K, n) trajectory for an (n, K) parameter -- is a caller bug that
        # cvxpy rejects, and reshaping it would scramble the data silently
        if a.shape != self.shape and tuple(d for d in a.shape if d != 1) == tuple(d for d in self.shape if d != 1):
            a = a.reshape(self.shape)
        if a.shape != self.shape:
            raise ValueError(f"Invalid dimensions {a.shape} for {type(self).__name__} value of shape {self.shape}.")
        if self.nonneg and np.any(a < 0):
            raise ValueError(f"{type(self).__name__} value must be nonnegative.")
        self._value = a if a.shape else float(a)

    def __repr__(self):
        return f"{type(self).__name__}({self.shape}, name={self._name})"


class Variable(_Leaf):
    pass


class Parameter(_Leaf):
    def require(self):
        if self._value is None:
            raise ParameterError(f"A Parameter (whose name is '{self._name}') does not have a value associated "
                                 "with it; all Parameter objects must have values before solving a problem.")
        return self._value


class ProblemResult:
    """What callers read off cvxpy.Problem after a solve: .status and .value (optimal objective)."""

    def __init__(self):
        self.status = None
        self.value = None
        self.solver_stats = {}

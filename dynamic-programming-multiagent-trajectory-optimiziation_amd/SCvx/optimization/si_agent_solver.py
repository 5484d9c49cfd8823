"""SI_AgentSolver -- drop-in replacement of the reference SCvx/optimization/si_agent_solver.py:10-105:
AgentSolver with 3-D positions (X[0:3]), Y / Lambda of shape (3, K)."""
from .agent_solver import AgentSolver


class SI_AgentSolver(AgentSolver):  # noqa: N801  (reference name)
    pos_dim = 3

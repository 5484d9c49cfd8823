"""SI_ADMMCoordinator -- drop-in replacement of the reference SCvx/optimization/si_admm_coordinator.py:13-127:
the ADMMCoordinator round structure with 3-D single-integrator agents (SI_AgentSolver, Y / Lambda
(3, K)) and, as in the reference (:83-86), the ORIGINAL X_refs[i] / U_refs[i] as the subproblem's
reference trajectory while the discretization uses the current iterate."""
from .admm_coordinator import ADMMCoordinator
from .si_agent_solver import SI_AgentSolver


class SI_ADMMCoordinator(ADMMCoordinator):  # noqa: N801  (reference name)
    agent_cls = SI_AgentSolver
    pos_dim = 3
    trust_ref_is_initial = True

"""SI_AgentBestResponse -- drop-in replacement of the reference SCvx/optimization/si_agent_best_response.py:17-127
(3-D single-integrator agents): AgentBestResponse with (3, K) neighbour positions, the model's
inter-sample rows added after the slabs (update_intersample_constraints, :64-75; it replaces the slab
rows, as in the reference -- see SCvx/models/game_si_model.py) and the reference's failure report."""
from .agent_best_response import AgentBestResponse


class SI_AgentBestResponse(AgentBestResponse):  # noqa: N801  (reference name)
    """Solve one agent's best-response with fixed time-scale (single-integrator)."""

    pos_dim = 3

    def _extra_constraints_hook(self, X_ref, U_ref, sigma_ref):
        self.model.update_intersample_constraints(X_v=self.scp.var["X"], U_v=self.scp.var["U"], X_nom=X_ref,
                                                  U_nom=U_ref, foh=self.foh, sigma_ref=sigma_ref)

    def _failed(self):
        print(f"!! Solver for Agent {self.i} failed with status: {self.scp.prob.status} !!")
        return RuntimeError(f"SCProblem for agent {self.i} was not solved successfully.")

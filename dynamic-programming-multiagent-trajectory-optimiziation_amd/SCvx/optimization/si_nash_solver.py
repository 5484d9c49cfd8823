"""SI_NashSolver -- drop-in replacement of the reference SCvx/optimization/si_nash_solver.py:22-124: the
NashSolver iteration (SCvx/optimization/nash_solver.py) with 3-D single-integrator agents
(SI_AgentBestResponse) and the reference's `show_progress` flag (a one-line progress report per
outer iteration instead of tqdm bars)."""
from .nash_solver import NashSolver
from .si_agent_best_response import SI_AgentBestResponse


class SI_NashSolver(NashSolver):  # noqa: N801  (reference name)
    """Non-cooperative Nash equilibrium via Iterative Best Response (3-D SI agents)."""

    br_cls = SI_AgentBestResponse

    def solve(self, X_refs, U_refs, sigma_ref: float = 1.0, verbose: bool = False, show_progress: bool = True):
        X, U, hist = super().solve(X_refs, U_refs, sigma_ref, verbose=verbose)
        if show_progress:
            print(f"Nash iters: {len(hist)} | max_change={hist[-1]:.2e}" if hist else "Nash iters: 0")
        return X, U, hist

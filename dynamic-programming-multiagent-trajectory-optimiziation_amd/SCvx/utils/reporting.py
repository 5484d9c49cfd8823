"""Console lines of the iterative solvers (the two functions of the reference
SCvx/utils/reporting.py:4-30, used by the Nash solver); same text, host-side only."""


def print_iteration(it, nu_norm, slack_norm, primal_res, dual_res, dx, ds, sigma, tr_radius):
    print(f"Iter {it:2d} | v={nu_norm:7.3e} | slack={slack_norm:7.3e} | p_res={primal_res:7.3e} "
          f"| d_res={dual_res:7.3e} | Δx={dx:6.2e} | Δs={ds:6.2e} | o={sigma:5.3f} | tr={tr_radius:5.3f}")


def print_summary(total_iters, sigma_final, runtime=None):
    out = ["", "=== Solver Summary ===", f"  Total iterations: {total_iters}", f"  Final o:         {sigma_final:.3f}"]
    if runtime is not None:
        out.append(f"  Runtime:         {runtime:.2f}s")
    out.append("======================\n")
    print("\n".join(out))

"""Per-round console output of the ADMM coordinators: the two functions of the reference
SCvx/utils/multi_agent_logging.py:1-15, producing the same text."""

_FIELDS = (("v", "7.3e"), ("slack", "7.3e"), ("p_res", "7.3e"), ("d_res", "7.3e"), ("Δx", "6.2e"), ("Δs", "6.2e"),
           ("o", "6.3f"), ("tr", "6.3f"))


def print_iteration(it, nu_norm, slack_norm, primal_res, dual_res, dx, ds, sigma, tr_radius):
    vals = (nu_norm, slack_norm, primal_res, dual_res, dx, ds, sigma, tr_radius)
    cols = [f"Iter {it:2d}"] + [f"{name}={format(v, spec)}" for (name, spec), v in zip(_FIELDS, vals)]
    print(" | ".join(cols))


def print_summary(total_iters, sigma_final, runtime=None):
    lines = ["", "=== SCvx+ADMM Summary ===", f"  Total iterations: {total_iters}",
             f"  Final time scale o: {sigma_final:.3f}"]
    if runtime is not None:
        lines.append(f"  Total runtime:    {runtime:.2f}s")
    lines.append("=" * 25 + "\n")
    print("\n".join(lines))

"""ORACLE / TEST INFRASTRUCTURE ONLY: second-order-cone step length shared by the dense checkers
(oracle/qp_dense.py, oracle/scp_dense.py)."""
import numpy as np


def soc_max_step(x, d):
    """Largest t >= 0 with x + t d in the second-order cone {v : v0 >= ||v[1:]||} (x inside it); inf if the
    ray never leaves.  The quadratic J(x + t d) = 0 (J(v) = v0^2 - ||v1||^2) is solved for the direction
    normalised to max |d| = 1, with J evaluated as (v0 - ||v1||)(v0 + ||v1||) and the roots by the stable
    form q = -(b + sign(b) sqrt(b^2 - 4ac)) / 2, t1 = q / a, t2 = c / q: no overflow for huge directions
    and no cancellation near the cone boundary.  A non-finite direction raises FloatingPointError (the
    callers treat it as a numerical breakdown)."""
    sc = float(np.max(np.abs(d))) if d.size else 0.0
    if not np.isfinite(sc):
        raise FloatingPointError("non-finite direction")
    if sc == 0.0:
        return np.inf
    dd = d / sc
    n1d, n1x = np.linalg.norm(dd[1:]), np.linalg.norm(x[1:])
    qa = (dd[0] - n1d) * (dd[0] + n1d)
    qb = 2.0 * (x[0] * dd[0] - x[1:] @ dd[1:])
    qc = (x[0] - n1x) * (x[0] + n1x)
    roots = []
    if abs(qa) <= 1e-15 * (dd[0] * dd[0] + n1d * n1d):     # J linear along the ray
        if qb < 0:
            roots.append(-qc / qb)
    else:
        disc = qb * qb - 4.0 * qa * qc
        if disc >= 0:
            q = -0.5 * (qb + np.copysign(np.sqrt(disc), qb))
            roots.append(q / qa)
            if q != 0:
                roots.append(qc / q)
    a = np.inf
    for r in roots:
        if r > 0 and x[0] + r * dd[0] >= -1e-14 * max(1.0, abs(x[0])):
            a = min(a, r)
    if dd[0] < 0:
        a = min(a, -x[0] / dd[0])
    return a / sc

"""Obstacle-aware warm start for the unicycle agents -- drop-in for the reference
SCvx/utils/initial_guess.py:1-98 (used by the ADMM / Nash example drivers, e.g.
SCvx/examples/compare_admm_vs_nash.py:104-110).

For every circular obstacle (inflated by `clearance`) that the straight start->goal segment crosses, the
path detours through the pair of tangent points (one from the start, one from the goal) of least total
length; the polyline is then resampled to exactly K points (segment i gets max(2, round(K L_i / L))
samples, the last segment the remainder; only the last segment includes its end point).  Headings are
the directions of consecutive samples, the last one repeated; inputs are zero.  Host-side data
preparation (no kernel): it runs once per scenario."""
import numpy as np


def line_circle_intersect(p, q, center, r):
    """True if the open segment p->q meets the circle (center, r) (a root of |p + t(q-p) - c| = r in (0,1))."""
    d, f = q - p, p - center
    a, b, c = d @ d, 2.0 * (f @ d), f @ f - r * r
    disc = b * b - 4.0 * a * c
    if disc < 0:
        return False
    roots = (-b + np.sqrt(disc)) / (2.0 * a), (-b - np.sqrt(disc)) / (2.0 * a)
    return any(0.0 < t < 1.0 for t in roots)


def compute_tangent_points(p, center, r):
    """The two points where lines from the external point p touch the circle (center, r)."""
    v = p - center
    dist = np.linalg.norm(v)
    if dist <= r:
        raise ValueError("Point inside/on circle; no tangents.")
    half = np.arcsin(r / dist)
    base = np.arctan2(v[1], v[0])
    return tuple(center + r * np.array([np.cos(base + s * half), np.sin(base + s * half)]) for s in (1.0, -1.0))


def generate_piecewise_linear(p0, p1, waypoints, K):
    """Resample the polyline p0 -> waypoints -> p1 to exactly K points (2 x K)."""
    pts = [p0, *waypoints, p1]
    seg = [np.linalg.norm(b - a) for a, b in zip(pts[:-1], pts[1:])]
    total = sum(seg)
    counts = [max(2, round(K * s / total)) for s in seg]
    counts[-1] = K - sum(counts[:-1])
    last = len(pts) - 2
    pieces = [np.linspace(pts[i], pts[i + 1], counts[i], endpoint=(i == last)) for i in range(len(pts) - 1)]
    return np.vstack(pieces).T


def initial_guess(p0, p1, obstacles, clearance, K):
    """(X0 (3, K), U0 (2, K)) from start / goal states [x, y, theta] and obstacles [(center, radius)]."""
    a, b = np.asarray(p0[:2], dtype=float), np.asarray(p1[:2], dtype=float)
    waypoints = []
    for c, r in obstacles:
        c, r = np.asarray(c, dtype=float), r + clearance
        if not line_circle_intersect(a, b, c, r):
            continue
        ts, gs = compute_tangent_points(a, c, r), compute_tangent_points(b, c, r)
        best = min(((np.linalg.norm(a - t) + np.linalg.norm(t - g) + np.linalg.norm(g - b), k, t, g)
                    for k, (t, g) in enumerate((t, g) for t in ts for g in gs)), key=lambda e: (e[0], e[1]))
        waypoints += [best[2], best[3]]
    path = generate_piecewise_linear(a, b, waypoints, K)
    X0 = np.zeros((3, K))
    X0[:2] = path
    step = np.diff(path, axis=1)
    X0[2, :-1] = np.arctan2(step[1], step[0])
    X0[2, -1] = X0[2, -2]
    return X0, np.zeros((2, K))

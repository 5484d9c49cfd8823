"""Synthetic SCvx workloads of SURVEY §8(d) (host-side data construction, no compute).

    synthetic_di       C2 / C3: random starts and goals in [-spread, spread]^3 at rest, straight-line
                       warm start (as x_initial, Distributed_opt/dist_scvx_3d.py:122-128), U = 0,
                       optional spheres (centres U[-8, 8]^3, radii U[0.5, 1.5]).
    synthetic_lattice  C4: starts on a cubic lattice whose spacing exceeds 2R (dist_scvx_3d.py:211),
                       goals a random permutation of the lattice sites inside 2x2x2 cells, so straight
                       paths cross (and every goal is reachable under the trust region).
    synthetic_quad     C5: 12-state quadrotor (models.hpp Quadrotor) from hover: positions as C2,
                       attitude / rates 0, U = hover thrust (m g, 0, 0, 0).  QUAD_BOX adds a roll /
                       pitch envelope |phi|, |theta| <= 1 rad to the x / y box: the model is build-defined
                        with Euler angles, whose kinematics are singular at |theta| = pi/2;
                       without the envelope the trust region on the inputs alone lets a subproblem
                       solution tilt past 90 degrees, and the next FOH linearisation is degenerate.

All arrays are agent-major (N, K, n) / (N, K, m) float64, the layout of include/scvx_hip.h.
"""
import numpy as np

BOX = [(0, -12.0, 12.0), (1, -12.0, 12.0)]                 # C2/C3/C5 x, y box (dist_scvx_3d.py:87-90 widened)
QUAD_BOX = BOX + [(6, -1.0, 1.0), (7, -1.0, 1.0)]        # C5: + roll / pitch envelope (rad)


def _obstacles(obstacles, obs_seed):
    if not obstacles:
        return []
    ro = np.random.default_rng(obs_seed)
    ctr = ro.uniform(-8, 8, (obstacles, 3))
    rad = ro.uniform(0.5, 1.5, obstacles)
    return [(ctr[o], rad[o]) for o in range(obstacles)]


def _straight(p0, pf, K, n):
    a = np.linspace(0, 1, K)
    X = np.zeros((p0.shape[0], K, n))
    X[:, :, 0:3] = p0[:, None, :] * (1 - a)[None, :, None] + pf[:, None, :] * a[None, :, None]
    return X


def synthetic_di(N, K=50, seed=0, sigma=30.0, spread=10.0, obstacles=0, obs_seed=11):
    rng = np.random.default_rng(seed)
    p0 = rng.uniform(-spread, spread, (N, 3))
    pf = rng.uniform(-spread, spread, (N, 3))
    X = _straight(p0, pf, K, 6)
    U = np.zeros((N, K, 3))
    return dict(X=X, U=U, x_init=X[:, 0, :].copy(), x_final=X[:, -1, :].copy(), sigma=np.full(N, sigma),
                obs=_obstacles(obstacles, obs_seed))


def synthetic_lattice(side=16, K=50, seed=2, sigma=30.0, spacing=6.0, obstacles=0, obs_seed=11, block=2):
    """N = side^3 agents; lattice centred on the origin.  Goals are a random permutation of the lattice
    sites composed of independent permutations inside every block x block x block cell of sites, so the
    straight paths of a cell's agents cross at its centre.  (A permutation of the whole lattice sends
    agents up to 90 m away, beyond what the trust region ||w_t||_1 <= 0.25 can reach in sigma = 30 s
    (at most a sigma^2 / 4 ~ 56 m per axis): most subproblems are then infeasible, where the reference's
    dist_scvx_3d.py:110-112 would get s_i.value = None from Clarabel and fail.)"""
    rng = np.random.default_rng(seed)
    g = (np.arange(side) - 0.5 * (side - 1)) * spacing
    sites = np.stack(np.meshgrid(g, g, g, indexing="ij"), -1).reshape(-1, 3)
    ijk = np.stack(np.meshgrid(*(np.arange(side),) * 3, indexing="ij"), -1).reshape(-1, 3)
    cell = ((ijk // block) * np.array([side * side, side, 1])).sum(1)
    perm = np.arange(sites.shape[0])
    for c in np.unique(cell):
        members = np.nonzero(cell == c)[0]
        perm[members] = members[rng.permutation(members.size)]
    goals = sites[perm]
    X = _straight(sites, goals, K, 6)
    N = sites.shape[0]
    return dict(X=X, U=np.zeros((N, K, 3)), x_init=X[:, 0, :].copy(), x_final=X[:, -1, :].copy(),
                sigma=np.full(N, sigma), obs=_obstacles(obstacles, obs_seed))


def synthetic_quad(N, K=50, seed=3, sigma=30.0, spread=10.0, obstacles=0, obs_seed=11, mass=1.0, g=9.81):
    rng = np.random.default_rng(seed)
    p0 = rng.uniform(-spread, spread, (N, 3))
    pf = rng.uniform(-spread, spread, (N, 3))
    X = _straight(p0, pf, K, 12)
    U = np.zeros((N, K, 4))
    U[:, :, 0] = mass * g
    return dict(X=X, U=U, x_init=X[:, 0, :].copy(), x_final=X[:, -1, :].copy(), sigma=np.full(N, sigma),
                obs=_obstacles(obstacles, obs_seed))

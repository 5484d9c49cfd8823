"""ORACLE / TEST INFRASTRUCTURE ONLY: synthetic problem instances shared by tests and bench.

Builds the same per-agent subproblem in two encodings:
  * the reference-form dict consumed by oracle/qp_dense.py (dense CVXPY-style formulation), and
  * the batched agent-major arrays of include/scvx_hip.h (scvx_qp_solve_batched).
Scenarios follow SURVEY §8(d): the dist_scvx_3d 3-robot case (Distributed_opt/dist_scvx_3d.py:199-231)
and the C2/C3 double-integrator constructions.
"""
import numpy as np


def zoh_di(dt):
    """Exact ZOH of the 3-D double integrator (== scipy.signal to_discrete, dist_scvx_3d.py:9-28)."""
    Ad = np.eye(6)
    Ad[0:3, 3:6] = dt * np.eye(3)
    Bd = np.zeros((6, 3))
    Bd[0:3] = 0.5 * dt * dt * np.eye(3)
    Bd[3:6] = dt * np.eye(3)
    return Ad, Bd


def pack_disc(A, B, C=None, S=None, z=None):
    """(K-1,n,n),(K-1,n,m)... -> [K-1][n(n+2m+2)] column-major blocks (include/scvx_hip.h)."""
    Km1, n, _ = A.shape
    m = B.shape[2]
    C = np.zeros_like(B) if C is None else C
    S = np.zeros((Km1, n)) if S is None else S
    z = np.zeros((Km1, n)) if z is None else z
    out = np.zeros((Km1, n * (n + 2 * m + 2)))
    for t in range(Km1):
        out[t] = np.concatenate([A[t].T.reshape(-1), B[t].T.reshape(-1), C[t].T.reshape(-1), S[t], z[t]])
    return out


def unpack_disc(d, n, m):
    Km1 = d.shape[0]
    o = np.cumsum([0, n * n, n * m, n * m, n, n])
    A = d[:, o[0]:o[1]].reshape(Km1, n, n).transpose(0, 2, 1)
    B = d[:, o[1]:o[2]].reshape(Km1, m, n).transpose(0, 2, 1)
    C = d[:, o[2]:o[3]].reshape(Km1, m, n).transpose(0, 2, 1)
    return A, B, C, d[:, o[3]:o[4]], d[:, o[4]:o[5]]


def dist3_scenario():
    """The reference's 3-robot scenario at its first Jacobi iteration (dist_scvx_3d.py:199-236)."""
    T, dt, R, tr = 51, 0.6, 2.3, 0.25
    Ad, Bd = zoh_di(dt)
    xi = [np.array([0, c * 5.1, 10, 0, 0, 0, 0, 0, 0.0]) for c in range(3)]
    xd = [np.array([14, (2 - c) * 5, 10 + c * 1, 0, 0, 0, 0, 0, 0.0]) for c in range(3)]
    Xt = [np.linspace(xi[c], xd[c], T) for c in range(3)]
    return dict(T=T, dt=dt, R=R, tr=tr, Ad=Ad, Bd=Bd, x_ini=xi, x_des=xd, X_traj=Xt)


def collision_rows(X_traj, i, R, pos_dim=3):
    """dist_scvx_3d.py:93-107: rows (g, b) with b - g'p_t <= S_t, g=(p_i-p_j)/|p_i-p_j|,
    b = 2R - |p_i-p_j| + g'p_i  (i.e. c - g'd with c = 2R - |.|)."""
    T = X_traj[i].shape[0]
    rows = []
    for t in range(T):
        rr = []
        for j in range(len(X_traj)):
            if j == i:
                continue
            diff = X_traj[i][t, :pos_dim] - X_traj[j][t, :pos_dim]
            nr = np.linalg.norm(diff)
            g = diff / nr
            rr.append(np.concatenate([g, [2 * R - nr + g @ X_traj[i][t, :pos_dim]]]))
        rows.append(np.array(rr))
    return rows


def dense_prob_from_rows(Ad_seq, Bd_seq, Xref, Uref, x_final, tr, rows, R_unused=None, **kw):
    """Convert (g,b) rows to the dense oracle's (g, c) with c = b - g'pbar."""
    pd = kw.get("pos_dim", 3)
    coll = None
    if rows is not None:
        coll = []
        for t in range(Xref.shape[0] - 1):
            r = rows[t]
            c = r[:, pd] - r[:, :pd] @ Xref[t, :pd]
            coll.append(np.hstack([r[:, :pd], c[:, None]]))
    p = dict(A=Ad_seq, B=Bd_seq, Xref=Xref, Uref=Uref, x_final=x_final, tr=tr, coll=coll)
    p.update(kw)
    return p


def synthetic_di(N, K=50, seed=0, sigma=30.0, spread=10.0, obstacles=0, obs_seed=11):
    """C2/C3 construction -- the same data the bench feeds the kernels
    (scvx_hip/workloads.py, host-side data construction only)."""
    from scvx_hip import workloads
    return workloads.synthetic_di(N, K=K, seed=seed, sigma=sigma, spread=spread, obstacles=obstacles,
                                  obs_seed=obs_seed)

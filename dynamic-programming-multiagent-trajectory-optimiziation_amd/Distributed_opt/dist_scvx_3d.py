"""Drop-in for the reference Distributed_opt/dist_scvx_3d.py (3-robot, 3-D double-integrator Jacobi SCP)
with the per-robot CVXPY+Clarabel solves replaced by ONE batched MI355X solve per iteration.

Module surface kept: the globals (T, n, m, dt, trust_region, R, robots_name, x_ini, x_des, Ad, Bd,
max_iter, cost_list), descete_f (:9-28), x_traj_opt (:31-118), x_initial (:122-128), cost_fcn
(:131-138) and the __main__ loop with its trust-region halving rule (:242-252).  Semantics kept:
  * every robot solves against the PREVIOUS iterate of the others (Jacobi) and X_traj is updated only
    after all solves (:113-118);
  * per-robot subproblem exactly as :59-107 (see include/scvx_hip.h), collision normals without epsilon;
  * the unused control row w[T-1] (:63) is pinned to 0, so X_traj[T-1, n:] is left unchanged: in the
    reference s_i[T-1, n:] appears in no constraint and no objective term, so every value is optimal
    and Clarabel's regularised KKT system returns 0 for it (same update);
  * a failed robot subproblem aborts the iteration with RuntimeError, as the reference aborts.
Plotting (:141-196) is optional (matplotlib, only when run as a script with --plot).
"""
import numpy as np

import scvx_hip


def descete_f(dt):
    """Exact zero-order hold of the 3-D double integrator (== scipy.signal StateSpace.to_discrete)."""
    Ad = np.eye(6)
    Ad[0:3, 3:6] = dt * np.eye(3)
    Bd = np.zeros((6, 3))
    Bd[0:3] = 0.5 * dt * dt * np.eye(3)
    Bd[3:6] = dt * np.eye(3)
    return [Ad, Bd]


def _device():
    import torch
    return torch.device("cuda")


def x_traj_opt(X_traj, trust_region):
    """One Jacobi sweep: all robots' trust-region QPs solved in one batched kernel launch."""
    import torch
    dev = _device()
    names = list(robots_name)
    N = len(names)
    Xr = np.stack([X_traj[nm][0:T, 0:n] for nm in names])
    Ur = np.stack([X_traj[nm][0:T, n:n + m] for nm in names])
    disc = np.zeros((T - 1, n * (n + 2 * m + 2)))
    for t in range(T - 1):
        disc[t, :n * n] = Ad.T.reshape(-1)
        disc[t, n * n:n * n + n * m] = Bd.T.reshape(-1)
    t_ = lambda a, dt=torch.float64: torch.as_tensor(np.ascontiguousarray(a), dtype=dt, device=dev)
    Xd = t_(Xr)
    jmax = max(N - 1, 0)
    rows = count = None
    if jmax > 0:
        rows, count = scvx_hip.collision_rows(Xd, 0, N, R, jmax, pos_dim=3, cull_radius=0.0)
    spec = scvx_hip.QPSpec(model="di", K=T, pos_dim=3, has_final=True, fix_last_input=True,
                           box=[(0, -1.0, 22.0), (1, -1.0, 20.0)], j_max=jmax, w_coll=10000.0, tol=1e-8,
                           max_iter=80)
    out = scvx_hip.qp_solve_batched(spec, t_(np.broadcast_to(disc, (N,) + disc.shape)), t_(np.zeros(N)), Xd,
                                    t_(Ur), t_(Xr[:, 0]), t_(np.stack([x_des[nm][0:n] for nm in names])),
                                    t_(np.full(N, float(trust_region))), rows, count)
    Xn, Un = out["X"].cpu().numpy(), out["U"].cpu().numpy()
    status = out["status"].cpu().numpy()
    print("update X")
    bad = [nm for a, nm in enumerate(names) if status[a] == 2]
    if bad:
        # the reference aborts here: cvxpy raises SolverError, or an infeasible solve leaves
        # s_i.value = None and `s_val[name].all()` (:115) raises AttributeError
        raise RuntimeError(f"x_traj_opt: subproblem of {bad} failed (solver_error)")
    for a, nm in enumerate(names):
        X_traj[nm][0:T, 0:n] += Xn[a] - Xr[a]
        X_traj[nm][0:T, n:n + m] += Un[a] - Ur[a]
    return X_traj


def x_initial(x_ini, x_des):
    return {nm: np.linspace(x_ini[nm], x_des[nm], T) for nm in robots_name}


def cost_fcn(X_traj):
    c = 0.0
    for nm in robots_name:
        u = X_traj[nm][0:T - 1, n:n + m]
        c += float(np.sum(u * u))
    return c


# global constants (:199-233)
Tf = 30
T0 = 0
T = 51
t_traj = np.linspace(T0, Tf, T)
dt = t_traj[1] - t_traj[0]
n = 6
m = 3
trust_region = 0.25
max_iter = 1000
N_agents = 3
robots_name = ["robot01", "robot02", "robot03"]
R = 2.3
x_ini = {}
x_des = {}
for count, name in enumerate(robots_name):
    x_ini[name] = np.array([0, count * 5.1, 10, 0, 0, 0, 0, 0, 0], dtype=float)
    x_des[name] = np.array([14, (N_agents - count - 1) * 5, 10 + count * 1, 0, 0, 0, 0, 0, 0], dtype=float)
[Ad, Bd] = descete_f(dt)
cost_list = np.zeros(max_iter)

if __name__ == "__main__":
    import sys
    iters = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else max_iter
    X_traj = x_initial(x_ini, x_des)
    for it in range(iters):
        print(trust_region)
        X_traj = x_traj_opt(X_traj, trust_region)
        cost_list[it] = cost_fcn(X_traj)
        print("Actual cost: ", cost_list[it])
        if it >= 1 and cost_list[it] > cost_list[it - 1]:
            trust_region = trust_region / 2

"""ORACLE / TEST INFRASTRUCTURE ONLY -- CPU restatement of the Nash iterative-best-response path.

Only tests/ use this module; the product path (scvx_hip, SCvx/...) never imports it.

  best_response   AgentBestResponse.setup + solve (SCvx/optimization/agent_best_response.py:46-113):
                  the SCProblem of oracle/scp_dense.py (reference formulation, independent sparse
                  conic IPM) plus GameUnicycleModel's cost and slab rows (SCvx/models/game_model.py:84-124)
                  and sigma == sigma_ref;
  slab_normals    GameUnicycleModel.update_slabs (game_model.py:54-66);
  ibr             NashSolver.solve (SCvx/optimization/nash_solver.py:66-143): Gauss-Seidel best
                  responses with the ACS inner loop, discretized by the C FOH restatement
                  (oracle/foh_ref.c, pinned to the reference's FirstOrderHold by tests/golden).

Trajectories are node-major here: X (K, n) is the reference's X.T.  Parity of the dense
formulation against ECOS itself is unpinned (ECOS/cvxpy are not installed); the pin on
the whole path is the reference's documented NASH row (tests/ref_pins.py)."""
import numpy as np

from . import foh_oracle, scp_dense, scp_problems


def slab_normals(p_i, P_j):
    """p_i, P_j (K, d) -> z (K, d): d_k/|d_k|, 0 where |d_k| < 1e-6."""
    z = np.zeros_like(p_i, dtype=float)
    for k in range(p_i.shape[0]):
        d = p_i[k] - P_j[k]
        nd = np.linalg.norm(d)
        if not nd < 1e-6:
            z[k] = d / nd
    return z


def game_problem(model, Xref, Uref, sigma_ref, cons, weights, X_prev, slabs, r_slab, tr=scp_problems.TRUST_RADIUS0,
                 nsub=16, disc=None, w=None):
    """The best-response problem dict for oracle/scp_dense.py.  cons: model_constraints(...) dict;
    weights: dict(control_weight, control_rate_weight, curvature_weight, inertia_weight);
    slabs: [(z (K,pd), P (K,pd))]; disc: (A, B, C, S, z) node-major stacks, else the C FOH."""
    K, n = Xref.shape
    m = Uref.shape[1]
    if disc is None:
        Ab, Bb, Cb, Sb, zb = foh_oracle.foh(model, Xref.T.copy(), Uref.T.copy(), sigma_ref, nsub=nsub)
        disc = (Ab.T.reshape(K - 1, n, n).transpose(0, 2, 1), Bb.T.reshape(K - 1, m, n).transpose(0, 2, 1),
                Cb.T.reshape(K - 1, m, n).transpose(0, 2, 1), Sb.T.copy(), zb.T.copy())
    p = dict(cons)
    w_nu, w_slack, w_sigma = w if w is not None else (scp_problems.WEIGHT_NU, scp_problems.WEIGHT_SLACK,
                                                      scp_problems.WEIGHT_SIGMA)
    p.update(A=disc[0], B=disc[1], C=disc[2], S=disc[3], z=disc[4], Xref=np.asarray(Xref, float),
             Uref=np.asarray(Uref, float), sigma_ref=float(sigma_ref), tr=float(tr), w_nu=w_nu, w_slack=w_slack,
             w_sigma=w_sigma)
    p["game"] = dict(w_u2=weights["control_weight"], w_du=weights["control_rate_weight"],
                     w_dth=weights.get("curvature_weight", 0.0), theta_idx=2 if model == "unicycle" else None,
                     w_in=weights.get("inertia_weight", 0.0), X_prev=np.asarray(X_prev, float), slabs=list(slabs),
                     r_slab=float(r_slab))
    return p


def disc_stacks(disc, n, m):
    """Kernel disc rows (K-1, n(n+2m+2): F-order A | B | C | S | z per node) -> node-major stacks."""
    K1 = disc.shape[0]
    o = np.cumsum([0, n * n, n * m, n * m, n, n])
    return (disc[:, o[0]:o[1]].reshape(K1, n, n).transpose(0, 2, 1), disc[:, o[1]:o[2]].reshape(K1, m, n).transpose(0, 2, 1),
            disc[:, o[2]:o[3]].reshape(K1, m, n).transpose(0, 2, 1), disc[:, o[3]:o[4]].copy(), disc[:, o[4]:o[5]].copy())


def best_response(p, tol=1e-10, maxit=300):
    return scp_dense.solve_scproblem(p, tol=tol, maxit=maxit)


def ibr(model, X_refs, U_refs, cons, weights, r_slab, sigma_ref=1.0, max_iter=20, tol=1e-3, max_acs_iters=5,
        acs_tol=1e-3, nsub=16, tr=scp_problems.TRUST_RADIUS0, w=None, log=None):
    """NashSolver.solve restated (nash_solver.py:66-143).  X_refs / U_refs: per agent (K, n) / (K, m);
    cons / weights / r_slab per agent lists.  Returns (X list, U list, change_hist)."""
    N = len(X_refs)
    pd = cons[0]["pos_dim"]
    X = [np.asarray(x, float).copy() for x in X_refs]
    U = [np.asarray(u, float).copy() for u in U_refs]
    hist = []
    for it in range(max_iter):
        Xp = [x.copy() for x in X]
        max_change = 0.0
        for i in range(N):
            nbr = [j for j in range(N) if j != i]
            z = [slab_normals(Xp[i][:, :pd], Xp[j][:, :pd]) for j in nbr]          # setup(): update_slabs
            P = [X[j][:, :pd] for j in nbr]
            Xn = Un = None
            for acs in range(max_acs_iters):
                pr = game_problem(model, X[i], U[i], sigma_ref, cons[i], weights[i], Xp[i], zip(z, P), r_slab[i],
                                  tr=tr, nsub=nsub, w=w)
                r = best_response(pr)
                if r["status"] not in ("optimal", "optimal_inaccurate"):
                    raise RuntimeError(f"oracle best response: iteration {it} agent {i} ACS step {acs} status "
                                       f"{r['status']} (after {r['iters']} IPM iterations)")
                Xn, Un = r["X"], r["U"]
                z = [slab_normals(Xn[:, :pd], X[j][:, :pd]) for j in nbr]
                if np.linalg.norm(Xn - X[i]) < acs_tol:
                    break
            delta = np.linalg.norm(Xn - X[i])
            max_change = max(max_change, delta)
            if log is not None:
                log.append((it, i, delta, r["obj"], r["iters"]))
            X[i], U[i] = Xn, Un
        hist.append(max_change)
        if max_change < tol:
            break
    return X, U, hist

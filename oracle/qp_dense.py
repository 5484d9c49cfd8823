"""ORACLE / TEST INFRASTRUCTURE ONLY -- QP/SOCP parity checker for the batched trust-region solve.

The reference solves each agent's convex subproblem with CVXPY -> Clarabel/ECOS
(Distributed_opt/dist_scvx_3d.py:51-111, SCvx/optimization/sc_problem.py:15-105).  None of
cvxpy/ECOS/Clarabel is installed here, so the reference's *solver* cannot be
run; its *formulation* can.  This module

  1. assembles the per-agent problem exactly as the reference writes it, in the reference's
     own variables (perturbations d, w, the shared collision slack S, the L1 trust region via
     CVXPY's epigraph canonicalization -v <= w <= v, sum v <= tr), as a dense conic QP
        min 1/2 z'Pz + q'z   s.t.  Az = b,  h - Gz in (R+^l x Q^{q1} x ...);
  2. solves it with a generic dense primal-dual interior-point method (Mehrotra
     predictor-corrector, Nesterov-Todd scaling for second-order cones -- the same algorithm
     family as Clarabel/ECOS), with plain numpy LU on the full KKT matrix;
  3. certifies the answer independently of the solver path (KKT residuals, cone membership,
     complementarity) -- `kkt_certificate`.

It shares no code and no formulation choices with the HIP solver (which works in absolute
variables, eliminates slacks per node, enumerates the L1 ball's 2^m facets and factors the KKT
by a Riccati recursion).  Solutions of these strictly-convex-in-u problems are unique, so
trajectories are comparable.  Parity against the reference's numerical solver output itself is
UNPINNED (no reference solver available offline); the reference formulation is what is pinned.
"""
import numpy as np

from .cone import soc_max_step


# ----------------------------------------------------------------------------------------------
# generic dense conic QP interior-point solver
# ----------------------------------------------------------------------------------------------
def _soc_J(x):
    return x[0] * x[0] - x[1:] @ x[1:]


def _soc_det(x):
    """_soc_J without cancellation, floored at a tiny positive value (NT scaling of a boundary iterate)."""
    n1 = np.linalg.norm(x[1:])
    return max((x[0] - n1) * (x[0] + n1), 1e-300)


def _jprod(dims, a, b):
    out = np.empty_like(a)
    nl = dims["l"]
    out[:nl] = a[:nl] * b[:nl]
    i = nl
    for k in dims["q"]:
        x, y = a[i:i + k], b[i:i + k]
        out[i] = x @ y
        out[i + 1:i + k] = x[0] * y[1:] + y[0] * x[1:]
        i += k
    return out


def _jdiv(dims, x, r):
    """rho with x o rho = r."""
    out = np.empty_like(r)
    nl = dims["l"]
    out[:nl] = r[:nl] / x[:nl]
    i = nl
    for k in dims["q"]:
        xx, rr = x[i:i + k], r[i:i + k]
        d = _soc_J(xx)
        r0 = (xx[0] * rr[0] - xx[1:] @ rr[1:]) / d
        out[i] = r0
        out[i + 1:i + k] = (rr[1:] - r0 * xx[1:]) / xx[0]
        i += k
    return out


def _identity(dims):
    e = np.zeros(dims["l"] + sum(dims["q"]))
    e[:dims["l"]] = 1.0
    i = dims["l"]
    for k in dims["q"]:
        e[i] = 1.0
        i += k
    return e


def _min_eig(dims, x):
    vals = []
    if dims["l"]:
        vals.append(np.min(x[:dims["l"]]))
    i = dims["l"]
    for k in dims["q"]:
        vals.append(x[i] - np.linalg.norm(x[i + 1:i + k]))
        i += k
    return min(vals) if vals else 1.0


def _nt_scaling(dims, s, z):
    """Dense W, W^-1 (block diagonal) with W z = W^-1 s."""
    m = len(s)
    W = np.zeros((m, m))
    Wi = np.zeros((m, m))
    nl = dims["l"]
    d = np.sqrt(s[:nl] / z[:nl])
    W[np.arange(nl), np.arange(nl)] = d
    Wi[np.arange(nl), np.arange(nl)] = 1.0 / d
    i = nl
    for k in dims["q"]:
        ss, zz = s[i:i + k], z[i:i + k]
        Js, Jz = _soc_det(ss), _soc_det(zz)
        sb, zb = ss / np.sqrt(Js), zz / np.sqrt(Jz)
        gam = np.sqrt((1.0 + sb @ zb) / 2.0)
        Jzb = zb.copy()
        Jzb[1:] *= -1
        w = (sb + Jzb) / (2.0 * gam)
        eta = (Js / Jz) ** 0.25
        # hyperbolic-rotation form of the NT scaling (W z = W^-1 s); W^2 = eta^2 (2 w w' - J)
        blk = np.eye(k)
        blk[1:, 1:] += np.outer(w[1:], w[1:]) / (1.0 + w[0])
        blk[0, 0] = w[0]
        Wb, Wib = blk.copy(), blk.copy()
        Wb[0, 1:] = Wb[1:, 0] = w[1:]
        Wib[0, 1:] = Wib[1:, 0] = -w[1:]
        W[i:i + k, i:i + k] = eta * Wb
        Wi[i:i + k, i:i + k] = Wib / eta
        i += k
    return W, Wi


def _max_step(dims, x, dx):
    a = np.inf
    nl = dims["l"]
    neg = dx[:nl] < 0
    if np.any(neg):
        a = min(a, np.min(-x[:nl][neg] / dx[:nl][neg]))
    i = nl
    for k in dims["q"]:
        a = min(a, soc_max_step(x[i:i + k], dx[i:i + k]))
        i += k
    return a


def solve_conic_qp(P, q, A, b, G, h, dims, tol=1e-11, maxit=80, verbose=False):
    """min 1/2 x'Px + q'x  s.t. Ax = b, Gx + s = h, s in K.  Returns dict(x, y, s, z, status, iters)."""
    n, p, m = len(q), len(b), len(h)
    e = _identity(dims)
    deg = dims["l"] + len(dims["q"])

    def kkt_solve(Wi2, rx, ry):
        K = np.zeros((n + p, n + p))
        K[:n, :n] = P + G.T @ Wi2 @ G
        K[:n, n:] = A.T
        K[n:, :n] = A
        sol = np.linalg.solve(K, np.concatenate([rx, ry]))
        return sol[:n], sol[n:]

    # initial point: W = I
    x, y = kkt_solve(np.eye(m), -q + G.T @ h, b)
    s = h - G @ x
    z = G @ x - h
    a_s, a_z = _min_eig(dims, s), _min_eig(dims, z)
    s = s + max(0.0, 1.0 - a_s) * e
    z = z + max(0.0, 1.0 - a_z) * e
    status = "max_iter"
    it = 0
    for it in range(maxit):
        rd = P @ x + q + A.T @ y + G.T @ z
        rp = A @ x - b
        rc = G @ x + s - h
        mu = (s @ z) / deg
        pres = max(np.linalg.norm(rp, np.inf), np.linalg.norm(rc, np.inf))
        dres = np.linalg.norm(rd, np.inf)
        pscale = 1.0 + max(np.linalg.norm(h, np.inf), np.linalg.norm(b, np.inf))
        dscale = 1.0 + np.linalg.norm(q, np.inf)
        pobj = 0.5 * x @ P @ x + q @ x
        if verbose:
            print(it, pres, dres, mu)
        if pres < tol * pscale and dres < tol * dscale and s @ z < tol * max(1.0, abs(pobj)):
            status = "optimal"
            break
        try:
            # an overflowing or invalid direction (a conditioning floor) ends the run: status stays "max_iter"
            with np.errstate(over="raise", invalid="raise"):
                W, Wi = _nt_scaling(dims, s, z)
                Wi2 = Wi @ Wi
                lam = W @ z

                def solve_dir(rcomp):
                    rho = _jdiv(dims, lam, rcomp)
                    t = Wi @ rho + Wi2 @ rc
                    dx, dy = kkt_solve(Wi2, -rd - G.T @ t, -rp)
                    dz = Wi @ rho + Wi2 @ (rc + G @ dx)
                    ds = -rc - G @ dx
                    return dx, dy, ds, dz

                lam2 = _jprod(dims, lam, lam)
                dxa, dya, dsa, dza = solve_dir(-lam2)
                alpha = min(1.0, _max_step(dims, s, dsa), _max_step(dims, z, dza))
                mu_a = ((s + alpha * dsa) @ (z + alpha * dza)) / deg
                sig = (mu_a / mu) ** 3
                corr = _jprod(dims, Wi @ dsa, W @ dza)
                dx, dy, ds, dz = solve_dir(-lam2 - corr + sig * mu * e)
                alpha = min(1.0, 0.99 * min(_max_step(dims, s, ds), _max_step(dims, z, dz)))
        except (FloatingPointError, np.linalg.LinAlgError):
            break
        x, y, s, z = x + alpha * dx, y + alpha * dy, s + alpha * ds, z + alpha * dz
    return dict(x=x, y=y, s=s, z=z, status=status, iters=it)


def kkt_certificate(P, q, A, b, G, h, dims, sol):
    """Solver-independent optimality certificate: max of scaled KKT residuals."""
    x, y, s, z = sol["x"], sol["y"], sol["s"], sol["z"]
    scale = 1.0 + max(np.abs(q).max(initial=0), np.abs(h).max(initial=0), np.abs(b).max(initial=0))
    rd = np.abs(P @ x + q + A.T @ y + G.T @ z).max(initial=0) / scale
    rp = max(np.abs(A @ x - b).max(initial=0), np.abs(G @ x + s - h).max(initial=0)) / scale
    cone = min(_min_eig(dims, s), _min_eig(dims, z))
    gap = abs(s @ z) / scale
    return dict(stationarity=rd, primal=rp, cone_min=cone, gap=gap)


# ----------------------------------------------------------------------------------------------
# reference formulation of one agent's Jacobi subproblem (Distributed_opt/dist_scvx_3d.py:51-111)
# ----------------------------------------------------------------------------------------------
def build_agent_problem(prob):
    """Assemble the dense conic QP for one agent, in the reference's own variables.

    prob keys (float64 numpy):
      A (K-1,n,n), B (K-1,n,m), C (K-1,n,m) or None, c (K-1,n) affine term (S sigma + z) or None
      Xref (K,n), Uref (K,m)            -- the current iterate X_traj[i] (rows) of dist_scvx_3d.py
      x_final (n,) or None              -- d_{T-1} + x_{T-1} == x_des   (:74)
      tr                                 -- ||w_t||_1 <= tr, t < T-1     (:84)
      box: list of (idx, lo, hi)         -- lo <= x_t[idx] + d_t[idx] <= hi, t < T-1 (:87-90)
      coll: list over t<T-1 of arrays (J_t, 4) rows (g0,g1,g2,c): c - g'd_t[0:3] <= S_t, S_t>=0 (:93-107)
      w_coll                             -- weight of sum S (1e4, :72)
      obs: list of (center(3), radius) ; w_obs -- a_t'(p_t - c) >= r - s_t, s_t >= 0
           a_t = (pbar_t - c)/(||pbar_t - c|| + 1e-6)  (single_integrator_model.py:113-126)
      umax or None                       -- ||u_t + w_t||_2 <= umax  (single_integrator_model.py:103-104)
      w_last                             -- weight on ||u_{T-1}+w_{T-1}||^2 (0 in dist_scvx_3d: unused row)
      w_final                            -- > 0: soft terminal w_final ||x_{T-1} + d_{T-1} - x_final||^2 in
                                            place of the row (:74) (build-side option, QPSpec.w_final)
      fix_last_input (bool)              -- pin w_{T-1} = 0 (dist_scvx_3d leaves it free & unused)
      w_nu                               -- > 0: virtual control nu_t (t < T-1) added to every dynamics row
                                            (the SCvx form of SCvx/optimization/sc_problem.py:60-68) with the
                                            exact penalty w_nu sum_t ||nu_t||_1 (CVXPY's epigraph
                                            -e <= nu <= e, + w_nu sum e; build-side option QPSpec.w_nu)
      w_prox                             -- > 0: + w_prox sum_t ||d_t||^2 (QPSpec.w_prox, a soft state trust region)
      pos_dim (3)
    Returns (P, q, A, b, G, h, dims, index dict).
    """
    Am, Bm = prob["A"], prob["B"]
    K = prob["Xref"].shape[0]
    n, m = prob["Xref"].shape[1], prob["Uref"].shape[1]
    Cm = prob.get("C")
    cm = prob.get("c")
    pd = prob.get("pos_dim", 3)
    Xr, Ur = prob["Xref"], prob["Uref"]
    coll = prob.get("coll") or []
    obs = prob.get("obs") or []
    has_coll = any(len(r) for r in coll)
    # variable layout
    idx = {}
    off = 0

    def alloc(name, size):
        nonlocal off
        idx[name] = (off, off + size)
        off += size

    alloc("d", K * n)
    alloc("w", K * m)
    alloc("v", (K - 1) * m)          # L1 epigraph (CVXPY canonicalization of norm(w,1))
    if has_coll:
        alloc("S", K - 1)
    if obs:
        alloc("so", (K - 1) * len(obs))
    w_nu = prob.get("w_nu", 0.0)
    if w_nu > 0:
        alloc("nu", (K - 1) * n)         # virtual control (sc_problem.py:25, 67)
        alloc("e", (K - 1) * n)          # its L1 epigraph
    nv = off

    def vd(t, i):
        return idx["d"][0] + t * n + i

    def vw(t, j):
        return idx["w"][0] + t * m + j

    P = np.zeros((nv, nv))
    q = np.zeros(nv)
    w_last = prob.get("w_last", 0.0)
    for t in range(K):
        wt = 1.0 if t < K - 1 else w_last
        for j in range(m):
            P[vw(t, j), vw(t, j)] += 2.0 * wt
            q[vw(t, j)] += 2.0 * wt * Ur[t, j]
    w_final = prob.get("w_final", 0.0)
    if w_final > 0:
        for i in range(n):
            P[vd(K - 1, i), vd(K - 1, i)] += 2.0 * w_final
            q[vd(K - 1, i)] += 2.0 * w_final * (Xr[K - 1, i] - prob["x_final"][i])
    w_prox = prob.get("w_prox", 0.0)
    if w_prox > 0:   # w_prox ||x_t - xbar_t||^2 = w_prox ||d_t||^2, every node (QPSpec.w_prox)
        for t in range(K):
            for i in range(n):
                P[vd(t, i), vd(t, i)] += 2.0 * w_prox
    if has_coll:
        q[idx["S"][0]:idx["S"][1]] = prob["w_coll"]
    if obs:
        q[idx["so"][0]:idx["so"][1]] = prob["w_obs"]
    if w_nu > 0:
        q[idx["e"][0]:idx["e"][1]] = w_nu

    Aeq, beq = [], []

    def eqrow():
        r = np.zeros(nv)
        Aeq.append(r)
        return r

    for i in range(n):                       # d_0 == 0            (:73)
        r = eqrow(); r[vd(0, i)] = 1.0; beq.append(0.0)
    if prob.get("x_final") is not None and not w_final > 0:   # d_{T-1} + x_{T-1} == x_des   (:74)
        for i in range(n):
            r = eqrow(); r[vd(K - 1, i)] = 1.0; beq.append(prob["x_final"][i] - Xr[K - 1, i])
    for t in range(K - 1):                   # x_{t+1}+d_{t+1} == A(x_t+d_t) + B(u_t+w_t) [+C(..)+c]  (:80-83)
        rhs0 = Am[t] @ Xr[t] + Bm[t] @ Ur[t] - Xr[t + 1]
        if Cm is not None:
            rhs0 = rhs0 + Cm[t] @ Ur[t + 1]
        if cm is not None:
            rhs0 = rhs0 + cm[t]
        for i in range(n):
            r = eqrow()
            r[vd(t + 1, i)] = 1.0
            for k in range(n):
                r[vd(t, k)] -= Am[t][i, k]
            for j in range(m):
                r[vw(t, j)] -= Bm[t][i, j]
                if Cm is not None:
                    r[vw(t + 1, j)] -= Cm[t][i, j]
            if w_nu > 0:
                r[idx["nu"][0] + t * n + i] -= 1.0
            beq.append(rhs0[i])
    if prob.get("fix_last_input", False):
        for j in range(m):
            r = eqrow(); r[vw(K - 1, j)] = 1.0; beq.append(0.0)
    Aeq = np.array(Aeq)
    beq = np.array(beq)

    Gl, hl = [], []

    def ineq(coefs, rhs):
        r = np.zeros(nv)
        for k, v in coefs:
            r[k] += v
        Gl.append(r)
        hl.append(rhs)

    tr = prob["tr"]
    for t in range(K - 1):
        for j in range(m):
            vv = idx["v"][0] + t * m + j
            ineq([(vw(t, j), 1.0), (vv, -1.0)], 0.0)     # w <= v
            ineq([(vw(t, j), -1.0), (vv, -1.0)], 0.0)    # -w <= v
        ineq([(idx["v"][0] + t * m + j, 1.0) for j in range(m)], tr)   # sum v <= tr
        for (bi, lo, hi) in prob.get("box", []):
            ineq([(vd(t, bi), 1.0)], hi - Xr[t, bi])
            ineq([(vd(t, bi), -1.0)], Xr[t, bi] - lo)
        if has_coll:
            St = idx["S"][0] + t
            for row in coll[t]:
                g, c = row[:pd], row[pd]
                ineq([(vd(t, i), -g[i]) for i in range(pd)] + [(St, -1.0)], -c)
            ineq([(St, -1.0)], 0.0)
        for o, (ctr, rad) in enumerate(obs):
            so = idx["so"][0] + t * len(obs) + o
            diff = Xr[t, :pd] - np.asarray(ctr)
            a = diff / (np.linalg.norm(diff) + 1e-6)
            # a'(pbar + d - c) >= r - s   <=>  -a'd - s <= a'(pbar - c) - r
            ineq([(vd(t, i), -a[i]) for i in range(pd)] + [(so, -1.0)], a @ diff - rad)
            ineq([(so, -1.0)], 0.0)
        if w_nu > 0:
            for i in range(n):
                vn, ve = idx["nu"][0] + t * n + i, idx["e"][0] + t * n + i
                ineq([(vn, 1.0), (ve, -1.0)], 0.0)     # nu <= e
                ineq([(vn, -1.0), (ve, -1.0)], 0.0)    # -nu <= e
    nl = len(Gl)
    qdims = []
    umax = prob.get("umax")
    if umax is not None:
        for t in range(K - 1):
            # (umax, u_t + w_t) in Q^{m+1}: h - G z with h = (umax, ubar), G = (0, -I on w)
            r0 = np.zeros(nv)
            Gl.append(r0); hl.append(umax)
            for j in range(m):
                r = np.zeros(nv); r[vw(t, j)] = -1.0
                Gl.append(r); hl.append(Ur[t, j])
            qdims.append(m + 1)
    G = np.array(Gl)
    h = np.array(hl)
    dims = {"l": nl, "q": qdims}
    return P, q, Aeq, beq, G, h, dims, idx


def solve_agent(prob, sparse=False, **kw):
    """Solve one agent's reference-form subproblem; returns X_new (K,n), U_new (K,m), obj, info.
    sparse=True: the same problem through oracle/scp_dense.py's sparse conic IPM (scipy splu on the
    KKT matrix; the large quadrotor / virtual-control instances, where the dense LU takes minutes)."""
    P, q, A, b, G, h, dims, idx = build_agent_problem(prob)
    if sparse:
        import scipy.sparse as sp
        from .scp_dense import solve_conic_qp_sparse
        osc = max(1.0, float(np.abs(q).max(initial=0.0)))
        sol = solve_conic_qp_sparse(sp.csr_matrix(P), q, sp.csr_matrix(A), b, sp.csr_matrix(G), h, dims,
                                    tol=kw.get("tol", 1e-10), maxit=kw.get("maxit", 150), osc=osc)
    else:
        sol = solve_conic_qp(P, q, A, b, G, h, dims, **kw)
    x = sol["x"]
    K, n = prob["Xref"].shape
    m = prob["Uref"].shape[1]
    d = x[idx["d"][0]:idx["d"][1]].reshape(K, n)
    w = x[idx["w"][0]:idx["w"][1]].reshape(K, m)
    obj = 0.5 * x @ P @ x + q @ x
    Ur = prob["Uref"]
    w_last = prob.get("w_last", 0.0)
    obj += np.sum(Ur[:-1] ** 2) + w_last * np.sum(Ur[-1] ** 2)
    if prob.get("w_final", 0.0) > 0:
        obj += prob["w_final"] * np.sum((prob["Xref"][-1] - prob["x_final"]) ** 2)
    info = dict(status=sol["status"], iters=sol["iters"], cert=kkt_certificate(P, q, A, b, G, h, dims, sol))
    if "S" in idx:
        info["S"] = x[idx["S"][0]:idx["S"][1]]
    if "nu" in idx:
        info["nu"] = x[idx["nu"][0]:idx["nu"][1]].reshape(K - 1, n)
    return prob["Xref"] + d, Ur + w, obj, info


def constraint_violation(prob, X, U, S=None, nu=None):
    """Max violation of the reference-form constraints (build_agent_problem) at absolute (X, U, S).

    Independent of any solver: the feasibility half of a parity certificate."""
    Xr, Ur = prob["Xref"], prob["Uref"]
    K, n = Xr.shape
    pd = prob.get("pos_dim", 3)
    d, w = X - Xr, U - Ur
    viol = {}
    viol["init"] = np.abs(d[0]).max()
    if prob.get("x_final") is not None and not prob.get("w_final", 0.0) > 0:
        viol["final"] = np.abs(X[K - 1] - prob["x_final"]).max()
    dyn = 0.0
    for t in range(K - 1):
        r = prob["A"][t] @ X[t] + prob["B"][t] @ U[t] - X[t + 1]
        if prob.get("C") is not None:
            r = r + prob["C"][t] @ U[t + 1]
        if prob.get("c") is not None:
            r = r + prob["c"][t]
        if nu is not None:
            r = r + nu[t]
        dyn = max(dyn, np.abs(r).max())
    viol["dyn"] = dyn
    viol["tr"] = max(0.0, max(np.abs(w[t]).sum() - prob["tr"] for t in range(K - 1)))
    bx = 0.0
    for (bi, lo, hi) in prob.get("box", []):
        bx = max(bx, np.max(X[:K - 1, bi] - hi), np.max(lo - X[:K - 1, bi]))
    viol["box"] = max(bx, 0.0)
    if prob.get("coll"):
        cv = 0.0
        for t in range(K - 1):
            for row in prob["coll"][t]:
                cv = max(cv, row[pd] - row[:pd] @ d[t, :pd] - S[t])
            cv = max(cv, -S[t])
        viol["coll"] = max(cv, 0.0)
    if prob.get("umax") is not None:
        viol["soc"] = max(0.0, max(np.linalg.norm(U[t]) - prob["umax"] for t in range(K - 1)))
    return viol

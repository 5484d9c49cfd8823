"""ORACLE / TEST INFRASTRUCTURE ONLY -- parity checker for the batched SCProblem / AgentSolver solve.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this module; the product
path (scvx_hip, SCvx/...) never imports it.

The reference's SCvx convex subproblem (SCvx/optimization/sc_problem.py:15-83, with the model
constraints of SCvx/models/unicycle_model.py:88-114 / single_integrator_model.py:80-126 and the ADMM
terms of SCvx/optimization/agent_solver.py:78-102 / si_agent_solver.py:70-92) is assembled here in the
reference's OWN variables X (n,K), U (m,K), nu (n,K-1), sigma, s_prime_j (K), S_j (K), with the
induced matrix 1-norms written the way CVXPY canonicalises them (per-column epigraph: |d_ik| <= a_ik,
sum_i a_ik <= t), and solved by a sparse primal-dual interior-point method (Mehrotra
predictor-corrector, Nesterov-Todd scaling for the second-order cones -- the ECOS/Clarabel algorithm
family) on the full KKT matrix with scipy's sparse LU.  It shares no formulation choices with the
HIP kernel (which enumerates the L1 balls' facets, carries sigma and the norm epigraphs as
augmented Riccati states and eliminates nu_{K-2} against the terminal condition).

LPs (unicycle, no ADMM terms) have non-unique optimisers, so parity is stated on the optimal
VALUE, primal feasibility and a KKT certificate; the ADMM problems are strictly convex in the
positions only.  Parity against ECOS/Clarabel output itself is UNPINNED: neither is installed (SURVEY
§8c, ordinary ImportError); the reference *formulation* is what this file pins.
"""
import numpy as np
import scipy.sparse as sp
import scipy.sparse.linalg as spla

from .cone import soc_max_step

WEIGHT_COLLISION_SLACK = 1e5  # SCvx/optimization/admm_utils.py:5


# ----------------------------------------------------------------------------------------------
# sparse conic QP interior point:  min 1/2 x'Px + q'x  s.t.  Ax = b,  Gx + s = h,  s in R+^l x Q...
# ----------------------------------------------------------------------------------------------
def _cone_blocks(dims):
    blocks, i = [], dims["l"]
    for k in dims["q"]:
        blocks.append((i, k))
        i += k
    return blocks


def _jprod(dims, a, b):
    out = np.empty_like(a)
    nl = dims["l"]
    out[:nl] = a[:nl] * b[:nl]
    for i, k in _cone_blocks(dims):
        x, y = a[i:i + k], b[i:i + k]
        out[i] = x @ y
        out[i + 1:i + k] = x[0] * y[1:] + y[0] * x[1:]
    return out


def _jdiv(dims, x, r):
    out = np.empty_like(r)
    nl = dims["l"]
    out[:nl] = r[:nl] / x[:nl]
    for i, k in _cone_blocks(dims):
        xx, rr = x[i:i + k], r[i:i + k]
        d = xx[0] * xx[0] - xx[1:] @ xx[1:]
        r0 = (xx[0] * rr[0] - xx[1:] @ rr[1:]) / d
        out[i] = r0
        out[i + 1:i + k] = (rr[1:] - r0 * xx[1:]) / xx[0]
    return out


def _unit(dims, m):
    e = np.zeros(m)
    e[:dims["l"]] = 1.0
    for i, _ in _cone_blocks(dims):
        e[i] = 1.0
    return e


def _min_eig(dims, x):
    v = [np.min(x[:dims["l"]])] if dims["l"] else []
    for i, k in _cone_blocks(dims):
        v.append(x[i] - np.linalg.norm(x[i + 1:i + k]))
    return min(v) if v else 1.0


def _max_step(dims, x, dx):
    a = np.inf
    nl = dims["l"]
    neg = dx[:nl] < 0
    if np.any(neg):
        a = min(a, np.min(-x[:nl][neg] / dx[:nl][neg]))
    for i, k in _cone_blocks(dims):
        a = min(a, soc_max_step(x[i:i + k], dx[i:i + k]))
    return a


def _soc_det(x):
    """x0^2 - ||x1||^2 as (x0 - ||x1||)(x0 + ||x1||): no cancellation near the cone boundary, and floored
    at a tiny positive value so the NT scaling of an iterate that rounding put on the boundary stays
    finite (the square root / fourth root of a negative number was NaN)."""
    n1 = np.linalg.norm(x[1:])
    return max((x[0] - n1) * (x[0] + n1), 1e-300)


def _nt_scaling(dims, s, z):
    """Sparse block-diagonal W, W^-1 with W z = W^-1 s (hyperbolic-rotation form for SOC)."""
    nl = dims["l"]
    d = np.sqrt(s[:nl] / z[:nl])
    Wb, Wib = [sp.diags(d)], [sp.diags(1.0 / d)]
    for i, k in _cone_blocks(dims):
        ss, zz = s[i:i + k], z[i:i + k]
        Js, Jz = _soc_det(ss), _soc_det(zz)
        sb, zb = ss / np.sqrt(Js), zz / np.sqrt(Jz)
        gam = np.sqrt((1.0 + sb @ zb) / 2.0)
        Jzb = zb.copy()
        Jzb[1:] *= -1
        w = (sb + Jzb) / (2.0 * gam)
        eta = (Js / Jz) ** 0.25
        blk = np.eye(k)
        blk[1:, 1:] += np.outer(w[1:], w[1:]) / (1.0 + w[0])
        blk[0, 0] = w[0]
        W, Wi = blk.copy(), blk.copy()
        W[0, 1:] = W[1:, 0] = w[1:]
        Wi[0, 1:] = Wi[1:, 0] = -w[1:]
        Wb.append(sp.csr_matrix(eta * W))
        Wib.append(sp.csr_matrix(Wi / eta))
    return sp.block_diag(Wb, format="csr"), sp.block_diag(Wib, format="csr")


def solve_conic_qp_sparse(P, q, A, b, G, h, dims, tol=1e-10, maxit=100, osc=1.0, trace=None):
    """Returns dict(x, y, s, z, status, iters).  P, A, G scipy sparse.  osc: objective scale (the
    iteration runs on (P, q)/osc, the duals are returned in the caller's units; the gap test stays
    relative to the unscaled objective)."""
    P, q = P / osc, q / osc
    n, p, m = len(q), len(b), len(h)
    e = _unit(dims, m)
    deg = dims["l"] + len(dims["q"])
    P, A, G = sp.csr_matrix(P), sp.csr_matrix(A), sp.csr_matrix(G)

    def factor(Wi2):
        H = P + G.T @ Wi2 @ G
        try:
            return spla.splu(sp.bmat([[H, A.T], [A, None]], format="csc"))
        except RuntimeError:     # exactly singular (a pivot underflowed): static regularisation; the
            d = 1e-11 * max(1.0, abs(H).max())  # residuals stay exact, later iterations absorb it
            return spla.splu(sp.bmat([[H + d * sp.identity(n), A.T], [A, -d * sp.identity(p)]], format="csc"))

    def ksolve(lu, rx, ry):
        sol = lu.solve(np.concatenate([rx, ry]))
        return sol[:n], sol[n:]

    lu = factor(sp.identity(m, format="csr"))
    x, y = ksolve(lu, -q + G.T @ h, b)
    s = h - G @ x
    z = G @ x - h
    s = s + max(0.0, 1.0 - _min_eig(dims, s)) * e
    z = z + max(0.0, 1.0 - _min_eig(dims, z)) * e
    status, it = "max_iter", 0
    best = (np.inf, 0, x, y, s, z)
    pscale = 1.0 + max(np.abs(h).max(initial=0), np.abs(b).max(initial=0))
    dscale = 1.0 + np.abs(q).max(initial=0)
    for it in range(maxit):
        rd = P @ x + q + A.T @ y + G.T @ z
        rp = A @ x - b
        rc = G @ x + s - h
        mu = (s @ z) / deg
        pobj = 0.5 * x @ (P @ x) + q @ x
        pres = max(np.abs(rp).max(initial=0), np.abs(rc).max(initial=0))
        if trace is not None:
            trace.append((pres / pscale, np.abs(rd).max() / dscale, s @ z, pobj * osc))
        if pres < tol * pscale and np.abs(rd).max() < tol * dscale and s @ z < tol * max(1.0 / osc, abs(pobj)):
            status = "optimal"
            break
        # ECOS-style reduced accuracy: keep the best iterate by max(scaled residuals, relative gap);
        # when 15 iterations bring no improvement (a conditioning floor), or at the cap, the best
        # iterate within 1e-8 feasibility and 1e-6 relative gap is returned as "optimal_inaccurate"
        merit = max(pres / pscale, np.abs(rd).max() / dscale, (s @ z) / max(1.0 / osc, abs(pobj)))
        if merit < best[0]:
            best = (merit, it, x.copy(), y.copy(), s.copy(), z.copy())
        if it - best[1] > 15:
            break
        try:
            # an overflowing or invalid direction (the Newton system at a conditioning floor) is a breakdown:
            # the best iterate so far is returned below, as ECOS does
            with np.errstate(over="raise", invalid="raise"):
                W, Wi = _nt_scaling(dims, s, z)
                Wi2 = Wi @ Wi
                lam = W @ z
                lu = factor(Wi2)

                def direction(rcomp):
                    rho = _jdiv(dims, lam, rcomp)
                    t = Wi @ rho + Wi2 @ rc
                    dx, dy = ksolve(lu, -rd - G.T @ t, -rp)
                    dz = Wi @ rho + Wi2 @ (rc + G @ dx)
                    ds = -rc - G @ dx
                    return dx, dy, ds, dz

                lam2 = _jprod(dims, lam, lam)
                dxa, dya, dsa, dza = direction(-lam2)
                alpha = min(1.0, _max_step(dims, s, dsa), _max_step(dims, z, dza))
                mu_a = ((s + alpha * dsa) @ (z + alpha * dza)) / deg
                sig = (mu_a / mu) ** 3
                corr = _jprod(dims, Wi @ dsa, W @ dza)
                dx, dy, ds, dz = direction(-lam2 - corr + sig * mu * e)
                alpha = min(1.0, 0.99 * min(_max_step(dims, s, ds), _max_step(dims, z, dz)))
                if not (np.isfinite(alpha) and np.all(np.isfinite(dx)) and np.all(np.isfinite(dz))):
                    raise FloatingPointError("non-finite direction")
        except (RuntimeError, FloatingPointError):   # boundary round-off (SOC J < 0) or a singular
            break                                     # factor: the best iterate is returned below
        x, y, s, z = x + alpha * dx, y + alpha * dy, s + alpha * ds, z + alpha * dz
    if status != "optimal" and best[0] < 1e-6:
        # (merit mixes scaled residuals and the relative gap: 1e-6 bounds all three)
        status, (x, y, s, z) = "optimal_inaccurate", best[2:]
    return dict(x=x, y=y * osc, s=s, z=z * osc, status=status, iters=it)


def kkt_certificate(P, q, A, b, G, h, dims, sol):
    x, y, s, z = sol["x"], sol["y"], sol["s"], sol["z"]
    scale = 1.0 + max(np.abs(q).max(initial=0), np.abs(h).max(initial=0), np.abs(b).max(initial=0))
    rd = np.abs(P @ x + q + A.T @ y + G.T @ z).max(initial=0) / scale
    rp = max(np.abs(A @ x - b).max(initial=0), np.abs(G @ x + s - h).max(initial=0)) / scale
    return dict(stationarity=rd, primal=rp, cone_min=min(_min_eig(dims, s), _min_eig(dims, z)),
                gap=abs(s @ z) / scale)


# ----------------------------------------------------------------------------------------------
# the reference's SCProblem (+ AgentSolver terms), in its own variables
# ----------------------------------------------------------------------------------------------
def obstacle_normals(Xref, center, pd):
    """a_k = (xbar_k - c)/(||xbar_k - c|| + 1e-6) (unicycle_model.py:103-114, single_integrator_model.py:113-126)."""
    d = Xref[:, :pd] - np.asarray(center, float)[None, :pd]
    return d / (np.linalg.norm(d, axis=1, keepdims=True) + 1e-6)


def build_scproblem(prob):
    """Assemble the reference's convex subproblem as a sparse conic QP.

    prob keys (float64 numpy; node index first, i.e. X is (K,n) = reference X.T):
      A (K-1,n,n), B, C (K-1,n,m), S, z (K-1,n)       discretization (sc_problem.py:29-34, :53-68)
      Xref (K,n), Uref (K,m), sigma_ref, tr            (:36-44, :71-74)
      w_nu, w_slack, w_sigma                           objective weights (:77-83)
      x_init, x_final (n,)                             BCs X[:,0], X[:,-1]; U[:,0] = U[:,-1] = 0
      u_bounds: [(j, lo, hi)]                          unicycle_model.py:96 (0<=v<=vmax, |w|<=wmax)
      u_soc: vmax or None                              single_integrator_model.py:103-104
      x_bounds: [(i, lo, hi)]                          position box with robot radius (:98-101 / :107-110)
      obs: [(center, r_total)], pos_dim               linearized obstacles with slack s_prime (:103-114)
      nbrs: [dict(Pref (K,pd), Y (K,pd), Lam (K,pd))], rho, d_min    AgentSolver terms (agent_solver.py:78-95)
      game: dict(w_u2, w_du, w_dth, theta_idx, w_in, X_prev (K,n), slabs [(z (K,pd), P (K,pd))], r_slab)
            Nash best response (agent_best_response.py:46-81 with game_model.py:84-124): the cost
            terms, the slab rows z_k'(p_k - P_k) >= r_slab and sigma == sigma_ref
    Returns (P, q, A, b, G, h, dims, idx).
    """
    A_, B_, C_, S_, z_ = prob["A"], prob["B"], prob["C"], prob["S"], prob["z"]
    Xr, Ur = prob["Xref"], prob["Uref"]
    K, n = Xr.shape
    m = Ur.shape[1]
    pd = prob.get("pos_dim", 2)
    obs = prob.get("obs") or []
    nbrs = prob.get("nbrs") or []
    idx, off = {}, 0

    def alloc(name, size):
        nonlocal off
        idx[name] = (off, off + size)
        off += size

    alloc("X", K * n)
    alloc("U", K * m)
    alloc("nu", (K - 1) * n)
    alloc("sigma", 1)
    alloc("sp", K * len(obs))
    alloc("S", K * len(nbrs))
    alloc("ax", K * n)        # epigraph of norm(dx, 1): |dx_ik| <= ax_ik
    alloc("au", K * m)
    alloc("anu", (K - 1) * n)
    alloc("t", 4)             # tx, tu, ts, tnu
    nv = off
    X = lambda k, i: idx["X"][0] + k * n + i          # noqa: E731
    U = lambda k, j: idx["U"][0] + k * m + j          # noqa: E731
    NU = lambda k, i: idx["nu"][0] + k * n + i        # noqa: E731
    SG = idx["sigma"][0]
    SP = lambda o, k: idx["sp"][0] + o * K + k        # noqa: E731
    SC = lambda j, k: idx["S"][0] + j * K + k         # noqa: E731
    AX = lambda k, i: idx["ax"][0] + k * n + i        # noqa: E731
    AU = lambda k, j: idx["au"][0] + k * m + j        # noqa: E731
    AN = lambda k, i: idx["anu"][0] + k * n + i       # noqa: E731
    TX, TU, TS, TN = (idx["t"][0] + i for i in range(4))

    eq_r, eq_c, eq_v, beq = [], [], [], []

    def eq(coefs, rhs):
        r = len(beq)
        for c, v in coefs:
            eq_r.append(r), eq_c.append(c), eq_v.append(v)
        beq.append(rhs)

    # model BCs (unicycle_model.py:94, single_integrator_model.py:95-100)
    for i in range(n):
        eq([(X(0, i), 1.0)], prob["x_init"][i])
        eq([(X(K - 1, i), 1.0)], prob["x_final"][i])
    for j in range(m):
        eq([(U(0, j), 1.0)], 0.0)
        eq([(U(K - 1, j), 1.0)], 0.0)
    game = prob.get("game")
    if game is not None:
        eq([(SG, 1.0)], prob["sigma_ref"])                      # agent_best_response.py:77
    # dynamics X_{k+1} = A X_k + B U_k + C U_{k+1} + S sigma + z + nu   (sc_problem.py:53-68)
    for k in range(K - 1):
        for i in range(n):
            co = [(X(k + 1, i), 1.0), (SG, -S_[k, i]), (NU(k, i), -1.0)]
            co += [(X(k, l), -A_[k, i, l]) for l in range(n)]
            co += [(U(k, j), -B_[k, i, j]) for j in range(m)]
            co += [(U(k + 1, j), -C_[k, i, j]) for j in range(m)]
            eq(co, z_[k, i])

    lin_r, lin_c, lin_v, hl = [], [], [], []

    def le(coefs, rhs):
        r = len(hl)
        for c, v in coefs:
            lin_r.append(r), lin_c.append(c), lin_v.append(v)
        hl.append(rhs)

    for (j, lo, hi) in prob.get("u_bounds") or []:
        for k in range(K):
            if k in (0, K - 1) and (lo is None or lo <= 0.0) and (hi is None or hi >= 0.0):
                continue        # U[:,0] = U[:,-1] = 0 satisfies the bound: a row without interior
            if hi is not None:
                le([(U(k, j), 1.0)], hi)
            if lo is not None:
                le([(U(k, j), -1.0)], -lo)
    for (i, lo, hi) in prob.get("x_bounds") or []:
        for k in range(K):
            le([(X(k, i), 1.0)], hi)
            le([(X(k, i), -1.0)], -lo)
    for o, (c, r_tot) in enumerate(obs):
        a = obstacle_normals(Xr, c, pd)
        cc = np.asarray(c, float)[:pd]
        for k in range(K):
            # a'(X[0:pd,k] - c) >= r_tot - s'_k
            le([(X(k, i), -a[k, i]) for i in range(pd)] + [(SP(o, k), -1.0)], -r_tot - a[k] @ cc)
            le([(SP(o, k), -1.0)], 0.0)
    for jn, nb in enumerate(nbrs):
        d = Xr[:, :pd] - nb["Pref"]
        a = d / (np.linalg.norm(d, axis=1, keepdims=True) + 1e-6)      # multi_agent_model.py:61-79
        for k in range(K):
            # a'(p_k - Y_k) + S_k >= d_min   (agent_solver.py:85-90)
            le([(X(k, i), -a[k, i]) for i in range(pd)] + [(SC(jn, k), -1.0)],
               -prob["d_min"] - a[k] @ nb["Y"][k])
            le([(SC(jn, k), -1.0)], 0.0)
    if game is not None:
        for (zs, Ps) in game["slabs"]:
            for k in range(K):
                # z_k'(p_k - P_k) >= r   (game_model.py:121-124)
                le([(X(k, i), -zs[k, i]) for i in range(pd)], -game["r_slab"] - zs[k] @ Ps[k])
    # trust region  norm(dx,1) + norm(du,1) + |ds| <= tr   (induced norms, sc_problem.py:71-74)
    for k in range(K):
        for i in range(n):
            le([(X(k, i), 1.0), (AX(k, i), -1.0)], Xr[k, i])
            le([(X(k, i), -1.0), (AX(k, i), -1.0)], -Xr[k, i])
        le([(AX(k, i), 1.0) for i in range(n)] + [(TX, -1.0)], 0.0)
        for j in range(m):
            le([(U(k, j), 1.0), (AU(k, j), -1.0)], Ur[k, j])
            le([(U(k, j), -1.0), (AU(k, j), -1.0)], -Ur[k, j])
        le([(AU(k, j), 1.0) for j in range(m)] + [(TU, -1.0)], 0.0)
    le([(SG, 1.0), (TS, -1.0)], prob["sigma_ref"])
    le([(SG, -1.0), (TS, -1.0)], -prob["sigma_ref"])
    le([(TX, 1.0), (TU, 1.0), (TS, 1.0)], prob["tr"])
    le([(SG, -1.0)], 0.0)                                   # sigma nonneg (sc_problem.py:25)
    # norm(nu, 1) epigraph
    for k in range(K - 1):
        for i in range(n):
            le([(NU(k, i), 1.0), (AN(k, i), -1.0)], 0.0)
            le([(NU(k, i), -1.0), (AN(k, i), -1.0)], 0.0)
        le([(AN(k, i), 1.0) for i in range(n)] + [(TN, -1.0)], 0.0)
    nl = len(hl)
    # SOC ||U[:,k]|| <= vmax  ->  (vmax, U[:,k]) in Q^{m+1}
    soc_r, soc_c, soc_v, hs, qd = [], [], [], [], []
    if prob.get("u_soc") is not None:
        for k in range(K):
            base = len(hs)
            hs.append(prob["u_soc"])
            for j in range(m):
                soc_r.append(base + 1 + j), soc_c.append(U(k, j)), soc_v.append(-1.0)
                hs.append(0.0)
            qd.append(m + 1)
    G = sp.vstack([sp.csr_matrix((lin_v, (lin_r, lin_c)), shape=(nl, nv)),
                   sp.csr_matrix((soc_v, (soc_r, soc_c)), shape=(len(hs), nv))], format="csr")
    h = np.concatenate([np.array(hl), np.array(hs)])
    Aeq = sp.csr_matrix((eq_v, (eq_r, eq_c)), shape=(len(beq), nv))
    # objective  w_nu norm(nu,1) + w_slack sum s' + w_sigma sigma   (sc_problem.py:77-83)
    q = np.zeros(nv)
    q[TN] = prob["w_nu"]
    q[SG] = prob["w_sigma"]
    for o in range(len(obs)):
        for k in range(K):
            q[SP(o, k)] = prob["w_slack"]
    Pd = np.zeros(nv)
    rho = prob.get("rho", 0.0)
    for jn, nb in enumerate(nbrs):
        # sum Lam o (p - Y) + rho/2 ||p - Y||^2 + W_COLL sum S  (agent_solver.py:92-95)
        for k in range(K):
            for i in range(pd):
                q[X(k, i)] += nb["Lam"][k, i] - rho * nb["Y"][k, i]
                Pd[X(k, i)] += rho
            q[SC(jn, k)] = WEIGHT_COLLISION_SLACK
    Pr, Pc, Pv = list(range(nv)), list(range(nv)), list(Pd)
    const = sum(float(np.sum(-nb["Lam"] * nb["Y"]) + 0.5 * rho * np.sum(nb["Y"] ** 2)) for nb in nbrs)
    if game is not None:
        def sq(a, b, w):        # w (z_a - z_b)^2
            Pr.extend([a, b, a, b]), Pc.extend([a, b, b, a]), Pv.extend([2 * w, 2 * w, -2 * w, -2 * w])
        for k in range(K):
            for j in range(m):
                Pr.append(U(k, j)), Pc.append(U(k, j)), Pv.append(2 * game["w_u2"])     # game_model.py:88
                if k < K - 1 and game["w_du"] > 0:
                    sq(U(k + 1, j), U(k, j), game["w_du"])                                # :91-93
            if k < K - 1 and game["w_dth"] > 0 and game["theta_idx"] is not None:
                th = game["theta_idx"]
                sq(X(k + 1, th), X(k, th), game["w_dth"])                                 # :94-96
            if game["w_in"] > 0:                                                          # :99-100
                for i in range(n):
                    Pr.append(X(k, i)), Pc.append(X(k, i)), Pv.append(2 * game["w_in"])
                    q[X(k, i)] -= 2 * game["w_in"] * game["X_prev"][k, i]
        if game["w_in"] > 0:
            const += game["w_in"] * float(np.sum(game["X_prev"] ** 2))
    P = sp.csr_matrix((Pv, (Pr, Pc)), shape=(nv, nv))
    idx["const"] = const
    return P, q, Aeq, np.array(beq), G, h, dict(l=nl, q=qd), idx


def solve_scproblem(prob, tol=1e-10, maxit=100):
    """Returns dict(X (K,n), U (K,m), nu (K-1,n), sigma, s_prime (nobs,K), S (nnb,K), obj, status, cert)."""
    P, q, A, b, G, h, dims, idx = build_scproblem(prob)
    osc = max(1.0, np.abs(q).max(initial=0.0), abs(P).max() if P.nnz else 0.0)
    sol = solve_conic_qp_sparse(P, q, A, b, G, h, dims, tol=tol, maxit=maxit, osc=osc)
    x = sol["x"]
    K, n = prob["Xref"].shape
    m = prob["Uref"].shape[1]
    g = lambda name: x[idx[name][0]:idx[name][1]]  # noqa: E731
    out = dict(X=g("X").reshape(K, n), U=g("U").reshape(K, m), nu=g("nu").reshape(K - 1, n), sigma=float(g("sigma")[0]),
               s_prime=g("sp").reshape(-1, K), S=g("S").reshape(-1, K),
               obj=float(0.5 * x @ (P @ x) + q @ x + idx["const"]), status=sol["status"], iters=sol["iters"],
               cert=kkt_certificate(P, q, A, b, G, h, dims, sol))
    # duality gap of the returned point relative to its objective (caller's units): an optimal_inaccurate
    # answer (the best iterate at a conditioning floor) is as good as this says
    out["rel_gap"] = abs(float(sol["s"] @ sol["z"])) / max(1.0, abs(float(0.5 * x @ (P @ x) + q @ x)))
    return out


def scp_objective(prob, X, U, nu, sigma, s_prime=None, S=None):
    """The reference objective evaluated at a point (induced 1-norm of nu, sc_problem.py:77-83 +
    agent_solver.py:92-95); slacks default to their optimal values given X."""
    K = X.shape[0]
    pd = prob.get("pos_dim", 2)
    obj = prob["w_nu"] * np.abs(nu).sum(axis=1).max() + prob["w_sigma"] * sigma
    game = prob.get("game")
    if game is not None:
        obj += game["w_u2"] * np.sum(U ** 2) + game["w_du"] * np.sum(np.diff(U, axis=0) ** 2)
        if game["theta_idx"] is not None:
            obj += game["w_dth"] * np.sum(np.diff(X[:, game["theta_idx"]]) ** 2)
        if game["w_in"] > 0:
            obj += game["w_in"] * np.sum((X - game["X_prev"]) ** 2)
    for o, (c, r_tot) in enumerate(prob.get("obs") or []):
        a = obstacle_normals(prob["Xref"], c, pd)
        viol = np.maximum(0.0, r_tot - np.einsum("ki,ki->k", a, X[:, :pd] - np.asarray(c, float)[None, :pd]))
        obj += prob["w_slack"] * (viol.sum() if s_prime is None else s_prime[o].sum())
    rho = prob.get("rho", 0.0)
    for jn, nb in enumerate(prob.get("nbrs") or []):
        d = prob["Xref"][:, :pd] - nb["Pref"]
        a = d / (np.linalg.norm(d, axis=1, keepdims=True) + 1e-6)
        diff = X[:, :pd] - nb["Y"]
        viol = np.maximum(0.0, prob["d_min"] - np.einsum("ki,ki->k", a, diff))
        obj += np.sum(nb["Lam"] * diff) + 0.5 * rho * np.sum(diff ** 2)
        obj += WEIGHT_COLLISION_SLACK * (viol.sum() if S is None else S[jn].sum())
    return float(obj)


def scp_violation(prob, X, U, nu, sigma):
    """Max violation of the hard constraints of build_scproblem at (X, U, nu, sigma)."""
    K, n = X.shape
    pd = prob.get("pos_dim", 2)
    v = [np.abs(X[0] - prob["x_init"]).max(), np.abs(X[-1] - prob["x_final"]).max(),
         np.abs(U[0]).max(), np.abs(U[-1]).max(), max(0.0, -sigma)]
    for k in range(K - 1):
        pred = prob["A"][k] @ X[k] + prob["B"][k] @ U[k] + prob["C"][k] @ U[k + 1] + prob["S"][k] * sigma \
            + prob["z"][k] + nu[k]
        v.append(np.abs(X[k + 1] - pred).max())
    for (j, lo, hi) in prob.get("u_bounds") or []:
        if hi is not None:
            v.append(max(0.0, (U[:, j] - hi).max()))
        if lo is not None:
            v.append(max(0.0, (lo - U[:, j]).max()))
    for (i, lo, hi) in prob.get("x_bounds") or []:
        v.append(max(0.0, (X[:, i] - hi).max(), (lo - X[:, i]).max()))
    if prob.get("u_soc") is not None:
        v.append(max(0.0, (np.linalg.norm(U, axis=1) - prob["u_soc"]).max()))
    game = prob.get("game")
    if game is not None:
        v.append(abs(sigma - prob["sigma_ref"]))
        for (zs, Ps) in game["slabs"]:
            v.append(max(0.0, (game["r_slab"] - np.einsum("ki,ki->k", zs, X[:, :pd] - Ps)).max()))
    tr_used = np.abs(X - prob["Xref"]).sum(axis=1).max() + np.abs(U - prob["Uref"]).sum(axis=1).max() \
        + abs(sigma - prob["sigma_ref"])
    v.append(max(0.0, tr_used - prob["tr"]))
    return float(max(v))

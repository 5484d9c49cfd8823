"""ORACLE / TEST INFRASTRUCTURE ONLY -- CPU restatement (numpy) of the structured SCProblem IPM that
csrc/scp_ipm.hip runs on the GPU (same formulation, same iteration), used to pin the kernel
iterate-by-iterate and to develop the algorithm on the CPU.  Never imported by the product path.

Problem: the reference's SCvx convex subproblem (SCvx/optimization/sc_problem.py:15-83) with the
model constraints of unicycle_model.py:88-114 / single_integrator_model.py:80-126 and optionally the
ADMM terms of agent_solver.py:78-95 / si_agent_solver.py:70-88.  Reformulation (exact):

  * per node k the variables z_k = [xi_k (n) | g (4) | u_k (m) | nu_k (n)] with
    xi_k = x_k - C_{k-1} u_k (FOH transform, so the dynamics lose the u_{k+1} term) and
    g = (sigma, tau_x, tau_u, tau_nu) carried as augmented Riccati STATE with g_{k+1} = g_k;
  * the induced 1-norms (sc_problem.py:74, :78) as L1-ball facets  s'(x_k - xbar_k) <= tau_x,
    s'(u_k - ubar_k) <= tau_u, s'nu_k <= tau_nu  (s in {-1,1}^dim), |sigma - sigma_ref| + tau_x +
    tau_u <= tr at node 0; objective w_nu tau_nu + w_sigma sigma + w_slack sum s';
  * x_{K-1} = x_final is eliminated by substituting nu_{K-2} = x_final - (A x + B u + C u_{K-1} +
    S sigma + z)_{K-2} into its facets (the K-2 dynamics then pin xi_{K-1}); U[:,0] = U[:,-1] = 0
    and nu_{K-1} (absent) are pinned inputs; x_0 = x_init is the Riccati initial state, g_0 free;
  * soft rows (obstacles, ADMM collision rows) keep their slack, eliminated per row.
Newton systems are solved by a Riccati recursion over the nodes (state n+4, input m+n).
"""
import itertools

import os

import numpy as np
from scipy.linalg import solve_triangular

NG = 4  # sigma, tau_x, tau_u, tau_nu
SCP_TAU_END = 0.99999  # end-game step fraction (csrc/scp_kernel.hpp)


def signs(d):
    return np.array(list(itertools.product((1.0, -1.0), repeat=d)))


class Layout:
    def __init__(self, n, m):
        self.n, self.m = n, m
        self.nxa, self.nua = n + NG, m + n
        self.nz = self.nxa + self.nua
        self.X = np.arange(0, n)
        self.G = n + np.arange(NG)
        self.U = n + NG + np.arange(m)
        self.N = n + NG + m + np.arange(n)
        self.SIG, self.TX, self.TU, self.TN = self.G


def build_nodes(p):
    """Per node: hard rows (a, h), soft rows (a, h, w), SOC blocks [(G (q,NZ), h (q))], q, P, pinned
    mask -- all in z-coordinates; dynamics At, Bt, ct."""
    K, n = p["Xref"].shape
    m = p["Uref"].shape[1]
    L = Layout(n, m)
    pd = p["pos_dim"]
    has_final = p.get("x_final") is not None
    A, B, C, S, zc = p["A"], p["B"], p["C"], p["S"], p["z"]
    Sx, Su = signs(n), signs(m)
    # objective scale: the kernel divides every cost term by cs so the duals are O(1) (weights of
    # 1e4..1e6 otherwise put the IPM's barrier curvatures lambda/s across > 1e24 in the end-game)
    nb_all = p.get("nbrs") or []
    cs = max([1.0, p["w_nu"], p["w_sigma"], p["w_slack"] if p.get("obs") else 0.0, 1e5 if nb_all else 0.0,
              p.get("rho", 0.0)] + [float(np.abs(nb["Lam"] - p.get("rho", 0.0) * nb["Y"]).max()) for nb in nb_all])
    nodes = []
    for k in range(K):
        hard, soft, socs = [], [], []

        def row(coefs):
            a = np.zeros(L.nz)
            for idx, v in coefs:
                a[idx] += v
            return a

        for s in Sx:                                   # TR facets on x
            a = row([(L.TX, -1.0)]); a[L.X] = s
            hard.append((a, s @ p["Xref"][k]))
        for s in Su:                                   # TR facets on u
            a = row([(L.TU, -1.0)]); a[L.U] = s
            hard.append((a, s @ p["Uref"][k]))
        if k < K - 1:                                  # ||nu_k||_1 <= tau_nu facets
            for s in Sx:
                a = row([(L.TN, -1.0)]); a[L.N] = s
                hard.append((a, 0.0))
        for (j, lo, hi) in p.get("u_bounds") or []:
            if k == 0 or k == K - 1:                   # pinned inputs: constant rows dropped (kernel too)
                continue
            if hi is not None:
                hard.append((row([(L.U[j], 1.0)]), hi))
            if lo is not None:
                hard.append((row([(L.U[j], -1.0)]), -lo))
        for (i, lo, hi) in p.get("x_bounds") or []:
            hard.append((row([(L.X[i], 1.0)]), hi))
            hard.append((row([(L.X[i], -1.0)]), -lo))
        if k == 0:
            hard.append((row([(L.SIG, -1.0)]), 0.0))
            hard.append((row([(L.SIG, 1.0), (L.TX, 1.0), (L.TU, 1.0)]), p["tr"] + p["sigma_ref"]))
            hard.append((row([(L.SIG, -1.0), (L.TX, 1.0), (L.TU, 1.0)]), p["tr"] - p["sigma_ref"]))
        for (c, r_tot) in p.get("obs") or []:
            cc = np.asarray(c, float)[:pd]
            d = p["Xref"][k, :pd] - cc
            an = d / (np.linalg.norm(d) + 1e-6)
            a = np.zeros(L.nz); a[L.X[:pd]] = -an
            soft.append((a, -r_tot - an @ cc, p["w_slack"] / cs))
        for nb in p.get("nbrs") or []:
            d = p["Xref"][k, :pd] - nb["Pref"][k]
            an = d / (np.linalg.norm(d) + 1e-6)
            a = np.zeros(L.nz); a[L.X[:pd]] = -an
            soft.append((a, -p["d_min"] - an @ nb["Y"][k], 1e5 / cs))
        if p.get("u_soc") is not None:
            Gs = np.zeros((m + 1, L.nz)); hs = np.zeros(m + 1)
            hs[0] = p["u_soc"]
            Gs[1 + np.arange(m), L.U] = -1.0
            socs.append((Gs, hs))
        q = np.zeros(L.nz)
        P = np.zeros((L.nz, L.nz))
        if k == 0:
            q[L.SIG] += p["w_sigma"] / cs
            q[L.TN] += p["w_nu"] / cs
        rho = p.get("rho", 0.0)
        for nb in p.get("nbrs") or []:
            q[L.X[:pd]] += (nb["Lam"][k] - rho * nb["Y"][k]) / cs
            P[L.X[:pd], L.X[:pd]] += rho / cs
        # nu_{K-2} substitution against x_{K-1} = x_final (u_{K-1} pinned at 0)
        if has_final and k == K - 2:
            def subst(a, h):
                an = a[L.N].copy()
                a = a.copy()
                a[L.X] -= A[k].T @ an
                a[L.U] -= B[k].T @ an
                a[L.SIG] -= S[k] @ an
                a[L.N] = 0.0
                return a, h - an @ (p["x_final"] - zc[k])
            hard = [subst(a, h) for a, h in hard]
        # FOH transform x_k = xi_k + C_{k-1} u_k
        T = np.eye(L.nz)
        if k > 0:
            T[np.ix_(L.X, L.U)] = C[k - 1]
        hard = [(T.T @ a, h) for a, h in hard]
        soft = [(T.T @ a, h, w) for a, h, w in soft]
        socs = [(Gs @ T, hs) for Gs, hs in socs]
        q = T.T @ q
        P = T.T @ P @ T
        pin = np.zeros(L.nz, bool)
        if k == 0 or k == K - 1:
            pin[L.U] = True
        if k == K - 1 or (has_final and k == K - 2):
            pin[L.N] = True
        # dynamics to node k+1 in Riccati coordinates
        dyn = None
        if k < K - 1:
            At = np.zeros((L.nxa, L.nxa)); Bt = np.zeros((L.nxa, L.nua)); ct = np.zeros(L.nxa)
            At[n:, n:] = np.eye(NG)
            if has_final and k == K - 2:
                ct[:n] = p["x_final"]              # xi_{K-1} = x_final - C_{K-2} * 0
            else:
                Cp = C[k - 1] if k > 0 else np.zeros((n, m))
                At[:n, :n] = A[k]
                At[:n, n] = S[k]
                Bt[:n, :m] = B[k] + A[k] @ Cp
                Bt[:n, m:] = np.eye(n)
                ct[:n] = zc[k]
            dyn = (At, Bt, ct)
        nodes.append(dict(hard=hard, soft=soft, socs=socs, q=q, P=P, pin=pin, dyn=dyn))
    return nodes, L


def ldl_solve(M, b, rel=1e-13):
    """LDL' solve of a symmetric (quasi-)definite block, pivots below rel * max|diag| clamped --
    the dynamic regularisation the kernel applies (csrc/scp_ipm.hip ldl_factor; IPM end-game normal
    matrices lose definiteness in rounding when barrier curvatures span > 1e16).

    Near the optimum the LP-like directions (nu, the norm epigraphs) carry curvature ~reg against ~1e6
    elsewhere, so the Riccati Schur complements are conditioned ~1e16; rounding can then leave a pivot
    clearly negative (-7e-2 on the ADMM unicycle instance of tests/test_scp_gpu.py), the clamp turns it
    into a 1e12 gain and the recursion overflows within a few stages.  The kernel (different rounding
    order) did not hit it on that instance.  Both treat a non-finite factor or direction as a breakdown
    (reduced-accuracy exit), so the overflow is an expected, handled event here: no FP warnings.  A
    max(|d|, clamp) pivot rule removes the overflow but perturbed the kernel's directions enough to fail
    two GPU parity tests, so it is not used."""
    nn = M.shape[0]
    Lm = np.eye(nn)
    d = np.zeros(nn)
    A = M.copy()
    dmax = np.abs(np.diag(M)).max()
    with np.errstate(over="ignore", invalid="ignore"):
        return _ldl_solve(A, Lm, d, dmax, nn, b, rel)


def _ldl_solve(A, Lm, d, dmax, nn, b, rel):
    for j in range(nn):
        dj = A[j, j] - (Lm[j, :j] ** 2) @ d[:j]
        dj = max(dj, rel * dmax + 1e-300)
        d[j] = dj
        for i in range(j + 1, nn):
            Lm[i, j] = (A[i, j] - (Lm[i, :j] * Lm[j, :j]) @ d[:j]) / dj
    if not np.isfinite(Lm).all():          # the kernel propagates the non-finite values to its guard
        return np.full(np.shape(b), np.nan)
    y = solve_triangular(Lm, b, lower=True, unit_diagonal=True, check_finite=False)
    y = (y.T / d).T
    return solve_triangular(Lm.T, y, lower=False, unit_diagonal=True, check_finite=False)


# ---- cone helpers (per node: LP part then SOC blocks)
def _soc_nt(s, z):
    Js, Jz = s[0] ** 2 - s[1:] @ s[1:], z[0] ** 2 - z[1:] @ z[1:]
    sb, zb = s / np.sqrt(Js), z / np.sqrt(Jz)
    gam = np.sqrt((1.0 + sb @ zb) / 2.0)
    Jzb = zb.copy(); Jzb[1:] *= -1
    w = (sb + Jzb) / (2.0 * gam)
    eta = (Js / Jz) ** 0.25
    k = len(s)
    blk = np.eye(k)
    blk[1:, 1:] += np.outer(w[1:], w[1:]) / (1.0 + w[0])
    blk[0, 0] = w[0]
    W, Wi = blk.copy(), blk.copy()
    W[0, 1:] = W[1:, 0] = w[1:]
    Wi[0, 1:] = Wi[1:, 0] = -w[1:]
    return eta * W, Wi / eta


def _jprod_soc(x, y):
    out = np.empty_like(x)
    out[0] = x @ y
    out[1:] = x[0] * y[1:] + y[0] * x[1:]
    return out


def _jdiv_soc(x, r):
    d = x[0] * x[0] - x[1:] @ x[1:]
    r0 = (x[0] * r[0] - x[1:] @ r[1:]) / d
    out = np.empty_like(r)
    out[0] = r0
    out[1:] = (r[1:] - r0 * x[1:]) / x[0]
    return out


def _soc_step(x, dx):
    a = np.inf
    qa = dx[0] ** 2 - dx[1:] @ dx[1:]
    qb = 2 * (x[0] * dx[0] - x[1:] @ dx[1:])
    qc = x[0] ** 2 - x[1:] @ x[1:]
    if abs(qa) > 1e-300:
        disc = qb * qb - 4 * qa * qc
        if disc >= 0:
            for r in ((-qb - np.sqrt(disc)) / (2 * qa), (-qb + np.sqrt(disc)) / (2 * qa)):
                if r > 0 and x[0] + r * dx[0] >= -1e-14:
                    a = min(a, r)
    elif qb != 0 and -qc / qb > 0:
        a = min(a, -qc / qb)
    if dx[0] < 0:
        a = min(a, -x[0] / dx[0])
    return a


class SCPSolver:
    """Structured Mehrotra predictor-corrector IPM with Riccati KKT solves (the kernel's algorithm)."""

    def __init__(self, p, tol=1e-9, max_iter=100, reg=1e-10):
        self.p, self.tol, self.max_iter, self.reg = p, tol, max_iter, reg
        self._regv = reg
        self.nodes, self.L = build_nodes(p)
        self.K = len(self.nodes)

    # node rows as one LP block: hard rows, soft row pairs (a z - sig + s1 = h ; -sig + s2 = 0)
    def _lp(self, nd):
        return len(nd["hard"]) + 2 * len(nd["soft"])

    def solve(self):
        L, K, nodes, p = self.L, self.K, self.nodes, self.p
        n = L.n
        # ---- starting point (W = I): min 1/2 z'Pz + q'z + 1/2||Gz - h||^2 s.t. dynamics
        z = np.zeros((K, L.nz))
        sig = [np.zeros(len(nd["soft"])) for nd in nodes]
        lin = []
        for nd in nodes:
            H = nd["P"].copy()
            f = nd["q"].copy()
            for a, h in nd["hard"]:
                H += np.outer(a, a); f -= a * h
            fs = []
            for a, h, w in nd["soft"]:
                # sigma_r: H_ss = 2, H_zs = -a ; f_s = w + h   -> eliminate
                rhs_s = -w - h
                H += 0.5 * np.outer(a, a)
                f -= a * h + 0.5 * a * rhs_s
                fs.append(rhs_s)
            for Gs, hs in nd["socs"]:
                H += Gs.T @ Gs; f -= Gs.T @ hs
            lin.append((H, f, fs))
        rp = [nd["dyn"][2].copy() if nd["dyn"] is not None else None for nd in nodes]
        r_init = -p["x_init"].copy()
        dz, yplus, yinit = self._lq([x[0] for x in lin], [x[1] for x in lin], rp, r_init)
        z = dz
        for k, nd in enumerate(nodes):
            for r, (a, h, w) in enumerate(nd["soft"]):
                sig[k][r] = (lin[k][2][r] + a @ z[k]) / 2.0
        s, lam = [], []
        for k, nd in enumerate(nodes):
            gz = self._Gz(nd, z[k], sig[k])
            hh = self._h(nd)
            s.append(hh - gz)
            lam.append(gz - hh)
        a_s = min(self._min_eig(nd, s[k]) for k, nd in enumerate(nodes))
        a_z = min(self._min_eig(nd, lam[k]) for k, nd in enumerate(nodes))
        for k, nd in enumerate(nodes):
            e = self._unit(nd)
            s[k] = s[k] + max(0.0, 1.0 - a_s) * e
            lam[k] = lam[k] + max(0.0, 1.0 - a_z) * e
        y = np.zeros((K - 1, L.nxa))
        y0 = np.zeros(n)
        deg = sum(self._lp(nd) + len(nd["socs"]) for nd in nodes)
        hmax = max(max((abs(self._h(nd)).max(initial=0) for nd in nodes)), np.abs(p["x_init"]).max(),
                   max(np.abs(nd["dyn"][2]).max() for nd in nodes if nd["dyn"] is not None))
        qmax = max(max(np.abs(nd["q"]).max() for nd in nodes), max((w for nd in nodes for _, _, w in nd["soft"]),
                                                                     default=0.0))
        pscale, dscale = 1.0 + hmax, 1.0 + qmax
        status, it, near_ok = "max_iter", 0, False
        pres_best = dres_best = np.inf
        score_best, snap = np.inf, None   # best iterate once the reduced tolerances hold (kernel: o_zb / o_sgb)
        self.restored = False
        self.trace = []
        self._regv = self.reg     # kernel: regv (x100 retry after a breakdown, x0.01 after a step)
        for it in range(self.max_iter):
            # residuals
            rd, rsig, rc, rpv = [], [], [], []
            for k, nd in enumerate(nodes):
                r = nd["P"] @ z[k] + nd["q"] + self._GTl(nd, lam[k])
                if nd["dyn"] is not None:
                    At, Bt, ct = nd["dyn"]
                    r[:L.nxa] += At.T @ y[k]
                    r[L.nxa:] += Bt.T @ y[k]
                if k > 0:
                    r[:L.nxa] -= y[k - 1]
                else:
                    r[:n] -= y0
                r[nd["pin"]] = 0.0
                rd.append(r)
                nh = len(nd["hard"])
                rsig.append(np.array([w for _, _, w in nd["soft"]]) - lam[k][nh:nh + 2 * len(nd["soft"]):2]
                            - lam[k][nh + 1:nh + 2 * len(nd["soft"]):2])
                rc.append(self._Gz(nd, z[k], sig[k]) + s[k] - self._h(nd))
                if nd["dyn"] is not None:
                    At, Bt, ct = nd["dyn"]
                    rpv.append(At @ z[k][:L.nxa] + Bt @ z[k][L.nxa:] + ct - z[k + 1][:L.nxa])
                else:
                    rpv.append(None)
            r_init = z[0][:n] - p["x_init"]
            gap = sum(s[k] @ lam[k] for k in range(K))
            mu = gap / deg
            pobj = sum(0.5 * z[k] @ nd["P"] @ z[k] + nd["q"] @ z[k] + sum(w * sig[k][r] for r, (_, _, w) in
                                                                          enumerate(nd["soft"]))
                       for k, nd in enumerate(nodes))
            pres = max(max(np.abs(x).max() for x in rpv if x is not None), np.abs(r_init).max(),
                       max(np.abs(x).max(initial=0) for x in rc))
            dres = max(max(np.abs(x).max() for x in rd), max((np.abs(x).max(initial=0) for x in rsig), default=0))
            self.trace.append((pres, dres, gap, pobj))
            if pres < self.tol * pscale and dres < self.tol * dscale and gap < self.tol * max(1.0, abs(pobj)):
                status = "optimal"
                break
            # reduced (ECOS-style "inaccurate") tolerances, used if the solve ends early (kernel: near_ok)
            near_ok = (pres < max(1e-4, self.tol) * pscale and dres < max(1e-4, self.tol) * dscale
                       and gap < max(5e-5, self.tol) * max(1.0, abs(pobj)))   # ECOS reduced tolerances
            # insufficient progress (kernel: pres_best / dres_best): a residual jumping 100x above its best
            # (ECOS returns its best iterate there: restore the snapshot below)
            if near_ok and (pres > max(100.0 * pres_best, self.tol * pscale)
                            or dres > max(100.0 * dres_best, self.tol * dscale)):
                status = "inaccurate"
                if snap is not None:
                    z, sig = snap[0].copy(), [x.copy() for x in snap[1]]
                    self.restored = True
                break
            pres_best, dres_best = min(pres_best, pres), min(dres_best, dres)
            score = max(pres / pscale, dres / dscale, gap / max(1.0, abs(pobj)))
            if near_ok and score < score_best:
                score_best, snap = score, (z.copy(), [x.copy() for x in sig])
            # scaling
            Wn = [self._nt(nd, s[k], lam[k]) for k, nd in enumerate(nodes)]
            lt = [self._Wmul(nd, Wn[k], lam[k], 0) for k, nd in enumerate(nodes)]   # lambda~ = W lam
            Hs = []
            if os.environ.get("SCP_DEBUG"):
                dm = max((float((1.0 / Wn[k][0] ** 2).max(initial=0)), k) for k in range(K))
                kk = dm[1]
                dd = 1.0 / Wn[kk][0] ** 2
                rr = int(np.argmax(dd))
                print(f"it {it} pres {pres:.2e} dres {dres:.2e} gap {gap:.2e} max D {dm[0]:.3e} node {kk} row {rr} "
                      f"s {s[kk][rr]:.3e} lam {lam[kk][rr]:.3e} nh {len(nodes[kk]['hard'])}")
            for k, nd in enumerate(nodes):
                H = nd["P"].copy()
                wl, socW = Wn[k]
                nh = len(nd["hard"])
                d = 1.0 / wl ** 2
                for r, (a, h) in enumerate(nd["hard"]):
                    H += d[r] * np.outer(a, a)
                for r, (a, h, w) in enumerate(nd["soft"]):
                    d1, d2 = d[nh + 2 * r], d[nh + 2 * r + 1]
                    H += (d1 * d2 / (d1 + d2)) * np.outer(a, a)
                for b, (Gs, hs) in enumerate(nd["socs"]):
                    Wi = socW[b][1]
                    H += Gs.T @ (Wi @ Wi) @ Gs
                Hs.append(H)

            def direction(rcomp):
                # rcomp: per node vector (rows); returns dz, dsig, ds, dlam, yplus, y0plus
                fs, aux = [], []
                for k, nd in enumerate(nodes):
                    rho = self._jdiv(nd, lt[k], rcomp[k])
                    t = self._Wmul(nd, Wn[k], rho, 1) + self._Wmul(nd, Wn[k], self._Wmul(nd, Wn[k], rc[k], 1), 1)
                    f = nd["P"] @ z[k] + nd["q"] + self._GTl(nd, lam[k]) + self._GTl(nd, t, soft_first_only=True)
                    wl, socW = Wn[k]
                    d = 1.0 / wl ** 2
                    nh = len(nd["hard"])
                    rs = []
                    for r, (a, h, w) in enumerate(nd["soft"]):
                        d1, d2 = d[nh + 2 * r], d[nh + 2 * r + 1]
                        t1, t2 = t[nh + 2 * r], t[nh + 2 * r + 1]
                        rhs_s = -rsig[k][r] + t1 + t2
                        f -= a * d1 * rhs_s / (d1 + d2)
                        rs.append(rhs_s)
                    fs.append(f)
                    aux.append((rho, t, rs))
                dz, yp, y0p = self._lq(Hs, fs, rpv, r_init)
                out_dsig, out_ds, out_dl = [], [], []
                for k, nd in enumerate(nodes):
                    rho, t, rs = aux[k]
                    wl, socW = Wn[k]
                    d = 1.0 / wl ** 2
                    nh = len(nd["hard"])
                    dsg = np.zeros(len(nd["soft"]))
                    for r, (a, h, w) in enumerate(nd["soft"]):
                        d1, d2 = d[nh + 2 * r], d[nh + 2 * r + 1]
                        dsg[r] = (rs[r] + d1 * (a @ dz[k])) / (d1 + d2)
                    gdz = self._Gz(nd, dz[k], dsg)
                    ds = -rc[k] - gdz
                    dl = self._Wmul(nd, Wn[k], rho, 1) + self._Wmul(nd, Wn[k], self._Wmul(nd, Wn[k], rc[k] + gdz, 1), 1)
                    out_dsig.append(dsg); out_ds.append(ds); out_dl.append(dl)
                return dz, out_dsig, out_ds, out_dl, yp, y0p

            lam2 = [self._jprod(nd, lt[k], lt[k]) for k, nd in enumerate(nodes)]
            dza, dsga, dsa, dla, _, _ = direction([-x for x in lam2])
            alpha = min(1.0, min(min(self._step(nd, s[k], dsa[k]), self._step(nd, lam[k], dla[k]))
                                 for k, nd in enumerate(nodes)))
            mu_a = sum((s[k] + alpha * dsa[k]) @ (lam[k] + alpha * dla[k]) for k in range(K)) / deg
            sg = (mu_a / mu) ** 3
            rcomp = []
            for k, nd in enumerate(nodes):
                corr = self._jprod(nd, self._Wmul(nd, Wn[k], dsa[k], 1), self._Wmul(nd, Wn[k], dla[k], 0))
                rcomp.append(-lam2[k] - corr + sg * mu * self._unit(nd))
            dz, dsg, ds, dl, yp, y0p = direction(rcomp)
            # step fraction 0.99, 1 - 1e-5 once the affine step is (nearly) full (kernel: SCP_TAU_END)
            tau = SCP_TAU_END if alpha >= 0.99 else 0.99
            alpha = min(1.0, tau * min(min(self._step(nd, s[k], ds[k]), self._step(nd, lam[k], dl[k]))
                                       for k, nd in enumerate(nodes)))
            # breakdown guard (kernel: wave_max(badl)): stop on the current finite iterate
            fin = np.isfinite(alpha) and alpha > 0 and np.isfinite(dz).all() and np.isfinite(yp).all() and \
                np.isfinite(y0p).all() and all(np.isfinite(x).all() for x in dsg + ds + dl)
            if not fin:
                if self._regv < 1e-5:
                    self._regv *= 100.0
                    continue
                status = "inaccurate" if near_ok else "numerical"
                break
            z = z + alpha * dz
            for k in range(K):
                sig[k] = sig[k] + alpha * dsg[k]
                s[k] = s[k] + alpha * ds[k]
                lam[k] = lam[k] + alpha * dl[k]
            y = y + alpha * (yp - y)
            y0 = y0 + alpha * (y0p - y0)
            self._regv = max(self.reg, 0.01 * self._regv)
        else:
            it = self.max_iter
            if not near_ok:
                status = "numerical"
        self.z, self.sig, self.s, self.lam = z, sig, s, lam
        return self._outputs(status, it)

    # ---- Riccati LQ solve: min sum 1/2 dz'H dz + f'dz s.t. xi~_{k+1} = At xi~ + Bt u~ + rp_k,
    # xi_0 (x part) = -r_init, g_0 free, pinned inputs zero.  Returns dz, costates y+ (K-1), y0+.
    def _lq(self, Hs, fs, rp, r_init):
        # a breakdown (overflowing Riccati factor at an extreme barrier scaling) yields non-finite directions,
        # which solve() detects and handles like the kernel (regularised retry, then the reduced-accuracy exit)
        with np.errstate(over="ignore", invalid="ignore", divide="ignore"):
            return self._lq_raw(Hs, fs, rp, r_init)

    def _lq_raw(self, Hs, fs, rp, r_init):
        L, K, nodes = self.L, self.K, self.nodes
        nx, n = L.nxa, L.n
        Ps, ps, Ks, ks = [None] * K, [None] * K, [None] * K, [None] * K
        Hm = []
        for k, nd in enumerate(nodes):
            H = Hs[k] + self._regv * np.eye(L.nz); f = fs[k].copy()
            pin = nd["pin"]
            H[pin, :] = 0.0; H[:, pin] = 0.0
            H[pin, pin] = 1.0
            f[pin] = 0.0
            Hm.append((H, f))
        P, pv = None, None
        for k in range(K - 1, -1, -1):
            H, f = Hm[k]
            Qxx, Qux, Quu = H[:nx, :nx].copy(), H[nx:, :nx].copy(), H[nx:, nx:].copy()
            qx, qu = f[:nx].copy(), f[nx:].copy()
            if k < K - 1:
                At, Bt, _ = nodes[k]["dyn"]
                Ppr = P @ rp[k] + pv
                Qxx += At.T @ P @ At; Qux += Bt.T @ P @ At; Quu += Bt.T @ P @ Bt
                qx += At.T @ Ppr; qu += Bt.T @ Ppr
            pin = nodes[k]["pin"][nx:]
            Qux[pin, :] = 0.0; Quu[pin, :] = 0.0; Quu[:, pin] = 0.0; Quu[pin, pin] = 1.0; qu[pin] = 0.0
            Kk = -ldl_solve(Quu, Qux)
            kk = -ldl_solve(Quu, qu)
            P = Qxx + Qux.T @ Kk
            P = 0.5 * (P + P.T)

            pv = qx + Qux.T @ kk
            Ps[k], ps[k], Ks[k], ks[k] = P, pv, Kk, kk
        # stage 0: x part fixed, g part free
        xi = np.zeros(nx)
        xi[:n] = -r_init
        gi = np.arange(n, nx)
        xi[gi] = -ldl_solve(Ps[0][np.ix_(gi, gi)], ps[0][gi] + Ps[0][gi, :n] @ xi[:n])
        dz = np.zeros((K, L.nz))
        yp = np.zeros((K - 1, nx))
        y0p = (Ps[0] @ xi + ps[0])[:n]
        for k in range(K):
            u = Ks[k] @ xi + ks[k]
            dz[k, :nx], dz[k, nx:] = xi, u
            if k < K - 1:
                At, Bt, _ = nodes[k]["dyn"]
                xi = At @ xi + Bt @ u + rp[k]
                yp[k] = Ps[k + 1] @ xi + ps[k + 1]
        return dz, yp, y0p

    # ---- per-node cone algebra
    def _h(self, nd):
        parts = [np.array([h for _, h in nd["hard"]])]
        sh = []
        for a, h, w in nd["soft"]:
            sh += [h, 0.0]
        parts.append(np.array(sh))
        parts += [hs for _, hs in nd["socs"]]
        return np.concatenate(parts)

    def _Gz(self, nd, z, sig):
        out = [np.array([a @ z for a, _ in nd["hard"]])]
        sh = []
        for r, (a, h, w) in enumerate(nd["soft"]):
            sh += [a @ z - sig[r], -sig[r]]
        out.append(np.array(sh))
        out += [Gs @ z for Gs, _ in nd["socs"]]
        return np.concatenate(out)

    def _GTl(self, nd, lam, soft_first_only=False):
        """G' lam restricted to z (soft rows: only their first row touches z)."""
        g = np.zeros(self.L.nz)
        nh = len(nd["hard"])
        for r, (a, _) in enumerate(nd["hard"]):
            g += a * lam[r]
        for r, (a, h, w) in enumerate(nd["soft"]):
            g += a * lam[nh + 2 * r]
        o = self._lp(nd)
        for Gs, hs in nd["socs"]:
            g += Gs.T @ lam[o:o + len(hs)]
            o += len(hs)
        return g

    def _unit(self, nd):
        e = np.zeros(self._lp(nd) + sum(len(hs) for _, hs in nd["socs"]))
        e[:self._lp(nd)] = 1.0
        o = self._lp(nd)
        for _, hs in nd["socs"]:
            e[o] = 1.0
            o += len(hs)
        return e

    def _min_eig(self, nd, x):
        nl = self._lp(nd)
        v = [x[:nl].min()] if nl else []
        o = nl
        for _, hs in nd["socs"]:
            q = len(hs)
            v.append(x[o] - np.linalg.norm(x[o + 1:o + q]))
            o += q
        return min(v)

    def _nt(self, nd, s, lam):
        nl = self._lp(nd)
        wl = np.sqrt(s[:nl] / lam[:nl])
        soc = []
        o = nl
        for _, hs in nd["socs"]:
            q = len(hs)
            soc.append(_soc_nt(s[o:o + q], lam[o:o + q]))
            o += q
        return wl, soc

    def _Wmul(self, nd, Wn, v, inv):
        wl, soc = Wn
        nl = self._lp(nd)
        out = np.empty_like(v)
        out[:nl] = v[:nl] / wl if inv else v[:nl] * wl
        o = nl
        for b, (_, hs) in enumerate(nd["socs"]):
            q = len(hs)
            out[o:o + q] = soc[b][1 if inv else 0] @ v[o:o + q]
            o += q
        return out

    def _jprod(self, nd, a, b):
        nl = self._lp(nd)
        out = np.empty_like(a)
        out[:nl] = a[:nl] * b[:nl]
        o = nl
        for _, hs in nd["socs"]:
            q = len(hs)
            out[o:o + q] = _jprod_soc(a[o:o + q], b[o:o + q])
            o += q
        return out

    def _jdiv(self, nd, x, r):
        nl = self._lp(nd)
        out = np.empty_like(r)
        out[:nl] = r[:nl] / x[:nl]
        o = nl
        for _, hs in nd["socs"]:
            q = len(hs)
            out[o:o + q] = _jdiv_soc(x[o:o + q], r[o:o + q])
            o += q
        return out

    def _step(self, nd, x, dx):
        nl = self._lp(nd)
        a = np.inf
        neg = dx[:nl] < 0
        if np.any(neg):
            a = np.min(-x[:nl][neg] / dx[:nl][neg])
        o = nl
        for _, hs in nd["socs"]:
            q = len(hs)
            a = min(a, _soc_step(x[o:o + q], dx[o:o + q]))
            o += q
        return a

    def _outputs(self, status, it):
        L, K, p, z = self.L, self.K, self.p, self.z
        n, m = L.n, L.m
        X = np.zeros((K, n)); U = z[:, L.U].copy()
        for k in range(K):
            X[k] = z[k, L.X] + (p["C"][k - 1] @ U[k] if k > 0 else 0.0)
        nu = z[:K - 1, L.N].copy()
        sigma = float(z[0, L.SIG])
        if p.get("x_final") is not None:
            k = K - 2
            nu[k] = p["x_final"] - (p["A"][k] @ X[k] + p["B"][k] @ U[k] + p["C"][k] @ U[k + 1] + p["S"][k] * sigma
                                    + p["z"][k])
        nobs = len(p.get("obs") or [])
        s_prime = np.array([[self.sig[k][o] for k in range(K)] for o in range(nobs)]).reshape(nobs, K)
        S = np.array([[self.sig[k][nobs + j] for k in range(K)] for j in range(len(p.get("nbrs") or []))])
        return dict(X=X, U=U, nu=nu, sigma=sigma, s_prime=s_prime, S=S.reshape(-1, K), status=status, iters=it,
                    g=z[0, L.G].copy())

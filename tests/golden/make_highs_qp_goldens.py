"""Generator of tests/golden/highs_qp_*.npz: Q1 trust-region subproblems solved by a THIRD-PARTY QP solver.

The reference solves each agent's subproblem of Distributed_opt/dist_scvx_3d.py:51-111 with CVXPY -> Clarabel
(:110), which is not installed here.  SciPy ships HiGHS (scipy.optimize._highspy, HiGHS 1.8),
whose QP solver is a primal active-set method for convex QPs -- an algorithm that shares nothing with the
interior-point methods of oracle/qp_dense.py, oracle/scvx_cpu.cpp and the HIP kernel.  This script

  1. builds C3-family (spheres, box, no SOC) and C4-shard-family (lattice, pairwise collision rows with the
     shared slack S_t) instances on the CPU (scvx_hip.workloads data construction, oracle/foh_oracle.py FOH),
  2. assembles each agent's problem HERE, independently of oracle/qp_dense.build_agent_problem, in ABSOLUTE
     variables (x_t, u_t, the L1 epigraph v_t of u_t - ubar_t, S_t, the obstacle slacks), straight from the
     reference's constraint list (dist_scvx_3d.py:72-107: cost sum ||u_t||^2 + w_coll sum S_t, x_0 = x_init,
     x_{T-1} = x_des, FOH dynamics, ||u_t - ubar_t||_1 <= tr, box, collision rows b - g'p_t <= S_t, S_t >= 0;
     sphere rows as single_integrator_model.py:113-126),
  3. solves it with HiGHS (tight feasibility tolerances, 5 s limit).  HiGHS 1.8's QP solver stops within its own
     tolerances (measured: objective a few 1e-9 relative above the optimum) and on some of these instances
     reports KKT failures or cycles, so its answer is not taken as is: the rows and bounds active at its point
     define an equality-constrained QP whose KKT system is solved exactly (sparse LU + refinement), and the
     result is kept only if it CERTIFIES as the optimum by the convex-QP KKT conditions, independently of any
     solver: primal feasible on every row and bound (<= 1e-12), stationary (<= 1e-14 relative), every
     inequality multiplier of the right sign (<= 1e-13 relative).  Such a point is the global optimum (KKT
     conditions are sufficient for a convex QP); HiGHS only supplied the active set,
  4. keeps instances with at least one ACTIVE box / obstacle / collision row at the optimum (the instances the
     all-inactive closed form of tests/test_independent_checks_cpu.py cannot pin) and stores the kernel-format
     inputs, the certified optimal value / trajectories and HiGHS's own (uncertified) value.

Consumers: tests/test_highs_qp_cpu.py (oracle/qp_dense.py and the CPU twin oracle/scvx_cpu.cpp against these) and
tests/test_highs_qp_gpu.py (the HIP kernel through the C-ABI against these).

    python tests/golden/make_highs_qp_goldens.py        # rewrites tests/golden/highs_qp_{c3,c4}.npz
"""
import os
import sys

import numpy as np
import scipy.sparse as sp

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "dynamic-programming-multiagent-trajectory-optimiziation_amd"))

from oracle import foh_oracle  # noqa: E402
from scvx_hip import workloads  # noqa: E402

K, N_X, N_U, PD = 50, 6, 3, 3
W_OBS, W_COLL = 1e6, 1e4


def assemble(disc, sigma, Xr, Ur, x_init, x_final, tr, box, obs, rows, cnt):
    """Sparse QP  min 1/2 z'Hz + c'z  s.t.  rl <= Az <= ru,  zl <= z <= zu  in absolute variables."""
    n, m = N_X, N_U
    o = np.cumsum([0, n * n, n * m, n * m, n, n])
    has_coll = rows is not None and cnt[:K - 1].sum() > 0
    nobs = len(obs)
    ix = lambda t, i: t * n + i                           # noqa: E731
    iu = lambda t, j: K * n + t * m + j                   # noqa: E731
    iv = lambda t, j: K * (n + m) + t * m + j             # noqa: E731
    base = K * (n + m) + (K - 1) * m
    iS = lambda t: base + t                               # noqa: E731
    base2 = base + (K - 1 if has_coll else 0)
    io = lambda t, k: base2 + t * nobs + k                # noqa: E731
    nv = base2 + (K - 1) * nobs
    cost = np.zeros(nv)
    hdiag = np.zeros(nv)
    for t in range(K - 1):                                # sum_{t<T-1} ||u_t||^2 (the last input is pinned)
        for j in range(m):
            hdiag[iu(t, j)] = 2.0
    if has_coll:
        cost[base:base + K - 1] = W_COLL
    if nobs:
        cost[base2:nv] = W_OBS
    zl, zu = np.full(nv, -np.inf), np.full(nv, np.inf)
    R, C, V, rl, ru, kind = [], [], [], [], [], []

    def row(coefs, lo, hi, kd):
        r = len(rl)
        for k, v in coefs:
            R.append(r); C.append(k); V.append(v)
        rl.append(lo); ru.append(hi); kind.append(kd)

    for i in range(n):
        zl[ix(0, i)] = zu[ix(0, i)] = x_init[i]
        zl[ix(K - 1, i)] = zu[ix(K - 1, i)] = x_final[i]
    for j in range(m):                                     # fix_last_input: w_{T-1} = 0
        zl[iu(K - 1, j)] = zu[iu(K - 1, j)] = Ur[K - 1, j]
    for t in range(K - 1):
        A = disc[t, o[0]:o[1]].reshape(n, n).T
        B = disc[t, o[1]:o[2]].reshape(m, n).T
        Cm = disc[t, o[2]:o[3]].reshape(m, n).T
        c = disc[t, o[3]:o[4]] * sigma + disc[t, o[4]:o[5]]
        for i in range(n):                                 # x_{t+1} - A x_t - B u_t - C u_{t+1} = c
            co = [(ix(t + 1, i), 1.0)] + [(ix(t, k), -A[i, k]) for k in range(n)]
            co += [(iu(t, j), -B[i, j]) for j in range(m)] + [(iu(t + 1, j), -Cm[i, j]) for j in range(m)]
            row(co, c[i], c[i], "dyn")
        for j in range(m):                                 # |u - ubar| <= v
            row([(iu(t, j), 1.0), (iv(t, j), -1.0)], -np.inf, Ur[t, j], "tr")
            row([(iu(t, j), -1.0), (iv(t, j), -1.0)], -np.inf, -Ur[t, j], "tr")
        row([(iv(t, j), 1.0) for j in range(m)], -np.inf, tr, "tr")
        for (bi, lo, hi) in box:
            row([(ix(t, bi), 1.0)], lo, hi, "box")
        if has_coll:
            zl[iS(t)] = 0.0
            for r in rows[t, :cnt[t]]:                     # b - g'p_t <= S_t
                row([(ix(t, i), -r[i]) for i in range(PD)] + [(iS(t), -1.0)], -np.inf, -r[PD], "coll")
        for k, (ctr, rad) in enumerate(obs):               # a'(p_t - ctr) >= rad - so, so >= 0
            diff = Xr[t, :PD] - np.asarray(ctr)
            a = diff / (np.linalg.norm(diff) + 1e-6)
            zl[io(t, k)] = 0.0
            row([(ix(t, i), a[i]) for i in range(PD)] + [(io(t, k), 1.0)], rad + a @ np.asarray(ctr), np.inf, "obs")
    A = sp.csc_matrix((V, (R, C)), shape=(len(rl), nv))
    return dict(hdiag=hdiag, cost=cost, A=A, rl=np.array(rl), ru=np.array(ru), kind=np.array(kind), zl=zl, zu=zu, nv=nv,
                iu=iu, ix=ix, iS=iS if has_coll else None, io=io, nobs=nobs, base=base, base2=base2)


def solve_highs(P):
    from scipy.optimize._highspy import _core as hc
    h = hc._Highs()
    h.setOptionValue("output_flag", False)
    for k in ("primal_feasibility_tolerance", "dual_feasibility_tolerance"):
        h.setOptionValue(k, 1e-10)
    lp = hc.HighsLp()
    lp.num_col_, lp.num_row_ = P["nv"], P["A"].shape[0]
    inf = hc.kHighsInf
    fix = lambda a: np.clip(a, -inf, inf)   # noqa: E731
    lp.col_cost_ = P["cost"]
    lp.col_lower_, lp.col_upper_ = fix(P["zl"]), fix(P["zu"])
    lp.row_lower_, lp.row_upper_ = fix(P["rl"]), fix(P["ru"])
    Am = P["A"]
    lp.a_matrix_.format_ = hc.MatrixFormat.kColwise
    lp.a_matrix_.num_col_, lp.a_matrix_.num_row_ = Am.shape[1], Am.shape[0]
    lp.a_matrix_.start_, lp.a_matrix_.index_, lp.a_matrix_.value_ = Am.indptr, Am.indices, Am.data
    assert h.passModel(lp) == hc.HighsStatus.kOk
    H = hc.HighsHessian()
    nz = np.nonzero(P["hdiag"])[0]
    H.dim_, H.format_ = P["nv"], hc.HessianFormat.kTriangular
    start = np.zeros(P["nv"] + 1, np.int32)
    start[nz + 1] = 1
    H.start_, H.index_, H.value_ = np.cumsum(start).astype(np.int32), nz.astype(np.int32), P["hdiag"][nz]
    assert h.passHessian(H) == hc.HighsStatus.kOk
    h.setOptionValue("time_limit", 5.0)
    h.run()
    ok = h.getModelStatus() == hc.HighsModelStatus.kOptimal
    z = np.array(h.getSolution().col_value)
    return ok, z, h.getInfo().objective_function_value


def certify(P, z, tol_act=1e-9):
    """Exact optimum on the active set of z, with its KKT certificate (see the module docstring, step 3)."""
    import scipy.sparse.linalg as sla
    A = P["A"].tocsr()
    rl, ru, zl, zu = P["rl"], P["ru"], P["zl"], P["zu"]
    h, c = P["hdiag"], P["cost"]

    def infeas(w):
        aw = A @ w
        return max(np.max(np.maximum(rl - aw, 0)), np.max(np.maximum(aw - ru, 0)),
                   np.max(np.maximum(zl - w, 0)), np.max(np.maximum(w - zu, 0)))

    az = A @ z
    near = lambda v, bd: np.isfinite(bd) & (np.abs(v - bd) <= tol_act * (1 + np.abs(bd)))   # noqa: E731
    lo_r, hi_r, lo_c, hi_c = near(az, rl), near(az, ru), near(z, zl), near(z, zu)
    ract, cact = np.nonzero(lo_r | hi_r)[0], np.nonzero(lo_c | hi_c)[0]
    b = np.concatenate([np.where(lo_r, rl, ru)[ract], np.where(lo_c, zl, zu)[cact]])
    E = sp.csr_matrix((np.ones(len(cact)), (np.arange(len(cact)), cact)), shape=(len(cact), len(z)))
    M = sp.vstack([A[ract], E]).tocsr()
    nv, na = len(z), M.shape[0]
    try:
        lu = sla.splu(sp.bmat([[sp.diags(h), -M.T], [M, None]]).tocsc())
    except RuntimeError:   # degenerate active set: a tiny regularisation, corrected by the refinement below
        lu = sla.splu(sp.bmat([[sp.diags(h + 1e-10), -M.T], [M, sp.eye(na) * 1e-10]]).tocsc())
    zz, lam = z.copy(), np.zeros(na)
    for _ in range(8):     # Newton on the linear KKT system (= iterative refinement)
        d = lu.solve(np.concatenate([-(h * zz + c - M.T @ lam), b - M @ zz]))
        zz, lam = zz + d[:nv], lam + d[nv:]
    lsc = 1 + np.abs(c).max()
    lr = np.concatenate([lo_r[ract] & ~hi_r[ract], lo_c[cact] & ~hi_c[cact]])
    ur = np.concatenate([hi_r[ract] & ~lo_r[ract], hi_c[cact] & ~lo_c[cact]])
    cert = dict(infeas=infeas(zz), stat=np.abs(h * zz + c - M.T @ lam).max() / lsc,
                sign=max(np.max(-lam[lr], initial=0), np.max(lam[ur], initial=0)) / lsc)
    ok = cert["infeas"] <= 1e-12 and cert["stat"] <= 1e-14 and cert["sign"] <= 1e-13
    return ok, zz, cert


def unpack(P, z, Ur):
    X = z[:K * N_X].reshape(K, N_X)
    U = z[K * N_X:K * (N_X + N_U)].reshape(K, N_U)
    S = z[P["base"]:P["base"] + K - 1] if P["iS"] is not None else np.zeros(K - 1)
    obj = np.sum(U[:K - 1] ** 2) + W_COLL * S.sum()
    if P["nobs"]:
        obj += W_OBS * z[P["base2"]:P["nv"]].sum()
    return X, U, S, obj


def n_active(P, z):
    """Active box / obstacle / collision rows at z (row within 1e-7 of a finite bound), per kind."""
    act = P["A"] @ z
    rl, ru = P["rl"], P["ru"]
    near = ((np.isfinite(rl) & (np.abs(act - rl) <= 1e-7 * (1 + np.abs(rl))))
            | (np.isfinite(ru) & (np.abs(act - ru) <= 1e-7 * (1 + np.abs(ru)))))
    return np.array([np.sum(near & (P["kind"] == k)) for k in ("box", "obs", "coll")])


def c3_family(n_agents=64, seed=5):
    """C3 family without the SOC: the bench's 8 spheres (workloads obs_seed 11), box |x|, |y| <= 7.  Each agent's
    straight reference path crosses a sphere (start and goal 4 m either side of its centre, 0.2-0.6 m off-axis).
    (Box rows: no certified instance of this family has one active -- starts moving towards a wall made HiGHS end
    infeasible or at its time limit; the box rows are pinned by the dense-oracle tests only.)"""
    rng = np.random.default_rng(seed)
    obs = workloads._obstacles(8, 11)
    box = [(0, -7.0, 7.0), (1, -7.0, 7.0)]
    out = []
    for _ in range(100 * n_agents):
        if len(out) == n_agents:
            break
        a = len(out)
        ctr, rad = obs[rng.integers(len(obs))]
        d = rng.normal(size=3)
        d /= np.linalg.norm(d)
        perp = np.cross(d, rng.normal(size=3))
        perp *= rng.uniform(0.2, 0.6) / np.linalg.norm(perp)
        p0, pf = ctr + 4 * d + perp, ctr - 4 * d + perp
        if np.abs(p0[:2]).max() > 6.5 or np.abs(pf[:2]).max() > 6.5:
            continue
        X = workloads._straight(p0[None], pf[None], K, N_X)[0]
        out.append(dict(X=X, U=np.zeros((K, N_U)), x_init=X[0].copy(), x_final=X[-1].copy(), sigma=30.0,
                        tr=(0.25, 0.1)[(a // 2) % 2], box=box, obs=obs, rows=None, cnt=None))
    return out


def c4_family(side=4, R=2.3, j_max=8, seed=2):
    sc = workloads.synthetic_lattice(side=side, K=K, seed=seed, sigma=30.0)
    N = sc["X"].shape[0]
    P = sc["X"][:, :, :PD]
    box = [(0, -50.0, 50.0), (1, -50.0, 50.0)]
    out = []
    for a in range(N):
        rows = np.zeros((K, j_max, 4))
        cnt = np.zeros(K, np.int32)
        for t in range(K - 1):
            d = np.linalg.norm(P[a, t] - P[:, t], axis=1)
            d[a] = np.inf
            near = [j for j in np.argsort(d)[:j_max] if d[j] < 4 * R]
            for k, j in enumerate(near):
                diff = P[a, t] - P[j, t]
                g = diff / d[j]
                rows[t, k, :PD] = g
                rows[t, k, PD] = 2 * R - d[j] + g @ P[a, t]
            cnt[t] = len(near)
        out.append(dict(X=sc["X"][a], U=sc["U"][a], x_init=sc["x_init"][a], x_final=sc["x_final"][a], sigma=30.0,
                        tr=(0.25, 0.125)[a % 2], box=box, obs=[], rows=rows, cnt=cnt))
    return out


def build(name, insts, want):
    keep = []
    tried = 0
    for inst in insts:
        tried += 1
        disc = foh_oracle.foh_disc("di", inst["X"], inst["U"], inst["sigma"])
        P = assemble(disc, inst["sigma"], inst["X"], inst["U"], inst["x_init"], inst["x_final"], inst["tr"],
                     inst["box"], inst["obs"], inst["rows"], inst["cnt"])
        _, zh, fval = solve_highs(P)
        if len(zh) != P["nv"] or not np.all(np.isfinite(zh)):
            continue
        ok, z, cert = certify(P, zh)
        if not ok:
            continue
        na = n_active(P, z)
        X, U, S, obj = unpack(P, z, inst["U"])
        fh = unpack(P, zh, inst["U"])[3]
        assert abs(obj - (0.5 * P["hdiag"] @ z ** 2 + P["cost"] @ z)) <= 1e-9 * max(1, abs(obj))
        if na.sum() == 0:
            continue
        keep.append((inst, disc, X, U, S, obj, na, fh))
        if len(keep) == want:
            break
    print(name, "kept", len(keep), "of", tried, "active box / obs / coll rows per instance:", [tuple(int(v) for v in k[6]) for k in keep])
    st = lambda f: np.stack([f(k) for k in keep])   # noqa: E731
    inst0 = keep[0][0]
    obs = inst0["obs"]
    rows = st(lambda k: k[0]["rows"]) if inst0["rows"] is not None else np.zeros((len(keep), K, 1, 4))
    cnt = st(lambda k: k[0]["cnt"]) if inst0["cnt"] is not None else np.zeros((len(keep), K), np.int32)
    np.savez_compressed(
        os.path.join(HERE, f"highs_qp_{name}.npz"),
        disc=st(lambda k: k[1]), sigma=st(lambda k: k[0]["sigma"]), Xref=st(lambda k: k[0]["X"]),
        Uref=st(lambda k: k[0]["U"]), x_init=st(lambda k: k[0]["x_init"]), x_final=st(lambda k: k[0]["x_final"]),
        tr=st(lambda k: k[0]["tr"]), rows=rows, cnt=cnt.astype(np.int32),
        box=np.array(inst0["box"], np.float64), obs_c=np.array([c for c, r in obs], np.float64).reshape(-1, 3),
        obs_r=np.array([r for c, r in obs], np.float64), j_max=np.int32(rows.shape[2] if inst0["rows"] is not None
                                                                           else 0),
        X=st(lambda k: k[2]), U=st(lambda k: k[3]), S=st(lambda k: k[4]), obj=st(lambda k: k[5]),
        n_active=st(lambda k: k[6]), obj_highs=st(lambda k: k[7]), solver=np.array("HiGHS %s active-set QP (scipy.optimize._highspy) + exact KKT solve on its active set, certified" % ver()))


def ver():
    from scipy.optimize._highspy import _core as hc
    return "%d.%d.%d" % (hc.HIGHS_VERSION_MAJOR, hc.HIGHS_VERSION_MINOR, hc.HIGHS_VERSION_PATCH)


if __name__ == "__main__":
    build("c3", c3_family(), 24)
    build("c4", c4_family(), 24)

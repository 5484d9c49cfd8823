"""GPU parity of the coupled configurations and of the exactness machinery of the
culled coupling:

  * C4: a 512-agent shard (rank 0 of 8) of the 4096-agent lattice construction
    (scvx_hip.workloads.synthetic_lattice), j_max = 8 nearest rows per node, checked agent by agent
    against the dense reference-formulation oracle (oracle/qp_dense.py: dist_scvx_3d.py:51-111 as
    written) on the same rows, and against the full reference row set (all 4095 neighbours) through
    the a-posteriori check;
  * C5: 64 quadrotors (scvx_hip.workloads.synthetic_quad) with 8 spheres and coupling R = 0.5;
  * culled + check == all rows: a dense 33-agent cluster where j_max = 32 keeps every neighbour;
  * status honesty: an iterate that hits the iteration cap far from optimal is a failure (status 2).

The IPM stops at Clarabel's default tolerances (1e-8, normalised as Clarabel does), the solver
dist_scvx_3d.py:110 calls.  A solve that ends at Clarabel's reduced tolerances (status 1,
"optimal_inaccurate": the Newton system loses accuracy at extreme barrier scalings on a few degenerate
instances, where the dense oracle needs its full iteration budget too) is checked for feasibility at the
reduced tolerance.  Tolerances (float64): objective 1e-7 relative, constraint violation 1e-7 (status 0)
or 1e-5 (status 1), trajectories 1e-8 (culled + check vs all rows: the same problem solved twice)."""
import numpy as np
import pytest

import scvx_hip
from oracle import problems as pb, qp_dense as qd

pytestmark = pytest.mark.gpu


def _t(x, cuda, dtype=None):
    import torch
    return torch.tensor(np.ascontiguousarray(x), device=cuda, dtype=dtype or torch.float64)


def _dense_prob(model, disc_a, sigma_a, Xref, Uref, x_final, tr, rows_a, cnt_a, box, obs, pd=3):
    n, m = scvx_hip.MODEL_DIMS[model]
    A, B, C, S, z = pb.unpack_disc(disc_a, n, m)
    coll = None
    if rows_a is not None:
        coll = []
        for t in range(Xref.shape[0] - 1):
            r = rows_a[t, :cnt_a[t]]
            c = r[:, pd] - r[:, :pd] @ Xref[t, :pd]
            coll.append(np.hstack([r[:, :pd], c[:, None]]))
    return dict(A=A, B=B, C=C, c=S * sigma_a + z, Xref=Xref, Uref=Uref, x_final=x_final, tr=tr, box=box, obs=obs,
                w_obs=1e6, coll=coll, w_coll=1e4, umax=None, fix_last_input=True, pos_dim=pd)


def _check_inaccurate(model, agents, out, dn, sig, X, U, xf, tr, rows, cnt, box, obs):
    """status-1 solves: feasible to Clarabel's reduced tolerance (1e-4 relative; 1e-5 absolute asked here)."""
    Xg, Ug, Sg = (out[k].cpu().numpy() for k in ("X", "U", "slack_coll"))
    for a in agents:
        prob = _dense_prob(model, dn[a], sig[a], X[a], U[a], xf[a], tr[a], rows[a], cnt[a], box, obs)
        viol = qd.constraint_violation(prob, Xg[a], Ug[a], Sg[a])
        assert max(viol.values()) < 1e-5, (a, viol)


def _check_against_dense(model, agents, out, dn, sig, X, U, xf, tr, rows, cnt, box, obs, tol_obj=1e-7, want=None):
    """Agent by agent against the dense oracle; an agent the oracle itself cannot certify within its
    iteration budget (degenerate instances) is skipped, and `want` (default: all) must be checked."""
    Xg, Ug, Sg, og = (out[k].cpu().numpy() for k in ("X", "U", "slack_coll", "obj"))
    checked = 0
    for a in agents:
        prob = _dense_prob(model, dn[a], sig[a], X[a], U[a], xf[a], tr[a], rows[a], cnt[a], box, obs)
        with np.errstate(all="ignore"):
            Xd, Ud, objd, info = qd.solve_agent(prob, tol=1e-10, maxit=150)
        if info["status"] != "optimal":
            continue
        assert abs(og[a] - objd) <= tol_obj * max(1.0, abs(objd)), (a, og[a], objd)
        viol = qd.constraint_violation(prob, Xg[a], Ug[a], Sg[a])
        assert max(viol.values()) < 1e-7, (a, viol)
        checked += 1
        if want is not None and checked >= want:
            break
    assert checked >= (len(agents) if want is None else want), (checked, len(agents))


def test_c4_lattice_shard_matches_dense_and_full_rows(cuda):
    """Rank 0's 512 agents of C4 at the first Jacobi iteration: FOH -> culled rows (j_max 8) -> QP."""
    import torch
    from scvx_hip import workloads
    sc = workloads.synthetic_lattice(side=16, K=50, seed=2, sigma=30.0)
    n_loc, K = 512, 50
    X_all = _t(sc["X"], cuda)
    sl = slice(0, n_loc)
    X, U, sig = _t(sc["X"][sl], cuda), _t(sc["U"][sl], cuda), _t(sc["sigma"][sl], cuda)
    disc = scvx_hip.foh_batched("di", X, U, sig)
    rows, cnt = scvx_hip.collision_rows(X_all, 0, n_loc, 2.3, j_max=8)
    box = [(0, -50.0, 50.0), (1, -50.0, 50.0)]
    spec = scvx_hip.QPSpec(model="di", K=K, box=box, j_max=8, w_coll=1e4, tol=1e-8, max_iter=60)
    tr = np.full(n_loc, 0.25)
    out = scvx_hip.qp_solve_batched(spec, disc, sig, X, U, _t(sc["x_init"][sl], cuda), _t(sc["x_final"][sl], cuda),
                                    _t(tr, cuda), rows, cnt)
    st, it = out["status"].cpu().numpy(), out["iters"].cpu().numpy()
    assert (st == 0).mean() >= 0.97 and (st != 2).all(), np.bincount(st, minlength=3)
    assert (it > 0).all()
    rng = np.random.default_rng(0)
    sample = rng.choice(np.nonzero(st == 0)[0], 8, replace=False)
    args = (out, disc.cpu().numpy(), sc["sigma"][sl], sc["X"][sl], sc["U"][sl], sc["x_final"][sl], tr,
            rows.cpu().numpy(), cnt.cpu().numpy(), box, [])
    _check_against_dense("di", sample, *args, want=3)
    _check_inaccurate("di", np.nonzero(st == 1)[0], *args)
    # every one of the 4095 reference rows per node at the culled solution
    viol, vmax = scvx_hip.collision_check(X_all, 0, out["X"], out["slack_coll"], 2.3, tol=1e-7)
    viol, vmax = viol.cpu().numpy(), vmax.cpu().numpy()
    ok = viol.sum(1) == 0
    # where no dropped row binds, the culled solution satisfies the full reference problem: a
    # relaxation whose optimum is feasible for the full problem is its optimum
    a = int(np.nonzero(ok & (st == 0))[0][0])
    Xg, Sg = out["X"].cpu().numpy()[a], out["slack_coll"].cpu().numpy()[a]
    d = Xg - sc["X"][a]
    for t in range(K - 1):
        diff = sc["X"][a, t, :3] - sc["X"][:, t, :3]
        nr = np.linalg.norm(diff, axis=1)
        nr[a] = np.inf
        v = (4.6 - nr) - (diff @ d[t, :3]) / nr - Sg[t]
        assert v.max() <= 1e-7
        assert abs(v.max() - vmax[a, t]) < 1e-9


def test_c5_quadrotors_n64(cuda):
    """C5 construction at N = 64: every subproblem solves (no exit at 0 iterations), sampled agents
    match the dense oracle on the same rows; three coupled SCvx iterations stay healthy."""
    import torch
    from scvx_hip import workloads
    from scvx_hip.scvx import CouplingSpec, JacobiSCvx
    N, K = 64, 50
    sc = workloads.synthetic_quad(N, K=K, seed=3, obstacles=8)
    X, U, sig = _t(sc["X"], cuda), _t(sc["U"], cuda), _t(sc["sigma"], cuda)
    disc = scvx_hip.foh_batched("quad", X, U, sig)
    rows, cnt = scvx_hip.collision_rows(X, 0, N, 0.5, j_max=8)
    box = workloads.QUAD_BOX
    spec = scvx_hip.QPSpec(model="quad", K=K, box=box, obs=sc["obs"], w_obs=1e6, j_max=8, w_coll=1e4, tol=1e-8,
                           max_iter=60)
    tr = np.full(N, 0.25)
    out = scvx_hip.qp_solve_batched(spec, disc, sig, X, U, _t(sc["x_init"], cuda), _t(sc["x_final"], cuda),
                                    _t(tr, cuda), rows, cnt)
    st, it = out["status"].cpu().numpy(), out["iters"].cpu().numpy()
    assert (st != 2).all() and (st == 0).mean() >= 0.95 and (it > 0).all(), (np.bincount(st, minlength=3), it.min())
    rng = np.random.default_rng(1)
    sample = rng.choice(np.nonzero(st == 0)[0], 2, replace=False)
    args = (out, disc.cpu().numpy(), sc["sigma"], sc["X"], sc["U"], sc["x_final"], tr, rows.cpu().numpy(),
            cnt.cpu().numpy(), box, sc["obs"])
    _check_against_dense("quad", sample, *args, tol_obj=1e-6)
    _check_inaccurate("quad", np.nonzero(st == 1)[0], *args)
    drv = JacobiSCvx(spec, _t(sc["x_init"], cuda), _t(sc["x_final"], cuda), sig, 0.25,
                     coupling=CouplingSpec(R=0.5), tr_rule="global")
    Xc, Uc = X.clone(), U.clone()
    for k in range(3):
        Xp, Up, trp = Xc.clone(), Uc.clone(), drv.tr.clone()
        Xc, Uc, o = drv.step(Xc, Uc)
        s = o["status"].cpu().numpy()
        assert (o["iters"].cpu().numpy() > 0).all()
        # a failed subproblem (the Q1 form has no virtual control: with a nonlinear model and a fixed
        # x_final the linearisation can be infeasible inside the trust region) must be one the dense
        # oracle cannot solve either; the driver rejects its step
        for a in np.nonzero(s == 2)[0][:2]:
            rr, cc = drv.rows[a].cpu().numpy(), drv.count[a].cpu().numpy()
            prob = _dense_prob("quad", drv.disc[a].cpu().numpy(), sc["sigma"][a], Xp[a].cpu().numpy(),
                               Up[a].cpu().numpy(), sc["x_final"][a], trp[a].item(), rr, cc, box, sc["obs"])
            with np.errstate(all="ignore"):
                _, _, _, info = qd.solve_agent(prob, tol=1e-9, maxit=150)
            assert info["status"] != "optimal", (k, a, info["status"])
        assert (s != 2).mean() >= 0.9, np.bincount(s, minlength=3)
    assert torch.isfinite(Xc).all()


def _cluster(N=33, K=30, seed=5):
    """N double integrators crossing a small region: every pair comes within 2R somewhere."""
    rng = np.random.default_rng(seed)
    ang = rng.uniform(0, 2 * np.pi, N)
    el = rng.uniform(-0.5, 0.5, N)
    dirs = np.stack([np.cos(ang) * np.cos(el), np.sin(ang) * np.cos(el), np.sin(el)], 1)
    p0 = 6.0 * dirs + rng.normal(0, 0.3, (N, 3))
    pf = -6.0 * dirs + rng.normal(0, 0.3, (N, 3))
    a = np.linspace(0, 1, K)[None, :, None]
    X = np.zeros((N, K, 6))
    X[:, :, :3] = p0[:, None] * (1 - a) + pf[:, None] * a
    return X, np.zeros((N, K, 3))


def test_culled_plus_check_equals_all_rows(cuda):
    """33 agents, every neighbour within reach: j_max = 8 + full-row check + re-solve with 32 rows
    gives the j_max = 32 (= all N-1 neighbours, the reference's row set) result."""
    import torch
    from scvx_hip.scvx import CouplingSpec, JacobiSCvx
    N, K = 33, 30
    Xn, Un = _cluster(N, K)
    X, U = _t(Xn, cuda), _t(Un, cuda)
    sig = _t(np.full(N, 20.0), cuda)
    xi, xf = _t(Xn[:, 0], cuda), _t(Xn[:, -1], cuda)
    box = [(0, -20.0, 20.0), (1, -20.0, 20.0)]
    res = {}
    for name, jm, check in (("full", 32, False), ("culled", 8, True), ("raw", 8, False)):
        spec = scvx_hip.QPSpec(model="di", K=K, box=box, j_max=jm, w_coll=1e4, tol=1e-9, max_iter=80)
        drv = JacobiSCvx(spec, xi, xf, sig, 0.5, coupling=CouplingSpec(R=1.0, check=check), tr_rule="global")
        Xo, Uo, o = drv.step(X, U)
        res[name] = (Xo.cpu().numpy(), o["status"].cpu().numpy(), drv.last_check)
    sf, sc_ = res["full"][1], res["culled"][1]
    assert (sf != 2).all() and (sc_ != 2).all() and (sf == 0).mean() >= 0.85, (sf, sc_)
    chk = res["culled"][2]
    assert chk["violated"] > 0 and chk["overflow"] == 0, chk      # the check found culled rows that bind
    # the agents the full-row check flags in the raw (culled, no re-solve) run
    sc = scvx_hip.QPSpec(model="di", K=K, box=box, j_max=8, w_coll=1e4, tol=1e-9, max_iter=80)
    drv = JacobiSCvx(sc, xi, xf, sig, 0.5, coupling=CouplingSpec(R=1.0, check=False), tr_rule="global")
    Xo, Uo, o = drv.step(X, U)
    viol, _ = scvx_hip.collision_check(X, 0, o["X"], o["slack_coll"], 1.0, tol=1e-7)
    flagged = viol.sum(1).cpu().numpy() > 0
    assert flagged.sum() == chk["violated"]
    # flagged agents are re-solved with the 32 nearest rows = every neighbour: the same inputs as the
    # full run, so the same bits.  The others solved the 8-row relaxation, whose optimum satisfies every
    # dropped row and is therefore the full problem's optimum: equal to the IPM's accuracy at tol 1e-9
    # (two different row sets, so not bitwise; trajectories agree to ~1e-6)
    np.testing.assert_array_equal(res["culled"][0][flagged], res["full"][0][flagged])
    np.testing.assert_allclose(res["culled"][0][~flagged], res["full"][0][~flagged], rtol=0, atol=1e-5)
    # without the re-solve, the flagged agents are exactly those that differ from the all-rows answer
    diff = np.abs(res["raw"][0] - res["full"][0]).max(axis=(1, 2))
    assert (diff[~flagged] < 1e-5).all() and (diff[flagged] > 1e-4).all(), (diff, flagged)


def test_iteration_cap_far_from_optimum_is_a_failure(cuda):
    """An IPM stopped by max_iter far from the optimum reports status 2 (solver_error), never
    'optimal_inaccurate' (status 1): status 1 requires the reduced tolerances of ECOS / Clarabel."""
    N, K = 16, 50
    sc = pb.synthetic_di(N, K=K, seed=1, obstacles=8)
    X, U, sig = _t(sc["X"], cuda), _t(sc["U"], cuda), _t(sc["sigma"], cuda)
    disc = scvx_hip.foh_batched("di", X, U, sig)
    box = [(0, -12, 12), (1, -12, 12)]
    args = (disc, sig, X, U, _t(sc["x_init"], cuda), _t(sc["x_final"], cuda), _t(np.full(N, 0.25), cuda))
    capped = scvx_hip.qp_solve_batched(scvx_hip.QPSpec(model="di", K=K, box=box, obs=sc["obs"], u_max=1.0,
                                                       max_iter=3), *args)
    assert (capped["status"].cpu().numpy() == 2).all()
    assert (capped["iters"].cpu().numpy() == 3).all()
    full = scvx_hip.qp_solve_batched(scvx_hip.QPSpec(model="di", K=K, box=box, obs=sc["obs"], u_max=1.0,
                                                     max_iter=60), *args)
    assert (full["status"].cpu().numpy() == 0).all()


def test_collision_check_kernel_exact_on_every_row(cuda):
    """scvx_collision_check_batched against numpy on every (agent, node): the violation count and the
    largest row value, with clustered agents (rows near the threshold), far agents (skipped by the
    kernel's distance bound) and one coincident pair (NaN, as the reference's 0/0)."""
    import torch
    rng = np.random.default_rng(7)
    N, K, R, tol = 300, 8, 0.5, 1e-7
    X_all = np.zeros((N, K, 6))
    X_all[:, :, :3] = rng.normal(scale=3.0, size=(N, K, 3))
    X_all[:40, :, :3] = rng.normal(scale=0.4, size=(40, K, 3))   # a dense cluster
    X_all[41, 3, :3] = X_all[40, 3, :3]                          # coincident at node 3
    X_new = X_all + rng.normal(scale=0.2, size=X_all.shape)
    S = np.abs(rng.normal(scale=0.3, size=(N, K)))
    viol, vmax = scvx_hip.collision_check(_t(X_all, cuda), 0, _t(X_new, cuda), _t(S, cuda), R, tol=tol)
    viol, vmax = viol.cpu().numpy(), vmax.cpu().numpy()
    with np.errstate(all="ignore"):
        for a in range(N):
            for t in range(K - 1):
                diff = X_all[a, t, :3] - np.delete(X_all[:, t, :3], a, axis=0)
                nr = np.linalg.norm(diff, axis=1)
                v = (2 * R - nr) - diff @ (X_new[a, t, :3] - X_all[a, t, :3]) / nr - S[a, t]
                assert viol[a, t] == int(np.sum((v > tol) | np.isnan(v))), (a, t)
                if np.isnan(v).any():
                    assert np.isnan(vmax[a, t]), (a, t)
                else:
                    assert abs(vmax[a, t] - v.max()) <= 1e-12 * max(1.0, abs(v.max())), (a, t, vmax[a, t], v.max())
            assert viol[a, K - 1] == 0


@pytest.mark.parametrize("j_max", [8, 16])
def test_collision_rows_keep_the_nearest_neighbours(cuda, j_max):
    """scvx_collision_rows_batched's culled selection against numpy on every (agent, node): the j_max
    rows of the nearest neighbours (dist_scvx_3d.py:93-107 rows, compared as sets), for 200 local
    agents of 300 (a dense cluster and a sparse cloud, so the wave-local bound is tight for some
    waves and loose for others)."""
    rng = np.random.default_rng(11)
    N, K, R, i0, n_loc = 300, 6, 0.5, 50, 200
    X_all = np.zeros((N, K, 6))
    X_all[:, :, :3] = rng.normal(scale=4.0, size=(N, K, 3))
    X_all[60:140, :, :3] = rng.normal(scale=0.5, size=(80, K, 3))
    rows, cnt = scvx_hip.collision_rows(_t(X_all, cuda), i0, n_loc, R, j_max=j_max)
    rows, cnt = rows.cpu().numpy(), cnt.cpu().numpy()
    for a in range(n_loc):
        gi = i0 + a
        for t in range(K - 1):
            assert cnt[a, t] == j_max
            diff = X_all[gi, t, :3] - X_all[:, t, :3]
            nr = np.linalg.norm(diff, axis=1)
            nr[gi] = np.inf
            near = np.argsort(nr, kind="stable")[:j_max]
            g = diff[near] / nr[near, None]
            ref = np.hstack([g, (2 * R - nr[near] + g @ X_all[gi, t, :3])[:, None]])
            got = rows[a, t, :j_max]
            np.testing.assert_allclose(got[np.lexsort(got.T)], ref[np.lexsort(ref.T)], rtol=1e-12, atol=1e-12)
        assert cnt[a, K - 1] == 0


def test_indexed_rows_and_partial_solve_match_the_full_launch(cuda):
    """The re-solve path of the full-row check (scvx_hip/scvx.py JacobiSCvx._enforce_all_rows): rows of an
    arbitrary subset of agents (scvx_collision_rows_indexed) equal, as sets, the rows the contiguous launch
    gives those agents; a QPSolver sized for N solving only its first n agents (QPSolver.solve(n=...)) gives
    bit-identical results to a solver sized for n."""
    import torch
    rng = np.random.default_rng(12)
    N, K, R = 300, 6, 0.5
    X_all = np.zeros((N, K, 6))
    X_all[:, :, :3] = rng.normal(scale=2.0, size=(N, K, 3))
    Xt = _t(X_all, cuda)
    full, cfull = scvx_hip.collision_rows(Xt, 0, N, R, j_max=16)
    idx = np.sort(rng.choice(N, 40, replace=False)).astype(np.int32)
    rows = torch.zeros((64, K, 16, 4), dtype=torch.float64, device=cuda)     # larger buffer: leading 40 written
    cnt = torch.zeros((64, K), dtype=torch.int32, device=cuda)
    scvx_hip.collision_rows_indexed(Xt, torch.tensor(idx, device=cuda), R, 16, rows=rows, count=cnt)
    full, cfull, rows, cnt = full.cpu().numpy(), cfull.cpu().numpy(), rows.cpu().numpy(), cnt.cpu().numpy()
    for a, gi in enumerate(idx):
        np.testing.assert_array_equal(cnt[a], cfull[gi])
        for t in range(K - 1):
            got, ref = rows[a, t, :cnt[a, t]], full[gi, t, :cfull[gi, t]]
            np.testing.assert_array_equal(got[np.lexsort(got.T)], ref[np.lexsort(ref.T)])
    # partial solve
    from scvx_hip import workloads
    sc = workloads.synthetic_di(48, K=50, seed=2, obstacles=8)
    X, U, sig = _t(sc["X"], cuda), _t(sc["U"], cuda), _t(sc["sigma"], cuda)
    disc = scvx_hip.foh_batched("di", X, U, sig)
    spec = scvx_hip.QPSpec(model="di", K=50, box=[(0, -12, 12), (1, -12, 12)], obs=sc["obs"], w_obs=1e6, u_max=1.0)
    n = 17
    ins = [disc, sig, X, U, _t(sc["x_init"], cuda), _t(sc["x_final"], cuda), _t(np.full(48, 0.25), cuda)]
    big = scvx_hip.QPSolver(spec, 48, device=cuda).solve(*[v[:n].contiguous() for v in ins], n=n)
    small = scvx_hip.QPSolver(spec, n, device=cuda).solve(*[v[:n].contiguous() for v in ins])
    for k in ("X", "U", "obj", "status", "iters"):
        assert torch.equal(big[k], small[k]), k

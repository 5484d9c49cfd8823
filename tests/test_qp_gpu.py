"""GPU parity: the HIP batched trust-region solve (scvx_qp_solve_batched through the C-ABI)
against the dense reference-formulation oracle (oracle/qp_dense.py: dist_scvx_3d.py:51-111 as
written, generic dense IPM + KKT certificate) and the CPU restatement (oracle/scvx_cpu.cpp).

Tolerances (float64): trajectories 1e-6 absolute, objective 1e-8 relative, feasibility 1e-8."""
import numpy as np
import pytest

import scvx_hip
from oracle import foh_oracle, problems as pb, qp_cpu, qp_dense as qd

pytestmark = pytest.mark.gpu


def _t(x, cuda, dtype=None):
    import torch
    return torch.tensor(np.ascontiguousarray(x), device=cuda, dtype=dtype or torch.float64)


def _kernel_pnorm(X, U, S, Xref, Uref, x_init, x_final, tr, box, rows, cnt, c_dyn=0.0):
    """The kernel's primal normalisation max(1, ||b|| + ||x|| + ||s||) (qp_ipm.hpp residual phase: Clarabel's relative
    primal test, inf-norms over every constant, variable and slack of its formulation) evaluated at a returned
    solution: b = x_init, x_final, the dynamics constants, every row's right-hand side (trust-region facets
    tr + s'ubar, box bounds, collision rows -b); x = (X, U, the shared collision slack S); s = every row's slack
    (facets tr - s'(u - ubar) at most tr + ||u - ubar||_1, box hi - x / x - lo, collision rows -b + g'p + S, the
    slack's sign row S).  Inequality rows live on nodes t < K-1 (ineq_last = 0)."""
    K = X.shape[0]
    nb = max(np.abs(x_init).max(), np.abs(x_final).max(), float(np.max(np.abs(c_dyn))))
    nb = max(nb, tr + np.abs(Uref[:K - 1]).sum(axis=1).max(), max(max(abs(lo), abs(hi)) for _, lo, hi in box))
    nx = max(np.abs(X).max(), np.abs(U).max(), np.abs(S).max())
    ns = (tr + np.abs(U[:K - 1] - Uref[:K - 1]).sum(axis=1)).max()
    for b, lo, hi in box:
        ns = max(ns, (hi - X[:K - 1, b]).max(), (X[:K - 1, b] - lo).max())
    ns = max(ns, np.abs(S[:K - 1]).max())
    for t in range(K - 1):
        for j in range(cnt[t]):
            g, bb = rows[t, j, :3], rows[t, j, 3]
            nb = max(nb, abs(bb))
            ns = max(ns, -bb + g @ X[t, :3] + S[t])
    return max(1.0, nb + nx + ns)


def test_dist_scvx_3d_first_iteration_matches_dense_oracle(cuda):
    sc = pb.dist3_scenario()
    T = sc["T"]
    A = np.repeat(sc["Ad"][None], T - 1, 0)
    B = np.repeat(sc["Bd"][None], T - 1, 0)
    disc = np.stack([pb.pack_disc(A, B)] * 3)
    Xref = np.stack([x[:, 0:6] for x in sc["X_traj"]])
    Uref = np.stack([x[:, 6:9] for x in sc["X_traj"]])
    xdes = np.stack([x[0:6] for x in sc["x_des"]])
    J = 2
    rows = np.zeros((3, T, J, 4))
    cnt = np.zeros((3, T), np.int32)
    dense_rows = [pb.collision_rows(sc["X_traj"], i, sc["R"]) for i in range(3)]
    for i in range(3):
        for t in range(T - 1):
            rows[i, t] = dense_rows[i][t]
            cnt[i, t] = 2
    box = [(0, -1, 22), (1, -1, 20)]
    spec = scvx_hip.QPSpec(model="di", K=T, box=box, j_max=J, w_coll=1e4, tol=1e-9, max_iter=80)
    import torch
    out = scvx_hip.qp_solve_batched(spec, _t(disc, cuda), _t(np.zeros(3), cuda), _t(Xref, cuda), _t(Uref, cuda),
                                    _t(Xref[:, 0], cuda), _t(xdes, cuda), _t(np.full(3, sc["tr"]), cuda),
                                    _t(rows, cuda), _t(cnt, cuda, torch.int32))
    st = out["status"].cpu().numpy()
    assert (st == 0).all(), st
    for i in range(3):
        prob = pb.dense_prob_from_rows(A, B, Xref[i], Uref[i], xdes[i], sc["tr"], dense_rows[i], box=box,
                                       w_coll=1e4, fix_last_input=True)
        Xd, Ud, objd, info = qd.solve_agent(prob, tol=1e-11, maxit=120)
        assert info["status"] == "optimal"
        X = out["X"][i].cpu().numpy()
        U = out["U"][i].cpu().numpy()
        S = out["slack_coll"][i].cpu().numpy()
        viol = qd.constraint_violation(prob, X, U, S)
        # Clarabel's primal test is relative: tol (1e-9) x (||b|| + ||x|| + ||s||) of the kernel's own formulation
        # (_kernel_pnorm at this solution: ~66 here, positions and box bounds ~22, box slacks ~23); the reference-form
        # violation of a row is at most its residual in the kernel's form, plus the rounding of d = X - Xref
        bound = spec.tol * _kernel_pnorm(X, U, S, Xref[i], Uref[i], Xref[i, 0], xdes[i], sc["tr"], box, rows[i],
                                         cnt[i]) + 1e-14 * max(1.0, np.abs(X).max())
        assert max(viol.values()) <= bound, (viol, bound)
        obj = out["obj"][i].item()
        assert abs(obj - objd) <= 1e-8 * max(1.0, abs(objd))
        if objd < 1e3:  # slack-free agents: the quadratic part pins the trajectory
            assert np.abs(X - Xd).max() < 1e-6
            assert np.abs(U - Ud).max() < 1e-6


@pytest.mark.parametrize("umax,nobs", [(None, 0), (1.0, 8), (0.12, 8)])
def test_c3_family_matches_cpu_and_dense(cuda, umax, nobs):
    N, K = 12, 50
    sc = pb.synthetic_di(N, K=K, seed=1, obstacles=nobs)
    import torch
    X, U, sig = _t(sc["X"], cuda), _t(sc["U"], cuda), _t(sc["sigma"], cuda)
    disc = scvx_hip.foh_batched("di", X, U, sig)
    box = [(0, -12, 12), (1, -12, 12)]
    spec = scvx_hip.QPSpec(model="di", K=K, box=box, obs=sc["obs"], w_obs=1e6, u_max=umax, tol=1e-10, max_iter=80)
    tr = np.full(N, 0.25)
    out = scvx_hip.qp_solve_batched(spec, disc, sig, X, U, _t(sc["x_init"], cuda), _t(sc["x_final"], cuda), _t(tr, cuda))
    tpl = qp_cpu.make_template(6, 3, K, box=box, obs=sc["obs"], w_obs=1e6, u_max=umax, tol=1e-10, max_iter=80)
    dn = disc.cpu().numpy()
    cpu = qp_cpu.solve_batched(tpl, dn, sc["sigma"], sc["X"], sc["U"], sc["x_init"], sc["x_final"], tr)
    st = out["status"].cpu().numpy()
    ok = cpu["status"] == 0
    assert ok.all(), cpu["status"]  # every agent of the family solves (tests/test_qp_twin_cpu.py: twin == dense)
    assert (st == 0).all(), st
    Xg, Ug, og = out["X"].cpu().numpy(), out["U"].cpu().numpy(), out["obj"].cpu().numpy()
    for a in np.nonzero(ok)[0]:
        assert abs(og[a] - cpu["obj"][a]) <= 1e-8 * max(1.0, abs(cpu["obj"][a]))
        assert np.abs(Xg[a] - cpu["X"][a]).max() < 1e-6
        assert np.abs(Ug[a] - cpu["U"][a]).max() < 1e-6
    for a in range(N):   # every agent against the reference form (sparse KKT path of the dense oracle)
        A, B, C, S, z = pb.unpack_disc(dn[a], 6, 3)
        prob = dict(A=A, B=B, C=C, c=S * sc["sigma"][a] + z, Xref=sc["X"][a], Uref=sc["U"][a],
                    x_final=sc["x_final"][a], tr=0.25, box=box, obs=sc["obs"], w_obs=1e6, umax=umax,
                    fix_last_input=True)
        with np.errstate(all="ignore"):
            Xd, Ud, objd, info = qd.solve_agent(prob, sparse=True, tol=1e-10)
        assert info["status"] == "optimal", (a, info["status"])
        assert abs(og[a] - objd) <= 1e-8 * max(1.0, abs(objd)), (a, og[a], objd)
        viol = qd.constraint_violation(prob, Xg[a], Ug[a])
        assert max(viol.values()) < 1e-7, viol


@pytest.mark.parametrize("umax", [1.0, 0.12])
def test_c3_bench_construction_sample_matches_dense_oracle(cuda, umax):
    """The headline workload itself (bench.py C3: workloads.synthetic_di(1024, seed=1), 8 spheres, SOC, box
    |x|,|y| <= 12, tr 0.25, the bench's tolerance 1e-8) solved for all 1024 agents in one launch; 16 agents
    (every 64th) checked against the reference-form oracle, each one of them (no sampling escape), plus
    the tight u_max = 0.12 variant (the longest IPM runs).  Objective 1e-8 relative, feasibility 1e-7."""
    from scvx_hip import workloads
    N, K = 1024, 50
    sc = workloads.synthetic_di(N, K=K, seed=1, obstacles=8)
    X, U, sig = _t(sc["X"], cuda), _t(sc["U"], cuda), _t(sc["sigma"], cuda)
    disc = scvx_hip.foh_batched("di", X, U, sig)
    box = [(0, -12, 12), (1, -12, 12)]
    spec = scvx_hip.QPSpec(model="di", K=K, box=box, obs=sc["obs"], w_obs=1e6, u_max=umax, tol=1e-8, max_iter=60)
    out = scvx_hip.qp_solve_batched(spec, disc, sig, X, U, _t(sc["x_init"], cuda), _t(sc["x_final"], cuda),
                                    _t(np.full(N, 0.25), cuda))
    st = out["status"].cpu().numpy()
    dn = disc.cpu().numpy()
    Xg, Ug, og = out["X"].cpu().numpy(), out["U"].cpu().numpy(), out["obj"].cpu().numpy()

    def dense(a, maxit=150):
        A, B, C, S, z = pb.unpack_disc(dn[a], 6, 3)
        prob = dict(A=A, B=B, C=C, c=S * sc["sigma"][a] + z, Xref=sc["X"][a], Uref=sc["U"][a],
                    x_final=sc["x_final"][a], tr=0.25, box=box, obs=sc["obs"], w_obs=1e6, umax=umax,
                    fix_last_input=True)
        with np.errstate(all="ignore"):
            return prob, qd.solve_agent(prob, sparse=True, tol=1e-11, maxit=maxit)

    for a in range(0, N, 64):   # the sample: every one optimal and equal to the reference form
        assert st[a] == 0, (a, st[a])
        prob, (Xd, Ud, objd, info) = dense(a)
        assert info["status"] == "optimal", (a, info["status"])
        assert abs(og[a] - objd) <= 1e-8 * max(1.0, abs(objd)), (a, og[a], objd)
        assert max(qd.constraint_violation(prob, Xg[a], Ug[a]).values()) < 1e-7, a
    # optimal_inaccurate (Clarabel's reduced tolerances) within 1e-5 of the optimum
    for a in np.nonzero(st == 1)[0]:
        prob, (Xd, Ud, objd, info) = dense(a)
        assert abs(og[a] - objd) <= 1e-5 * max(1.0, abs(objd)), (a, og[a], objd)
    # a solver_error is an agent whose subproblem is infeasible: at u_max = 0.12 a goal more than
    # u_max sigma^2 / 4 = 27 m away cannot be reached (the reference's Clarabel would report infeasible)
    for a in np.nonzero(st == 2)[0]:
        prob, (Xd, Ud, objd, info) = dense(a, maxit=60)
        assert info["status"] != "optimal", a
        assert np.linalg.norm(sc["x_final"][a][:3] - sc["x_init"][a][:3]) > 0.8 * umax * sc["sigma"][a] ** 2 / 4
    assert (st == 0).mean() >= 0.99, np.bincount(st, minlength=3)


def test_collision_rows_match_reference_formula(cuda):
    rng = np.random.default_rng(3)
    N, K = 9, 20
    Xall = rng.normal(0, 3.0, (N, K, 6))
    rows, cnt = scvx_hip.collision_rows(_t(Xall, cuda), 2, 4, 2.3, j_max=N - 1)
    rows, cnt = rows.cpu().numpy(), cnt.cpu().numpy()
    trajs = [Xall[i] for i in range(N)]
    for a in range(4):
        ref = pb.collision_rows(trajs, 2 + a, 2.3)
        for t in range(K - 1):
            assert cnt[a, t] == N - 1
            got = rows[a, t, :cnt[a, t]]
            np.testing.assert_allclose(got[np.lexsort(got.T)], ref[t][np.lexsort(ref[t].T)], rtol=1e-13, atol=1e-13)
        assert cnt[a, K - 1] == 0


@pytest.mark.parametrize("j_max", [0, 8])
def test_quad_family_matches_cpu_and_dense(cuda, j_max):
    """C5 family: 12-state quadrotor from hover (scvx_hip/workloads.synthetic_quad), 8 obstacles,
    optionally collision rows (R=0.5) -- GPU vs the C++ restatement and the dense oracle."""
    import torch
    from scvx_hip import workloads
    N, K = 8, 50
    sc = workloads.synthetic_quad(N, K=K, seed=3, obstacles=8)
    X, U, sig = _t(sc["X"], cuda), _t(sc["U"], cuda), _t(sc["sigma"], cuda)
    disc = scvx_hip.foh_batched("quad", X, U, sig)
    box = [(0, -12, 12), (1, -12, 12)]
    rows = cnt = None
    if j_max:
        rows, cnt = scvx_hip.collision_rows(X, 0, N, 0.5, j_max=j_max)
    spec = scvx_hip.QPSpec(model="quad", K=K, box=box, obs=sc["obs"], w_obs=1e6, j_max=j_max, w_coll=1e4,
                           tol=1e-9, max_iter=80)
    tr = np.full(N, 0.25)
    out = scvx_hip.qp_solve_batched(spec, disc, sig, X, U, _t(sc["x_init"], cuda), _t(sc["x_final"], cuda),
                                    _t(tr, cuda), rows, cnt)
    st = out["status"].cpu().numpy()
    assert (st == 0).all(), st
    tpl = qp_cpu.make_template(12, 4, K, box=box, obs=sc["obs"], w_obs=1e6, j_max=j_max, w_coll=1e4, tol=1e-9, model_id=3,
                               max_iter=80)
    dn = disc.cpu().numpy()
    cpu = qp_cpu.solve_batched(tpl, dn, sc["sigma"], sc["X"], sc["U"], sc["x_init"], sc["x_final"], tr,
                               None if rows is None else rows.cpu().numpy(),
                               None if cnt is None else cnt.cpu().numpy())
    assert (cpu["status"] == 0).all()
    og = out["obj"].cpu().numpy()
    np.testing.assert_allclose(og, cpu["obj"], rtol=1e-8)
    assert np.abs(out["X"].cpu().numpy() - cpu["X"]).max() < 1e-6
    if not j_max:
        A, B, C, S, z = pb.unpack_disc(dn[0], 12, 4)
        prob = dict(A=A, B=B, C=C, c=S * sc["sigma"][0] + z, Xref=sc["X"][0], Uref=sc["U"][0],
                    x_final=sc["x_final"][0], tr=0.25, box=box, obs=sc["obs"], w_obs=1e6, umax=None,
                    fix_last_input=True)
        with np.errstate(all="ignore"):
            Xd, Ud, objd, info = qd.solve_agent(prob, tol=1e-10, maxit=150)
        assert info["status"] == "optimal"
        assert abs(og[0] - objd) <= 1e-7 * max(1.0, abs(objd))


@pytest.mark.parametrize("model", ["unicycle", "si"])
def test_unicycle_and_si_classes_match_cpu_and_dense(cuda, model):
    """The unicycle (n=3, m=2, planar positions) and single-integrator (n=3, m=3, SOC ||u|| <= 3)
    instantiations of the trust-region QP kernel -- GPU vs the C++ restatement and the dense oracle."""
    N, K = 6, 30
    rng = np.random.default_rng(11)
    n, m = scvx_hip.MODEL_DIMS[model]
    pd = 2 if model == "unicycle" else 3
    a = np.linspace(0, 1, K)[None, :, None]
    p0 = rng.uniform(-8, -5, (N, 1, n))
    p1 = rng.uniform(5, 8, (N, 1, n))
    X = p0 * (1 - a) + p1 * a
    if model == "unicycle":
        X[:, :, 2] = np.pi / 4 + rng.normal(0, 0.1, (N, K))
        U = np.stack([np.full((N, K), 0.8), rng.normal(0, 0.1, (N, K))], -1)
        sig = np.full(N, 24.0)
        obs = [(np.array([0.5, -0.5]), 1.5), (np.array([-3.0, -2.0]), 1.0)]
        umax = None
    else:
        U = np.repeat(((p1 - p0)[:, 0] / 12.0)[:, None, :], K, 1) + rng.normal(0, 0.05, (N, K, 3))
        sig = np.full(N, 12.0)
        obs = [(np.array([0.3, -0.4, 0.2]), 1.5), (np.array([-4.0, -3.0, -4.0]), 1.0)]
        umax = 3.0
    box = [(0, -10, 10), (1, -10, 10)]
    Xt, Ut, st_ = _t(X, cuda), _t(U, cuda), _t(sig, cuda)
    disc = scvx_hip.foh_batched(model, Xt, Ut, st_)
    tr = np.full(N, 0.5)
    spec = scvx_hip.QPSpec(model=model, K=K, pos_dim=pd, box=box, obs=obs, w_obs=1e6, u_max=umax, tol=1e-10,
                           max_iter=80)
    out = scvx_hip.qp_solve_batched(spec, disc, st_, Xt, Ut, _t(X[:, 0], cuda), _t(X[:, -1], cuda), _t(tr, cuda))
    dn = disc.cpu().numpy()
    tpl = qp_cpu.make_template(n, m, K, pos_dim=pd, box=box, obs=obs, w_obs=1e6, u_max=umax, tol=1e-10, max_iter=80,
                               model_id=scvx_hip.MODEL_IDS[model])
    cpu = qp_cpu.solve_batched(tpl, dn, sig, X, U, X[:, 0], X[:, -1], tr)
    st = out["status"].cpu().numpy()
    assert (cpu["status"] == 0).all(), cpu["status"]   # every agent (round 2 let half of them fail)
    assert (st == 0).all(), st
    og, Xg = out["obj"].cpu().numpy(), out["X"].cpu().numpy()
    for i in range(N):
        assert abs(og[i] - cpu["obj"][i]) <= 1e-8 * max(1.0, abs(cpu["obj"][i]))
        assert np.abs(Xg[i] - cpu["X"][i]).max() < 1e-6
        A, B, C, S, z = pb.unpack_disc(dn[i], n, m)
        prob = dict(A=A, B=B, C=C, c=S * sig[i] + z, Xref=X[i], Uref=U[i], x_final=X[i, -1], tr=0.5, box=box,
                    obs=obs, w_obs=1e6, umax=umax, fix_last_input=True, pos_dim=pd)
        with np.errstate(all="ignore"):
            Xd, Ud, objd, info = qd.solve_agent(prob, sparse=True, tol=1e-11)
        assert info["status"] == "optimal"
        assert abs(og[i] - objd) <= 1e-8 * max(1.0, abs(objd)), (i, og[i], objd)
        assert max(qd.constraint_violation(prob, Xg[i], out["U"].cpu().numpy()[i]).values()) < 1e-7


def test_soft_terminal_matches_twin_and_dense(cuda):
    """QPSpec.w_final (soft terminal, has_final=False): the kernel equals the CPU twin on every agent of
    a 64-agent C3-family batch and the dense reference form (x_final row replaced by the penalty) on a
    sample; tolerances as above."""
    N, K, wf = 64, 50, 50.0
    sc = pb.synthetic_di(N, K=K, seed=4, obstacles=8)
    box = [(0, -12, 12), (1, -12, 12)]
    import torch
    X, U, sig = _t(sc["X"], cuda), _t(sc["U"], cuda), _t(sc["sigma"], cuda)
    disc = scvx_hip.foh_batched("di", X, U, sig)
    tr = np.full(N, 0.25)
    spec = scvx_hip.QPSpec(model="di", K=K, box=box, obs=sc["obs"], w_obs=1e6, u_max=1.0, has_final=False,
                           w_final=wf, tol=1e-10, max_iter=80)
    out = scvx_hip.qp_solve_batched(spec, disc, sig, X, U, _t(sc["x_init"], cuda), _t(sc["x_final"], cuda),
                                    _t(tr, cuda))
    st = out["status"].cpu().numpy()
    assert (st == 0).all(), np.bincount(st, minlength=3)
    dn = disc.cpu().numpy()
    tpl = qp_cpu.make_template(6, 3, K, has_final=False, w_final=wf, box=box, obs=sc["obs"], w_obs=1e6, u_max=1.0,
                               tol=1e-10, max_iter=80)
    cpu = qp_cpu.solve_batched(tpl, dn, sc["sigma"], sc["X"], sc["U"], sc["x_init"], sc["x_final"], tr, nthreads=8)
    assert (cpu["status"] == 0).all()
    Xg, Ug = out["X"].cpu().numpy(), out["U"].cpu().numpy()
    assert np.abs(Xg - cpu["X"]).max() < 1e-6
    assert np.abs(Ug[:, :-1] - cpu["U"][:, :-1]).max() < 1e-6
    for a in (0, 17):
        A, B, C, S, z = pb.unpack_disc(dn[a], 6, 3)
        prob = dict(A=A, B=B, C=C, c=S * sc["sigma"][a] + z, Xref=sc["X"][a], Uref=sc["U"][a],
                    x_final=sc["x_final"][a], w_final=wf, tr=0.25, box=box, obs=sc["obs"], w_obs=1e6, umax=1.0,
                    fix_last_input=True)
        with np.errstate(all="ignore"):
            Xd, Ud, objd, info = qd.solve_agent(prob, tol=1e-11, maxit=150)
        assert info["status"] == "optimal"
        assert np.abs(Xg[a] - Xd).max() < 1e-6 and np.abs(Ug[a][:-1] - Ud[:-1]).max() < 1e-6
        assert abs(out["obj"][a].item() - objd) <= 1e-6 * max(1.0, abs(objd))


def test_min_energy_closed_form(cuda):
    """Known answer: with every inequality inactive (trust region 1e3, no box / obstacles / SOC / coupling)
    the Q1 subproblem (dist_scvx_3d.py:51-111) is the minimum-energy transfer of the FOH-discretized double
    integrator, u* = M'(M M')^-1 r (tests/test_independent_checks_cpu.min_energy_transfer) -- no solver
    involved in the reference answer."""
    from test_independent_checks_cpu import gramian_case, min_energy_transfer
    sc, disc = gramian_case(N=16)
    N, K = disc.shape[0], disc.shape[1] + 1
    spec = scvx_hip.QPSpec(model="di", K=K, tol=1e-12, max_iter=80)
    out = scvx_hip.qp_solve_batched(spec, _t(disc, cuda), _t(sc["sigma"], cuda), _t(sc["X"], cuda), _t(sc["U"], cuda),
                                    _t(sc["x_init"], cuda), _t(sc["x_final"], cuda), _t(np.full(N, 1e3), cuda))
    st = out["status"].cpu().numpy()
    assert (st == 0).all(), st
    Xg, Ug, og = out["X"].cpu().numpy(), out["U"].cpu().numpy(), out["obj"].cpu().numpy()
    for a in range(N):
        A, B, C, S, z = pb.unpack_disc(disc[a], 6, 3)
        Xc, Uc, objc = min_energy_transfer(A, B, C, S * sc["sigma"][a] + z, sc["x_init"][a], sc["x_final"][a],
                                           sc["U"][a][-1])
        assert np.abs(Xg[a] - Xc).max() < 1e-8 and np.abs(Ug[a] - Uc).max() < 1e-9, a
        assert abs(og[a] - objc) <= 1e-9 * max(1.0, objc), (a, og[a], objc)

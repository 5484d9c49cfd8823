"""GPU parity of the batched SCProblem / AgentSolver kernel (scvx_scp_solve_batched) against
  * oracle/scp_dense.py -- the reference's own formulation (sc_problem.py:15-83, agent_solver.py:78-102)
    solved by an independent sparse conic IPM: optimal VALUE (LPs have non-unique optimisers),
    feasibility and, where the problem is strictly convex in the positions (ADMM), positions;
  * oracle/scp_cpu.py -- the CPU restatement of the kernel's own iteration.
Tolerances: objective relative 1e-7, constraint violation 1e-7, ADMM positions within the strong-convexity bound ||p - p*||^2 <= 2 gap / (rho n_nbr) implied by the measured optimal-value gap."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def spec_and_tensors(probs, torch, dev, max_iter=100, tol=1e-9, waves_per_agent=0):
    import scvx_hip
    p0 = probs[0]
    nn = len(p0.get("nbrs") or [])
    spec = scvx_hip.SCPSpec(model=p0["model"], K=p0["Xref"].shape[0], pos_dim=p0["pos_dim"],
                            u_bounds=p0["u_bounds"], u_soc=p0["u_soc"], x_bounds=p0["x_bounds"], obs=p0["obs"],
                            w_nu=p0["w_nu"], w_slack=p0["w_slack"], w_sigma=p0["w_sigma"], n_nbr=nn,
                            rho=p0.get("rho", 0.0), d_min=p0.get("d_min", 1.0), max_iter=max_iter, tol=tol,
                            waves_per_agent=waves_per_agent)
    T = lambda a: torch.tensor(np.ascontiguousarray(a), dtype=torch.float64, device=dev)  # noqa: E731
    args = dict(disc=T(np.stack([p["disc"] for p in probs])), Xref=T(np.stack([p["Xref"] for p in probs])),
                Uref=T(np.stack([p["Uref"] for p in probs])), sigma_ref=T([p["sigma_ref"] for p in probs]),
                tr=T([p["tr"] for p in probs]), x_init=T(np.stack([p["x_init"] for p in probs])),
                x_final=T(np.stack([p["x_final"] for p in probs])))
    if nn:
        args["nbr_pos"] = T(np.stack([np.stack([nb["Pref"] for nb in p["nbrs"]]) for p in probs]))
        args["nbr_Y"] = T(np.stack([np.stack([nb["Y"] for nb in p["nbrs"]]) for p in probs]))
        args["nbr_Lam"] = T(np.stack([np.stack([nb["Lam"] for nb in p["nbrs"]]) for p in probs]))
    return spec, args


def solve_gpu(probs, torch, dev, **kw):
    import scvx_hip
    spec, args = spec_and_tensors(probs, torch, dev, **kw)
    out = scvx_hip.SCPSolver(spec, len(probs), device=dev).solve(**args)
    torch.cuda.synchronize()
    return {k: v.cpu().numpy() for k, v in out.items()}


def instances(model, K, n_agents, admm=False, seed=0):
    from oracle import scp_problems as sp_
    rng = np.random.default_rng(seed)
    out = []
    for a in range(n_agents):
        x0 = np.array([-8.0, -8.0, 0.0]) + (rng.uniform(-1, 1, 3) * [1, 1, 0.3] if a else 0)
        xf = np.array([8.0, 8.0, 0.0]) + (rng.uniform(-1, 1, 3) * [1, 1, 0.3] if a else 0)
        if model == "si":
            x0 = np.array([-8.0, -8.0, -8.0]) + (rng.uniform(-1, 1, 3) if a else 0)
            xf = np.array([8.0, 8.0, 8.0]) + (rng.uniform(-1, 1, 3) if a else 0)
        p = sp_.scp_instance(model, K=K, x_init=x0, x_final=xf, sigma_ref=1.0 + 2.0 * a)
        if admm:
            pd = p["pos_dim"]
            nbr = [sp_.straight(x0 + 3.0 * np.eye(3)[0], xf - 3.0 * np.eye(3)[0], K), sp_.straight(xf, x0, K)]
            Y = [r[:, :pd] + 0.1 * rng.standard_normal((K, pd)) for r in nbr]
            Lam = [0.5 * rng.standard_normal((K, pd)) for _ in nbr]
            p = sp_.add_admm(p, nbr, Y=Y, Lam=Lam, rho=1.0, d_min=1.0)
        out.append(p)
    return out


@pytest.mark.parametrize("model,K", [("unicycle", 30), ("unicycle", 100), ("si", 30), ("si", 100)])
def test_scproblem_matches_reference_formulation(cuda, model, K):
    import torch
    from oracle import scp_dense as sd
    probs = instances(model, K, 3)
    g = solve_gpu(probs, torch, cuda)
    assert np.isin(g["status"], (0, 1)).all(), g["status"]   # optimal or optimal_inaccurate (accuracy checked below)
    for a, p in enumerate(probs):
        ref = sd.solve_scproblem(p, tol=1e-10)
        X, U, nu, sig = g["X"][a], g["U"][a], g["nu"][a], float(g["sigma"][a])
        obj = sd.scp_objective(p, X, U, nu, sig)
        assert abs(obj - ref["obj"]) <= 1e-7 * abs(ref["obj"]), (a, obj, ref["obj"])
        assert abs(g["obj"][a] - obj) <= 1e-7 * abs(obj)          # kernel-reported objective
        assert sd.scp_violation(p, X, U, nu, sig) < 1e-7
        assert X.shape == (K, 3) and nu.shape == (K - 1, 3)


@pytest.mark.parametrize("model,admm,K", [("unicycle", False, 100), ("si", False, 100), ("unicycle", True, 100),
                                          ("unicycle", False, 200)])
def test_one_and_two_waves_per_agent(cuda, model, admm, K):
    """K > 64 nodes: the same agents through the one-wave mapping (node phases in two or more passes; what a
    launch that fills every SIMD uses) and the two-wave mapping (SCPSpec.waves_per_agent; what a
    single-agent launch uses; K = 200 takes two passes of 128 threads).  Both at the dense oracle's optimal
    value (1e-7, feasibility 1e-7); their reductions sum in different orders, so they agree to the
    stopping tolerance, not bit for bit."""
    import torch
    import scvx_hip
    from oracle import scp_dense as sd
    probs = instances(model, K, 3 if K <= 100 else 2, admm=admm, seed=5)
    out = {w: solve_gpu(probs, torch, cuda, waves_per_agent=w) for w in (1, 2)}   # the template's own mapping
    # the automatic mapping (waves_per_agent = 0) takes two waves here (K > 64, few agents): the same results
    dflt = solve_gpu(probs, torch, cuda)
    for k in ("X", "U", "obj", "iters"):
        np.testing.assert_array_equal(dflt[k], out[2 if K > 64 else 1][k])
    with pytest.raises(Exception):   # only 0, 1, 2
        solve_gpu(probs, torch, cuda, waves_per_agent=3)
    for a, p in enumerate(probs):
        ref = sd.solve_scproblem(p, tol=1e-10)
        objs = []
        for w in (1, 2):
            g = out[w]
            assert g["status"][a] in (0, 1), (w, g["status"])
            X, U, nu, sig = g["X"][a], g["U"][a], g["nu"][a], float(g["sigma"][a])
            obj = sd.scp_objective(p, X, U, nu, sig)
            assert abs(obj - ref["obj"]) <= 1e-7 * abs(ref["obj"]), (w, a, obj, ref["obj"])
            assert sd.scp_violation(p, X, U, nu, sig) < 1e-7
            objs.append(obj)
        assert abs(objs[0] - objs[1]) <= 1e-7 * abs(ref["obj"])


@pytest.mark.parametrize("model", ["unicycle", "si"])
def test_agent_solver_admm_matches_reference_formulation(cuda, model):
    import torch
    from oracle import scp_dense as sd, scp_cpu as sc
    probs = instances(model, 30, 2, admm=True, seed=3)
    g = solve_gpu(probs, torch, cuda)
    assert np.isin(g["status"], (0, 1)).all(), g["status"]
    for a, p in enumerate(probs):
        ref = sd.solve_scproblem(p, tol=1e-10)
        X, U, nu, sig = g["X"][a], g["U"][a], g["nu"][a], float(g["sigma"][a])
        obj = sd.scp_objective(p, X, U, nu, sig)
        assert abs(obj - ref["obj"]) <= 1e-7 * abs(ref["obj"]), (a, obj, ref["obj"])
        assert sd.scp_violation(p, X, U, nu, sig) < 1e-7
        pd = p["pos_dim"]
        # strong convexity in p (modulus rho per neighbour): ||p - p*||^2 <= 2 gap / (rho n_nbr)
        gap = abs(obj - ref["obj"]) + 1e-9 * abs(ref["obj"])
        ptol = np.sqrt(2.0 * gap / (p["rho"] * len(p["nbrs"]))) + 1e-6
        assert np.abs(X[:, :pd] - ref["X"][:, :pd]).max() < ptol
        cpu = sc.SCPSolver(p, tol=1e-9).solve()
        gap_c = abs(obj - sd.scp_objective(p, cpu["X"], cpu["U"], cpu["nu"], float(cpu["sigma"]))) + 1e-9 * abs(ref["obj"])
        assert np.abs(X[:, :pd] - cpu["X"][:, :pd]).max() < np.sqrt(2.0 * gap_c / (p["rho"] * len(p["nbrs"]))) + 1e-6
        assert g["s_nbr"].shape == (2, 2, 30)


def test_scproblem_second_iterate_and_iteration_count(cuda):
    """A second SCvx iterate (sigma_ref = 5, tr = 50) and the kernel's iteration count against the
    CPU restatement of the same algorithm."""
    import torch
    from oracle import scp_dense as sd, scp_problems as sp_, scp_cpu as sc
    p = sp_.scp_instance("unicycle", K=30)
    r = sd.solve_scproblem(p, tol=1e-10)
    p2 = sp_.scp_instance("unicycle", K=30, Xref=r["X"], Uref=r["U"], sigma_ref=5.0, tr=50.0)
    g = solve_gpu([p2], torch, cuda)
    cpu = sc.SCPSolver(p2, tol=1e-9).solve()
    ref = sd.solve_scproblem(p2, tol=1e-10)
    obj = sd.scp_objective(p2, g["X"][0], g["U"][0], g["nu"][0], float(g["sigma"][0]))
    assert g["status"][0] == 0
    assert abs(obj - ref["obj"]) <= 1e-7 * abs(ref["obj"])
    assert abs(g["sigma"][0] - ref["sigma"]) < 1e-6
    assert abs(int(g["iters"][0]) - cpu["iters"]) <= 2


@pytest.mark.parametrize("K", [30, 100])
def test_scproblem_lp_value_matches_highs(cuda, K):
    """The SCP kernel's optimal value on the SCProblem LPs (unicycle: no SOC, the objective is linear)
    against SciPy's HiGHS on the reference-form assembly -- a solver that shares nothing with either the
    kernel or oracle/scp_dense.py (tests/test_independent_checks_cpu.py checks the oracles the same way).
    Trust radii 100 (inactive), 5 and 1 (binding).  Value 1e-7 relative (the kernel's tolerance 1e-9)."""
    import torch
    from oracle import scp_dense as sd
    from test_independent_checks_cpu import _uni_instances, highs_value
    probs = _uni_instances(K)
    g = solve_gpu(probs, torch, cuda)
    assert np.isin(g["status"], (0, 1)).all(), g["status"]
    for a, p in enumerate(probs):
        v = highs_value(p)
        obj = sd.scp_objective(p, g["X"][a], g["U"][a], g["nu"][a], float(g["sigma"][a]))
        assert abs(obj - v) <= 1e-7 * max(1.0, abs(v)), (a, obj, v)
        assert sd.scp_violation(p, g["X"][a], g["U"][a], g["nu"][a], float(g["sigma"][a])) < 1e-7


@pytest.mark.parametrize("tr,tol", [(5.0, 1e-20), (1.0, 1e-15)])
def test_end_game_exit_returns_best_iterate(cuda, tr, tol):
    """A tolerance below what the Newton systems can reach drives the kernel into ECOS's
    insufficient-progress exit (status 1): the outputs are the best iterate since the reduced tolerances
    held (as the CPU twin, tests/test_independent_checks_cpu.py), and their value is HiGHS's to 1e-8.
    (Since the end-game step fraction both reach 1e-13 and the tr = 5 instance 1e-15, so they are asked for 1e-15
    and 1e-20.)"""
    import torch
    from oracle import scp_dense as sd, scp_problems as spp
    from test_independent_checks_cpu import highs_value
    p = spp.scp_instance("unicycle", K=30, tr=tr)
    g = solve_gpu([p], torch, cuda, tol=tol)
    assert g["status"][0] == 1, g["status"]
    v = highs_value(p)
    obj = sd.scp_objective(p, g["X"][0], g["U"][0], g["nu"][0], float(g["sigma"][0]))
    assert abs(obj - v) <= 1e-8 * max(1.0, abs(v)), (obj, v)
    assert sd.scp_violation(p, g["X"][0], g["U"][0], g["nu"][0], float(g["sigma"][0])) < 1e-7

"""CPU, no GPU: checks of the restated oracles by means that share nothing with them.

cvxpy / ECOS / Clarabel are not installed here, so the reference's own solver answers cannot be
produced (parity against them is unpinned).  What can be checked independently:

  * the LP family of SCProblem (unicycle: sc_problem.py:15-83 with unicycle_model.py:88-114, no SOC)
    against SciPy's vendored HiGHS (scipy.optimize.linprog(method="highs"), a simplex / IPM code
    with its own presolve): the optimal VALUE of oracle/scp_dense.py's reference-form assembly and
    of oracle/scp_cpu.py (the SCP kernel's CPU restatement) must equal HiGHS's;
  * the Q1 trust-region subproblem of Distributed_opt/dist_scvx_3d.py:51-111 with every inequality
    inactive (large trust region, no box / obstacles / coupling): a closed-form minimum-energy transfer
    (the controllability-Gramian solution u = M'(MM')^-1 r of the FOH-discretized double integrator),
    against oracle/qp_dense.py and the kernel's CPU twin oracle/scvx_cpu.cpp;
  * the virtual-control form (QPSpec.w_nu, the SCvx subproblem of sc_problem.py:60-68 with an
    elementwise ||nu||_1) on the twin against the dense oracle's own assembly of it.
"""
import numpy as np
import pytest
from scipy.optimize import linprog

from oracle import foh_oracle, problems as pb, qp_cpu, qp_dense as qd, scp_cpu, scp_dense as sd, scp_problems as sp_


def _uni_instances(K):
    rng = np.random.default_rng(0)
    out = []
    for a, tr in enumerate((100.0, 5.0, 1.0)):   # TRUST_RADIUS0 (inactive), then a binding trust region
        x0 = np.array([-8.0, -8.0, 0.0]) + (rng.uniform(-1, 1, 3) * [1, 1, 0.3] if a else 0)
        xf = np.array([8.0, 8.0, 0.0]) + (rng.uniform(-1, 1, 3) * [1, 1, 0.3] if a else 0)
        out.append(sp_.scp_instance("unicycle", K=K, x_init=x0, x_final=xf, sigma_ref=1.0 + 2.0 * a, tr=tr))
    return out


def highs_value(p):
    """Optimal value of the reference-form LP (oracle/scp_dense.build_scproblem) by HiGHS."""
    P, q, A, b, G, h, dims, idx = sd.build_scproblem(p)
    assert (P.nnz == 0 or abs(P).max() == 0) and not dims["q"], "not an LP instance"
    r = linprog(q, A_ub=G, b_ub=h, A_eq=A, b_eq=b, bounds=(None, None), method="highs")
    assert r.status == 0, r.message
    return r.fun + idx["const"]


@pytest.mark.parametrize("K", [30, 100])
def test_scproblem_lp_value_matches_highs(K):
    """scp_dense (reference formulation, our IPM) and scp_cpu (the kernel's iteration) reach HiGHS's
    optimal value to 1e-8 relative on the SCProblem LPs (the objective is linear: w_nu max_k||nu_k||_1 +
    w_slack sum s' + w_sigma sigma, so only the value is unique)."""
    for p in _uni_instances(K):
        v = highs_value(p)
        ref = sd.solve_scproblem(p, tol=1e-10)
        # (the oracles' ECOS-style reduced-accuracy exit is taken on 2 of these 6 LPs; the value is what matters)
        assert ref["status"] in ("optimal", "optimal_inaccurate")
        assert abs(ref["obj"] - v) <= 1e-8 * max(1.0, abs(v)), (ref["obj"], v)
        o = scp_cpu.SCPSolver(p, tol=1e-10).solve()
        obj = sd.scp_objective(p, o["X"], o["U"], o["nu"], o["sigma"])
        assert abs(obj - v) <= 1e-8 * max(1.0, abs(v)), (obj, v)
        assert sd.scp_violation(p, o["X"], o["U"], o["nu"], o["sigma"]) < 1e-7


def min_energy_transfer(A, B, C, c, x0, xf, u_last):
    """Closed form of min sum_{t<K-1} ||u_t||^2 s.t. x_{t+1} = A_t x_t + B_t u_t + C_t u_{t+1} + c_t,
    x_0 = x0, x_{K-1} = xf, u_{K-1} = u_last: x_{K-1} = a + M u (u = u_0..u_{K-2} stacked), so
    u* = M'(M M')^-1 (xf - a) -- the discrete controllability-Gramian solution."""
    Km1, n, m = B.shape
    K = Km1 + 1
    a = np.asarray(x0, float).copy()
    M = np.zeros((n, Km1 * m))
    for t in range(Km1):
        a = A[t] @ a + c[t]
        M = A[t] @ M
        M[:, t * m:(t + 1) * m] += B[t]
        if t + 1 < Km1:
            M[:, (t + 1) * m:(t + 2) * m] += C[t]
        else:
            a = a + C[t] @ u_last
    u = M.T @ np.linalg.solve(M @ M.T, xf - a)
    U = np.vstack([u.reshape(Km1, m), u_last[None]])
    X = np.zeros((K, n))
    X[0] = x0
    for t in range(Km1):
        X[t + 1] = A[t] @ X[t] + B[t] @ U[t] + C[t] @ U[t + 1] + c[t]
    return X, U, float(np.sum(U[:-1] ** 2))


def gramian_case(N=4, K=50, seed=7):
    """C2 construction (random starts / goals at rest, straight-line warm start, sigma = 30), trust region
    1e3 (never active), no box, obstacles, SOC or coupling."""
    sc = pb.synthetic_di(N, K=K, seed=seed)
    disc = np.stack([np.hstack([o.T for o in foh_oracle.foh("di", sc["X"][a].T, sc["U"][a].T, sc["sigma"][a])])
                     for a in range(N)])
    return sc, disc


def test_min_energy_closed_form_pins_dense_oracle_and_twin():
    sc, disc = gramian_case()
    N, K = disc.shape[0], disc.shape[1] + 1
    tr = np.full(N, 1e3)
    tpl = qp_cpu.make_template(6, 3, K, tol=1e-12, max_iter=80)
    cpu = qp_cpu.solve_batched(tpl, disc, sc["sigma"], sc["X"], sc["U"], sc["x_init"], sc["x_final"], tr)
    assert (cpu["status"] == 0).all(), cpu["status"]
    for a in range(N):
        A, B, C, S, z = pb.unpack_disc(disc[a], 6, 3)
        c = S * sc["sigma"][a] + z
        Xc, Uc, objc = min_energy_transfer(A, B, C, c, sc["x_init"][a], sc["x_final"][a], sc["U"][a][-1])
        assert np.abs(cpu["X"][a] - Xc).max() < 1e-8
        assert np.abs(cpu["U"][a] - Uc).max() < 1e-9
        assert abs(cpu["obj"][a] - objc) <= 1e-9 * max(1.0, objc)
        prob = dict(A=A, B=B, C=C, c=c, Xref=sc["X"][a], Uref=sc["U"][a], x_final=sc["x_final"][a], tr=1e3,
                    fix_last_input=True)
        Xd, Ud, objd, info = qd.solve_agent(prob, sparse=True, tol=1e-12)
        assert info["status"] == "optimal"
        assert np.abs(Xd - Xc).max() < 1e-7 and abs(objd - objc) <= 1e-9 * max(1.0, objc)


BOX = [(0, -12, 12), (1, -12, 12)]


@pytest.mark.parametrize("tr0,w_nu,w_prox", [(0.01, 1e3, 0.0), (0.01, 50.0, 1.0), (0.25, 1e3, 0.0)])
def test_twin_virtual_control_matches_dense_oracle(tr0, w_nu, w_prox):
    """Virtual control on the C3 family: with tr = 0.01 the goal is out of reach of the input trust region
    and nu carries the difference (max |nu| ~ 0.1-0.4); with tr = 0.25 nu is 0.  Objective 1e-9 relative;
    trajectories and nu 1e-5 (the nu part of the objective is piecewise linear: the inputs are unique through
    their quadratic cost, nu only up to the IPM's end-game accuracy, measured 1.2e-6)."""
    N, K = 3, 50
    sc = pb.synthetic_di(N, K=K, seed=1, obstacles=8)
    disc = np.stack([np.hstack([o.T for o in foh_oracle.foh("di", sc["X"][a].T, sc["U"][a].T, sc["sigma"][a])])
                     for a in range(N)])
    tr = np.full(N, tr0)
    tpl = qp_cpu.make_template(6, 3, K, box=BOX, obs=sc["obs"], w_obs=1e6, u_max=1.0, tol=1e-10, max_iter=80,
                               w_nu=w_nu, w_prox=w_prox)
    cpu = qp_cpu.solve_batched(tpl, disc, sc["sigma"], sc["X"], sc["U"], sc["x_init"], sc["x_final"], tr)
    assert (cpu["status"] == 0).all(), cpu["status"]
    if tr0 < 0.1:
        assert np.abs(cpu["nu"]).max() > 1e-2
    else:
        assert np.abs(cpu["nu"]).max() < 1e-9
    for a in range(N):
        A, B, C, S, z = pb.unpack_disc(disc[a], 6, 3)
        prob = dict(A=A, B=B, C=C, c=S * sc["sigma"][a] + z, Xref=sc["X"][a], Uref=sc["U"][a],
                    x_final=sc["x_final"][a], tr=tr0, box=BOX, obs=sc["obs"], w_obs=1e6, umax=1.0,
                    fix_last_input=True, w_nu=w_nu, w_prox=w_prox)
        with np.errstate(all="ignore"):
            Xd, Ud, objd, info = qd.solve_agent(prob, sparse=True, tol=1e-11)
        assert info["status"] == "optimal"
        # the gap test is relative to the objective WITHOUT the proximal term's constant w_prox sum ||xbar||^2
        # (as the soft terminal's, and Clarabel's without CVXPY's offset), here ~2e2 times the objective
        ref = max(1.0, abs(objd)) + w_prox * float(np.sum(sc["X"][a] ** 2))
        assert abs(cpu["obj"][a] - objd) <= 1e-9 * ref, (a, cpu["obj"][a], objd)
        assert np.abs(cpu["X"][a] - Xd).max() < 1e-5 and np.abs(cpu["nu"][a] - info["nu"]).max() < 1e-5
        # strong convexity in U (Hessian 2I): ||U - U*||^2 <= gap, the stopping rule's 1e-10 x objective
        assert np.abs(cpu["U"][a][:-1] - Ud[:-1]).max() < max(1e-6, 3.0 * np.sqrt(1e-10 * ref))
        assert max(qd.constraint_violation(prob, cpu["X"][a], cpu["U"][a], nu=cpu["nu"][a]).values()) < 1e-8


@pytest.mark.parametrize("tr", [5.0, 1.0])
def test_twin_end_game_exit_returns_best_iterate(tr):
    """ECOS's insufficient-progress exit (oracle/scp_cpu.py, csrc/scp_ipm.hip): at tol 1e-15 the LP's
    Newton systems hit their accuracy floor, a residual jumps 100x above its best and the solve ends as
    optimal_inaccurate on the BEST iterate seen since the reduced tolerances held (restored), whose value
    HiGHS confirms to 1e-8."""
    from oracle import scp_problems as spp
    p = spp.scp_instance("unicycle", K=30, tr=tr)
    sol = scp_cpu.SCPSolver(p, tol=1e-15, max_iter=100)   # (1e-13 is reached since the end-game step fraction)
    o = sol.solve()
    assert o["status"] == "inaccurate" and sol.restored
    v = highs_value(p)
    obj = sd.scp_objective(p, o["X"], o["U"], o["nu"], float(o["sigma"]))
    assert abs(obj - v) <= 1e-8 * max(1.0, abs(v)), (obj, v)
    assert sd.scp_violation(p, o["X"], o["U"], o["nu"], float(o["sigma"])) < 1e-7

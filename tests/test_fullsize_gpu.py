"""GPU: the headline configuration at full size (BASELINE.json config C3: N=1024 agents, K=50, 8
spheres, SOC ||u|| <= 1, box), checked through size-independent properties plus a sampled
comparison with the CPU restatement:

  * FOH of the double integrator for all 1024 agents: Phi = Ad(h) exactly, B + C = Bd(h),
    S sigma + z = 0 (the reference's LSODA reproduces these to 3e-9);
  * trust-region QP for all agents: every agent that reports optimal satisfies the reference-form
    constraints of Distributed_opt/dist_scvx_3d.py:73-90 (+ SOC, soft obstacles) to 1e-7
    (oracle/qp_dense.constraint_violation); 32 sampled agents match oracle/scvx_cpu.cpp to 1e-8 in
    objective and 1e-6 in trajectory; a repeated launch is bit-identical (determinism);
  * three Jacobi SCvx iterations: the per-agent trust radius only ever halves (dist_scvx_3d.py:250-252)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
N, K, SIGMA, TR = 1024, 50, 30.0, 0.25
BOX = [(0, -12.0, 12.0), (1, -12.0, 12.0)]


@pytest.fixture(scope="module")
def c3(cuda):
    import torch
    import scvx_hip
    from scvx_hip import workloads
    sc = workloads.synthetic_di(N, K=K, seed=1, sigma=SIGMA, obstacles=8)
    t = {k: torch.tensor(sc[k], device=cuda) for k in ("X", "U", "x_init", "x_final", "sigma")}
    disc = scvx_hip.foh_batched("di", t["X"], t["U"], t["sigma"])
    spec = scvx_hip.QPSpec(model="di", K=K, box=BOX, obs=sc["obs"], w_obs=1e6, u_max=1.0, tol=1e-9, max_iter=60)
    solver = scvx_hip.QPSolver(spec, N, device=cuda)
    trt = torch.full((N,), TR, dtype=torch.float64, device=cuda)
    out = solver.solve(disc, t["sigma"], t["X"], t["U"], t["x_init"], t["x_final"], trt)
    host = {k: v.cpu().numpy().copy() for k, v in out.items()}
    return dict(sc=sc, t=t, disc=disc, spec=spec, solver=solver, trt=trt, out=host)


def test_foh_invariants_all_agents(c3):
    from oracle import problems as pb
    h = SIGMA / (K - 1)
    Ad, Bd = pb.zoh_di(h)
    d = c3["disc"].cpu().numpy()
    for a in range(0, N, 1):
        A, B, C, S, z = pb.unpack_disc(d[a], 6, 3)
        assert np.abs(A - Ad[None]).max() < 1e-12
        assert np.abs(B + C - Bd[None]).max() < 1e-12
        assert np.abs(S * SIGMA + z).max() < 1e-12


def test_qp_feasibility_all_agents(c3):
    from oracle import problems as pb, qp_dense as qd
    sc, out = c3["sc"], c3["out"]
    d = c3["disc"].cpu().numpy()
    ok = np.flatnonzero(out["status"] == 0)
    assert ok.size >= 0.99 * N, np.bincount(out["status"], minlength=3)
    worst = 0.0
    for a in ok:
        A, B, C, S, z = pb.unpack_disc(d[a], 6, 3)
        prob = dict(A=A, B=B, C=C, c=S * SIGMA + z, Xref=sc["X"][a], Uref=sc["U"][a], x_final=sc["x_final"][a],
                    tr=TR, box=BOX, obs=sc["obs"], w_obs=1e6, umax=1.0, fix_last_input=True)
        worst = max(worst, max(qd.constraint_violation(prob, out["X"][a], out["U"][a]).values()))
    assert worst < 1e-7, worst


def test_qp_sampled_agents_match_cpu_restatement(c3):
    from oracle import qp_cpu
    sc, out = c3["sc"], c3["out"]
    idx = np.random.default_rng(0).choice(N, 32, replace=False)
    tpl = qp_cpu.make_template(6, 3, K, box=BOX, obs=sc["obs"], w_obs=1e6, u_max=1.0, tol=1e-9, max_iter=60)
    d = c3["disc"].cpu().numpy()[idx]
    cpu = qp_cpu.solve_batched(tpl, d, sc["sigma"][idx], sc["X"][idx], sc["U"][idx], sc["x_init"][idx],
                               sc["x_final"][idx], np.full(idx.size, TR), nthreads=4)
    both = (cpu["status"] == 0) & (out["status"][idx] == 0)
    assert both.sum() >= 30
    for j in np.flatnonzero(both):
        a = idx[j]
        assert abs(out["obj"][a] - cpu["obj"][j]) <= 1e-8 * max(1.0, abs(cpu["obj"][j]))
        assert np.abs(out["X"][a] - cpu["X"][j]).max() < 1e-6


def test_qp_relaunch_is_bit_identical(c3):
    t, s = c3["t"], c3["solver"]
    again = s.solve(c3["disc"], t["sigma"], t["X"], t["U"], t["x_init"], t["x_final"], c3["trt"])
    for k in ("X", "U", "obj", "status", "iters"):
        assert np.array_equal(again[k].cpu().numpy(), c3["out"][k]), k


def test_jacobi_iterations_trust_radius_only_halves(c3):
    from scvx_hip.scvx import JacobiSCvx
    t = c3["t"]
    drv = JacobiSCvx(c3["spec"], t["x_init"], t["x_final"], t["sigma"], TR, tr_rule="per_agent")
    X, U = t["X"].clone(), t["U"].clone()
    prev = drv.tr.cpu().numpy().copy()
    for _ in range(3):
        Xn, Un, out = drv.step(X, U)
        X.copy_(Xn)
        U.copy_(Un)
        cur = drv.tr.cpu().numpy()
        assert np.all((cur == prev) | (cur == 0.5 * prev))
        prev = cur.copy()
    assert np.isfinite(X.cpu().numpy()).all()

"""CPU, no GPU: the kernel's CPU twin (oracle/scvx_cpu.cpp, the structured Riccati IPM the GPU tests
compare the HIP kernel with on EVERY agent) against the independent dense reference-formulation
oracle (oracle/qp_dense.py: Distributed_opt/dist_scvx_3d.py:51-111 as written -- perturbation
variables, CVXPY's L1 epigraph, a generic dense KKT IPM) on every agent of C3-family batches.

Together with the GPU tests (kernel == twin on every agent, 1e-6 / 1e-8) this makes the chain
kernel -> twin -> reference formulation hold agent by agent, not on a 1-2 agent sample.
Tolerances (float64): objective 1e-8 relative, trajectories 1e-6 absolute (as the GPU tests), the
twin's solution feasible for the dense form to 1e-7."""
import numpy as np
import pytest

from oracle import foh_oracle, problems as pb, qp_cpu, qp_dense as qd

BOX = [(0, -12, 12), (1, -12, 12)]


def _disc(sc, model, N):
    return np.stack([np.hstack([o.T for o in foh_oracle.foh(model, sc["X"][a].T, sc["U"][a].T, sc["sigma"][a])])
                     for a in range(N)])


def _check_agent(prob, cpu, a):
    with np.errstate(all="ignore"):
        Xd, Ud, objd, info = qd.solve_agent(prob, sparse=True, tol=1e-10)
    assert info["status"] == "optimal", (a, info["status"])
    assert abs(cpu["obj"][a] - objd) <= 1e-8 * max(1.0, abs(objd)), (a, cpu["obj"][a], objd)
    assert np.abs(cpu["X"][a] - Xd).max() < 1e-6, a
    assert np.abs(cpu["U"][a][:-1] - Ud[:-1]).max() < 1e-6, a
    assert max(qd.constraint_violation(prob, cpu["X"][a], cpu["U"][a]).values()) < 1e-7, a


@pytest.mark.parametrize("umax,nobs,agents", [(1.0, 8, (0, 1, 2, 3)), (0.12, 8, (1, 8))])
def test_twin_matches_dense_oracle_on_every_c3_agent(umax, nobs, agents):
    """C3 construction (bench.py: K=50, sigma=30, tr=0.25, box |x|,|y| <= 12, 8 soft spheres, SOC
    ||u|| <= u_max); the tight u_max = 0.12 case is the one with the longest IPM runs (agents 1 and 8:
    18 and 17 iterations; on agent 9 the dense checker itself stops at its iteration cap).  The dense
    oracle takes ~10 s per agent, so the sample is bounded here; the GPU tests compare the kernel with
    the twin on every agent."""
    N, K = 12, 50
    sc = pb.synthetic_di(N, K=K, seed=1, obstacles=nobs)
    disc = _disc(sc, "di", N)
    tr = np.full(N, 0.25)
    tpl = qp_cpu.make_template(6, 3, K, box=BOX, obs=sc["obs"], w_obs=1e6, u_max=umax, tol=1e-10, max_iter=80)
    cpu = qp_cpu.solve_batched(tpl, disc, sc["sigma"], sc["X"], sc["U"], sc["x_init"], sc["x_final"], tr)
    assert (cpu["status"] == 0).all(), cpu["status"]
    for a in agents:
        A, B, C, S, z = pb.unpack_disc(disc[a], 6, 3)
        prob = dict(A=A, B=B, C=C, c=S * sc["sigma"][a] + z, Xref=sc["X"][a], Uref=sc["U"][a],
                    x_final=sc["x_final"][a], tr=0.25, box=BOX, obs=sc["obs"], w_obs=1e6, umax=umax,
                    fix_last_input=True)
        _check_agent(prob, cpu, a)


def test_twin_soft_terminal_matches_dense_oracle():
    """QPSpec.w_final (soft terminal, the build's option for nonlinear models): has_final = 0 and
    w_final ||x_{K-1} - x_final||^2 in the objective, on the twin and on the dense form (no x_final
    row there either); the objective includes the constant w_final ||x_final||^2 in both."""
    N, K, wf = 3, 50, 50.0
    sc = pb.synthetic_di(N, K=K, seed=4, obstacles=8)
    disc = _disc(sc, "di", N)
    tr = np.full(N, 0.25)
    tpl = qp_cpu.make_template(6, 3, K, has_final=False, w_final=wf, box=BOX, obs=sc["obs"], w_obs=1e6, u_max=1.0,
                               tol=1e-12, max_iter=80)   # 1e-12: the 1e6-weighted obstacle slacks move the
    #                                                         objective by ~1e-7 at 1e-10 (agent 1)
    cpu = qp_cpu.solve_batched(tpl, disc, sc["sigma"], sc["X"], sc["U"], sc["x_init"], sc["x_final"], tr)
    assert (cpu["status"] == 0).all(), cpu["status"]
    for a in range(N):
        A, B, C, S, z = pb.unpack_disc(disc[a], 6, 3)
        prob = dict(A=A, B=B, C=C, c=S * sc["sigma"][a] + z, Xref=sc["X"][a], Uref=sc["U"][a],
                    x_final=sc["x_final"][a], w_final=wf, tr=0.25, box=BOX, obs=sc["obs"], w_obs=1e6, umax=1.0,
                    fix_last_input=True)
        _check_agent(prob, cpu, a)
        # the terminal state is pulled towards x_final but not pinned to it
        assert np.abs(cpu["X"][a][-1] - sc["x_final"][a]).max() > 1e-6

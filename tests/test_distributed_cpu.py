"""CPU, multi-process: the sharded Jacobi SCvx driver (scvx_hip.scvx.JacobiSCvx) over torch.distributed
gloo (world_size 2) gives the same iterates as one process owning all agents.

Agents are sharded contiguously; the only data-path exchange is the all_gather of the states
(RCCL on the GPU path), plus one scalar all_reduce for the global trust-region rule
(Distributed_opt/dist_scvx_3d.py:248-252).  The kernels are replaced by the CPU restatements
(oracle/) through the driver's backend hook, so this test runs without a GPU."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from oracle import foh_oracle, problems as pb, qp_cpu

N_TOTAL, K, ITERS = 6, 20, 3


class OracleBackend:
    def foh(self, model, X, U, sigma, nsub, out):
        Xn, Un, sn = X.numpy(), U.numpy(), sigma.numpy()
        d = np.stack([np.hstack([o.T for o in foh_oracle.foh(model, Xn[a].T, Un[a].T, sn[a], nsub=nsub)])
                      for a in range(Xn.shape[0])])
        return torch.from_numpy(d)

    def collision_rows(self, X_all, i0, n_local, R, j_max, pos_dim, cull, rows, count):
        return self.collision_rows_indexed(X_all, torch.arange(i0, i0 + n_local), R, j_max, pos_dim, cull, rows, count)

    def collision_rows_indexed(self, X_all, idx, R, j_max, pos_dim, cull, rows, count):
        """The j_max nearest neighbours' rows per node (the kernel's selection: largest 2R - |d|), kept in
        neighbour-index order."""
        Xa = X_all.numpy()
        trajs = [Xa[i] for i in range(Xa.shape[0])]
        rows.zero_(); count.zero_()
        for a, gi in enumerate(idx.tolist()):
            rr = pb.collision_rows(trajs, gi, R, pos_dim)
            others = [j for j in range(Xa.shape[0]) if j != gi]
            for t in range(Xa.shape[1] - 1):
                dist = [np.linalg.norm(Xa[gi, t, :pos_dim] - Xa[j, t, :pos_dim]) for j in others]
                keep = sorted(sorted(range(len(others)), key=lambda k: dist[k])[:j_max])
                rows[a, t, :len(keep)] = torch.from_numpy(rr[t][keep])
                count[a, t] = len(keep)
        return rows, count

    def collision_check(self, X_all, i0, X_new, slack, R, pos_dim, tol):
        Xa, Xn, S = X_all.numpy(), X_new.numpy(), slack.numpy()
        n_local, K = Xn.shape[0], Xn.shape[1]
        viol = np.zeros((n_local, K), np.int32)
        vmax = np.zeros((n_local, K))
        for a in range(n_local):
            for t in range(K - 1):
                pi = Xa[i0 + a, t, :pos_dim]
                dp = Xn[a, t, :pos_dim] - pi
                v = [2 * R - np.linalg.norm(pi - Xa[j, t, :pos_dim])
                     - (pi - Xa[j, t, :pos_dim]) @ dp / np.linalg.norm(pi - Xa[j, t, :pos_dim]) - S[a, t]
                     for j in range(Xa.shape[0]) if j != i0 + a]
                viol[a, t] = sum(x > tol for x in v)
                vmax[a, t] = max(v)
        return torch.from_numpy(viol), torch.from_numpy(vmax)

    def qp_solver(self, spec, N, device):
        return _CpuQP(spec)


class _CpuQP:
    def __init__(self, spec):
        self.tpl = qp_cpu.make_template(6, 3, spec.K, box=spec.box, j_max=spec.j_max, w_coll=spec.w_coll,
                                        tol=spec.tol, max_iter=spec.max_iter)

    def solve(self, disc, sigma, Xref, Uref, x_init, x_final, tr, rows=None, count=None, n=None, warm=None):
        o = qp_cpu.solve_batched(self.tpl, disc.numpy(), sigma.numpy(), Xref.numpy(), Uref.numpy(), x_init.numpy(),
                                 x_final.numpy(), tr.numpy(), None if rows is None else rows.numpy(),
                                 None if count is None else count.numpy())
        return {k: torch.from_numpy(np.asarray(v)) for k, v in o.items()}


def _problem(n=N_TOTAL):
    sc = pb.synthetic_di(n, K=K, seed=4, spread=3.0)  # close starts/goals -> active coupling
    return sc


def _run(rank, world, port, q):
    import scvx_hip
    from scvx_hip.scvx import CouplingSpec, JacobiSCvx
    if world > 1:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    sc = _problem()
    n_loc = N_TOTAL // world
    sl = slice(rank * n_loc, (rank + 1) * n_loc)
    T = lambda a: torch.tensor(np.ascontiguousarray(a))
    spec = scvx_hip.QPSpec(model="di", K=K, box=[(0, -20, 20)], j_max=N_TOTAL - 1, w_coll=1e4, tol=1e-10, max_iter=80)
    drv = JacobiSCvx(spec, T(sc["x_init"][sl]), T(sc["x_final"][sl]), T(sc["sigma"][sl]), 0.3,
                     coupling=CouplingSpec(R=1.0), tr_rule="global", backend=OracleBackend())
    X, U = T(sc["X"][sl]).clone(), T(sc["U"][sl]).clone()
    for _ in range(ITERS):
        Xn, Un, out = drv.step(X, U)
        X, U = Xn.clone(), Un.clone()
    assert drv.last_check["violated"] == 0   # every row is in the solve (j_max = N_total - 1)
    q.put((rank, X.numpy(), drv.tr.numpy(), int(out["status"].max())))
    if world > 1:
        torch.distributed.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_sharded_jacobi_matches_single_process():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    _run(0, 1, 0, q)
    _, X_single, tr_single, st = q.get()
    assert st == 0
    port = _free_port()
    procs = [ctx.Process(target=_run, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict((r, (x, tr, s)) for r, x, tr, s in (q.get(timeout=300) for _ in procs))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    X_multi = np.concatenate([res[0][0], res[1][0]])
    np.testing.assert_array_equal(X_multi, X_single)
    np.testing.assert_array_equal(res[0][1], tr_single[:N_TOTAL // 2])
    assert all(res[r][2] == 0 for r in res)
    # the coupling is live: some node of some agent is pushed by a neighbour row
    assert not np.allclose(X_single, _problem()["X"])


N_CULL, J_MAX = 8, 2


def _run_culled(rank, world, port, q, order=None):
    """The culled coupling path of the C4 / C5 configurations: the QP keeps the J_MAX nearest rows per node,
    every reference row is checked at the solution, violating agents are re-solved with all N - 1 rows
    (j_max_hi), the global trust-region rule all-reduces the cost.  order: agent order of the shards
    (scvx_hip.scvx.balanced_order; rank r owns order[r*n:(r+1)*n]); None = contiguous."""
    import scvx_hip
    from scvx_hip.scvx import CouplingSpec, JacobiSCvx
    if world > 1:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    sc = _problem(N_CULL)
    if order is not None:
        sc = {k: (v[order] if isinstance(v, np.ndarray) and v.shape[:1] == (N_CULL,) else v) for k, v in sc.items()}
    n_loc = N_CULL // world
    sl = slice(rank * n_loc, (rank + 1) * n_loc)
    T = lambda a: torch.tensor(np.ascontiguousarray(a))
    spec = scvx_hip.QPSpec(model="di", K=K, box=[(0, -20, 20)], j_max=J_MAX, w_coll=1e4, tol=1e-10, max_iter=80)
    drv = JacobiSCvx(spec, T(sc["x_init"][sl]), T(sc["x_final"][sl]), T(sc["sigma"][sl]), 0.3,
                     coupling=CouplingSpec(R=1.0, j_max_hi=N_CULL - 1), tr_rule="global", backend=OracleBackend())
    X, U = T(sc["X"][sl]).clone(), T(sc["U"][sl]).clone()
    checks = []
    for _ in range(ITERS):
        Xn, Un, out = drv.step(X, U)
        X, U = Xn.clone(), Un.clone()
        checks.append(dict(drv.last_check))
    q.put((rank, X.numpy(), drv.tr.numpy(), checks, int(out["status"].max())))
    if world > 1:
        torch.distributed.destroy_process_group()


def test_sharded_culled_coupling_matches_single_process():
    """World 1 against world 2 (gloo) on the culled path: bit-identical iterates and radii, and the check's
    counts (violated / re-solved / overflow) summed over the ranks equal to the single process's, at every
    step.  The dropped rows bind here (some agents violate and are re-solved), so the re-solve path runs."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    _run_culled(0, 1, 0, q)
    _, X_single, tr_single, ck_single, st = q.get()
    assert st == 0
    assert sum(c["violated"] for c in ck_single) > 0           # the culled rows bind: the re-solve path ran
    assert all(c["overflow"] == 0 for c in ck_single)           # and made every step exact
    port = _free_port()
    procs = [ctx.Process(target=_run_culled, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict((r, (x, tr, ck, s_)) for r, x, tr, ck, s_ in (q.get(timeout=300) for _ in procs))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    np.testing.assert_array_equal(np.concatenate([res[0][0], res[1][0]]), X_single)
    np.testing.assert_array_equal(res[0][1], tr_single[:N_CULL // 2])
    for k in range(ITERS):
        for key in ("violated", "resolved", "overflow"):
            assert res[0][2][k][key] + res[1][2][k][key] == ck_single[k][key], (k, key)


def test_balanced_shard_order_matches_single_process():
    """Shards of a non-identity agent order (scvx_hip.scvx.balanced_order: every rank gets the same mix of
    per-agent IPM iteration counts): gloo world 2 gives bit-identical iterates, radii and check counts to one
    process owning all agents in that order.  Against the contiguous order the iterates agree to the
    subproblems' accuracy, not bitwise: a node's collision rows are listed in neighbour-index order, so the order
    changes the IPM's summation order, and the shared collision slack makes the coupled subproblem LP-like in S
    (its minimiser is not unique).  The Jacobi update itself is order-free."""
    from scvx_hip.scvx import balanced_order
    iters = np.array([9, 5, 5, 12, 5, 6, 14, 5])          # e.g. the last step's IPM iterations
    order = balanced_order(iters, 2)
    assert sorted(order.tolist()) == list(range(N_CULL)) and not np.array_equal(order, np.arange(N_CULL))
    assert {14, 12} & set(iters[order[:4]].tolist()) in ({14}, {12})      # the two longest solves split
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    _run_culled(0, 1, 0, q, order)
    _, X_single, tr_single, ck_single, st = q.get()
    assert st == 0
    port = _free_port()
    procs = [ctx.Process(target=_run_culled, args=(r, 2, port, q, order)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict((r, (x, tr, ck, s_)) for r, x, tr, ck, s_ in (q.get(timeout=300) for _ in procs))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    np.testing.assert_array_equal(np.concatenate([res[0][0], res[1][0]]), X_single)
    np.testing.assert_array_equal(np.concatenate([res[0][1], res[1][1]]), tr_single)
    for k in range(ITERS):
        for key in ("violated", "resolved", "overflow"):
            assert res[0][2][k][key] + res[1][2][k][key] == ck_single[k][key], (k, key)
    _run_culled(0, 1, 0, q)                                   # contiguous order, one process
    _, X_contig, _, ck_contig, _ = q.get()
    inv = np.argsort(order)
    np.testing.assert_allclose(X_single[inv], X_contig, rtol=0, atol=1e-3)
    assert [c["overflow"] for c in ck_single] == [c["overflow"] for c in ck_contig] == [0] * ITERS


@pytest.mark.parametrize("balanced", [False, True])
def test_world4_culled_coupling_matches_single_process(balanced):
    """The C4 path at world 4 (gloo; the 8-GPU driver run deals 512 agents per rank the same way): the culled
    coupling rows, the full-row check and the re-solve of violating agents, the global trust-region rule's scalar
    all_reduce -- contiguous or balanced shards (scvx_hip.scvx.balanced_order over 4 ranks).  Bit-identical iterates,
    radii and per-step check counts to one process owning all agents in the same order."""
    from scvx_hip.scvx import balanced_order
    order = None
    if balanced:
        order = balanced_order(np.array([9, 5, 5, 12, 5, 6, 14, 5]), 4)
        assert sorted(order.tolist()) == list(range(N_CULL))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    _run_culled(0, 1, 0, q, order)
    _, X_single, tr_single, ck_single, st = q.get()
    assert st < 2
    port = _free_port()
    procs = [ctx.Process(target=_run_culled, args=(r, 4, port, q, order)) for r in range(4)]
    for p in procs:
        p.start()
    res = dict((r, (x, tr, ck, s_)) for r, x, tr, ck, s_ in (q.get(timeout=300) for _ in procs))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    np.testing.assert_array_equal(np.concatenate([res[r][0] for r in range(4)]), X_single)
    np.testing.assert_array_equal(np.concatenate([res[r][1] for r in range(4)]), tr_single)
    for k in range(ITERS):
        for key in ("violated", "resolved", "overflow"):
            assert sum(res[r][2][k][key] for r in range(4)) == ck_single[k][key], (k, key)


def _run_indep(rank, world, port, q):
    """The headline's C3 form: independent agents (no coupling), the reference's global trust-region rule over every
    rank's agents (one scalar all_reduce per step, JacobiSCvx tensor path; the fused kernel path does the same with a
    fixed-order local sum, tests/test_jacobi_update_gpu.py)."""
    import scvx_hip
    from scvx_hip.scvx import JacobiSCvx
    if world > 1:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    sc = pb.synthetic_di(N_TOTAL, K=K, seed=7, spread=6.0)
    n_loc = N_TOTAL // world
    sl = slice(rank * n_loc, (rank + 1) * n_loc)
    T = lambda a: torch.tensor(np.ascontiguousarray(a))  # noqa: E731
    spec = scvx_hip.QPSpec(model="di", K=K, box=[(0, -20, 20)], tol=1e-10, max_iter=80)
    drv = JacobiSCvx(spec, T(sc["x_init"][sl]), T(sc["x_final"][sl]), T(sc["sigma"][sl]), 0.3, tr_rule="global",
                     backend=OracleBackend())
    X, U = T(sc["X"][sl]).clone(), T(sc["U"][sl]).clone()
    totals = []
    for _ in range(ITERS + 1):
        X, U, out = drv.step(X, U)
        X, U = X.clone(), U.clone()
        totals.append(float(drv.prev_total.item()))
    q.put((rank, X.numpy(), drv.tr.numpy(), totals, int(out["status"].max())))
    if world > 1:
        torch.distributed.destroy_process_group()


def test_sharded_global_rule_independent_agents_matches_single_process():
    """bench.py's default line at --gpus 2 (C3 form: every rank its own agents, the global rule's summed cost
    all-reduced): world 2 (gloo) against one process owning all agents -- the same totals (to the summation order's
    rounding), the same radius and the same iterates at every step."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    _run_indep(0, 1, 0, q)
    _, X_single, tr_single, tot_single, st = q.get()
    assert st == 0
    port = _free_port()
    procs = [ctx.Process(target=_run_indep, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict((r, (x, tr, tot, s)) for r, x, tr, tot, s in (q.get(timeout=300) for _ in procs))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    np.testing.assert_allclose(res[0][2], tot_single, rtol=1e-13)
    np.testing.assert_allclose(res[1][2], tot_single, rtol=1e-13)
    np.testing.assert_array_equal(np.concatenate([res[0][1], res[1][1]]), tr_single)
    np.testing.assert_array_equal(np.concatenate([res[0][0], res[1][0]]), X_single)
    assert all(res[r][3] == 0 for r in res)

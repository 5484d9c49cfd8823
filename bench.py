"""Benchmark: SCvx-iterations/sec of the batched SCvx inner loop on MI355X.

Workload (BASELINE.json metric, config C3 of SURVEY §8(d)): per GPU, N=1024 agents, 3-D double
integrator (n=6, m=3), K=50 nodes, sigma=30 s (h=0.6 s as Distributed_opt/dist_scvx_3d.py:200-204),
trust region 0.25 (:207), 8 static spherical obstacles as linearized soft halfspaces
(single_integrator_model.py:113-126 semantics, weight 1e6), per-node SOC ||u_t|| <= 1.0
(:103-104 semantics), box |x|,|y| <= 12 (dist_scvx_3d.py:87-90 widened), straight-line warm start.

One SCvx iteration (= one "step") = batched FOH discretization (scvx_foh_batched) + batched
trust-region QP/SOCP solve to tolerance (scvx_qp_solve_batched) + trust-region bookkeeping, all
on device; inputs resident in HBM.  The headline `value` runs the reference's outer rule
(dist_scvx_3d.py:248-252: one trust radius, halved when the summed cost rises); the same invocation
then times this build's per-agent rule (each agent's radius halves on its own cost increase) from the
same initial iterate, with its own warmup, reported under `other_rule` (`--rules one` skips it).
Multi-GPU (--gpus N under torch.distributed.run): weak scaling, each rank owns its own 1024 agents; the
only exchange is the global rule's summed cost (one scalar all_reduce per step, RCCL); `value` counts
the N_gpus * 1024-agent SCvx iterations completed per second.

Also reported: roofline of the dominant kernel (qp_ipm_kernel, FP64 FLOP rate vs the FP64 peak,
timed with HIP events on the launch stream) and a CPU baseline (the C++ restatement of the same
algorithm, oracle/scvx_cpu.cpp + oracle/foh_ref.c, on a bounded agent sample, the headline's rule).

Optional workloads (--config; the default c3 is the headline line the driver records):
  c2  BASELINE.json configs[1]: N=128 double-integrator agents per GPU (seed 0, no
      obstacles, no SOC, box |x|,|y| <= 12), both rules as c3.
  c4  N=4096 double-integrator agents in total on a 16^3 lattice (spacing 6 > 2R, R=2.3) with
      permuted goals, pairwise collision coupling (dist_scvx_3d.py:93-107, one shared slack per node,
      the j_max=8 nearest neighbours per node kept), global trust-region rule (:248-252).  Agents
      are sharded contiguously over ranks; one RCCL all_gather of the states per iteration feeds the
      collision linearization (strong scaling: the 4096-agent problem is fixed).
  c5  N=1024 12-state quadrotors (models.hpp) from hover, 8 obstacles, coupling as c4 with R=0.5
      (strong scaling); the subproblem carries virtual control (QPSpec.w_nu = 1e4: nu_t in the dynamics
      priced w_nu ||nu_t||_1, the SCvx form of sc_problem.py:60-68) and a proximal state term
      (QPSpec.w_prox = 10), so it stays feasible under the Jacobi update of a nonlinear model.
"""
import argparse
import json

import numpy as np
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "dynamic-programming-multiagent-trajectory-optimiziation_amd"))
sys.path.insert(0, REPO)

N_AGENTS = 1024
K = 50
SIGMA = 30.0
TR0 = 0.25
U_MAX = 1.0
N_OBS = 8
BOX = [(0, -12.0, 12.0), (1, -12.0, 12.0)]
C5_W_NU, C5_W_PROX = 1e4, 10.0   # c5 subproblem: virtual control weight (WEIGHT_NU, global_parameters.py) and proximal term
FP64_PEAK_TFLOPS = 78.6   # MI355X FP64 vector (= FP64 matrix) dense peak, spec
HBM_PEAK_GBS = 8000.0


def foh_bytes_per_agent(n, m, K):
    """Algorithmic HBM bytes of the FOH stage per agent: read X (K,n), U (K,m), sigma;
    write disc (K-1, n(n+2m+2)).  DI, K=50: 36,536 B."""
    return 8 * (K * n + K * m + 1) + 8 * (K - 1) * n * (n + 2 * m + 2)


def foh_flops_per_agent(n, m, K, nsub=1, f_flops=None):
    """Algorithmic FLOPs of the FOH stage per agent: per RK4 step 4 RHS evaluations of
    F + 2n^3 + 4n^2 m + 7n^2 + 7nm + 4n + 3m (F = model f/A/B, dense mat-vecs 2(n^2 + nm): DI 108) plus
    11 L for the RK4 combination, L = n + n^2 + 2nm + 2n.  DI, K=50: 6,522 per interval-substep."""
    F = f_flops if f_flops is not None else 2 * (n * n + n * m)
    L = n + n * n + 2 * n * m + 2 * n
    rhs = F + 2 * n ** 3 + 4 * n * n * m + 7 * n * n + 7 * n * m + 4 * n + 3 * m
    return (K - 1) * nsub * (4 * rhs + 11 * L)


def qp_bytes_per_agent(n, m, K, j_max=0, pos_dim=3):
    """Algorithmic (interface) HBM bytes of one QP solve per agent: in disc, Xref, Uref, x_init, x_final,
    tr, sigma (+ collision rows and counts); out X, U, shared slack, obj, status, iters.  DI, K=50, no
    coupling: 36,640 + 4,016 = 40,656 B (~42.7 KB incl. the SCP-form outputs)."""
    b_in = 8 * ((K - 1) * n * (n + 2 * m + 2) + K * n + K * m + 2 * n + 2)
    b_in += (8 * K * j_max * (pos_dim + 1) + 4 * K) if j_max else 0
    b_out = 8 * (K * n + K * m + K + 1) + 8
    return b_in + b_out


def qp_flops_per_ipm_iter(n, m, K, rows):
    """Algorithmic FP64 FLOPs of one IPM iteration of one agent, SURVEY §8(d)'s count: the block-banded
    KKT factorization with block size b = n+m, (b^3/3 + 2 b^3) K, plus the residual / assembly work over
    the inequality rows, 2 (n+m) FLOPs per row per node.  DI (b=9), K=50, 32 rows: 85,050 + 28,800 =
    113,850 (~0.12 MFLOP).  The two Riccati solves per iteration are not counted: a lower bound."""
    b = n + m
    return K * (b ** 3 / 3 + 2 * b ** 3) + K * rows * 2 * (n + m)


def qp_rows(n, m, n_box, n_obs, j_max, soc):
    """Inequality rows per node of the QP template: 2^m trust-region facets, 2 per box constraint, an
    obstacle row and its slack sign row per obstacle, j_max collision rows + 1 shared-slack row, and the
    (m+1)-dimensional SOC counted as m+1 rows."""
    return (1 << m) + 2 * n_box + 2 * n_obs + (j_max + 1 if j_max else 0) + ((m + 1) if soc else 0)


def committed_traffic(kernel_prefix="scvx::qp_ipm_kernel<scvx::QPCfg<6, 3, 2, 8, 0, 0>"):
    """HBM-side bytes per launch of the dominant kernel from the newest committed rocprofv3 --pmc
    summary (profiles/*_pmc_traffic.json, made by tools/pmc_summary.py from separate FETCH_SIZE /
    WRITE_SIZE passes of this same bench, gfx950 FETCH_SIZE x2 correction applied); None if absent."""
    import glob
    files = sorted(glob.glob(os.path.join(REPO, "profiles", "*_pmc_traffic.json")))  # round-tagged names
    for f in reversed(files):
        d = json.load(open(f))
        if str(d.get("kernel", "")).startswith(kernel_prefix) and "traffic_bytes" in d:   # tools/pmc_summary.py
            return d["traffic_bytes"], os.path.relpath(f, REPO)
        for k, v in d.items():                                                            # round-1 format
            if k.startswith(kernel_prefix) and isinstance(v, dict):
                return v["traffic_bytes"], os.path.relpath(f, REPO)
    return None, None


def make_workload(N, seed, device, obstacles=N_OBS):
    import torch
    from scvx_hip import workloads
    sc = workloads.synthetic_di(N, K=K, seed=seed, sigma=SIGMA, obstacles=obstacles)
    t = {k: torch.tensor(sc[k], device=device) for k in ("X", "U", "x_init", "x_final", "sigma")}
    return sc, t


def make_coupled(config, world, rank, device):
    """c4 / c5: the full problem is built identically on every rank, each rank keeps its block."""
    import torch
    from scvx_hip import workloads
    if config == "c4":
        sc = workloads.synthetic_lattice(side=16, K=K, seed=2, sigma=SIGMA)
        model, R, obs, box, j_max = "di", 2.3, [], [(0, -50.0, 50.0), (1, -50.0, 50.0)], 8   # lattice spans +-45
    else:
        sc = workloads.synthetic_quad(1024, K=K, seed=3, sigma=SIGMA, obstacles=N_OBS)
        model, R, obs, box, j_max = "quad", 0.5, sc["obs"], workloads.QUAD_BOX, 8
    vc = dict(w_nu=C5_W_NU, w_prox=C5_W_PROX) if config == "c5" else {}
    N_total = sc["X"].shape[0]
    if N_total % world:
        raise SystemExit(f"{config}: {N_total} agents do not shard over {world} ranks")
    n_loc = N_total // world
    t = shard_tensors(sc, np.arange(rank * n_loc, (rank + 1) * n_loc), device)
    return sc, t, dict(model=model, R=R, obs=obs, box=box, j_max=j_max, N_total=N_total, n_loc=n_loc, vc=vc)


def shard_tensors(sc, idx, device):
    """The agents `idx` of a coupled construction (a contiguous block, or a balanced order's block) on device."""
    import torch
    return {k: torch.tensor(np.ascontiguousarray(sc[k][idx]), device=device)
            for k in ("X", "U", "x_init", "x_final", "sigma")}


def host_info():
    """What the CPU baseline ran on: nproc (CPUs this process may use), the machine's CPU count, the
    cgroup CPU quota if one is set, and the CPU model."""
    info = {"nproc": len(os.sched_getaffinity(0)), "cpu_count": os.cpu_count()}
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        info["cgroup_cpu_quota"] = None if q == "max" else float(q) / float(per)
    except (OSError, ValueError):
        info["cgroup_cpu_quota"] = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                info["cpu_model"] = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return info


def cpu_jacobi(sc, n_sample, threads, warmup, steps, tol=1e-8, max_seconds=30.0, warm_status=1, tr_rule="per_agent",
               soc=True):
    """The CPU restatement of the timed region, like for like: the same warm-started Jacobi loop as the GPU
    line (JacobiSCvx with the bench's settings) on the first n_sample agents -- per step the FOH
    (oracle/foh_ref.c), the QP twin (oracle/scvx_cpu.cpp, the kernel's algorithm, started from the previous
    step's primal-dual point exactly as the kernel's warm rule: warm = last status <= warm_status) and the per-agent
    trust-region bookkeeping of csrc/jacobi.hip (tie margin 1e-9; tr_rule "global": the reference's one radius, halved
    when the summed cost rises, JacobiSCvx's global rule -- summed over the n_sample agents simulated here: with
    n_sample = N on one GPU that is the GPU line's own sum; at --gpus > 1 the GPU line all-reduces the sum over every
    rank's agents, so there the CPU leg's halving decisions are a one-rank approximation).  `warmup` untimed steps,
    then up to `steps`
    timed steps (fewer if max_seconds runs out first).  Returns (SCvx iterations/s scaled to the N=1024-agent
    workload, timed steps, seconds, mean IPM iterations per agent over the timed steps)."""
    from oracle import foh_oracle, qp_cpu
    n_agents = sc["X"].shape[0]   # the GPU line's agents per GPU: the rate is scaled to that workload
    tpl = qp_cpu.make_template(6, 3, K, box=BOX, obs=sc["obs"], w_obs=1e6, u_max=U_MAX if soc else None, tol=tol,
                               max_iter=60)
    n = n_sample
    X, U = sc["X"][:n].copy(), sc["U"][:n].copy()
    sig, xi, xf = sc["sigma"][:n], sc["x_init"][:n], sc["x_final"][:n]
    tr = np.full(n, TR0)
    prev = np.full(n, np.inf)
    prev_total = np.inf
    wstate = np.zeros((n, qp_cpu.warm_doubles(tpl)))
    warm = None
    disc = np.zeros((n, K - 1, 6 * (6 + 6 + 2)))
    timed, t_el, it_sum = 0, 0.0, 0
    for k in range(warmup + steps):
        t0 = time.perf_counter()
        for a in range(n):
            disc[a] = foh_oracle.foh_disc("di", X[a], U[a], sig[a])
        o = qp_cpu.solve_batched(tpl, disc, sig, X, U, xi, xf, tr, nthreads=threads, warm=warm, wstate=wstate)
        ok = o["status"] != 2
        X = np.where(ok[:, None, None], o["X"], X)
        U = np.where(ok[:, None, None], o["U"], U)
        cost = (U[:, :-1] ** 2).sum(axis=(1, 2))
        if tr_rule == "global":
            tr = tr * (0.5 if cost.sum() > prev_total else 1.0)
            prev_total = cost.sum()
        else:
            tr = np.where(cost > prev * (1.0 + 1e-9), 0.5 * tr, tr)
        tr = np.where(ok, tr, 0.5 * tr)
        prev = cost
        warm = (o["status"] <= warm_status).astype(np.int32)
        if k >= warmup:
            t_el += time.perf_counter() - t0
            timed += 1
            it_sum += int(o["iters"].sum())
            if t_el >= max_seconds:
                break
    return timed * (n / n_agents) / t_el, timed, t_el, it_sum / (timed * n)


def cpu_baselines(sc, n_sample, tol, warmup, steps, warm_status=1, tr_rule="per_agent", obstacles=True, soc=True):
    """All-core and single-core CPU figures of the restatement on the GPU line's own loop (cpu_jacobi).  "All
    cores" is every CPU this process may run on: nproc, capped by the cgroup CPU quota when one is set (the GPU
    box grants 16 CPUs of a 256-thread host; more OpenMP threads than that only time-slice)."""
    info = host_info()
    quota = info.get("cgroup_cpu_quota")
    threads = max(1, min(info["nproc"], int(quota))) if quota else info["nproc"]
    v_all, steps_all, el, it_all = cpu_jacobi(sc, n_sample, threads, warmup, steps, tol=tol, warm_status=warm_status,
                                              tr_rule=tr_rule, soc=soc)
    n1 = min(n_sample, 64)
    v_one, steps1, el1, it1 = cpu_jacobi(sc, n1, 1, warmup, steps, tol=tol, warm_status=warm_status, tr_rule=tr_rule,
                                         soc=soc)
    N_ = sc["X"].shape[0]
    return dict(value=v_all, unit=f"SCvx-iterations/s (N={N_}-agent equivalent)", cores=threads, kind="port",
                tr_rule=tr_rule,
                sample=f"warm-started steady state, steps {warmup + 1}-{warmup + steps_all} of the GPU line's Jacobi "
                       f"loop ({warmup} untimed warm-up steps first, {tr_rule} trust-region rule) on {n_sample} of the "
                       f"{N_} agents: FOH C + "
                       f"the kernel's IPM in C++ with the same warm start and trust-region bookkeeping, -O3 x86-64-v3, "
                       f"OpenMP over agents on {threads} threads = the CPUs this process may use (nproc "
                       f"{info['nproc']}, cgroup quota {quota}); {el:.1f} s timed",
                ipm_iters_per_agent=it_all,
                single_core={"value": v_one, "cores": 1, "ipm_iters_per_agent": it1,
                             "sample": f"steps {warmup + 1}-{warmup + steps1} of the same loop on {n1} agents, 1 thread, "
                                       f"{el1:.1f} s timed"},
                host=info)


def is_flops_per_rollout(n, m, nsub):
    """Single-integrator roll-out to t: nsub RK4 steps (4 f-evals of m interpolation FMAs, 3 stage
    updates + final combination over n) + projection and norm."""
    return nsub * (4 * 2 * m + 3 * 2 * n + 4 * n) + 3 * n + 2


def bench_intersample(args, world, rank, device):
    """--config is: the inter-sample clearance scan (scvx_intersample_batched) over C3-sized data --
    N=1024 single-integrator agents (the reference's intersample user, game_si_model.py:156-176),
    K=50, the 8 C3 spheres, T = I, dt = 1, 100 samples.  value = segment x obstacle scans / s."""
    import torch
    import scvx_hip
    from scvx_hip import workloads
    N = args.agents
    sc = workloads.synthetic_di(N, K=K, seed=1 + rank, sigma=1.0, obstacles=N_OBS)
    X = np.ascontiguousarray(sc["X"][:, :, 0:3])
    U = np.repeat(((sc["x_final"] - sc["x_init"])[:, 0:3])[:, None, :], K, 1)   # straight-line velocities
    U = U + np.random.default_rng(7).normal(0, 0.5, U.shape)
    T = lambda a: torch.tensor(np.ascontiguousarray(a), dtype=torch.float64, device=device)  # noqa: E731
    Xd, Ud, sd = T(X), T(U), T(np.ones(N))
    obs = sc["obs"]
    run = lambda: scvx_hip.intersample_batched("si", Xd, Ud, sd, obs, max_crit=8)  # noqa: E731
    for _ in range(args.warmup):
        out = run()
    torch.cuda.synchronize()
    st = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(st)
    for _ in range(args.steps):
        out = run()
    e1.record(st)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    kms = e0.elapsed_time(e1) / args.steps
    scans = N * (K - 1) * len(obs)
    minima = int(out["n_crit"].sum().item())
    flops = scans * 2 * 100 * is_flops_per_rollout(3, 3, 1)   # grid phi only: a lower bound
    achieved = flops / (kms * 1e-3) / 1e12
    cpu = None
    if not args.no_cpu:
        from oracle import intersample_np
        t1, done = time.perf_counter(), 0
        while time.perf_counter() - t1 < 10.0:
            a, rem = divmod(done, (K - 1) * len(obs))
            k, o = divmod(rem, len(obs))
            a %= N
            intersample_np.segment("si", X[a, k], U[a, k], U[a, k + 1], 1.0 / (K - 1), np.eye(3), obs[o][0],
                                   obs[o][1], nsub=1)
            done += 1
        cel = time.perf_counter() - t1
        cpu = dict(value=done / cel, unit="segment-obstacle scans/s", cores=1, kind="port",
                   sample=f"{done} scans of the same workload (oracle/intersample_np.py, numpy, 1 thread), {cel:.1f} s")
    if rank != 0:
        return
    print(json.dumps({
        "metric": "inter-sample clearance scans/sec (segment x obstacle), N=1024 agents x K=50 x 8 obstacles",
        "value": scans / (el / args.steps), "unit": "scans/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": 1e3 * el / args.steps, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f64", "data": "synthetic (C3 starts/goals and spheres, SI velocities + noise)",
        "config": {"workload": "intersample: N=1024 SI agents, K=50, 8 spheres, T=I, dt=1, 100 samples, eps 1e-4",
                   "agents_per_gpu": N, "K": K, "parallelism": f"agents sharded x{world}"},
        "roofline": {"bound": "fp64_valu", "achieved": achieved, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": achieved / FP64_PEAK_TFLOPS, "traffic": None, "kernel": "intersample_kernel",
                     "kernel_ms": kms, "note": "FP64 VALU; algorithmic FLOPs = grid central differences only "
                                               "(lower bound: bisection / linearisation roll-outs not counted)"},
        "minima_found": minima, "cpu_baseline": cpu}), flush=True)


def bench_scproblem(args, world, rank, device):
    """--config scp: the SCProblem path (SCvx/optimization/sc_problem.py + scvx_solver.py) -- N=1024
    independent unicycle agents (the reference's UnicycleModel, K=100 = global_parameters.K, 3
    obstacles) stepping BatchedSCVXSolver in lockstep: one FOH launch + one scvx_scp_solve_batched
    launch + device metrics per step.  Convergence is disabled so exactly `steps` iterations run."""
    import torch
    sys.path.insert(0, os.path.join(REPO, "dynamic-programming-multiagent-trajectory-optimiziation_amd"))
    from SCvx.models.unicycle_model import UnicycleModel
    from SCvx.optimization.scvx_solver import BatchedSCVXSolver
    N = args.agents
    rng = np.random.default_rng(1 + rank)
    models = [UnicycleModel(r_init=np.array([-8.0, -8.0, 0.0]) + np.r_[rng.uniform(-1, 1, 2), 0.0],
                            r_final=np.array([8.0, 8.0, 0.0]) + np.r_[rng.uniform(-1, 1, 2), 0.0]) for _ in range(N)]
    bat = BatchedSCVXSolver(models, device=device)
    bat.conv_tol = -1.0
    bat.max_iter = args.warmup
    bat.solve()
    torch.cuda.synchronize()
    bat.max_iter = args.steps
    t0 = time.perf_counter()
    bat.solve()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    iters = np.concatenate(bat.ipm_iters) if bat.ipm_iters else np.zeros(1)
    cpu = None
    if not args.no_cpu:
        from oracle import scp_problems as sp_, scp_cpu
        t1, done = time.perf_counter(), 0
        while time.perf_counter() - t1 < 10.0:
            m = models[done % N]
            p = sp_.scp_instance("unicycle", K=100, x_init=m.x_init, x_final=m.x_final)
            scp_cpu.SCPSolver(p, tol=1e-9).solve()
            done += 1
        cel = time.perf_counter() - t1
        cpu = dict(value=done / cel / N, unit="SCvx-iterations/s (N=1024-agent equivalent)", cores=1, kind="port",
                   sample=f"{done} SCProblem solves (oracle/scp_cpu.py numpy restatement, 1 thread; FOH excluded), "
                          f"{cel:.1f} s")
    if rank != 0:
        return
    print(json.dumps({
        "metric": "SCvx-iterations/sec of the SCProblem path, N=1024 unicycle agents x K=100",
        "value": world * args.steps / el, "unit": "SCvx-iterations/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": 1e3 * el / args.steps, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f64", "data": "synthetic (reference UnicycleModel defaults, jittered BCs)",
        "config": {"workload": "scp: BatchedSCVXSolver, N=1024 unicycle agents, K=100, 3 obstacles, ECOS-form LP",
                   "agents_per_gpu": N, "K": 100, "parallelism": f"agents sharded x{world}"},
        "ipm_iters_per_agent": float(iters.mean()), "ipm_iters_max": int(iters.max()),
        "cpu_baseline": cpu}), flush=True)


def bench_nash(args, world, rank, device):
    """--config nash: the Nash best-response path (SCvx/optimization/nash_solver.py + agent_best_response.py).
    (1) NashSolver, Gauss-Seidel (the reference's order), on the default 3-agent game (SCvx/config/
    default_game.py agents, K = global K = 100, warm start SCvx/utils/initial_guess.py): `steps` outer
    iterations (tol < 0, so exactly that many), each = 3 agents x max_acs_iters ACS solves; one agent per
    launch, so this is the latency-bound sequential path.  (2) The game kernel's throughput: N = 1024
    best responses (the three agents' first problems, neighbour positions jittered) in one
    scvx_scp_game_solve_batched launch, timed with HIP events on the launch stream."""
    import torch
    import scvx_hip
    sys.path.insert(0, os.path.join(REPO, "dynamic-programming-multiagent-trajectory-optimiziation_amd"))
    from SCvx.config import default_game as G
    from SCvx.global_parameters import K as KG
    from SCvx.models.game_model import GameUnicycleModel
    from SCvx.models.multi_agent_model import MultiAgentModel
    from SCvx.optimization.nash_solver import NashSolver
    from SCvx.optimization.sc_problem import _solver
    from SCvx.utils.initial_guess import initial_guess
    X0, U0 = (list(v) for v in zip(*(initial_guess(p["r_init"], p["r_final"], G.OBSTACLES, G.CLEARANCE, KG)
                                     for p in G.AGENT_PARAMS)))
    mam = MultiAgentModel(G.AGENT_PARAMS)
    for i, p in enumerate(G.AGENT_PARAMS):       # compare_admm_vs_nash.py:84-95
        mam.models[i] = GameUnicycleModel(**{k: p[k] for k in ("r_init", "r_final", "obstacles", "control_weight",
                                                               "collision_weight", "collision_radius",
                                                               "control_rate_weight", "curvature_weight")})
    ns = NashSolver(mam, max_iter=max(args.warmup, 1), tol=-1.0)
    ns.solve(X0, U0, 1.0)
    torch.cuda.synchronize()
    ns.max_iter = args.steps
    t0 = time.perf_counter()
    ns.solve(X0, U0, 1.0)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    solves = ns.solves
    # (2) batched throughput on the game kernel
    br = ns.br_solvers
    N = args.agents
    rng = np.random.default_rng(5 + rank)
    T = lambda a: torch.as_tensor(np.ascontiguousarray(a), dtype=torch.float64, device=device)  # noqa: E731
    ins = [b.scp.host_inputs() for b in br]
    pick = [a % len(br) for a in range(N)]
    args_b = {k: T(np.stack([ins[i][k] for i in pick]) if np.ndim(ins[0][k]) else [ins[i][k] for i in pick])
              for k in ins[0]}
    spec = br[0].spec()
    X_prev = T(np.stack([np.asarray(br[i].X_prev_param.require(), float).T for i in pick]))
    P = np.stack([np.stack([np.asarray(br[i].Y_params[j].require(), float).T for j in sorted(br[i].Y_params)])
                  for i in pick])
    P = T(P + rng.uniform(-0.05, 0.05, P.shape))
    z = scvx_hip.slab_update(X_prev, P, spec.pos_dim)
    solver = _solver(spec, N, device)
    for _ in range(2):
        solver.solve_game(X_prev=X_prev, slab_z=z, slab_P=P, **args_b)
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    reps = 5
    ev[0].record()
    for _ in range(reps):
        out = solver.solve_game(X_prev=X_prev, slab_z=z, slab_P=P, **args_b)
    ev[1].record()
    torch.cuda.synchronize()
    launch_ms = ev[0].elapsed_time(ev[1]) / reps
    st = out["status"].cpu().numpy()
    it = out["iters"].cpu().numpy()
    cpu = None
    if not args.no_cpu:
        from oracle import nash_ref, scp_problems as sp_
        b0 = br[0]
        i0 = b0.scp.host_inputs()
        p0 = G.AGENT_PARAMS[0]
        cons = sp_.model_constraints("unicycle", p0["r_init"], p0["r_final"], obstacles=G.OBSTACLES)
        wts = {k: p0[k] for k in ("control_weight", "control_rate_weight", "curvature_weight")}
        slabs = [(np.stack([zz.require() for zz in row]), np.asarray(b0.Y_params[j].require(), float).T)
                 for row, j in zip(b0.model.z_params, sorted(b0.Y_params))]
        pr = nash_ref.game_problem("unicycle", i0["Xref"], i0["Uref"], 1.0, cons, wts,
                                   np.asarray(b0.X_prev_param.require(), float).T, slabs, p0["collision_radius"],
                                   disc=nash_ref.disc_stacks(i0["disc"], 3, 2))
        t1, done = time.perf_counter(), 0
        while time.perf_counter() - t1 < 10.0:
            nash_ref.best_response(pr)
            done += 1
        cel = time.perf_counter() - t1
        cpu = dict(value=done / cel, unit="best-responses/s", cores=1, kind="port",
                   sample=f"{done} solves of agent 0's best response (oracle/nash_ref.py: the reference formulation, "
                          f"sparse conic IPM in numpy/scipy, 1 thread), {cel:.1f} s")
    if rank != 0:
        return
    print(json.dumps({
        "metric": "Nash best responses/sec (default 3-agent game, K=100), Gauss-Seidel IBR + ACS",
        "value": solves / el, "unit": "best-responses/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": 1e3 * el / args.steps, "ms_per_best_response": 1e3 * el / max(solves, 1),
        "higher_is_better": True, "scaling": "replicas only", "vs_baseline": None, "dtype": "f64",
        "data": "SCvx/config/default_game.py agents, initial_guess warm start",
        "config": {"workload": f"nash: NashSolver GS, 3 agents, K={KG}, max_acs_iters=5; an outer iteration = "
                               "3 x 5 best responses", "agents_per_gpu": 3, "K": KG, "parallelism": "none (GS order)"},
        "batched_game_kernel": {"agents": N, "launch_ms": launch_ms, "best_responses_per_s": N / (launch_ms * 1e-3),
                                "ipm_iters_mean": float(it.mean()), "ipm_iters_max": int(it.max()),
                                "status_counts": {str(k): int((st == k).sum()) for k in (0, 1, 2)}},
        "cpu_baseline": cpu}), flush=True)


def _free_port():
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def launch_ranks(args):
    """--gpus N > 1 without a torch.distributed environment: start the N ranks as a child process
    (python -m torch.distributed.run, one rank per GPU, rendezvous on 127.0.0.1) before this process
    touches the GPU, and exit with its return code."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def stage_times(marks_per_step):
    """Per-stage milliseconds (median over steps) from the (name, event) marks of JacobiSCvx.step, and
    the per-step GPU-timeline durations (consecutive 'start' marks, the last step to its last mark)."""
    stages, steps = {}, []
    for marks in marks_per_step:
        for (n0, e0), (n1, e1) in zip(marks[:-1], marks[1:]):
            stages.setdefault(n1, []).append(e0.elapsed_time(e1))
        steps.append(marks[0][1].elapsed_time(marks[-1][1]))
    return {k: float(np.median(v)) for k, v in stages.items()}, steps


def dry_run_shards(args, world, rank):
    """The coupled configs' shard arithmetic on CPU: every rank builds the full problem (make_coupled, host data
    only), keeps its block -- contiguous, or with --balance the block of scvx_hip.scvx.balanced_order over a
    deterministic stand-in for the first step's IPM iterations -- and the ranks all_gather their agent indices and a
    checksum of their initial states, so rank 0 can check that the shards tile the agents exactly once and that every
    rank holds the data of its own agents."""
    import torch
    import torch.distributed as dist
    from scvx_hip.scvx import balanced_order
    sc, w, cfg = make_coupled(args.config, world, rank, torch.device("cpu"))
    N_total, n_loc = cfg["N_total"], cfg["n_loc"]
    idx = np.arange(rank * n_loc, (rank + 1) * n_loc)
    if args.balance and world > 1:
        iters = 3 + (np.arange(N_total) * 2654435761 % 97) % 29     # stand-in iteration counts, 3..31
        order = balanced_order(iters, world)
        idx = order[rank * n_loc:(rank + 1) * n_loc]
        w = shard_tensors(sc, idx, torch.device("cpu"))
    mine = torch.tensor(idx, dtype=torch.int64)
    chk = torch.tensor([float(w["X"].sum()), float(w["x_final"].sum())], dtype=torch.float64)
    if world > 1:
        allidx = [torch.empty_like(mine) for _ in range(world)]
        allchk = [torch.empty_like(chk) for _ in range(world)]
        dist.all_gather(allidx, mine)
        dist.all_gather(allchk, chk)
    else:
        allidx, allchk = [mine], [chk]
    ok = True
    if rank == 0:
        cat = torch.cat(allidx).numpy()
        ok = bool(np.array_equal(np.sort(cat), np.arange(N_total)))
        for r in range(world):
            ir = allidx[r].numpy()
            ok = ok and bool(np.isclose(allchk[r][0].item(), sc["X"][ir].sum(), rtol=1e-12, atol=1e-9))
            ok = ok and bool(np.isclose(allchk[r][1].item(), sc["x_final"][ir].sum(), rtol=1e-12, atol=1e-9))
    return dict(N_total=N_total, agents_per_rank=n_loc, balanced=bool(args.balance and world > 1),
                shard_first_agents=[int(a[0]) for a in allidx], shards_tile_agents=ok)


def dry_run(args, world, rank):
    """--dry-run: the launcher / rendezvous / barrier / max-over-ranks timing path on CPU (gloo), with
    no GPU work -- used by tests/test_bench_cpu.py to check that --gpus N really runs N ranks; for c4 / c5
    also the shard arithmetic of the coupled configs (dry_run_shards)."""
    import torch
    import torch.distributed as dist
    if world > 1:
        dist.init_process_group("gloo")
        dist.barrier()
    shards = dry_run_shards(args, world, rank) if args.config in ("c4", "c5") else None
    t0 = time.perf_counter()
    for _ in range(args.steps):
        time.sleep(0.001)
    el_t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
    if world > 1:
        dist.barrier()
        dist.all_reduce(el_t, op=dist.ReduceOp.MAX)
    if rank == 0:
        line = {"metric": "dry-run", "value": None, "n_gpus": world, "steps": args.steps,
                "ms_per_step": 1e3 * el_t.item() / args.steps, "dry_run": True, "config": {"workload": args.config}}
        if shards is not None:
            line["config"].update(shards)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def timed_leg(drv, w, args, world, device):
    """Warmup + exactly args.steps timed SCvx iterations of `drv` from the initial iterate w (X, U), bracketed by a
    barrier + torch.cuda.synchronize() on both sides; the elapsed time is the max over ranks.  Every stage of a timed
    step is bracketed by HIP events on the launch stream (the QP kernel's mark pair gives its launch duration)."""
    import torch
    import torch.distributed as dist
    it_state = [w["X"].clone(), w["U"].clone()]   # the current iterate (X, U), rebound every step

    def step(marks=None):
        it_state[0], it_state[1], out = drv.step(it_state[0], it_state[1], marks=marks)
        return out

    hist = torch.empty((max(args.steps, 1), 2, w["X"].shape[0]), dtype=torch.int32, device=device)

    def record(out, i):
        """Per-step device-side bookkeeping of the timed region: ONE launch copies the step's IPM iteration counts
        and statuses into slot i of `hist` (reduced on the host after the timed region; no host sync inside it).  The
        warmup runs it too, so no torch kernel is loaded for the first time inside the timed region (a first use
        costs ~40-180 ms of module loading on a fresh box)."""
        torch.stack((out["iters"], out["status"]), out=hist[i])

    for _ in range(args.warmup):
        out = step()
        record(out, 0)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    marks, checks = [], []
    t0 = time.perf_counter()
    host_ms = []
    for i in range(args.steps):
        mk = []
        th = time.perf_counter()
        out = step(mk)
        host_ms.append(1e3 * (time.perf_counter() - th))
        marks.append(mk)
        record(out, i)
        if drv.last_check is not None:
            checks.append(dict(drv.last_check))
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    el_t = torch.tensor([el], dtype=torch.float64, device=device)
    if world > 1:
        dist.all_reduce(el_t, op=dist.ReduceOp.MAX)
    st_ms, step_ms = stage_times(marks)
    if world > 1:   # every rank's stage medians (the all-gather time per rank for c4/c5)
        mine = torch.tensor([st_ms.get(k, 0.0) for k in ("foh", "gather", "rows", "qp", "check", "update")],
                            dtype=torch.float64, device=device)
        allr = [torch.empty_like(mine) for _ in range(world)]
        dist.all_gather(allr, mine)
        per_rank = [r.tolist() for r in allr]
    else:
        per_rank = None
    h = hist[:args.steps].cpu().numpy()   # (steps, 2, N): IPM iterations, status
    its, status = h[-1, 0], h[-1, 1]
    N = its.size
    stats = [[int((h[i, 1] == k).sum()) for k in (0, 1, 2)] for i in range(args.steps)]
    return dict(
        el=el_t.item(), st_ms=st_ms, step_ms=step_ms, per_rank=per_rank, host_ms=host_ms, checks=checks,
        ipm_iters=float(h[:, 0].sum()),
        fields={
            "ms_per_step_median": float(np.median(step_ms)),
            "stage_ms_median": st_ms,
            "stage_ms_per_rank": per_rank,
            "ipm_iters_per_agent": float(h[:, 0].sum()) / (args.steps * N),
            "ipm_iters_max_last": int(its.max()),
            "ipm_iters_hist_last": {str(int(v)): int(c) for v, c in zip(*np.unique(its, return_counts=True))},
            "status_counts": {str(k): int((status == k).sum()) for k in (0, 1, 2)},
            "status_counts_per_step": stats,
            "step_ms": [round(v, 4) for v in step_ms],
            "host_ms_per_step": [round(v, 4) for v in host_ms],
            "gap_ms_between_steps": [round(a[-1][1].elapsed_time(b[0][1]), 4) for a, b in zip(marks[:-1], marks[1:])],
            "ipm_iters_max_per_step": [int(v) for v in h[:, 0].max(axis=1)],
            "min_frac_status_0_1": min((c[0] + c[1]) / N for c in stats),
            "coupling_check": checks or None,
        })


def leg_roofline(res, args, n, m, K_, N, rows, j_max, model, nsub):
    """Roofline of the dominant kernel (qp_ipm_kernel, FP64 FLOPs of SURVEY §8(d) x executed IPM iterations over
    its HIP-event launch time) and of the whole step (t_min / t) for one timed leg."""
    qp_ms = res["st_ms"]["qp"]
    qp_flops = qp_flops_per_ipm_iter(n, m, K_, rows) * res["ipm_iters"] / args.steps          # per launch
    qp_bytes = qp_bytes_per_agent(n, m, K_, j_max) * N
    foh_bytes = foh_bytes_per_agent(n, m, K_) * N
    foh_flops = foh_flops_per_agent(n, m, K_, nsub=nsub) * N
    achieved = qp_flops / (qp_ms * 1e-3) / 1e12
    qp_gbs = qp_bytes / (qp_ms * 1e-3) / 1e9
    t_step = res["el"] / args.steps
    t_min = (max(foh_bytes / (HBM_PEAK_GBS * 1e9), foh_flops / (FP64_PEAK_TFLOPS * 1e12))
             + max(qp_bytes / (HBM_PEAK_GBS * 1e9), qp_flops / (FP64_PEAK_TFLOPS * 1e12)))
    roof = {"bound": "fp64_valu", "achieved": achieved, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
            "frac": achieved / FP64_PEAK_TFLOPS, "kernel": "qp_ipm_kernel", "kernel_ms": qp_ms,
            "algorithmic_flops_per_launch": qp_flops, "algorithmic_bytes_per_launch": qp_bytes,
            "hbm_achieved_gbs": qp_gbs, "hbm_frac": qp_gbs / HBM_PEAK_GBS}
    step_roof = {"hbm_frac": (foh_bytes + qp_bytes) / (t_step * HBM_PEAK_GBS * 1e9),
                 "fp64_frac": (foh_flops + qp_flops) / (t_step * FP64_PEAK_TFLOPS * 1e12),
                 "t_min_ms": 1e3 * t_min, "t_min_over_t": t_min / t_step,
                 "algorithmic_bytes_per_step": foh_bytes + qp_bytes,
                 "algorithmic_flops_per_step": foh_flops + qp_flops}
    return roof, step_roof


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", choices=("c2", "c3", "c4", "c5", "is", "scp", "nash"), default="c3")
    ap.add_argument("--agents", type=int, default=None, help="c2 / c3: agents per GPU (default 128 / 1024)")
    ap.add_argument("--cpu-sample", type=int, default=1024)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--balance", action="store_true",
                    help="c4/c5 at --gpus > 1: deal agents to ranks by their first-step IPM iterations (DESIGN §6)")
    ap.add_argument("--tol", type=float, default=1e-8,
                    help="IPM relative stopping tolerance; default = Clarabel's defaults (tol_feas = tol_gap_rel = "
                         "1e-8), the solver of the reference's dist_scvx_3d.py:110")
    ap.add_argument("--dry-run", action="store_true", help="launcher/rendezvous check on CPU, no GPU work")
    ap.add_argument("--tensor-update", action="store_true", help="c2/c3 per-agent rule: bookkeeping as tensor ops "
                                                                  "(not csrc/jacobi.hip)")
    ap.add_argument("--tr-rule", default="global", choices=("per_agent", "global"),
                    help="c2/c3 trust-region rule of the headline `value`: global (the reference's one radius, halved "
                         "when the summed cost rises: Distributed_opt/dist_scvx_3d.py:248-252; at --gpus > 1 the sum "
                         "is all-reduced over every rank's agents) or per_agent (each agent's radius halves on its "
                         "own cost increase: this build's extension for independent agents)")
    ap.add_argument("--rules", default="both", choices=("both", "one"),
                    help="c2/c3: both -- also time the other trust-region rule in the same invocation (its own "
                         "warmup and timed steps, reported under `other_rule`); one -- only --tr-rule")
    ap.add_argument("--tie-rtol", type=float, default=1e-9,
                    help="per-agent trust-region rule: relative margin of the cost-increase test (JacobiSCvx.tie_rtol)")
    ap.add_argument("--dispatch-order", default="lpt", choices=("lpt", "none"),
                    help="QP dispatch order of the Jacobi loop (JacobiSCvx.dispatch_order): lpt deals the agents "
                         "longest-first by their previous solve's IPM iterations where they outnumber the resident "
                         "waves (c4); none: agent order")
    ap.add_argument("--warm-status", type=int, default=1, choices=(0, 1),
                    help="JacobiSCvx.warm_max_status: warm-start agents whose last solve had status <= this "
                         "(1: optimal_inaccurate iterates too -- they meet the reduced tolerances; C4 80 -> 85 "
                         "SCvx-it/s, no status change; C3 / C5 end every solve optimal, so it does not apply there)")
    args = ap.parse_args()
    if args.agents is None:
        args.agents = 128 if args.config == "c2" else N_AGENTS

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    if args.dry_run:
        return dry_run(args, world, rank)

    import torch
    import torch.distributed as dist
    import scvx_hip
    from scvx_hip.scvx import CouplingSpec, JacobiSCvx, balanced_order

    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    device = torch.device("cuda", local)
    if args.config == "is":
        return bench_intersample(args, world, rank, device)
    if args.config == "scp":
        return bench_scproblem(args, world, rank, device)
    if args.config == "nash":
        return bench_nash(args, world, rank, device)
    independent = args.config in ("c2", "c3")
    if independent:
        # C2 / C3: independent agents, weak scaling (each rank owns its own N agents; the global rule's
        # summed cost is the only exchange, one scalar all_reduce per step)
        N = args.agents
        c3 = args.config == "c3"
        sc, w = make_workload(N, seed=(1 if c3 else 0) + rank, device=device, obstacles=N_OBS if c3 else 0)
        model, box, j_max, n, m = "di", BOX, 0, 6, 3
        spec = scvx_hip.QPSpec(model="di", K=K, box=BOX, obs=sc["obs"], w_obs=1e6, u_max=U_MAX if c3 else None,
                               tol=args.tol, max_iter=60)
        n_obs = len(sc["obs"])
        soc = c3

        def make_drv(rule):
            return JacobiSCvx(spec, w["x_init"], w["x_final"], w["sigma"], TR0, tr_rule=rule, tie_rtol=args.tie_rtol,
                              fused_update=not args.tensor_update, warm_max_status=args.warm_status,
                              dispatch_order=args.dispatch_order)
        rules = [args.tr_rule] + ([r for r in ("global", "per_agent") if r != args.tr_rule] if args.rules == "both"
                                  else [])
        drv = make_drv(rules[0])
    else:
        sc, w, cfg = make_coupled(args.config, world, rank, device)
        N, model, box, j_max = cfg["n_loc"], cfg["model"], cfg["box"], cfg["j_max"]
        n, m = scvx_hip.MODEL_DIMS[model]
        n_obs = len(cfg["obs"])
        soc = False
        spec = scvx_hip.QPSpec(model=model, K=K, box=box, obs=cfg["obs"], w_obs=1e6, j_max=j_max, w_coll=1e4,
                               tol=args.tol, max_iter=60, **cfg["vc"])
        drv = JacobiSCvx(spec, w["x_init"], w["x_final"], w["sigma"], TR0, coupling=CouplingSpec(R=cfg["R"]),
                         tr_rule="global", warm_max_status=args.warm_status, dispatch_order=args.dispatch_order)
        rules = ["global"]
        if args.balance and world > 1:
            # one untimed step on contiguous shards measures every agent's IPM iterations; the shards are then
            # re-dealt so each rank gets the same mix (scvx_hip.scvx.balanced_order), and the run
            # restarts from the initial iterate on the new shards (the warmup steps follow as usual)
            _, _, out0 = drv.step(w["X"].clone(), w["U"].clone())
            it_loc = out0["iters"].to(torch.int32).contiguous()
            allit = [torch.empty_like(it_loc) for _ in range(world)]
            dist.all_gather(allit, it_loc)
            order = balanced_order(torch.cat(allit).cpu().numpy(), world)
            w = shard_tensors(sc, order[rank * N:(rank + 1) * N], device)
            drv = JacobiSCvx(spec, w["x_init"], w["x_final"], w["sigma"], TR0, coupling=CouplingSpec(R=cfg["R"]),
                             tr_rule="global", warm_max_status=args.warm_status, dispatch_order=args.dispatch_order)
    rows = qp_rows(n, m, len(box), n_obs, j_max, soc)
    nsub = drv.nsub   # the FOH substeps the timed loop ran (scvx_hip.default_nsub for its interval)
    res = timed_leg(drv, w, args, world, device)
    roof, step_roof = leg_roofline(res, args, n, m, K, N, rows, j_max, model, nsub)
    primary_cfg = dict(tr_rule=drv.tr_rule, qp_dispatch="longest-first (last-step IPM iterations)"
                       if getattr(drv, "_lpt", False) else "agent order")
    other = None
    if independent and len(rules) > 1:
        del drv
        drv2 = make_drv(rules[1])
        res2 = timed_leg(drv2, w, args, world, device)
        roof2, step_roof2 = leg_roofline(res2, args, n, m, K, N, rows, j_max, model, nsub)
        other = dict(tr_rule=rules[1], value=world * args.steps / res2["el"], unit="SCvx-iterations/s",
                     ms_per_step=1e3 * res2["el"] / args.steps, **res2["fields"],
                     roofline={k: roof2[k] for k in ("achieved", "frac", "kernel_ms")}, step_roofline=step_roof2)
    t_step = res["el"] / args.steps
    traffic, traffic_src = committed_traffic() if args.config == "c3" else (None, None)
    if rank == 0:
        cpu = None
        if not args.no_cpu and independent:
            cpu = cpu_baselines(sc, min(args.cpu_sample, N), tol=args.tol, warmup=args.warmup, steps=args.steps,
                                warm_status=args.warm_status, tr_rule=rules[0], obstacles=n_obs > 0, soc=soc)
        rule_txt = ("global trust-region rule (dist_scvx_3d.py:248-252: one radius, halved when the summed cost rises)"
                    if rules[0] == "global" else "per-agent trust-region rule (this build's extension)")
        if independent:
            value, scaling = world * args.steps / res["el"], "weak"
            metric = f"SCvx-iterations/sec, N agents x K=50 nodes (N={N} per GPU)"
            if args.config == "c3":
                data = "synthetic (C3 construction, SURVEY §8d: seeded random starts/goals, 8 spheres)"
                workload = (f"C3: N={N} agents/GPU, 3-D double integrator n=6 m=3, K=50, FOH sigma=30, tr=0.25, "
                            f"8 obstacles (soft), SOC ||u||<=1, box |x|,|y|<=12, {rule_txt}")
            else:
                data = "synthetic (C2 construction, SURVEY §8d: seed 0, random starts/goals, no obstacles)"
                workload = (f"C2: N={N} agents/GPU, 3-D double integrator n=6 m=3, K=50, FOH sigma=30, tr=0.25, "
                            f"no coupling, no obstacles, no SOC, box |x|,|y|<=12, {rule_txt}")
        else:
            value, scaling = args.steps / res["el"], "strong"
            metric = f"SCvx-iterations/sec, N={cfg['N_total']} agents x K=50 nodes (whole problem)"
            data = ("synthetic (C4 construction, SURVEY §8d: 16^3 lattice, spacing 6, permuted goals)"
                    if args.config == "c4" else
                    "synthetic (C5 construction: quadrotors from hover, seeded starts/goals, 8 spheres)")
            workload = (f"{args.config.upper()}: N={cfg['N_total']} agents ({N}/GPU), model {model} n={n} m={m}, "
                        f"K=50, pairwise coupling R={cfg['R']} (j_max={j_max} nearest rows per node in the solve, "
                        f"every other row checked at the solution and violators re-solved with 32), {n_obs} "
                        f"obstacles, box |x|,|y|<={box[0][2]:g}, global trust-region rule, RCCL all_gather of states"
                        + (f", virtual control w_nu={cfg['vc']['w_nu']:g} + proximal w_prox={cfg['vc']['w_prox']:g}"
                           if cfg["vc"] else ""))
        roof.update({"traffic": traffic,
                     "traffic_unit": "bytes/launch (FETCH_SIZE x2 + WRITE_SIZE; warm-started launches as in the "
                                     "timed region: the PMC command's cold first launch excluded)",
                     "traffic_source": traffic_src,
                     "note": "FP64-VALU small dense linear algebra (no MFMA: 6x6 / 6x3 f64 blocks); peak = FP64 "
                             "dense peak; FLOPs = SURVEY §8(d) count (bench.qp_flops_per_ipm_iter) x executed IPM "
                             "iterations; bytes = interface bytes (bench.qp_bytes_per_agent)"})
        line = {
            "metric": metric,
            "value": value,
            "unit": "SCvx-iterations/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": 1e3 * t_step,
            "higher_is_better": True,
            "scaling": scaling,
            "vs_baseline": None,
            "dtype": "f64",
            "data": data,
            "config": {"workload": workload, "agents_per_gpu": N, "K": K,
                       "parallelism": f"agents sharded x{world}" + (" (balanced order)" if (args.balance and world > 1
                                                                         and not independent) else ""),
                       **primary_cfg,
                       # JacobiSCvx's default is 0 (warm-start only optimal solves); the bench warm-starts
                       # optimal_inaccurate ones too (C3 / C5 end every solve optimal: no effect there)
                       "warm_max_status": args.warm_status},
            "roofline": roof,
            "step_roofline": step_roof,
            **res["fields"],
            "other_rule": other,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

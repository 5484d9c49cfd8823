"""CPU checks of bench.py: the --gpus launcher really starts N ranks (dry run over gloo, no GPU work),
and the algorithmic byte / FLOP accounting the roofline is computed from."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*args):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), *args], capture_output=True, text=True,
                       timeout=240, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def test_launcher_runs_two_ranks():
    line = _run("--gpus", "2", "--steps", "3", "--warmup", "1", "--dry-run")
    assert line["n_gpus"] == 2 and line["steps"] == 3


def test_single_rank_default():
    line = _run("--steps", "2", "--dry-run")
    assert line["n_gpus"] == 1


def test_dry_run_c4_shards_at_8_ranks():
    """bench.py --dry-run --gpus 8 --config c4: the 4096-agent lattice over 8 gloo ranks (the driver's 8-GPU run),
    contiguous and --balance shards: 512 agents per rank, the shards tile the agents exactly once and every rank
    holds its own agents' data (bench.dry_run_shards)."""
    for extra in ((), ("--balance",)):
        line = _run("--gpus", "8", "--steps", "2", "--warmup", "1", "--dry-run", "--config", "c4", *extra)
        c = line["config"]
        assert line["n_gpus"] == 8 and c["N_total"] == 4096 and c["agents_per_rank"] == 512
        assert c["shards_tile_agents"] is True and c["balanced"] == bool(extra)
        if not extra:
            assert c["shard_first_agents"] == [512 * r for r in range(8)]


def test_world_size_mismatch_is_refused():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--dry-run"],
                       capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode != 0 and "WORLD_SIZE" in (r.stderr + r.stdout)


def test_algorithmic_counts_c3():
    sys.path.insert(0, REPO)
    import bench
    assert bench.foh_bytes_per_agent(6, 3, 50) == 36536
    assert bench.foh_flops_per_agent(6, 3, 50) == 49 * 6522
    assert bench.qp_bytes_per_agent(6, 3, 50) == 36640 + 4016
    rows = bench.qp_rows(6, 3, 2, 8, 0, True)
    assert rows == 32
    assert abs(bench.qp_flops_per_ipm_iter(6, 3, 50, rows) - 113850) < 1e-6

"""bench.py's multi-GPU coordination (replicas, no data-path collective) on CPU:
two ranks under torchrun share only a gloo barrier and the max over ranks of the timing."""
from __future__ import annotations

import os
import re
import socket
import subprocess
import sys

from conftest import ROOT


def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_two_rank_barrier_and_max():
    env = dict(os.environ, OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}",
           os.path.join(ROOT, "tests", "helpers", "group_probe.py")]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    # the two ranks share the launcher's stdout: their lines may interleave without a newline
    found = re.findall(r"rank (\d+) world (\d+) max ([0-9.]+) tokens (\d+)", r.stdout)
    assert sorted(f[0] for f in found) == ["0", "1"], r.stdout + r.stderr
    for _, world, mx, tokens in found:
        assert (world, mx, tokens) == ("2", "11.0", "14")


def test_bench_spawns_replicas_without_launcher():
    """`bench.py --gpus 2` with no WORLD_SIZE in the environment starts its own two ranks (child
    processes, before any GPU call) and rank 0 reports n_gpus 2 after the shared barriers and the
    max over ranks (--dry-run: the same launch/timing path with no engine)."""
    import json
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "1"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--batch", "64", "--dry-run"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["dry_run"] is True
    assert out["config"]["global_batch"] == 128
    assert abs(out["max_rank_s"] - 0.002) < 1e-12   # rank 1's duration wins the max


def test_bench_rejects_mismatched_launcher_world():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run"],
                       capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 2 and "WORLD_SIZE=1" in r.stderr


def test_bench_eight_replica_shard_of_configs3():
    """configs[3] (Llama-2-7B INT4, batch 512 over 8 GPUs) as the driver launches it: 8 ranks of
    `bench.py --gpus 8 --batch 64`, each an independent replica with 64 streams of its own (gloo
    rendezvous on CPU, --dry-run: no engine).  Rank 0 reports global_batch 512 as replicas8, the
    max over ranks of the per-rank durations, and every rank's shard plan: 64 streams each, distinct
    weight seeds, first tokens and KV seeds (no two replicas decode the same requests)."""
    import json
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "1"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8", "--batch", "64", "--dry-run"],
                       capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 8 and out["dry_run"] is True
    assert out["config"] == {"global_batch": 512, "parallelism": "replicas8"}
    assert abs(out["max_rank_s"] - 0.008) < 1e-12   # rank 7's duration wins the max
    plans = out["rank_plans"]
    assert [p["rank"] for p in plans] == list(range(8))
    assert all(p["streams"] == 64 for p in plans)
    for key in ("weight_seed", "first_token", "kv_seed_first"):
        assert len({p[key] for p in plans}) == 8, (key, plans)
    kv = sorted((p["kv_seed_first"], p["kv_seed_last"]) for p in plans)
    assert all(a[1] < b[0] for a, b in zip(kv, kv[1:])), kv   # the ranks' KV seed ranges are disjoint

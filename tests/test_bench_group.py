"""bench.py's multi-GPU coordination (replicas, no data-path collective) on CPU:
two ranks under torchrun share only a gloo barrier and the max over ranks of the timing."""
from __future__ import annotations

import os
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
    lines = [l for l in r.stdout.splitlines() if l.startswith("rank ")]
    assert len(lines) == 2, r.stdout + r.stderr
    for l in lines:
        assert "world 2" in l and "max 11.0" in l and "tokens 14" in l

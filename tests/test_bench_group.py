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

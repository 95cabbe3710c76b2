"""Rank body for tests/test_bench_group.py: bench.Group over gloo (barrier + max over ranks)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402

g = bench.Group()
g.barrier()
m = g.max(10.0 + g.rank)            # every rank must see the largest rank's value
tokens = 7 * g.world                 # value = tokens of all ranks / max time, as bench.py reports
print(f"rank {g.rank} world {g.world} max {m} tokens {tokens}", flush=True)
g.barrier()
g.close()

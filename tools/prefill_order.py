"""512-token prefill timed with the chunk limit alternating 512 / 1024 (same single 511-row chunk
either way), 3 timed generate() calls per setting, to tell an order / warm-up effect in
tools/prefill_bench.py from a real difference."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import turboinfer_amd as T  # noqa: E402

T.init(0)
e = T.Engine(32000, 4096, 32, 32, 32, 128, 11008, bits=4, max_seq=2048, max_batch=1)
e.synth(0x7157, 0.0)
prompt = np.random.RandomState(0).randint(0, 32000, size=512).tolist()
for rows in (512, 1024, 512, 1024, 1024, 512):
    e.set_prefill(rows)
    e.generate([prompt], 1)
    ts = []
    for _ in range(3):
        t = time.perf_counter()
        e.generate([prompt], 1)
        ts.append((time.perf_counter() - t) * 1e3)
    print(f"rows {rows:4d}: " + " ".join(f"{v:6.2f}" for v in ts) + " ms", flush=True)

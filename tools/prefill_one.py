"""One prefill configuration for profiling (GPU box): 7B INT4, a 512-token prompt in one
512-row chunk, warmed once and run `reps` times:  python tools/prefill_one.py [reps]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import turboinfer_amd as T  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
T.init(0)
e = T.Engine(32000, 4096, 32, 32, 32, 128, 11008, bits=4, max_seq=2048, max_batch=1)
e.synth(0x7157, 0.0)
prompt = np.random.RandomState(0).randint(0, 32000, size=512).tolist()
e.set_prefill(512)
e.generate([prompt], 1)
for _ in range(reps):
    t = time.perf_counter()
    tok = e.generate([prompt], 1)
    print(f"prefill 512 rows: {(time.perf_counter() - t) * 1e3:.2f} ms, next token {tok[0][0]}", flush=True)

"""Prompt processing time, prefill on vs one token per decode step (GPU box):
    python tools/prefill_bench.py [prompt_len]
Llama-2-7B shape, INT4, synthetic weights; times generate(prompt, 1) end to end."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import turboinfer_amd as T  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 512
T.init(0)
e = T.Engine(32000, 4096, 32, 32, 32, 128, 11008, bits=4, max_seq=2048, max_batch=1)
e.synth(0x7157, 0.0)
prompt = np.random.RandomState(0).randint(0, 32000, size=n).tolist()
e.set_prefill(T.GEMM_MAX_ROWS)
for _ in range(2):   # first-use costs (module loads, graph capture) outside every timed line
    e.generate([prompt], 1)
for rows in (T.GEMM_MAX_ROWS, 512, 256, 0):
    e.set_prefill(rows)
    e.generate([prompt], 1)   # warm (graphs, kernels)
    t = time.perf_counter()
    tok = e.generate([prompt], 1)
    dt = time.perf_counter() - t
    print(f"prefill rows {rows:2d}: {n} prompt tokens in {dt * 1e3:8.1f} ms ({n / dt:8.0f} tok/s), next token {tok[0][0]}",
          flush=True)

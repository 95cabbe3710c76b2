"""Non-greedy decode speed: on-device sampling (ti_engine_generate_sampled) vs logits to the
host every step + the host sampler (the C++ API's path for batched requests), vs greedy.
    python tools/sample_bench.py [new_tokens]
Llama-2-7B shape, INT4, synthetic weights, 8-token prompt, top-k 40 / top-p 0.9 / T 0.8."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import turboinfer_amd as T  # noqa: E402

new = int(sys.argv[1]) if len(sys.argv) > 1 else 128
T.init(0)
e = T.Engine(32000, 4096, 32, 32, 32, 128, 11008, bits=4, max_seq=2048, max_batch=1)
e.synth(0x7157, 0.0)
e.set_prefill(0)   # token-by-token prompt on all three paths: identical logits, comparable tokens
prompt = [1, 15, 25, 35, 45, 55, 65, 75]
draws = np.random.RandomState(1).uniform(0, 1, new).astype(np.float32)
e.generate([prompt], new)
e.generate_sampled([prompt], new, 0.8, 40, 0.9, draws)   # warm graphs
t = time.perf_counter()
e.generate([prompt], new)
greedy = time.perf_counter() - t
t = time.perf_counter()
tok, _ = e.generate_sampled([prompt], new, 0.8, 40, 0.9, draws)
dev = time.perf_counter() - t
t = time.perf_counter()
toks = list(prompt)
for pos in range(len(prompt) + new - 1):
    lg = e.step([toks[pos]], [pos])[0]
    if pos >= len(prompt) - 1:
        toks.append(T.sample_token(lg, 0.8, 40, 0.9, float(draws[len(toks) - len(prompt)]))[0])
host = time.perf_counter() - t
same = toks[len(prompt):] == tok[0].tolist()
print(f"{new} new tokens after an {len(prompt)}-token prompt (end to end, incl. prefill):")
print(f"  greedy, device loop           {greedy * 1e3:8.1f} ms  {new / greedy:7.1f} tok/s")
print(f"  sampled, device sampler       {dev * 1e3:8.1f} ms  {new / dev:7.1f} tok/s")
print(f"  sampled, host loop + sampler  {host * 1e3:8.1f} ms  {new / host:7.1f} tok/s  (same tokens: {same})")

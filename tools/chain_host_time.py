"""Host enqueue cost of chained vs graph decode steps (diagnostic, GPU box)."""
import sys, time
sys.path.insert(0, ".")
import turboinfer_amd as T

T.init(0)
e = T.Engine(32000, 4096, 32, 32, 32, 128, 11008, bits=4, max_seq=2048, max_batch=1)
e.synth(0x7157, 0.0)
e.fill_kv(0, 2047, 99)
for chain in (False, True, False, True):
    e.set_chain(chain)
    e.replay_prepare(1, 2048, 7)
    e.replay_run(8)
    e.sync()
    n = 64
    t0 = time.perf_counter()
    e.replay_run(n)
    t1 = time.perf_counter()
    e.sync()
    t2 = time.perf_counter()
    print(f"chain={chain}: enqueue {1e6 * (t1 - t0) / n:8.1f} us/step, wall {1e6 * (t2 - t0) / n:8.1f} us/step", flush=True)

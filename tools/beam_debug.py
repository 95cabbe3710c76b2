"""Debug: prompt logits through generate() (prefill + one step) vs step-by-step decode vs the
oracle, for short sequences of the beam test model."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "oracle")); sys.path.insert(0, os.path.join(ROOT, "tests"))
import turboinfer_amd as T
from pyoracle import Oracle, OracleModel
from test_gpu_beam import CFG, SEED, JIT, CASES
T.init(0)
c = CFG
o = Oracle()
m = OracleModel(o, CFG, SEED, JIT)
def oracle_lg(toks):
    m.fill_kv(0, 0)
    for t in toks: _, lg = m.step(t)
    return lg
for mb in (2, 8):
    e = T.Engine(c["vocab"], c["hidden"], c["layers"], c["heads"], c["kv_heads"], c["head_dim"], c["inter"], bits=4, max_seq=64, max_batch=mb)
    e.synth(SEED, JIT)
    for seq in ([231], [231, 439], [231, 217], [231, 439, 506], [231, 217, 217], [4, 39, 12]):
        _, lg = e.generate([seq], 1, want_logits=True)
        ref = oracle_lg(seq)
        steps = [e.step([t], [i])[0] for i, t in enumerate(seq)][-1]
        print(mb, seq, "gen-vs-oracle", float(np.abs(lg[0] - ref).max()), "step-vs-oracle", float(np.abs(steps - ref).max()), "max", float(np.abs(ref).max()), flush=True)
    prompt, new, beam, T_, k, p, lp = CASES[5]
    print(mb, "beam", e.beam_search(prompt, new, beam, T_, k, p, lp, 2))
    e.close()
print("oracle", o.beam_search(oracle_lg, *CASES[5][:3], *CASES[5][3:], eos=2))

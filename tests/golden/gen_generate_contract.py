"""Golden vectors for generate()'s stopping and timing contract, produced by the
compiled reference (oracle/_ref, `make -C oracle ref`) on its benchmark's plumbing model:

  * EOS is token id 2, hard-coded (inference_engine.cpp:759-760): with config.eos_token_id = 5
    the greedy run on create_test_model(7, 256, 4) emits 5 and continues, then stops at 2;
  * config.eos_token_id = 999 on the (1000, 256, 4) model, whose greedy token is always 999:
    the reference does not stop at it and runs to max_new_tokens;
  * max_sequence_length reached first: stop_reason "max_length" (:767-771).
Also recorded: the reference's total_time_ms (whole milliseconds, :778-780) and tokens_per_second.

    python tests/golden/gen_generate_contract.py   (build container; writes generate_contract.npz)
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
from pyoracle import Reference  # noqa: E402

CASES = [  # (vocab, hidden, layers, prompt, max_new, eos_token_id, max_sequence_length)
    (7, 256, 4, [1, 1], 10, 5, 2048),
    (1000, 256, 4, [1, 15, 25, 35], 12, 999, 2048),
    (1000, 256, 4, [1, 15, 25, 35], 12, 2, 7),
    (7, 256, 4, [1, 1, 1], 10, 1, 2048),
]


def main():
    ref = Reference()
    out = {"n": np.array([len(CASES)], np.int32)}
    for i, (V, H, L, prompt, mn, eos, ml) in enumerate(CASES):
        toks, fin, stop, ms, tps = ref.plumbing_generate_cfg(V, H, L, prompt, mn, eos, ml)
        out[f"cfg{i}"] = np.array([V, H, L, mn, eos, ml], np.int64)
        out[f"prompt{i}"] = np.array(prompt, np.int32)
        out[f"tokens{i}"] = np.array(toks, np.int32)
        out[f"stop{i}"] = np.array([stop, int(fin)], np.int32)
        out[f"time{i}"] = np.array([ms, tps], np.float32)
        print(i, toks, "finished" if fin else "", ["eos_token", "max_length", "max_new_tokens"][stop], ms, tps)
    np.savez(os.path.join(HERE, "generate_contract.npz"), **out)


if __name__ == "__main__":
    main()

"""GGUF fixtures for ModelLoader::load_gguf (tests/test_cpp_api.py), written by the oracle's
GGUF v3 writer (oracle/gguf_oracle.py; ggml's reference quantizers for the block types).

* gguf_ref_pin.gguf -- what the reference's own loader reads correctly (model_loader.cpp:
  710-873): scalar key/values of every type and ONE fp32 tensor.  The test runs the compiled
  reference (oracle/_ref) on it and requires the C++ API's ModelData to match field for field.
* gguf_mixed.gguf  -- a llama-shaped file as real checkpoints are: a tokenizer string array,
  general.alignment 64, and F32 / F16 / BF16 / Q4_0 / Q4_1 / Q8_0 tensors.  Checked against
  gguf_oracle.gguf_read (the reference cannot read this file: it skips arrays by count * 8
  bytes and seeks tensors relative to the previous read).

    python tests/golden/gen_gguf.py
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(HERE)), "oracle"))
import gguf_oracle as G  # noqa: E402


def main() -> None:
    rng = np.random.RandomState(0x66F)
    pin_kvs = [("general.architecture", G.STR, "llama"), ("general.name", G.STR, "pin_fixture"),
               ("llama.vocab_size", G.U32, 64), ("llama.embedding_length", G.U64, 32),
               ("llama.block_count", G.U32, 1), ("llama.attention.head_count", G.U32, 4),
               ("llama.feed_forward_length", G.I32, 48), ("llama.rope.theta", G.F32, 500000.0),
               ("llama.attention.head_count_kv", G.U32, 2), ("llama.attention.layer_norm_rms_epsilon", G.F32, 1e-5),
               ("general.file_type", G.U8, 2), ("test.i8", G.I8, -5), ("test.u16", G.U16, 65535),
               ("test.i16", G.I16, -300), ("test.i64", G.I64, -(1 << 40)), ("test.f64", G.F64, 3.25),
               ("test.bool", G.BOOL, 1)]
    G.gguf_write(os.path.join(HERE, "gguf_ref_pin.gguf"), pin_kvs,
                 [("token_embd.weight", rng.standard_normal((64, 32)).astype(np.float32), G.T_F32)])

    mixed_kvs = [("general.architecture", G.STR, "llama"), ("general.name", G.STR, "mixed_fixture"),
                 ("general.alignment", G.U32, 64), ("llama.vocab_size", G.U32, 64),
                 ("llama.embedding_length", G.U32, 64), ("llama.block_count", G.U32, 1),
                 ("llama.attention.head_count", G.U32, 4), ("llama.feed_forward_length", G.U32, 96),
                 ("tokenizer.ggml.tokens", G.ARR, (G.STR, ["<unk>", "<s>", "</s>", "hello", "wor", "ld"])),
                 ("tokenizer.ggml.scores", G.ARR, (G.F32, [0.0, -1.0, -2.5])),
                 ("llama.rope.theta", G.F32, 10000.0)]
    big = (rng.standard_normal((96, 64)) * 0.1).astype(np.float32)
    big[3, 7] = 2.0    # a block whose largest magnitude is positive (Q4_0 d < 0)
    big[5, 40] = -3.0  # and negative
    tensors = [("token_embd.weight", rng.standard_normal((64, 64)).astype(np.float32), G.T_F16),
               ("blk.0.attn_norm.weight", (1 + 0.1 * rng.standard_normal(64)).astype(np.float32), G.T_F32),
               ("blk.0.attn_q.weight", (rng.standard_normal((64, 64)) * 0.1).astype(np.float32), G.T_Q4_0),
               ("blk.0.attn_k.weight", (rng.standard_normal((64, 64)) * 0.1).astype(np.float32), G.T_Q8_0),
               ("blk.0.ffn_up.weight", big, G.T_Q4_1),
               ("blk.0.ffn_down.weight", big.T.copy(), G.T_Q4_0),
               ("output_norm.weight", rng.standard_normal(64).astype(np.float32), G.T_BF16),
               ("output.weight", (rng.standard_normal((64, 64)) * 0.1).astype(np.float32), G.T_Q8_0)]
    G.gguf_write(os.path.join(HERE, "gguf_mixed.gguf"), mixed_kvs, tensors, alignment=64)


if __name__ == "__main__":
    main()

"""Generate the golden vectors in tests/golden/ from the COMPILED REFERENCE.

Runs in the build container only (needs oracle/_ref/libti_ref.so, built by `make -C oracle ref`
from the unmodified sources under /root/reference).  Every expected output below is produced
by the reference's own TensorEngine / Quantizer / InferenceEngine code through
oracle/ref_shim.cpp; inputs are seeded numpy data (stored in the fixture) or the synthetic
model of SURVEY 8(d) (regenerated from its seed by the oracle).

    python tests/golden/gen_golden.py

Fixtures are data only (inputs + expected outputs); no reference source is copied.
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
from pyoracle import Oracle, Reference  # noqa: E402

ref = Reference()
orc = Oracle()

manifest = {"generator": "tests/golden/gen_golden.py", "reference": "juliuspleunes4/TurboInfer @ 2025-09-05, "
            "compiled by oracle/Makefile (g++ 11.4, -std=c++20 -O3 -mavx2 -mfma -fopenmp)", "files": {}}


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def save(name: str, desc: str, **arrays) -> None:
    path = os.path.join(HERE, name + ".npz")
    np.savez_compressed(path, **arrays)
    manifest["files"][name + ".npz"] = desc
    print(f"wrote {name}.npz ({os.path.getsize(path) // 1024} KiB)")


f32 = np.float32
BIG = 64 * 1024  # outputs above this many bytes are stored as sha256 + leading slice


def inp(seed: int, shape, scale: float = 1.0) -> np.ndarray:
    """Seeded input; numpy's legacy RandomState stream is frozen across versions."""
    return (np.random.RandomState(seed).standard_normal(shape) * scale).astype(f32)


def put(cases: dict, key: str, y: np.ndarray) -> None:
    y = np.ascontiguousarray(y)
    if y.nbytes > BIG:
        cases[key + "_sha"] = np.frombuffer(bytes.fromhex(sha(y)), np.uint8)
        cases[key + "_head"] = y.reshape(-1)[:512]
    else:
        cases[key] = y


# ---------------------------------------------------------------- op level (O1)
cases = {}
for i, (B, M, K, N) in enumerate([(1, 1, 37, 29), (1, 1, 256, 256), (1, 2, 64, 48), (2, 3, 128, 130),
                                  (1, 1, 1024, 1000), (1, 1, 4096, 4096)]):
    sa, sb = 100 + 2 * i, 101 + 2 * i
    a, b = inp(sa, (B, M, K)), inp(sb, (K, N), 0.05)
    cases[f"shape{i}"] = np.array([B, M, K, N])
    cases[f"seeds{i}"] = np.array([sa, sb])
    put(cases, f"y{i}", ref.matmul(a, b))
save("matmul", "TensorEngine::matmul 3Dx2D (matmul_3d_2d); inputs RandomState(seed).standard_normal (b *0.05)", **cases)

cases = {}
for i, (rows, n) in enumerate([(2, 5), (2, 100), (1, 256), (3, 4096), (2, 4099)]):
    x = inp(200 + i, (rows, n))
    w = (f32(1.0) + inp(300 + i, (n,), 0.1)).astype(f32)
    cases[f"shape{i}"] = np.array([rows, n])
    put(cases, f"y{i}", ref.rms_norm(x, w))
save("rms_norm", "TensorEngine::rms_norm eps=1e-5; x = RandomState(200+i), w = 1 + 0.1*RandomState(300+i)", **cases)

cases = {}
rope_specs = [((1, 32, 1, 128), [0.0], 1e4), ((1, 32, 1, 128), [1.0], 1e4), ((1, 32, 1, 128), [2047.0], 1e4),
              ((1, 8, 1, 128), [8191.0], 5e5), ((1, 4, 1, 64), [17.0], 1e4), ((2, 3, 5, 12), [0, 3, 9, 300, 4000], 1e4),
              ((2, 5, 16), [1, 2, 3, 4, 5], 1e4)]
for i, (shape, pos, theta) in enumerate(rope_specs):
    x = inp(400 + i, shape)
    p = np.array(pos, f32)
    cases[f"shape{i}"], cases[f"pos{i}"], cases[f"theta{i}"] = np.array(shape), p, np.array([theta], f32)
    put(cases, f"y{i}", ref.apply_rope(x, p, theta))
save("rope", "TensorEngine::apply_rope (4-D [B,heads,S,D] and 3-D); x = RandomState(400+i)", **cases)

x, x2 = inp(500, (1001,), 4.0), inp(501, (1001,))
save("eltwise", "silu, relu, add, multiply on n=1001; x = 4*RandomState(500), x2 = RandomState(501)",
     silu=ref.silu(x), relu=ref.relu(x), add=ref.add(x, x2), mul=ref.multiply(x, x2))

cases = {}
for i, (rows, n, T) in enumerate([(3, 5, 1.0), (2, 16, 1.0), (2, 37, 0.7), (2, 1000, 1.0), (1, 32000, 1.0),
                                  (1, 32000, 0.7), (1, 128256, 1.0)]):
    x = inp(600 + i, (rows, n), 5.0)
    cases[f"shape{i}"], cases[f"T{i}"] = np.array([rows, n]), np.array([T], f32)
    put(cases, f"y{i}", ref.softmax(x, T))
save("softmax", "TensorEngine::softmax (AVX2 fast_exp path for n>=16); x = 5*RandomState(600+i)", **cases)

cases = {}
for i, (B, S, D) in enumerate([(1, 1, 128), (1, 7, 128), (2, 19, 64), (1, 13, 12), (1, 2048, 128), (1, 300, 64)]):
    q, k, v = inp(700 + 3 * i, (B, 1, D)), inp(701 + 3 * i, (B, S, D)), inp(702 + 3 * i, (B, S, D))
    cases[f"shape{i}"] = np.array([B, S, D])
    put(cases, f"y{i}", ref.attention_incremental(q, k, v))
save("attention", "TensorEngine::attention_fast_incremental; q,k,v = RandomState(700+3i, +1, +2)", **cases)

cases = {}
for i, (S, H, heads) in enumerate([(1, 256, 4), (17, 256, 4), (33, 512, 4), (2048, 4096, 32)]):
    q, k, v = inp(800 + 3 * i, (1, 1, H)), inp(801 + 3 * i, (1, S, H)), inp(802 + 3 * i, (1, S, H))
    cases[f"shape{i}"] = np.array([S, H, heads])
    put(cases, f"y{i}", ref.multi_head_attention(q, k, v, heads))
save("mha", "TensorEngine::multi_head_attention (decode shape); q,k,v = RandomState(800+3i, +1, +2)", **cases)

cases = {}
qin = [inp(900, (1000,), 3.0),
       np.linspace(-10, 10, 16).astype(f32),            # tests/test_quantization_complete.cpp:20-78 grid
       np.linspace(-2, 2, 9).astype(f32),                # :80-131 grid
       np.array([0.5, 1.5, 2.5, -0.5, -1.5, 7.0, -7.0, 3.5], f32)]
k = 0
for xi, x in enumerate(qin):
    for bits in (8, 4):
        for sym in (1, 0):
            q, s, z = ref.quantize(x, bits, bool(sym))
            cases[f"x{k}"], cases[f"bits{k}"], cases[f"sym{k}"] = x, np.array([bits]), np.array([sym])
            cases[f"q{k}"], cases[f"scale{k}"], cases[f"zp{k}"] = q, np.array([s], f32), np.array([z], f32)
            cases[f"deq{k}"] = ref.dequantize(q, bits, s, z)
            k += 1
save("quant", "Quantizer::calculate_quantization_info + quantize_tensor + dequantize_from_int{8,4}", n=np.array([k]), **cases)

cases = {}
for i, p in enumerate([[1, 15, 25, 35], [1, 10, 20, 30, 40, 50], [1, 5, 15, 25, 35, 45, 55, 65]]):
    cases[f"prompt{i}"] = np.array(p, np.int32)
    cases[f"tokens{i}"] = np.array(ref.plumbing_generate(1000, 256, 4, p, 20), np.int32)
save("plumbing_generate", "InferenceEngine::generate, benchmark_inference create_test_model(1000,256,4), top_k=1, "
     "20 new tokens (BASELINE config 1)", **cases)

# The reference's own sampler through its public generate() (include_logprobs = true): one
# realisation of its clock-seeded draws per config, (token, log-prob) per sampled step.
cases = {}
SAMPLE_CFGS = [(1.0, 50, 0.9), (0.7, 40, 0.9), (1.3, 0, 0.95), (1.0, 3, 1.0), (0.5, 1000, 0.5), (2.0, 7, 0.99),
               (1.0, 2, 1.0), (0.9, 9, 1.0)]
for i, (T, k, p) in enumerate(SAMPLE_CFGS):
    toks, lps = ref.plumbing_generate_sampled(1000, 256, 4, [1, 15, 25, 35], 12, T, k, p)
    cases[f"cfg{i}"] = np.array([T, k, p], f32)
    cases[f"tokens{i}"], cases[f"logprobs{i}"] = np.array(toks, np.int32), lps
save("sample_plumbing", "InferenceEngine::generate(include_logprobs) with sampling configs (temperature, top_k, top_p) "
     "on create_test_model(1000,256,4), prompt 1 15 25 35, 12 new tokens; the draws are the reference's clock-seeded "
     "mt19937 (one realisation)", n=np.array([len(SAMPLE_CFGS)]), **cases)

# The reference's generate_beam_search on the plumbing model (deterministic: no draws).  Its
# forward_pass returns all seq_len x vocab logits and beam_search_decode reads them as one
# distribution (:1961-1966), so token ids run past the vocabulary; ties everywhere (the lm_head
# repeats every 500 columns) exercise its std::sort / priority_queue orders.
cases = {}
BEAM_CFGS = [(3, 2, 1.0, 0, 1.0, 1.0), (4, 3, 1.0, 50, 0.9, 1.0), (3, 4, 0.7, 0, 1.0, 0.6), (2, 2, 1.0, 2, 1.0, 1.0),
             (3, 3, 1.5, 7, 0.95, 1.3)]
for i, (mn, beam, T, k, p, lpen) in enumerate(BEAM_CFGS):
    res = ref.plumbing_beam_search(1000, 256, 4, [1, 15, 25, 35], mn, beam, T, k, p, lpen)
    cases[f"cfg{i}"] = np.array([mn, beam, T, k, p, lpen], f32)
    cases[f"tokens{i}"] = np.array([t + [-1] * (mn - len(t)) for t, _, _ in res], np.int32)
    cases[f"finished{i}"] = np.array([f for _, f, _ in res], np.int32)
    cases[f"logprob{i}"] = np.array([lp for _, _, lp in res], f32)
save("beam_plumbing", "InferenceEngine::generate_beam_search(include_logprobs) on create_test_model(1000,256,4), "
     "prompt 1 15 25 35; cfg = (max_new, beam, temperature, top_k, top_p, length_penalty)",
     n=np.array([len(BEAM_CFGS)]), **cases)

# -------------------------------------------- reference-composed decode step (O2)
def synth_model(cfg, seed, jitter):
    """The weights or_model_synth builds, materialised in numpy (data for the reference)."""
    H, hd, nh, nkv, I, V = cfg["hidden"], cfg["head_dim"], cfg["heads"], cfg["kv_heads"], cfg["inter"], cfg["vocab"]
    bits = cfg["bits"]

    def lin(tid, K, N):
        w = orc.synth_linear(seed, tid, K, N)
        if bits == 16:
            return w.astype(np.float16).astype(f32)
        q, s = orc.quantize_groups(w, bits, 128, 0)
        return orc.dequantize_groups(q, s, 128)

    def unit(tid, n):
        return np.array([orc.lib.or_synth_unit(seed, tid, i) for i in range(n)], f32)

    m = {"emb": (unit(1, V * H) * f32(0.02)).astype(np.float16).astype(f32).reshape(V, H),
         "out_norm": (f32(1.0) + f32(jitter) * unit(2, H)).astype(f32), "lm": lin(3, H, V), "layers": []}
    for l in range(cfg["layers"]):
        t = 16 + 16 * l
        m["layers"].append({
            "an": (f32(1.0) + f32(jitter) * unit(t + 0, H)).astype(f32),
            "fn": (f32(1.0) + f32(jitter) * unit(t + 1, H)).astype(f32),
            "wq": lin(t + 2, H, nh * hd), "wk": lin(t + 3, H, nkv * hd), "wv": lin(t + 4, H, nkv * hd),
            "wo": lin(t + 5, nh * hd, H), "wg": lin(t + 6, H, I), "wu": lin(t + 7, H, I), "wd": lin(t + 8, I, H)})
    return m


def ref_decode(cfg, model, tokens):
    """Decode `tokens` one by one, composing ONLY reference TensorEngine ops."""
    H, hd, nh, nkv = cfg["hidden"], cfg["head_dim"], cfg["heads"], cfg["kv_heads"]
    grp = nh // nkv
    theta = cfg["rope_theta"]
    kc = [np.zeros((0, nkv * hd), f32) for _ in range(cfg["layers"])]
    vc = [np.zeros((0, nkv * hd), f32) for _ in range(cfg["layers"])]
    all_logits = []
    for pos, tok in enumerate(tokens):
        x = model["emb"][tok].reshape(1, 1, H).copy()
        p = np.array([float(pos)], f32)
        for l, L in enumerate(model["layers"]):
            xn = ref.rms_norm(x, L["an"])
            q = ref.matmul(xn, L["wq"])
            k = ref.matmul(xn, L["wk"])
            v = ref.matmul(xn, L["wv"])
            q = ref.apply_rope(q.reshape(1, nh, 1, hd), p, theta).reshape(1, 1, nh * hd)
            k = ref.apply_rope(k.reshape(1, nkv, 1, hd), p, theta).reshape(1, nkv * hd)
            kc[l] = np.concatenate([kc[l], k], 0)
            vc[l] = np.concatenate([vc[l], v.reshape(1, nkv * hd)], 0)
            S = kc[l].shape[0]
            kx = np.repeat(kc[l].reshape(S, nkv, hd), grp, axis=1).reshape(1, S, nh * hd)
            vx = np.repeat(vc[l].reshape(S, nkv, hd), grp, axis=1).reshape(1, S, nh * hd)
            att = ref.multi_head_attention(q, kx, vx, nh)
            x = ref.add(x, ref.matmul(att, L["wo"]))
            xn = ref.rms_norm(x, L["fn"])
            up = ref.matmul(xn, L["wu"])
            gate = ref.silu(ref.matmul(xn, L["wg"]))
            x = ref.add(x, ref.matmul(ref.multiply(up, gate), L["wd"]))
        logits = ref.matmul(ref.rms_norm(x, model["out_norm"]), model["lm"]).reshape(-1)
        all_logits.append(logits)
    return np.stack(all_logits)


def greedy(cfg, model, prompt, n_new):
    toks = list(prompt)
    logits = None
    for _ in range(n_new):
        logits = ref_decode(cfg, model, toks)     # full recompute: reference ops are stateless
        toks.append(int(np.argmax(logits[-1])))
    return toks, ref_decode(cfg, model, toks[:-1])


decode_cases = [
    ("mini_gqa_w4", dict(vocab=512, hidden=256, layers=2, heads=4, kv_heads=2, head_dim=64, inter=512,
                         rope_theta=10000.0, eps=1e-5, bits=4, group=128, max_seq=64), 11, 0.1, [1, 17, 42], 6),
    ("mini_hd128_w8", dict(vocab=256, hidden=256, layers=2, heads=2, kv_heads=2, head_dim=128, inter=384,
                           rope_theta=500000.0, eps=1e-5, bits=8, group=128, max_seq=64), 23, 0.1, [5, 9], 5),
]
for name, cfg, seed, jit, prompt, n_new in decode_cases:
    model = synth_model(cfg, seed, jit)
    toks, logits = greedy(cfg, model, prompt, n_new)
    save(f"decode_{name}", f"reference-composed Llama decode (O2), synthetic model seed {seed} jitter {jit}, "
         f"greedy from prompt {prompt}", tokens=np.array(toks, np.int32), logits=logits,
         cfg=np.array(json.dumps(cfg)), seed=np.array([seed]), jitter=np.array([jit], f32),
         prompt=np.array(prompt, np.int32))

with open(os.path.join(HERE, "manifest.json"), "w") as f:
    json.dump(manifest, f, indent=1)
print("done")

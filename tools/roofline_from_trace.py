"""The bench's roofline figure recomputed from a rocprofv3 kernel trace of decode steps.

    python tools/roofline_from_trace.py gpurun_out/prof/run_results.db [--model llama2-7b]

Finds every complete single-stream decode step in the trace (step_begin followed by
5 x layers kernels and the lm_head -- or 4 x layers where QKV and the attention run as one
launch, qkv_attn_kernel: DESIGN 4.19), labels the launches by their position in the step
(qkv, attention, o, gate/up, down per layer, the fused launch labelled qkv with the attention's
K/V bytes added, as bench.py does; lm_head), and prints per class the average
traced duration, the algorithmic bytes per launch (bench.py / ti_engine_time_kernel: packed
weights + group scales + the fp16 input row) and GB/s, then the W4 GEMV family's
sum(bytes) / sum(time) over a step's 4 x layers + 1 launches -- the quantity bench.py reports as
`roofline.achieved` from its own HIP-event timing."""
from __future__ import annotations

import argparse
import json
import sqlite3
import sys
from collections import defaultdict

MODELS = {
    "llama2-7b": (32000, 4096, 32, 32, 32, 128, 11008, 4),
    "tinyllama-1.1b": (32000, 2048, 22, 32, 4, 64, 5632, 8),
    "llama3-8b": (128256, 4096, 32, 32, 8, 128, 14336, 4),
}


def lin_bytes(bits, K, N):
    return K * N * bits // 8 + (K // 128) * N * 2 + K * 2


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--model", default="llama2-7b", choices=sorted(MODELS))
    ap.add_argument("--kv", type=int, default=2048, help="keys the replayed step reads (bench.py --kv)")
    ap.add_argument("--json", action="store_true")
    a = ap.parse_args()
    V, H, layers, nh, nkv, hd, I, bits = MODELS[a.model]
    qd, kvd = nh * hd, nkv * hd
    cls_bytes = {"qkv": lin_bytes(bits, H, qd + 2 * kvd), "o": lin_bytes(bits, qd, H),
                 "gate_up": lin_bytes(bits, H, 2 * I), "down": lin_bytes(bits, I, H), "lm_head": lin_bytes(bits, H, V)}
    rows = sqlite3.connect(a.db).execute("select name, start, end from kernels order by start").fetchall()
    fused = any("qkv_attn_kernel" in r[0] for r in rows)
    lpl = 4 if fused else 5   # launches per layer
    if fused:   # the fused launch streams the attention's K/V too (ti_engine_time_kernel's attention bytes)
        cls_bytes["qkv"] += 2 * kvd * a.kv * 2 + qd * (4 + 2)
    per_step = 2 + lpl * layers
    order = ["qkv", "o", "gate_up", "down"] if fused else ["qkv", "attention", "o", "gate_up", "down"]
    gemv_pos = (1, 2, 3) if fused else (0, 2, 3, 4)
    dur = defaultdict(list)
    n_steps = 0
    i = 0
    while i + per_step <= len(rows):
        if "step_begin" not in rows[i][0]:
            i += 1
            continue
        blk = rows[i:i + per_step]
        if not all("gemv_wq_kernel" in blk[1 + lpl * l + j][0] for l in range(layers) for j in gemv_pos) or \
           (fused and not all("qkv_attn_kernel" in blk[1 + lpl * l][0] for l in range(layers))) or \
           "gemv_wq_kernel" not in blk[-1][0]:
            i += 1
            continue
        for l in range(layers):
            for j, name in enumerate(order):
                r = blk[1 + lpl * l + j]
                dur[name].append((r[2] - r[1]) / 1e3)
        dur["lm_head"].append((blk[-1][2] - blk[-1][1]) / 1e3)
        n_steps += 1
        i += per_step
    if not n_steps:
        sys.exit("no complete decode step in the trace")
    out = {"steps": n_steps, "classes": {}}
    fam_b = fam_t = 0.0
    for name, d in dur.items():
        avg = sum(d) / len(d)
        ent = {"avg_us": round(avg, 3)}
        if name in cls_bytes:
            cnt = 1 if name == "lm_head" else layers
            ent.update(bytes=cls_bytes[name], GBps=round(cls_bytes[name] / avg / 1e3, 1))
            fam_b += cls_bytes[name] * cnt
            fam_t += avg * cnt
        out["classes"][name] = ent
    out["family_achieved_GBps"] = round(fam_b / fam_t / 1e3, 1)
    out["family_frac"] = round(fam_b / fam_t / 1e3 / 8000.0, 4)
    out["family_avg_launch_us"] = round(fam_t / (4 * layers + 1), 3)
    if a.json:
        print(json.dumps(out))
        return
    print(f"{n_steps} complete decode steps")
    for name, ent in out["classes"].items():
        print(f"  {name:10s} {ent['avg_us']:8.3f} us" + (f"  {ent['bytes'] / 1e6:8.2f} MB  {ent['GBps']:8.1f} GB/s"
                                                        if "bytes" in ent else ""))
    print(f"W{bits} GEMV family{' (qkv = the fused QKV + attention launch)' if fused else ''}: "
          f"{out['family_achieved_GBps']} GB/s = {out['family_frac']} of 8 TB/s, "
          f"{out['family_avg_launch_us']} us per launch")


if __name__ == "__main__":
    main()

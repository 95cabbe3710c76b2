"""HBM traffic per launch from a rocprofv3 FETCH_SIZE pass (GPU-box output -> profiles/).

    rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc -o run -- \
        python3 bench.py --steps 4 --warmup 2 --kernel-reps 4 --no-cpu-baseline [--model M --batch B]
    python tools/pmc_traffic.py gpurun_out/pmc/run_counter_collection.csv profiles/r5_pmc_traffic.json \
        [--model llama2-7b --batch 1 --kv 2048]

FETCH_SIZE is reported in KiB and, on gfx950, counts a wide coalesced streaming read at
exactly half its bytes (MI355X_MICROARCH.md, HBM section: 128-B requests tallied as 64 B),
so bytes = FETCH_SIZE * 1024 * 2.  Infinity-Cache hits are counted as fetches.  The mean is
over every dispatch of the kernel family in the pass (the replayed decode steps plus the
bench's per-shape timing launches, same mixture of shapes).

Families: the decode GEMM (every launch of gemv_wq_kernel / gemm_rows_kernel / gemm_tile_kernel:
one projection each) and the attention (attn_split_kernel).
The GEMM family's key is the one bench.py's roofline names: "gemv_wq_kernel<BITS>" for one stream
(the fused kernel runs every projection), "gemm_family" for batched steps (rows / tile kernels)."""
import argparse
import csv
import json
from collections import defaultdict

MODELS = {   # bench.py MODELS: vocab, hidden, layers, heads, kv_heads, head_dim, inter, bits
    "llama2-7b": (32000, 4096, 32, 32, 32, 128, 11008, 4),
    "tinyllama-1.1b": (32000, 2048, 22, 32, 4, 64, 5632, 8),
    "llama3-8b": (128256, 4096, 32, 32, 8, 128, 14336, 4),
}
GEMM = ("gemv_wq_kernel", "gemm_rows_kernel", "gemm_tile_kernel", "gemv_mb_kernel", "gemv_mbr_kernel",
        "qkv_attn_kernel")   # (the fused QKV + attention of one stream, DESIGN 4.19: its step position is QKV's)


def lin_bytes(bits, K, N):
    """Packed tiles + fp16 group-128 scales (ti_wpack_tile_bytes + ti_wpack_scale_bytes)."""
    return K * N * bits // 8 + (K // 128) * N * 2


def class_bytes(model, B):
    V, H, layers, nh, nkv, hd, I, bits = MODELS[model]
    qd, kvd = nh * hd, nkv * hd
    act = lambda K: B * K * 2   # noqa: E731  fp16 activation rows
    algo = {"qkv": lin_bytes(bits, H, qd + 2 * kvd) + act(H), "o": lin_bytes(bits, qd, H) + act(qd),
            "gate_up": lin_bytes(bits, H, 2 * I) + act(H), "down": lin_bytes(bits, I, H) + act(I),
            "lm_head": lin_bytes(bits, H, V) + act(H)}
    n = {"qkv": layers, "o": layers, "gate_up": layers, "down": layers, "lm_head": 1}
    return algo, n, bits


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("dst")
    ap.add_argument("--model", default="llama2-7b", choices=sorted(MODELS))
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--kv", type=int, default=2048)
    a = ap.parse_args()
    algo, n, bits = class_bytes(a.model, a.batch)
    gemm_key = f"gemv_wq_kernel<{bits}>" if a.batch == 1 else "gemm_family"
    rows = [r for r in csv.DictReader(open(a.src)) if r["Counter_Name"] == "FETCH_SIZE"]
    if any("qkv_attn_kernel" in r["Kernel_Name"] for r in rows):   # the qkv class also streams the K/V (bench.py)
        V, H, layers_, nh, nkv, hd, I, _ = MODELS[a.model]
        algo["qkv"] += 2 * nkv * hd * a.kv * 2 + nh * hd * (4 + 2)
    fam = defaultdict(list)
    names = defaultdict(set)
    for r in rows:
        name = r["Kernel_Name"]
        key = gemm_key if any(g in name for g in GEMM) else (
            "attn_split_kernel" if "attn_split_kernel" in name else None)
        if key:
            fam[key].append(float(r["Counter_Value"]) * 1024.0 * 2.0)
            names[key].add(name.split("(")[0][:80])
    out = {"source": "rocprofv3 --pmc FETCH_SIZE (KiB, x2 gfx950 streaming-read correction)",
           "config": {"model": a.model, "batch": a.batch, "kv": a.kv}, "kernels": {}}
    for k, v in fam.items():
        out["kernels"][k] = {"dispatches": len(v), "traffic_bytes_per_launch": round(sum(v) / len(v)),
                             "min": round(min(v)), "max": round(max(v)), "kernel_names": sorted(names[k])}
    # The pass mixes the decode steps with the bench's per-class timing launches, so the plain
    # mean depends on that mixture.  Step-weighted: each GEMM dispatch is assigned to the projection
    # class whose algorithmic bytes are nearest, the per-class means are weighted by the step's own
    # mixture (layers x QKV, O, gate/up, down + 1 lm_head), comparable to the bench line's
    # bytes_per_launch.
    # Classes by position in each decode step: after a step_begin dispatch the step issues, per layer,
    # the QKV, O, gate/up and down GEMMs in that order and then the lm_head (layers x 4 + 1 GEMM
    # dispatches); the bench's per-class timing launches outside the steps are not labelled.  Fall
    # back to the nearest algorithmic bytes when no complete step is found.
    per = defaultdict(list)
    layers = n["qkv"]
    order = ["qkv", "o", "gate_up", "down"]
    pos = None
    for r in sorted(rows, key=lambda r: int(r["Dispatch_Id"])):
        name = r["Kernel_Name"]
        if "step_begin_kernel" in name:
            pos = 0
            continue
        if pos is None or not any(g in name for g in GEMM):
            continue
        cls = order[pos % 4] if pos < 4 * layers else "lm_head"
        per[cls].append(float(r["Counter_Value"]) * 1024.0 * 2.0)
        pos = pos + 1 if pos < 4 * layers else None
    out["class_labels"] = "step position"
    if len(per) != len(algo):
        out["class_labels"] = "nearest algorithmic bytes"
        per = defaultdict(list)
        for b in fam.get(gemm_key, []):
            per[min(algo, key=lambda c: abs(algo[c] - b))].append(b)
    if len(per) == len(algo):
        cls = {c: {"dispatches": len(per[c]), "traffic_bytes": round(sum(per[c]) / len(per[c])), "algorithmic_bytes": algo[c],
                   "ratio": round(sum(per[c]) / len(per[c]) / algo[c], 4)} for c in algo}
        tw = sum(n[c] * cls[c]["traffic_bytes"] for c in algo) / sum(n.values())
        aw = sum(n[c] * algo[c] for c in algo) / sum(n.values())
        out["kernels"][gemm_key].update({"classes": cls, "step_weighted_traffic_bytes_per_launch": round(tw),
                                         "step_weighted_algorithmic_bytes_per_launch": round(aw),
                                         "step_weighted_ratio": round(tw / aw, 4)})
    json.dump(out, open(a.dst, "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()

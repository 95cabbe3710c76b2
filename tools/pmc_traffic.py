"""HBM traffic per launch from a rocprofv3 FETCH_SIZE pass (GPU-box output -> profiles/).

    rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc -o run -- \
        python3 bench.py --steps 4 --warmup 2 --kernel-reps 4 --no-cpu-baseline
    python tools/pmc_traffic.py gpurun_out/pmc/run_counter_collection.csv profiles/r1_pmc_traffic.json

FETCH_SIZE is reported in KiB and, on gfx950, counts a wide coalesced streaming read at
exactly half its bytes (MI355X_MICROARCH.md, HBM section: 128-B requests tallied as 64 B),
so bytes = FETCH_SIZE * 1024 * 2.  Infinity-Cache hits are counted as fetches.  The mean is
over every dispatch of the kernel family in the pass (the replayed decode steps plus the
bench's per-shape timing launches, same mixture of shapes)."""
import csv
import json
import sys
from collections import defaultdict


def main():
    src, dst = sys.argv[1], sys.argv[2]
    rows = [r for r in csv.DictReader(open(src)) if r["Counter_Name"] == "FETCH_SIZE"]
    fam = defaultdict(list)
    for r in rows:
        name = r["Kernel_Name"]
        key = "gemv_wq_kernel<4>" if "gemv_wq_kernel<4" in name else (
            "attn_split_kernel" if "attn_split_kernel" in name else ("pds_kernel" if "pds_kernel" in name else None))
        if key:
            fam[key].append(float(r["Counter_Value"]) * 1024.0 * 2.0)
    out = {"source": "rocprofv3 --pmc FETCH_SIZE (KiB, x2 gfx950 streaming-read correction)", "kernels": {}}
    for k, v in fam.items():
        out["kernels"][k] = {"dispatches": len(v), "traffic_bytes_per_launch": round(sum(v) / len(v)),
                             "min": round(min(v)), "max": round(max(v))}
    # The pass mixes the decode steps with the bench's per-class timing launches, so the plain
    # mean depends on that mixture.  Step-weighted: each dispatch is assigned to the projection
    # class whose algorithmic bytes are nearest (7B shapes), the per-class means are weighted by
    # the step's own mixture (32 x QKV, O, gate/up, down + 1 lm_head), comparable to the bench
    # line's bytes_per_launch.
    algo = {"qkv": 25960448, "o": 8658944, "gate_up": 46505984, "down": 23270912, "lm_head": 67592192}
    per = defaultdict(list)
    for b in fam.get("gemv_wq_kernel<4>", []):
        per[min(algo, key=lambda c: abs(algo[c] - b))].append(b)
    if len(per) == len(algo):
        n = {"qkv": 32, "o": 32, "gate_up": 32, "down": 32, "lm_head": 1}
        cls = {c: {"dispatches": len(per[c]), "traffic_bytes": round(sum(per[c]) / len(per[c])), "algorithmic_bytes": algo[c],
                   "ratio": round(sum(per[c]) / len(per[c]) / algo[c], 4)} for c in algo}
        tw = sum(n[c] * cls[c]["traffic_bytes"] for c in algo) / sum(n.values())
        aw = sum(n[c] * algo[c] for c in algo) / sum(n.values())
        out["kernels"]["gemv_wq_kernel<4>"].update({"classes": cls, "step_weighted_traffic_bytes_per_launch": round(tw),
                                                    "step_weighted_algorithmic_bytes_per_launch": round(aw),
                                                    "step_weighted_ratio": round(tw / aw, 4)})
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()

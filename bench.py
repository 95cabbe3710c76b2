#!/usr/bin/env python3
"""bench.py -- decode tokens/s per GPU, Llama-2-7B-shape INT4 (group 128) at 2048-token KV,
and the achieved fraction of the HBM-read roofline (BASELINE.json `metric`, configs[2]).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--kv L] [--model llama2-7b]

One process per GPU (torchrun for N > 1).  Each rank holds an independent replica of the
model with B decode streams (requests) and their fp16 KV caches in its own HBM: the path
shards by request, there is no collective on the data path (torch.distributed/gloo only
carries the barrier and the max-over-ranks of the timing).  A step = one decode token for
each of the rank's B streams, replayed at position L-1 so every step reads exactly L cache
slots (SURVEY 8(d) replay mode), greedy feedback on the device.  Synthetic random weights of
the named architecture (no checkpoints are reachable); `data` says so.

rank 0 prints ONE JSON line with the contract fields plus `roofline` (dominant kernel:
the W4 decode GEMM, live HIP-event timing on the engine stream) and `cpu_baseline` (the
compiled reference's own CPU decode ops timed on this host, rank 0 / N=1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

MODELS = {
    # name: (vocab, hidden, layers, heads, kv_heads, head_dim, inter, bits, rope_theta)
    "llama2-7b": (32000, 4096, 32, 32, 32, 128, 11008, 4, 10000.0),
    "tinyllama-1.1b": (32000, 2048, 22, 32, 4, 64, 5632, 8, 10000.0),
    "llama3-8b": (128256, 4096, 32, 32, 8, 128, 14336, 4, 500000.0),
}
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level parameters)


def step_bytes(m, B, L):
    """Algorithmic HBM bytes of one decode step: weights once + B streams' KV."""
    import turboinfer_amd as T
    V, H, layers, nh, nkv, hd, I, bits, _ = m
    lib = T.lib()

    def lin(K, N):
        return lib.ti_wpack_tile_bytes(bits, K, N) + lib.ti_wpack_scale_bytes(bits, K, N)

    w = layers * (lin(H, nh * hd + 2 * nkv * hd) + lin(nh * hd, H) + lin(H, 2 * I) + lin(I, H))
    w += lin(H, V) + (2 * layers + 1) * H * 4 + B * H * 2          # lm_head, norms (fp32), embedding rows
    kv_read = 2 * layers * nkv * hd * 2 * L
    kv_write = 2 * layers * nkv * hd * 2
    return w + B * (kv_read + kv_write), w


class Group:
    """Barrier / max over ranks.  World 1: trivial; otherwise torch.distributed over gloo
    (CPU-side only: nothing of the decode path goes through it)."""

    def __init__(self):
        self.rank = int(os.environ.get("RANK", "0"))
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        self.dist = None
        if self.world > 1:
            import torch.distributed as dist
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            dist.init_process_group("gloo", rank=self.rank, world_size=self.world)
            self.dist = dist

    def barrier(self):
        if self.dist:
            self.dist.barrier()

    def max(self, v: float) -> float:
        if not self.dist:
            return v
        import torch
        t = torch.tensor([float(v)], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def close(self):
        if self.dist:
            self.dist.destroy_process_group()


def cpu_baseline(m, L):
    """The reference's own CPU decode (oracle/_ref: unmodified sources, g++ -O3 -mavx2 -mfma):
    one layer of the reference-composed decode step (rms_norm, q/k/v/o matmul_3d_2d, apply_rope,
    multi_head_attention over L cached tokens, SwiGLU FFN) with int32-stored INT4 weights as
    Quantizer::quantize_model hands them to the engine, plus the lm_head matmul; token time =
    layers * layer + lm_head.  Bounded sample (~5-10 s of CPU work)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    try:
        from pyoracle import Reference
        ref = Reference()
    except Exception as exc:  # reference library not shipped with this checkout
        return {"value": None, "unit": "tokens/s", "cores": 1, "kind": "reference",
                "sample": f"unavailable: {exc}"}
    V, H, layers, nh, nkv, hd, I, bits, _ = m
    layer_s, head_s = ref.time_decode(H, nh, I, V, L, weight_kind=1, n_layers=1)
    tok_s = layers * layer_s + head_s
    return {"value": round(1.0 / tok_s, 6), "unit": "tokens/s", "cores": 1, "kind": "reference",
            "cpu_model": cpu_info(), "omp_num_threads": os.environ.get("OMP_NUM_THREADS"),
            "sample": f"1 decode layer ({layer_s:.2f} s) x {layers} + lm_head ({head_s:.2f} s) at L={L}, "
                      f"INT4 held as int32 (reference quantized path), 1 stream; matmul_3d_2d is single-threaded "
                      f"(tensor_engine.cpp:620-633, no OpenMP on the decode path, so OMP_NUM_THREADS does not "
                      f"change it); host {os.uname().machine}, {os.cpu_count()} logical CPUs"}


def pmc_traffic(kernel: str, model: str, batch: int):
    """HBM bytes per launch of `kernel` from the newest committed FETCH_SIZE pass of this
    configuration (profiles/r*_pmc_traffic*.json, written by tools/pmc_traffic.py from a separate
    `rocprofv3 --pmc FETCH_SIZE` run of this bench; files without a "config" are the default
    llama2-7b one-stream pass), or None."""
    import glob
    best = None
    for f in glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_traffic*.json")):
        try:
            d = json.load(open(f))
            c = d.get("config", {"model": "llama2-7b", "batch": 1})
            if c.get("model") != model or int(c.get("batch", 1)) != batch or kernel not in d["kernels"]:
                continue
            k = d["kernels"][kernel]
            v = int(k.get("step_weighted_traffic_bytes_per_launch", k["traffic_bytes_per_launch"]))
        except (KeyError, ValueError, OSError):
            continue
        tag = os.path.basename(f).split("_")[0]          # r<N>: newest round wins
        rank = (int(tag[1:]) if tag[1:].isdigit() else 0, f)
        if best is None or rank > best[0]:
            best = (rank, v, os.path.relpath(f, ROOT))
    return (best[1], best[2]) if best else (None, None)


def rank_plan(args, rank: int, vocab: int) -> dict:
    """What rank `rank` of a replica job runs: its own B = --batch streams (the request shard:
    global_batch = B x world), its weight seed, each stream's KV seed and the replay's first
    token.  Distinct per rank, so no two replicas decode the same requests."""
    B = args.batch
    return {"streams": B, "weight_seed": args.seed + rank,
            "kv_seeds": [args.seed + 1000 * rank + s for s in range(B)],
            "first_token": (args.seed + rank) % vocab}


def dry_run(g: "Group", args) -> int:
    """The replica path without a GPU: every rank takes part in the same two barriers and the
    max over ranks as a real run, with a fixed per-rank duration in place of the timed steps,
    and rank 0 gathers every rank's shard plan (rank_plan) to report it."""
    g.barrier()
    dt = g.max(0.001 * (g.rank + 1))
    plan = rank_plan(args, g.rank, MODELS[args.model][0])
    plans = [plan]
    if g.dist:
        plans = [None] * g.world
        g.dist.all_gather_object(plans, plan)
    g.barrier()
    if g.rank == 0:
        print(json.dumps({"metric": "decode tokens/s/GPU, Llama-7B-shape INT4 @2048 ctx; % HBM-read roofline",
                          "value": None, "dry_run": True, "n_gpus": g.world, "max_rank_s": dt,
                          "config": {"global_batch": args.batch * g.world, "parallelism": f"replicas{g.world}"},
                          "rank_plans": [{"rank": r, "streams": p["streams"], "weight_seed": p["weight_seed"],
                                          "first_token": p["first_token"], "kv_seed_first": p["kv_seeds"][0],
                                          "kv_seed_last": p["kv_seeds"][-1]} for r, p in enumerate(plans)]}))
    g.close()
    return 0


def cpu_info() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_replicas(n: int, argv: list) -> int:
    """`--gpus N` without a launcher: start N ranks of this script (one per GPU) as child
    processes and wait for them.  This process never touches a GPU (nothing here makes a HIP
    call), so no program is exec'd after GPU initialisation.  The children do the same
    barrier / max-over-ranks timing as under torch.distributed.run; rank 0's JSON line is
    passed through."""
    import subprocess
    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env,
                                      stdout=subprocess.PIPE if r == 0 else subprocess.DEVNULL))
    out, _ = procs[0].communicate()
    rcs = [procs[0].returncode] + [p.wait() for p in procs[1:]]
    sys.stdout.write(out.decode())
    sys.stdout.flush()
    bad = [rc for rc in rcs if rc != 0]
    return bad[0] if bad else 0


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1, help="replicas, one process per GPU (spawned here when no "
                                                        "launcher has set WORLD_SIZE)")
    ap.add_argument("--steps", type=int, default=256)
    ap.add_argument("--warmup", type=int, default=16)
    ap.add_argument("--batch", type=int, default=1, help="decode streams per GPU")
    ap.add_argument("--kv", type=int, default=2048, help="KV length read per step")
    ap.add_argument("--model", default="llama2-7b", choices=sorted(MODELS))
    ap.add_argument("--seed", type=int, default=0x7157)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--kernel-reps", type=int, default=50)
    ap.add_argument("--stamp-steps", type=int, default=20, help="stamped step replays for the in-step roofline")
    ap.add_argument("--attn-splits", type=int, default=0, help="0 = the engine's policy")
    ap.add_argument("--dry-run", action="store_true",
                    help="CPU-only rehearsal of the replica launch / barrier / max-over-ranks path: no GPU, "
                         "no engine; prints the JSON line with value null (tests)")
    args = ap.parse_args()

    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None and args.gpus > 1:
        return spawn_replicas(args.gpus, sys.argv[1:])
    if world_env is not None and int(world_env) != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={world_env} ranks", file=sys.stderr)
        return 2

    g = Group()
    if args.dry_run:
        return dry_run(g, args)

    import turboinfer_amd as T

    T.init(g.local_rank)
    # same-run calibration of this box's HBM: every rate below can be read
    # against it (1 GiB read by 2 workgroups per CU; device-to-device copy, read + write bytes)
    hbm_read, hbm_copy = T.hbm_calibrate(1 << 30, 5)
    m = MODELS[args.model]
    V, H, layers, nh, nkv, hd, I, bits, theta = m
    B, L = args.batch, args.kv
    e = T.Engine(V, H, layers, nh, nkv, hd, I, bits=bits, max_seq=L, max_batch=B, rope_theta=theta,
                 device=g.local_rank, attn_splits=args.attn_splits)
    plan = rank_plan(args, g.rank, V)
    e.synth(plan["weight_seed"], 0.0)
    for s in range(B):
        e.fill_kv(s, L - 1, plan["kv_seeds"][s])
    e.replay_prepare(B, L, plan["first_token"])

    e.replay_run(args.warmup)
    e.sync()
    g.barrier()
    e.sync()
    t0 = time.perf_counter()
    e.replay_run(args.steps)
    e.sync()
    t1 = time.perf_counter()
    g.barrier()
    dt = g.max(t1 - t0)

    tokens = B * args.steps * g.world
    value = tokens / dt
    ms_per_step = dt / args.steps * 1000.0
    sb, wb = step_bytes(m, B, L)

    # Dominant kernel.  Live timing on the engine stream (ti_engine_time_kernel): the launches of
    # one class as the step runs them (same kernel, x mode and epilogue), cycling through the
    # layers so the weights come from HBM, captured into a graph and replayed back to back for
    # several ms between two HIP events.  The decode GEMM family: layers x (qkv, o, gate/up,
    # down) + lm_head launches, achieved = sum(bytes) / sum(time), which is what
    # profiles/*_kernel_stats.txt gives as sum(calls x bytes) / total time over the same rows;
    # each class names its kernel.
    names = ["qkv", "o", "gate_up", "down", "lm_head"]
    shapes = {"qkv": (nh * hd + 2 * nkv * hd, H), "o": (H, nh * hd), "gate_up": (2 * I, H), "down": (H, I),
              "lm_head": (V, H)}
    fold_on = B == 1 and e.set_fold(None)
    # one stream of a GQA head_dim-64 model: QKV and the attention run as ONE launch (ti_qkv_attn_partials,
    # DESIGN 4.19); its class "qkv" then carries the attention's bytes too and there is no attention class
    qa_on = B == 1 and hasattr(e, "set_qkv_attn") and e.set_qkv_attn(None)
    lib = T.lib()

    def class_kernel(name):
        N_, K_ = shapes[name]
        if name in ("qkv", "gate_up", "lm_head"):
            if fold_on:
                xk = T.X_F16_FOLDED
            elif bits == 4 and B > 1 and lib.ti_gemm_packed_rows_for(bits, B, N_, K_):
                xk = T.X_F16_PACKED
            elif lib.ti_gemm_max_rows(bits, T.X_F32_RMSNORM, N_, K_) < B:
                xk = T.X_F16
            else:
                xk = T.X_F32_RMSNORM
        elif name == "o" and B == 1:
            xk = T.X_ATTN_SPLITS
        else:
            xk = T.X_F16_PACKED if bits == 4 and lib.ti_gemm_packed_rows(bits, B) else T.X_F16
        return T.gemm_kernel_name(bits, xk, B, N_, K_)

    # In-step timing: the replay step graph captured with per-workgroup
    # s_memrealtime stamps (ti_engine_stamp_steps).  A launch's duration is its period in the step:
    # its first workgroup's entry -> the next launch's first entry (its boundary included; the
    # periods of a step add up to the step), averaged over the class's launches and `stamp_steps`
    # replays -- what a kernel trace's dispatch-to-completion duration measures.  The in-kernel span
    # (first entry -> last wave end) and the isolated class timing (ti_engine_time_kernel: graphs of
    # one class's launches; it also gives each class's algorithmic bytes) are reported beside it.
    stamps = e.stamp_steps(args.stamp_steps)
    in_step = {}
    for d in stamps:
        if d["workgroups"] == 0:
            continue
        c = in_step.setdefault(d["tag"], {"n": 0, "span": 0.0, "period": 0.0, "gap": 0.0, "cu_shared": 0.0})
        c["n"] += 1
        c["span"] += d["span_us"]
        c["period"] += d["period_us"]
        c["gap"] += d["gap_us"]
        c["cu_shared"] += d["cu_shared_wgs"]
    tag_of = {"qkv": "qkv", "o": "o", "gate_up": "gate_up", "down": "down", "lm_head": "lm_head", "attention": "attention"}
    per = {}
    gemv_bytes = gemv_us = gemv_iso_us = gemv_span_us = 0.0
    n_launch = 0
    kernels_used = {}
    att_iso = e.time_kernel(5, B, L, args.kernel_reps) if qa_on else None
    for w, name in enumerate(names + ["attention"]):
        if name == "attention" and qa_on:
            break
        iso_us, by = e.time_kernel(w, B, L, args.kernel_reps)
        c = in_step[tag_of[name]]
        us = c["period"] / c["n"]
        kname = "attn_split_kernel" if name == "attention" else class_kernel(name)
        if name == "qkv" and qa_on:   # the fused launch: the q / k / v weights and the K / V it attends over
            by += att_iso[1]
            iso_us += att_iso[0]      # (isolated: the two unfused launches, for comparison)
            kname = f"qkv_attn_kernel<{bits},{hd}> (QKV + attention, one launch)"
        per[name] = {"avg_us": round(us, 3), "bytes": int(by), "GBps": round(by / us / 1e3, 1), "kernel": kname,
                     "in_step_launches": c["n"], "span_us": round(c["span"] / c["n"], 3),
                     "gap_us": round(c["gap"] / c["n"], 3), "cu_shared_wgs": round(c["cu_shared"] / c["n"], 2),
                     "isolated_us": round(iso_us, 3)}
        if name == "attention":
            break
        cnt = c["n"]
        kernels_used.setdefault(kname, []).append(name)
        gemv_bytes += by * cnt
        gemv_us += us * cnt
        gemv_iso_us += iso_us * cnt
        gemv_span_us += c["span"]
        n_launch += cnt
    att_bytes = att_iso[1] if qa_on else per["attention"]["bytes"]
    dom = {"kernel": " + ".join(f"{k} ({', '.join(v)})" for k, v in kernels_used.items()),
           "bytes_per_launch": int(gemv_bytes / n_launch), "avg_launch_us": round(gemv_us / n_launch, 3),
           "timing": f"in-step: per-workgroup s_memrealtime stamps of the replay step graph, {args.stamp_steps} "
                     f"replays; launch duration = first workgroup entry -> next launch's first entry "
                     f"(ti_engine_stamp_steps)",
           "span_frac": round(gemv_bytes / gemv_span_us / 1e3 / HBM_PEAK_GBS, 4),
           "isolated_frac": round(gemv_bytes / gemv_iso_us / 1e3 / HBM_PEAK_GBS, 4),
           "step_stamped_us": round(sum(d["period_us"] for d in stamps), 1)}
    achieved = gemv_bytes / gemv_us / 1e3   # GB/s
    e.close()

    traffic, traffic_src = pmc_traffic(f"gemv_wq_kernel<{bits}>" if B == 1 else "gemm_family", args.model, B)
    att_traffic, _ = pmc_traffic("attn_split_kernel", args.model, B)
    result = None
    if g.rank == 0:
        result = {
            "metric": "decode tokens/s/GPU, Llama-7B-shape INT4 @2048 ctx; % HBM-read roofline",
            "value": round(value, 3),
            "unit": "tokens/s",
            "n_gpus": g.world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "w4a16" if bits == 4 else ("w8a16" if bits == 8 else "f16"),
            "data": "synthetic (seeded random weights of the named architecture, quantized per group of 128; "
                    "synthetic fp16 KV cache)",
            "config": {"workload": f"{args.model} INT{bits} g128 decode, {B} stream(s)/GPU, KV {L}, replay at pos {L - 1}",
                       "model": args.model, "global_batch": B * g.world, "seq_len": L,
                       "parallelism": f"replicas{g.world} (request-sharded, no collectives)"},
            "roofline": dict({"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                              "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                              "traffic_source": traffic_src}, **dom),
            "attention_roofline": ({"bound": "hbm", "kernel": "attn_split_kernel", "achieved": per["attention"]["GBps"],
                                    "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                    "frac": round(per["attention"]["GBps"] / HBM_PEAK_GBS, 4), "traffic": att_traffic,
                                    "share_of_step_bytes": round(layers * att_bytes / sb, 4)} if not qa_on else
                                   {"fused_into": "qkv", "share_of_step_bytes": round(layers * att_bytes / sb, 4)}),
            "calibration": {"hbm_read_GBps": round(hbm_read, 1), "hbm_copy_GBps": round(hbm_copy, 1),
                            "note": "same run, this GPU: 1 GiB streamed once by 2 workgroups per CU (read) and "
                                    "hipMemcpyAsync device-to-device (read + write bytes); best of 5"},
            "step_roofline": {"bytes_per_step": int(sb), "weight_bytes": int(wb),
                              "achieved_GBps": round(sb / (ms_per_step * 1e-3) / 1e9, 1),
                              "frac": round(sb / (ms_per_step * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                              "roofline_tokens_per_s_per_gpu": round(B * HBM_PEAK_GBS * 1e9 / sb, 1)},
            "kernels": per,
        }
        if g.world == 1 and not args.no_cpu_baseline:
            result["cpu_baseline"] = cpu_baseline(m, L)
        else:
            result["cpu_baseline"] = None
    g.barrier()
    g.close()
    if result is not None:
        print(json.dumps(result))
    return 0


if __name__ == "__main__":
    sys.exit(main())

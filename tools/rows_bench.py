"""Microbenchmark of ti_gemm_wq_a16's batched-rows path (M > 16) on the Llama-2-7B and
Llama-3-8B decode shapes, with cold weights (launches cycle through enough weight copies to
exceed the 256 MiB Infinity Cache), timed between HIP events.

    python tools/rows_bench.py [M ...]

Prints us per launch and GB/s of algorithmic bytes (packed weights + scales + fp16 rows).
Compare kernels with TI_GEMM_ROWS=0/1 and TI_GEMM_ROWS_RG=1/2; TI_GEMM_SPLITK=0 (or
ROWS_SPLITK_MB=0: no workspace) for the batched-rows kernel instead of the split-K tile GEMM."""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import turboinfer_amd as T  # noqa: E402

ROWMAJOR = os.environ.get("ROWS_X") == "rowmajor"
SPLITK_MB = int(os.environ.get("ROWS_SPLITK_MB", "64"))   # the engine's split-K workspace (0: none)
Ms = [int(a) for a in sys.argv[1:]] or [32, 64]
T.init(0)
L = T.lib()
shapes = [("7b qkv", 4096, 12288), ("7b o", 4096, 4096), ("7b gate_up", 4096, 22016), ("7b down", 11008, 4096),
          ("7b lm_head", 4096, 32000), ("l3 qkv", 4096, 6144), ("l3 gate_up", 4096, 28672), ("l3 down", 14336, 4096)]
ws = T.DeviceBuffer(max(SPLITK_MB, 1) << 20)
ws.zero()
ev0, ev1 = C.c_void_p(), C.c_void_p()
T.check(L.ti_event_create(C.byref(ev0)))
T.check(L.ti_event_create(C.byref(ev1)))
for name, K, N in shapes:
    tb, sb = L.ti_wpack_tile_bytes(4, K, N), L.ti_wpack_scale_bytes(4, K, N)
    copies = max(2, int(320e6 // (tb + sb)) + 1)
    W = []
    for c in range(copies):
        tiles, scales = T.DeviceBuffer(tb), T.DeviceBuffer(sb)
        T.check(L.ti_wsynth_device(1, 7 + c, K, N, N, 4, 0, 0, tiles.ptr, scales.ptr, None))
        W.append((tiles, scales))
    for M in Ms:
        XK = T.X_F16 if ROWMAJOR or not T.lib().ti_gemm_packed_rows(4, M) else T.X_F16_PACKED
        # (packed operands cover whole 16-row blocks: the buffer holds ceil(M / 16) * 16 rows)
        MP = (M + 15) // 16 * 16 if XK == T.X_F16_PACKED else M
        x16 = T.DeviceBuffer.from_array(np.random.RandomState(0).standard_normal((MP, K)).astype(np.float16))
        y = T.DeviceBuffer(M * N * 4)
        ep = T.Epilogue()
        ep.kind, ep.ldo, ep.out = T.EPI_STORE_F32, N, y.ptr
        if SPLITK_MB:
            ep.splitk_ws, ep.splitk_bytes = ws.ptr, SPLITK_MB << 20
        plan = ""
        a, b, c = C.c_int(), C.c_int(), C.c_int()
        if L.ti_gemm_tile_plan(4, M, N, K, (SPLITK_MB << 20) if SPLITK_MB else 0, C.byref(a), C.byref(b), C.byref(c)) == 0:
            plan = f" tile wmr{a.value} tpw{b.value} ks{c.value}"

        def run(i):
            t, s = W[i % copies]
            T.check(L.ti_gemm_wq_a16(t.ptr, s.ptr, 4, x16.ptr, XK, K, None, 1e-5, M, N, K, C.byref(ep), None))

        for i in range(copies):
            run(i)
        T.sync()
        reps = 4 * copies
        T.check(L.ti_event_record(ev0, None))
        for i in range(reps):
            run(i)
        T.check(L.ti_event_record(ev1, None))
        ms = C.c_float()
        T.check(L.ti_event_elapsed_ms(ev0, ev1, C.byref(ms)))
        us = ms.value * 1e3 / reps
        by = tb + sb + M * K * 2
        print(f"M={M:3d} {name:11s} K={K:6d} N={N:6d} {us:8.2f} us  {by / us / 1e3:8.1f} GB/s  {2 * M * K * N / us / 1e6:7.1f} TFLOP/s{plan}", flush=True)
    del W

import ctypes as C, os, sys
import numpy as np
sys.path.insert(0, os.environ["GRAFT_REPO_ROOT"])
import turboinfer_amd as T
T.init(0); L = T.lib()
ev0, ev1 = C.c_void_p(), C.c_void_p()
T.check(L.ti_event_create(C.byref(ev0))); T.check(L.ti_event_create(C.byref(ev1)))
for name, K, N in [("o", 4096, 4096), ("down", 11008, 4096)]:
    tb, sb = L.ti_wpack_tile_bytes(4, K, N), L.ti_wpack_scale_bytes(4, K, N)
    copies = max(2, int(320e6 // (tb + sb)) + 1)
    W = []
    for c in range(copies):
        t, s = T.DeviceBuffer(tb), T.DeviceBuffer(sb)
        T.check(L.ti_wsynth_device(1, 7 + c, K, N, N, 4, 0, 0, t.ptr, s.ptr, None)); W.append((t, s))
    for M in (33, 40, 47, 48, 49, 56, 63, 64):
        for xk in (T.X_F16_PACKED, T.X_F16):
            x16 = T.DeviceBuffer.from_array(np.random.RandomState(0).standard_normal((max(M, 64), K)).astype(np.float16))
            y = T.DeviceBuffer(M * N * 4); ep = T.Epilogue(); ep.kind, ep.ldo, ep.out = T.EPI_STORE_F32, N, y.ptr
            run = lambda i: T.check(L.ti_gemm_wq_a16(W[i % copies][0].ptr, W[i % copies][1].ptr, 4, x16.ptr, xk, K, None, 1e-5, M, N, K, C.byref(ep), None))
            for i in range(copies): run(i)
            T.sync(); reps = 4 * copies
            T.check(L.ti_event_record(ev0, None))
            for i in range(reps): run(i)
            T.check(L.ti_event_record(ev1, None)); ms = C.c_float(); T.check(L.ti_event_elapsed_ms(ev0, ev1, C.byref(ms)))
            print(name, M, "packed" if xk == T.X_F16_PACKED else "rowmajor", round(ms.value * 1e3 / reps, 2), flush=True)
    del W

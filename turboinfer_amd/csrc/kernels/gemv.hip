// gemv.hip -- fused weight-dequant x fp16 decode GEMM for gfx950 (ti_gemm_wq_a16).
//
// Replaces the decode projections of the reference: TensorEngine::matmul ->
// matmul_3d_2d (src/core/tensor_engine.cpp:594-640, scalar fp32, one core) with the
// int weights' convert_dtype (:2218-2284), plus the neighbouring element-wise ops of
// TransformerLayer::forward (src/model/inference_engine.cpp:203-233, 376-401).
//
// Shape of the work (M <= 16 decode rows, N outputs, K inputs):
//   * one workgroup = 8 waves = one 16-row output tile; the waves interleave over the
//     K/128 k-tiles (wave w takes k-tiles w, w+8, ...), each wave keeping B k-tiles of
//     packed weights in flight as plain dwordx4 loads straight into VGPRs (weights are
//     streamed once -- no LDS round trip, cdna_hip_programming.md "GEMV / M <= 16").
//   * the activation row(s) are staged once per workgroup in LDS as fp16 (the rms_norm
//     prologue is fused here), read back as MFMA A fragments with ds_read_b128.
//   * per k-tile: 4 x v_mfma_f32_16x16x32_f16 on (x, dequantized W) then one fp32 FMA by
//     the group scale; int4 nibbles -> fp16 with the 0x6400 magic (exact), int8 with
//     v_perm_b32 + the same magic.
//   * the 8 waves' partial tiles are summed in LDS in a fixed order (deterministic) and
//     the epilogue (residual add, SiLU*up, RoPE + KV append, logits + argmax) runs on the
//     16 x M results of the tile.
#include <math.h>

#include "common.hpp"

namespace ti {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int kGemvWaves = 8;
constexpr int kGemvThreads = kGemvWaves * kWave;

struct GemvArgs {
  const u32x4* tiles;
  const uint16_t* scales;
  const void* x;
  const float* norm_w;
  float eps;
  int32_t x_kind, ldx, M, N, K;
  ti_epilogue epi;
};

__host__ __device__ constexpr int align16(int b) { return (b + 15) & ~15; }

__host__ __device__ inline int gemv_lds_bytes(int M, int K) {
  const int KT = K >> 7;
  return align16(M * (K + 8) * 2) + align16(KT * 32) + kGemvWaves * kWave * 4 * 4;
}

// ------------------------------------------------------------------- dequant
// int4: word of 8 nibbles, nibble p holds element 2p, nibble p+4 element 2p+1, value q+8.
__device__ __forceinline__ f16x8 deq_int4_word(uint32_t w) {
  f16x8 r;
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const uint32_t t = ((w >> (4 * p)) & 0x000F000Fu) | 0x64006400u;   // fp16 1024+n, exact
    const f16x2 h = __builtin_bit_cast(f16x2, t) - (f16x2){(f16)1032.0f, (f16)1032.0f};
    r[2 * p] = h[0];
    r[2 * p + 1] = h[1];
  }
  return r;
}
// int8: 4 signed bytes in k order; (b ^ 0x80) = b + 128 -> fp16 1024 + b + 128 - 1152.
__device__ __forceinline__ f16x2 deq_int8_pair(uint32_t t, uint32_t sel) {
  const uint32_t v = __builtin_amdgcn_perm(0x64646464u, t, sel);
  return __builtin_bit_cast(f16x2, v) - (f16x2){(f16)1152.0f, (f16)1152.0f};
}
__device__ __forceinline__ void deq_int8_word(uint32_t w, f16x8& r, int o) {
  const uint32_t t = w ^ 0x80808080u;
  const f16x2 lo = deq_int8_pair(t, 0x04010400u), hi = deq_int8_pair(t, 0x04030402u);
  r[o + 0] = lo[0];
  r[o + 1] = lo[1];
  r[o + 2] = hi[0];
  r[o + 3] = hi[1];
}

template <int BITS>
__device__ __forceinline__ f16x8 dequant_step(const u32x4 (&w)[BITS / 4], int s4) {
  if constexpr (BITS == 4) {
    return deq_int4_word(w[0][s4]);
  } else if constexpr (BITS == 8) {
    f16x8 r;
    const u32x4 c = w[s4 >> 1];
    deq_int8_word(c[(s4 & 1) * 2 + 0], r, 0);
    deq_int8_word(c[(s4 & 1) * 2 + 1], r, 4);
    return r;
  } else {
    return __builtin_bit_cast(f16x8, w[s4]);
  }
}

// ------------------------------------------------------------- x staging (LDS)
__device__ __forceinline__ void stage_x(const GemvArgs& a, f16* xl, float* red) {
  const int tid = threadIdx.x, K = a.K, xs = K + 8, K8 = K >> 3;
  if (a.x_kind == TI_X_F32_RMSNORM) {
    // rms_norm (tensor_engine.cpp:1488-1505): y = (x / sqrt(sum(x^2)/K + eps)) * w.
    for (int m = 0; m < a.M; ++m) {
      const float* xr = (const float*)a.x + (size_t)m * a.ldx;
      float ss = 0.0f;
      for (int k8 = tid; k8 < K8; k8 += kGemvThreads) {
        const float4 v0 = *(const float4*)(xr + 8 * k8), v1 = *(const float4*)(xr + 8 * k8 + 4);
        ss = fmaf(v0.x, v0.x, ss); ss = fmaf(v0.y, v0.y, ss); ss = fmaf(v0.z, v0.z, ss); ss = fmaf(v0.w, v0.w, ss);
        ss = fmaf(v1.x, v1.x, ss); ss = fmaf(v1.y, v1.y, ss); ss = fmaf(v1.z, v1.z, ss); ss = fmaf(v1.w, v1.w, ss);
      }
      ss = wave_sum_xor<kWave>(ss);
      if ((tid & 63) == 0) red[tid >> 6] = ss;
      __syncthreads();
      float tot = 0.0f;
#pragma unroll
      for (int w = 0; w < kGemvWaves; ++w) tot += red[w];
      const float rms = sqrtf(tot / (float)K + a.eps);
      for (int k8 = tid; k8 < K8; k8 += kGemvThreads) {
        const float4 v0 = *(const float4*)(xr + 8 * k8), v1 = *(const float4*)(xr + 8 * k8 + 4);
        const float4 w0 = *(const float4*)(a.norm_w + 8 * k8), w1 = *(const float4*)(a.norm_w + 8 * k8 + 4);
        f16x8 h;
        h[0] = (f16)((v0.x / rms) * w0.x); h[1] = (f16)((v0.y / rms) * w0.y);
        h[2] = (f16)((v0.z / rms) * w0.z); h[3] = (f16)((v0.w / rms) * w0.w);
        h[4] = (f16)((v1.x / rms) * w1.x); h[5] = (f16)((v1.y / rms) * w1.y);
        h[6] = (f16)((v1.z / rms) * w1.z); h[7] = (f16)((v1.w / rms) * w1.w);
        *(f16x8*)(xl + m * xs + 8 * k8) = h;
      }
      __syncthreads();   // red reused by the next row
    }
  } else if (a.x_kind == TI_X_F32) {
    for (int i = tid; i < a.M * K8; i += kGemvThreads) {
      const int m = i / K8, k8 = i - m * K8;
      const float* xr = (const float*)a.x + (size_t)m * a.ldx + 8 * k8;
      const float4 v0 = *(const float4*)xr, v1 = *(const float4*)(xr + 4);
      f16x8 h;
      h[0] = (f16)v0.x; h[1] = (f16)v0.y; h[2] = (f16)v0.z; h[3] = (f16)v0.w;
      h[4] = (f16)v1.x; h[5] = (f16)v1.y; h[6] = (f16)v1.z; h[7] = (f16)v1.w;
      *(f16x8*)(xl + m * xs + 8 * k8) = h;
    }
  } else {
    for (int i = tid; i < a.M * K8; i += kGemvThreads) {
      const int m = i / K8, k8 = i - m * K8;
      *(u32x4*)(xl + m * xs + 8 * k8) = *(const u32x4*)((const f16*)a.x + (size_t)m * a.ldx + 8 * k8);
    }
  }
}

// ------------------------------------------------------------------ epilogue
__device__ __forceinline__ uint32_t float_order_key(float v) {
  const uint32_t u = __builtin_bit_cast(uint32_t, v);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

// Runs in waves 0..3: thread t holds y[m][n] of tile nt with l = t & 63, i = t >> 6,
// m = 4*(l>>4) + i, n = l & 15 (the v_mfma_f32_16x16x32 C layout, reduced over waves).
__device__ __forceinline__ void epilogue(const GemvArgs& a, int nt, int l, int i, float v) {
  const ti_epilogue& e = a.epi;
  const int m = 4 * (l >> 4) + i, n = l & 15, ng = nt * 16 + n;
  const bool live = m < a.M;
  switch (e.kind) {
    case TI_EPI_STORE_F32:
      if (live) ((float*)e.out)[(size_t)m * e.ldo + ng] = v;
      break;
    case TI_EPI_STORE_F16:
      if (live) ((uint16_t*)e.out)[(size_t)m * e.ldo + ng] = f2h(v);
      break;
    case TI_EPI_RESID_F32:
      if (live) ((float*)e.out)[(size_t)m * e.ldo + ng] += v;   // add(residual, y), :1626-1678
      break;
    case TI_EPI_SILU_MUL_F16: {
      // compute_ffn (inference_engine.cpp:386-391): multiply(up, silu(gate)).
      const float up = __shfl_down(v, 8, kWave);
      if (live && n < 8) {
        const float s = v / (1.0f + expf(-v));
        ((uint16_t*)e.out)[(size_t)m * e.ldo + nt * 8 + n] = f2h(up * s);
      }
      break;
    }
    case TI_EPI_QKV_ROPE_KV: {
      const float partner = __shfl_xor(v, 1, kWave);
      if (!live) break;
      const int p = e.pos[m];
      const int hd = e.head_dim;
      if (ng < e.q_dim + e.kv_dim) {
        const int base = ng < e.q_dim ? 0 : e.q_dim;
        const int d = (ng - base) % hd;
        const float2 cs = *(const float2*)(e.rope_cs + ((size_t)p * (hd >> 1) + (d >> 1)) * 2);
        // apply_rope (tensor_engine.cpp:1602-1612): even = x*c - y*s, odd = x*s + y*c,
        // evaluated with the reference build's contraction pattern.
        const float r = (d & 1) == 0 ? fmaf(-partner, cs.y, v * cs.x) : fmaf(v, cs.x, partner * cs.y);
        if (ng < e.q_dim) {
          ((float*)e.out)[(size_t)m * e.ldo + ng] = r;
        } else {
          const int kvh = (ng - e.q_dim) / hd;
          e.k_cache[(size_t)m * e.kv_stream_stride + ((size_t)kvh * e.max_seq + p) * hd + d] = f2h(r);
        }
      } else {
        const int c = ng - e.q_dim - e.kv_dim;
        const int kvh = c / hd, d = c - kvh * hd;
        e.v_cache[(size_t)m * e.kv_stream_stride + ((size_t)kvh * e.max_seq + p) * hd + d] = f2h(v);
      }
      break;
    }
    case TI_EPI_LOGITS_ARGMAX: {
      if (live) ((float*)e.out)[(size_t)m * e.ldo + ng] = v;
      unsigned long long key = live ? (((unsigned long long)float_order_key(v) << 32) |
                                       (unsigned long long)(0xFFFFFFFFu - (uint32_t)ng))
                                    : 0ull;
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {
        const unsigned long long other = __shfl_xor(key, o, kWave);
        key = other > key ? other : key;
      }
      if (live && n == 0) atomicMax(e.argmax + m, key);
      if (e.step_ctr && blockIdx.x == 0 && threadIdx.x == 0) *e.step_ctr += e.advance;
      break;
    }
    default:
      break;
  }
}

// --------------------------------------------------------------------- kernel
template <int BITS>
__global__ __launch_bounds__(kGemvThreads, 2) void gemv_wq_kernel(const GemvArgs a) {
  constexpr int C = TileFmt<BITS>::kChunks;
  constexpr int B = (BITS == 16) ? 2 : 4;                      // k-tiles per wave in flight
  constexpr int S = kGemvWaves;                                // k-tile stride between a wave's tiles
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int KT = a.K >> 7, xs = a.K + 8;
  const int nt = blockIdx.x;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  f16* xl = (f16*)smem;
  uint16_t* sl = (uint16_t*)(smem + align16(a.M * xs * 2));
  float* red = (float*)(smem + align16(a.M * xs * 2) + align16(KT * 32));

  // Issue the first weight batch before anything else so HBM latency overlaps the
  // x / scale staging.  Out-of-range k-tiles re-load the last tile (no branch around
  // the loads; their compute is skipped).
  const u32x4* tb = a.tiles + (size_t)nt * KT * (kWave * C);
  u32x4 cur[B][C];
#pragma unroll
  for (int i = 0; i < B; ++i) {
    const int kt = min(wave + i * S, KT - 1);
#pragma unroll
    for (int c = 0; c < C; ++c) cur[i][c] = tb[((size_t)kt * C + c) * kWave + lane];
  }

  if constexpr (BITS != 16) {
    const u32x4* sg = (const u32x4*)(a.scales + (size_t)nt * KT * 16);
    for (int i = tid; i < KT * 2; i += kGemvThreads) ((u32x4*)sl)[i] = sg[i];
  }
  stage_x(a, xl, red);
  __syncthreads();

  const int r = lane & 15, kq = lane >> 4;
  const f16* xrow = xl + (r < a.M ? r : a.M - 1) * xs + kq * 32;
  f32x4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
  for (int kb = wave; kb < KT; kb += B * S) {
    const int kn = kb + B * S;
    const bool more = kn < KT;
    u32x4 nxt[B][C];
    if (more) {
#pragma unroll
      for (int i = 0; i < B; ++i) {
        const int kt = min(kn + i * S, KT - 1);
#pragma unroll
        for (int c = 0; c < C; ++c) nxt[i][c] = tb[((size_t)kt * C + c) * kWave + lane];
      }
    }
#pragma unroll
    for (int i = 0; i < B; ++i) {
      const int kt = kb + i * S;
      if (kt < KT) {
        f32x4 t = {0.0f, 0.0f, 0.0f, 0.0f};
        if constexpr (BITS == 16) t = acc;
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) {
          const f16x8 bf = dequant_step<BITS>(cur[i], s4);
          const f16x8 af = *(const f16x8*)(xrow + kt * 128 + s4 * 8);
          t = __builtin_amdgcn_mfma_f32_16x16x32_f16(af, bf, t, 0, 0, 0);
        }
        if constexpr (BITS == 16) {
          acc = t;
        } else {
          const float sc = h2f(sl[kt * 16 + r]);
          acc[0] = fmaf(sc, t[0], acc[0]);
          acc[1] = fmaf(sc, t[1], acc[1]);
          acc[2] = fmaf(sc, t[2], acc[2]);
          acc[3] = fmaf(sc, t[3], acc[3]);
        }
      }
    }
    if (more) {
#pragma unroll
      for (int i = 0; i < B; ++i)
#pragma unroll
        for (int c = 0; c < C; ++c) cur[i][c] = nxt[i][c];
    }
  }

  // Cross-wave reduction in a fixed order, then the epilogue on waves 0..3.
  *(f32x4*)(red + (wave * kWave + lane) * 4) = acc;
  __syncthreads();
  if (tid < 4 * kWave) {
    const int l = tid & 63, i = tid >> 6;
    float v = 0.0f;
#pragma unroll
    for (int w = 0; w < kGemvWaves; ++w) v += red[(w * kWave + l) * 4 + i];
    epilogue(a, nt, l, i, v);
  }
}

template <int BITS>
static int launch_gemv(const GemvArgs& a, int lds, hipStream_t s) {
  hipLaunchKernelGGL(gemv_wq_kernel<BITS>, dim3(a.N / 16), dim3(kGemvThreads), lds, s, a);
  TI_LAUNCH_CHECK("gemv_wq_kernel");
  return TI_OK;
}

static bool g_prepared = false;

}  // namespace ti

// Raise the dynamic-LDS cap of the GEMM instantiations (call before any stream capture).
extern "C" int ti_gemm_prepare(void) {
  using namespace ti;
  if (g_prepared) return TI_OK;
  TI_HIP_CHECK(hipFuncSetAttribute((const void*)gemv_wq_kernel<4>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   160 * 1024), "hipFuncSetAttribute(gemv<4>)");
  TI_HIP_CHECK(hipFuncSetAttribute((const void*)gemv_wq_kernel<8>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   160 * 1024), "hipFuncSetAttribute(gemv<8>)");
  TI_HIP_CHECK(hipFuncSetAttribute((const void*)gemv_wq_kernel<16>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   160 * 1024), "hipFuncSetAttribute(gemv<16>)");
  g_prepared = true;
  return TI_OK;
}

extern "C" int ti_gemm_lds_bytes(int M, int K) { return ti::gemv_lds_bytes(M, K); }

extern "C" int ti_gemm_wq_a16(const void* tiles, const uint16_t* scales, int bits, const void* x,
                              int x_kind, int ldx, const float* norm_w, float eps, int M, int N, int K,
                              const ti_epilogue* epi, ti_stream_t stream) {
  using namespace ti;
  if (!tiles || !x || !epi || !epi->out) return ti_set_error(TI_ERR_ARG, "ti_gemm_wq_a16: null pointer");
  if (bits != 4 && bits != 8 && bits != 16)
    return ti_set_error(TI_ERR_ARG, "ti_gemm_wq_a16: bits must be 4, 8 or 16 (got %d)", bits);
  if (bits != 16 && !scales) return ti_set_error(TI_ERR_ARG, "ti_gemm_wq_a16: scales required for bits %d", bits);
  if (M < 1 || M > 16) return ti_set_error(TI_ERR_ARG, "ti_gemm_wq_a16: M must be in [1,16] (got %d)", M);
  if (K <= 0 || (K & 127) || N <= 0 || (N & 15))
    return ti_set_error(TI_ERR_ARG, "ti_gemm_wq_a16: K %% 128 and N %% 16 must be 0 (K=%d N=%d)", K, N);
  if (x_kind < TI_X_F16 || x_kind > TI_X_F32_RMSNORM)
    return ti_set_error(TI_ERR_ARG, "ti_gemm_wq_a16: bad x_kind %d", x_kind);
  if (x_kind == TI_X_F32_RMSNORM && !norm_w) return ti_set_error(TI_ERR_ARG, "ti_gemm_wq_a16: norm_w required");
  if (ldx < K) return ti_set_error(TI_ERR_ARG, "ti_gemm_wq_a16: ldx %d < K %d", ldx, K);
  switch (epi->kind) {
    case TI_EPI_STORE_F32: case TI_EPI_STORE_F16: case TI_EPI_RESID_F32:
      if (epi->ldo < N) return ti_set_error(TI_ERR_ARG, "ti_gemm_wq_a16: ldo %d < N %d", epi->ldo, N);
      break;
    case TI_EPI_SILU_MUL_F16:
      if (epi->ldo < N / 2) return ti_set_error(TI_ERR_ARG, "ti_gemm_wq_a16: ldo < N/2");
      break;
    case TI_EPI_QKV_ROPE_KV:
      if (!epi->pos || !epi->rope_cs || !epi->k_cache || !epi->v_cache || epi->head_dim <= 0 ||
          (epi->head_dim & 1) || epi->q_dim + 2 * epi->kv_dim != N || epi->q_dim % epi->head_dim ||
          epi->kv_dim % epi->head_dim || epi->ldo < epi->q_dim)
        return ti_set_error(TI_ERR_ARG, "ti_gemm_wq_a16: inconsistent QKV epilogue");
      break;
    case TI_EPI_LOGITS_ARGMAX:
      if (!epi->argmax || epi->ldo < N) return ti_set_error(TI_ERR_ARG, "ti_gemm_wq_a16: argmax/ldo");
      break;
    default:
      return ti_set_error(TI_ERR_ARG, "ti_gemm_wq_a16: unknown epilogue %d", epi->kind);
  }
  const int lds = gemv_lds_bytes(M, K);
  if (lds > 160 * 1024)
    return ti_set_error(TI_ERR_UNSUPPORTED, "ti_gemm_wq_a16: M*K too large for one LDS stage (M=%d K=%d)", M, K);
  if (lds > 64 * 1024 && !g_prepared) {
    const int rc = ti_gemm_prepare();
    if (rc != TI_OK) return rc;
  }
  GemvArgs a;
  a.tiles = (const u32x4*)tiles;
  a.scales = scales;
  a.x = x;
  a.norm_w = norm_w;
  a.eps = eps;
  a.x_kind = x_kind;
  a.ldx = ldx;
  a.M = M;
  a.N = N;
  a.K = K;
  a.epi = *epi;
  hipStream_t s = (hipStream_t)stream;
  if (bits == 4) return launch_gemv<4>(a, lds, s);
  if (bits == 8) return launch_gemv<8>(a, lds, s);
  return launch_gemv<16>(a, lds, s);
}

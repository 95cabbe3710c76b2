// misc.hip -- device-side decode loop step, synthetic weight / KV generation.
#include <algorithm>
#include <math.h>

#include "common.hpp"

namespace ti {

// --------------------------------------------------------------- step begin
// One block per stream m.  The decode loop runs entirely on the device: the token of
// step s is the prompt token while s < n_in[m], else the previous step's greedy argmax
// (the key packs (value, 0xFFFFFFFF - index), so the max is the lowest-index maximum).
__device__ __forceinline__ void step_begin_body(const ti_step_args a);
__global__ __launch_bounds__(256) void step_begin_kernel(const ti_step_args a, unsigned long long* stamp) {
  const unsigned long long t_entry = stamp_now();
  step_begin_body(a);
  stamp_end(stamp, t_entry);
}
__device__ __forceinline__ void step_begin_body(const ti_step_args a) {
  __shared__ int s_tok;
  const int m = blockIdx.x, tid = threadIdx.x;
  // With hidden % 8 == 0 (<= 8192): the embedding row moves in 16-byte pieces, all
  // of a thread's loads in flight together; the fold weights (independent of the token) are
  // loaded before the token is decided.
  constexpr int kPT = 4;   // pieces of 8 per thread
  const int H8 = a.hidden >> 3;
  const bool vec = (a.hidden & 7) == 0 && H8 <= 256 * kPT && a.placeholder_first < 0;
  float4 fw[kPT][2];
  if (vec && a.fold_x) {
#pragma unroll
    for (int p = 0; p < kPT; ++p) {
      const int i8 = min(tid + 256 * p, H8 - 1);
      fw[p][0] = *(const float4*)(a.fold_w + 8 * i8);
      fw[p][1] = *(const float4*)(a.fold_w + 8 * i8 + 4);
    }
  }
  const int s = *a.step_ctr;
  const int nin = a.n_in ? a.n_in[m] : 0;
  unsigned long long* am = a.argmax + (size_t)m * TI_ARGMAX_SLOTS;
  unsigned long long key = 0ull;
  if (tid < 64) {   // row m's key = max over its slots (wave 0)
    key = tid < TI_ARGMAX_SLOTS ? am[tid] : 0ull;
#pragma unroll
    for (int o = 1; o < TI_ARGMAX_SLOTS; o <<= 1) {
      const unsigned long long other = __shfl_xor(key, o, 64);
      key = other > key ? other : key;
    }
  }
  if (tid == 0) {
    int tok;
    if (s < nin) {
      tok = a.in_tokens[(size_t)m * a.in_stride + s];
    } else {
      tok = (int)(0xFFFFFFFFu - (uint32_t)(key & 0xFFFFFFFFull));
      if (a.out_tokens && s - nin < a.out_stride) {
        a.out_tokens[(size_t)m * a.out_stride + (s - nin)] = tok;
      }
    }
    if (tok < 0 || tok >= a.vocab) tok = 0;     // never index outside the table
    s_tok = tok;
    a.pos[m] = a.base_pos[m] + s;
  }
  __syncthreads();   // every slot read before any is cleared
  if (tid < TI_ARGMAX_SLOTS) am[tid] = 0ull;
  float* h = a.h + (size_t)m * a.hidden;
  if (a.placeholder_first >= 0) {
    // forward_pass / forward_pass_incremental placeholder rows (inference_engine.cpp:1444-1448,
    // 1509-1512): 0.1f * (flat_index % 100).
    const size_t off = s == 0 ? (size_t)a.placeholder_first : 0;
    for (int i = tid; i < a.hidden; i += 256) {
      h[i] = 0.1f * (float)((off + (size_t)i) % 100);
    }
  } else if (vec) {
    const uint16_t* e = a.emb + (size_t)s_tok * a.hidden;
    f16x8 ev[kPT];
#pragma unroll
    for (int p = 0; p < kPT; ++p) ev[p] = *(const f16x8*)(e + 8 * min(tid + 256 * p, H8 - 1));
    float ss = 0.0f;
#pragma unroll
    for (int p = 0; p < kPT; ++p) {
      const int i8 = tid + 256 * p;
      if (i8 >= H8) break;
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (float)ev[p][j];
      *(float4*)(h + 8 * i8) = make_float4(v[0], v[1], v[2], v[3]);
      *(float4*)(h + 8 * i8 + 4) = make_float4(v[4], v[5], v[6], v[7]);
      if (a.fold_x) {   // the first projection's TI_X_F16_FOLDED input (ti_hip.h)
        const float w[8] = {fw[p][0].x, fw[p][0].y, fw[p][0].z, fw[p][0].w, fw[p][1].x, fw[p][1].y, fw[p][1].z, fw[p][1].w};
        f16x8 fx;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          fx[j] = (f16)(v[j] * w[j]);
          ss = fmaf(v[j], v[j], ss);
        }
        *(f16x8*)(a.fold_x + (size_t)m * a.hidden + 8 * i8) = fx;
      }
    }
    if (a.fold_x) {
      __shared__ float s_red4[4];
      ss = group_sum<64>(ss);
      if ((tid & 63) == 0) s_red4[tid >> 6] = ss;
      __syncthreads();
      if (tid == 0) a.fold_ss[m] = (s_red4[0] + s_red4[1]) + (s_red4[2] + s_red4[3]);
    }
  } else {
    const uint16_t* e = a.emb + (size_t)s_tok * a.hidden;
    float ss = 0.0f;
    for (int i = tid; i < a.hidden; i += 256) {
      const float v = h2f(e[i]);
      h[i] = v;
      if (a.fold_x) {   // the first projection's TI_X_F16_FOLDED input (ti_hip.h)
        a.fold_x[(size_t)m * a.hidden + i] = f2h(v * a.fold_w[i]);
        ss = fmaf(v, v, ss);
      }
    }
    if (a.fold_x) {
      __shared__ float s_red[4];
      ss = group_sum<64>(ss);
      if ((tid & 63) == 0) s_red[tid >> 6] = ss;
      __syncthreads();
      if (tid == 0) a.fold_ss[m] = (s_red[0] + s_red[1]) + (s_red[2] + s_red[3]);
    }
  }
}

// ---------------------------------------------------------- synthetic weights
__host__ __device__ inline int map_row(int c, int row_map, int row_offset) {
  return row_map == TI_ROWS_INTERLEAVE8 ? 16 * (c >> 3) + (c & 7) + row_offset : row_offset + c;
}

// One thread per (source column c, k-group g): 128 seeded values -> per-group symmetric
// scale (absmax / 7 or / 127) -> q = clamp(round(w / s)) -> packed tile bytes + fp16 scale.
template <int BITS>
__global__ __launch_bounds__(128) void wsynth_kernel(uint64_t stream, int K, int N_src, int row_map,
                                                     int row_offset, float amp, uint8_t* tiles,
                                                     uint16_t* scales) {
  const int KT = K >> 7;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)N_src * KT) return;
  const int c = (int)(t % N_src), g = (int)(t / N_src);
  float w[128];
  float amax = 0.0f;
#pragma unroll
  for (int i = 0; i < 128; ++i) {
    w[i] = synth_unit(stream, (uint64_t)(g * 128 + i) * (uint64_t)N_src + (uint64_t)c) * amp;
    amax = fmaxf(amax, fabsf(w[i]));
  }
  const float qmax = BITS == 4 ? 7.0f : 127.0f, qlo = BITS == 4 ? -7.0f : -128.0f;
  const float sc = amax / qmax;
  const int n = map_row(c, row_map, row_offset), nt = n >> 4, r = n & 15;
  scales[((size_t)nt * KT + g) * 16 + r] = f2h_soft(sc);
  uint8_t* tile = tiles + ((size_t)nt * KT + g) * (size_t)TileFmt<BITS>::kBytes;
#pragma unroll
  for (int kq = 0; kq < 4; ++kq) {
    const int lane = kq * 16 + r;
    if constexpr (BITS == 4) {
      uint32_t words[4];
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) {
        uint32_t wd = 0;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          float q = roundf(w[kq * 32 + s4 * 8 + e] / sc);
          q = fmaxf(qlo, fminf(qmax, q));
          const uint32_t nib = (uint32_t)((int)q + 8) & 0xF;
          const int p = e >> 1;
          wd |= nib << ((e & 1) ? (16 + 4 * p) : (4 * p));
        }
        words[s4] = wd;
      }
      *(uint4*)(tile + lane * 16) = make_uint4(words[0], words[1], words[2], words[3]);
    } else {
#pragma unroll
      for (int ch = 0; ch < 2; ++ch) {
        uint32_t words[4];
#pragma unroll
        for (int wi = 0; wi < 4; ++wi) {
          uint32_t wd = 0;
#pragma unroll
          for (int b = 0; b < 4; ++b) {
            float q = roundf(w[kq * 32 + ch * 16 + wi * 4 + b] / sc);
            q = fmaxf(qlo, fminf(qmax, q));
            wd |= ((uint32_t)(int)q & 0xFFu) << (8 * b);
          }
          words[wi] = wd;
        }
        *(uint4*)(tile + ch * 1024 + lane * 16) = make_uint4(words[0], words[1], words[2], words[3]);
      }
    }
  }
}

// fp16 weights: element-parallel, no scale.
__global__ void wsynth_f16_kernel(uint64_t stream, int K, int N_src, int row_map, int row_offset, float amp,
                                  uint16_t* tiles) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)K * N_src) return;
  const int k = (int)(t / N_src), c = (int)(t % N_src);
  const float v = synth_unit(stream, (uint64_t)t) * amp;
  const int KT = K >> 7, n = map_row(c, row_map, row_offset), nt = n >> 4, r = n & 15;
  const int kt = k >> 7, kk = k & 127, kq = kk >> 5, ch = (kk & 31) >> 3, e = kk & 7;
  const size_t off = ((size_t)nt * KT + kt) * 2048 + (size_t)ch * 512 + (size_t)(kq * 16 + r) * 8 + e;
  tiles[off] = f2h_soft(v);
}

__global__ void fill_uniform_f16_kernel(uint64_t stream, uint64_t n, float mul, uint16_t* dst) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    dst[i] = f2h_soft(synth_unit(stream, i) * mul);
}
__global__ void fill_uniform_f32_kernel(uint64_t stream, uint64_t n, float mul, float add, float* dst) {
  // add + mul*u with two roundings, as the oracle's `1.0f + jitter * u` (no contraction)
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    dst[i] = __fadd_rn(add, __fmul_rn(mul, synth_unit(stream, i)));
}

// Synthetic KV (or_model_fill_kv): slot p of kv-head kvh, dim d takes element
// p*(kv_heads*hd) + kvh*hd + d of the oracle's [pos][kv*hd] stream.
__global__ void fill_kv_kernel(uint64_t stream, int n, int kv_heads, int hd, int max_seq, uint16_t* dst) {
  const int64_t total = (int64_t)n * kv_heads * hd;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int p = (int)(i / (kv_heads * hd));
    const int c = (int)(i - (int64_t)p * kv_heads * hd);
    const int kvh = c / hd, d = c - kvh * hd;
    dst[((size_t)kvh * max_seq + p) * hd + d] = f2h_soft(synth_unit(stream, (uint64_t)i));
  }
}

// --------------------------------------------------------------- KV slot copy
// Beam search (ti_engine_beam_search): a beam that forks copies its parent's cache prefix into
// a free stream slot.  For each of n_tab caches (layer K / V base pointers in `tab`), `rows`
// rows (kv heads) of `row_elems` fp16 each, row pitch `row_pitch`, from element offset
// src_off to dst_off.  16 bytes per thread (row_elems % 8 == 0, 16-byte aligned rows).
__global__ __launch_bounds__(256) void kv_copy_kernel(uint16_t* const* tab, int64_t src_off, int64_t dst_off,
                                                      int64_t row_pitch, int64_t row_chunks) {
  uint16_t* base = tab[blockIdx.z];
  const int64_t r = blockIdx.y;
  for (int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x; c < row_chunks; c += (int64_t)gridDim.x * 256) {
    const uint4 v = *(const uint4*)(base + src_off + r * row_pitch + 8 * c);
    *(uint4*)(base + dst_off + r * row_pitch + 8 * c) = v;
  }
}

// HBM read calibration (ti_hbm_calibrate): every workgroup streams a contiguous slice with 16-byte
// non-temporal loads, 4 in flight per thread, and folds them into one word (never 0 in practice).
typedef uint32_t hbm_u32x4 __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(512) void hbm_read_kernel(const hbm_u32x4* src, size_t n16, uint32_t* sink) {
  const size_t per = (n16 + gridDim.x - 1) / gridDim.x, b0 = blockIdx.x * per, b1 = b0 + per < n16 ? b0 + per : n16;
  uint32_t acc = 0;
  for (size_t i = b0 + threadIdx.x; i < b1; i += 4 * blockDim.x) {
    hbm_u32x4 v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const size_t k = i + (size_t)j * blockDim.x;
      v[j] = k < b1 ? __builtin_nontemporal_load(src + k) : (hbm_u32x4){0u, 0u, 0u, 0u};
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) acc ^= v[j][0] ^ v[j][1] ^ v[j][2] ^ v[j][3];
  }
  if (acc == 0x9e3779b9u) sink[blockIdx.x] = acc;   // keeps the loads; practically never stores
}

}  // namespace ti

extern "C" int ti_step_begin(const ti_step_args* a, ti_stream_t stream) {
  using namespace ti;
  if (!a || !a->h || !a->argmax || !a->pos || !a->base_pos || !a->step_ctr || a->M < 1 || a->hidden < 1)
    return ti_set_error(TI_ERR_ARG, "ti_step_begin: bad arguments");
  if (a->placeholder_first < 0 && !a->emb) return ti_set_error(TI_ERR_ARG, "ti_step_begin: emb required");
  if (a->n_in && !a->in_tokens) return ti_set_error(TI_ERR_ARG, "ti_step_begin: in_tokens required");
  if (a->fold_x && (!a->fold_w || !a->fold_ss || a->placeholder_first >= 0))
    return ti_set_error(TI_ERR_ARG, "ti_step_begin: fold_x needs fold_w, fold_ss and the embedding gather");
  hipLaunchKernelGGL(step_begin_kernel, dim3(a->M), dim3(256), 0, (hipStream_t)stream, *a,
                     ti_stamp_next(STAMP_BEGIN, a->M));
  TI_LAUNCH_CHECK("step_begin_kernel");
  return TI_OK;
}


extern "C" int ti_wsynth_device(uint64_t seed, uint32_t tensor_id, int K, int N_src, int N_total, int bits,
                                int row_map, int row_offset, void* tiles, uint16_t* scales, ti_stream_t stream) {
  using namespace ti;
  if (!tiles || K <= 0 || (K & 127) || N_total <= 0 || (N_total & 15) || N_src <= 0)
    return ti_set_error(TI_ERR_ARG, "ti_wsynth_device: bad shape K=%d N_src=%d N_total=%d", K, N_src, N_total);
  if (map_row(N_src - 1, row_map, row_offset) >= N_total || (row_map == TI_ROWS_INTERLEAVE8 && (N_src & 7)))
    return ti_set_error(TI_ERR_ARG, "ti_wsynth_device: rows do not fit N_total");
  const float amp = sqrtf(3.0f) / sqrtf((float)K);
  const uint64_t stream_id = synth_stream(seed, tensor_id);
  hipStream_t s = (hipStream_t)stream;
  if (bits == 16) {
    const int64_t n = (int64_t)K * N_src;
    hipLaunchKernelGGL(wsynth_f16_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, stream_id, K, N_src,
                       row_map, row_offset, amp, (uint16_t*)tiles);
    TI_LAUNCH_CHECK("wsynth_f16_kernel");
    return TI_OK;
  }
  if (!scales) return ti_set_error(TI_ERR_ARG, "ti_wsynth_device: scales required");
  const int64_t n = (int64_t)N_src * (K >> 7);
  const dim3 grid((unsigned)((n + 127) / 128));
  if (bits == 4)
    hipLaunchKernelGGL(wsynth_kernel<4>, grid, dim3(128), 0, s, stream_id, K, N_src, row_map, row_offset, amp,
                       (uint8_t*)tiles, scales);
  else if (bits == 8)
    hipLaunchKernelGGL(wsynth_kernel<8>, grid, dim3(128), 0, s, stream_id, K, N_src, row_map, row_offset, amp,
                       (uint8_t*)tiles, scales);
  else
    return ti_set_error(TI_ERR_ARG, "ti_wsynth_device: bits %d", bits);
  TI_LAUNCH_CHECK("wsynth_kernel");
  return TI_OK;
}

extern "C" int ti_fill_uniform_f16(uint64_t seed, uint32_t tensor_id, uint64_t n, float mul, uint16_t* dst,
                                   ti_stream_t stream) {
  using namespace ti;
  if (!dst) return ti_set_error(TI_ERR_ARG, "ti_fill_uniform_f16: null");
  if (n == 0) return TI_OK;
  const unsigned blocks = (unsigned)((n + 255) / 256 < 65536 ? (n + 255) / 256 : 65536);
  hipLaunchKernelGGL(fill_uniform_f16_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream,
                     synth_stream(seed, tensor_id), n, mul, dst);
  TI_LAUNCH_CHECK("fill_uniform_f16_kernel");
  return TI_OK;
}

extern "C" int ti_fill_kv_uniform(uint64_t seed, uint32_t tensor_id, int n, int kv_heads, int head_dim,
                                  int max_seq, uint16_t* dst, ti_stream_t stream) {
  using namespace ti;
  if (!dst || n < 0 || n > max_seq || kv_heads < 1 || head_dim < 1)
    return ti_set_error(TI_ERR_ARG, "ti_fill_kv_uniform: bad arguments");
  if (n == 0) return TI_OK;
  const int64_t total = (int64_t)n * kv_heads * head_dim;
  const unsigned blocks = (unsigned)((total + 255) / 256 < 65536 ? (total + 255) / 256 : 65536);
  hipLaunchKernelGGL(fill_kv_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, synth_stream(seed, tensor_id),
                     n, kv_heads, head_dim, max_seq, dst);
  TI_LAUNCH_CHECK("fill_kv_kernel");
  return TI_OK;
}

extern "C" int ti_fill_uniform_f32(uint64_t seed, uint32_t tensor_id, uint64_t n, float mul, float add, float* dst,
                                   ti_stream_t stream) {
  using namespace ti;
  if (!dst) return ti_set_error(TI_ERR_ARG, "ti_fill_uniform_f32: null");
  if (n == 0) return TI_OK;
  const unsigned blocks = (unsigned)((n + 255) / 256 < 65536 ? (n + 255) / 256 : 65536);
  hipLaunchKernelGGL(fill_uniform_f32_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream,
                     synth_stream(seed, tensor_id), n, mul, add, dst);
  TI_LAUNCH_CHECK("fill_uniform_f32_kernel");
  return TI_OK;
}

extern "C" int ti_kv_copy_slots(uint16_t* const* tab, int n_tab, int64_t src_off, int64_t dst_off, int rows,
                                int64_t row_pitch, int64_t row_elems, ti_stream_t stream) {
  using namespace ti;
  if (!tab || n_tab < 1 || n_tab > 65535 || rows < 1 || rows > 65535 || row_elems < 0 || (row_elems & 7) ||
      row_pitch < row_elems || (row_pitch & 7) || (src_off & 7) || (dst_off & 7) || src_off < 0 || dst_off < 0)
    return ti_set_error(TI_ERR_ARG, "ti_kv_copy_slots: bad arguments");
  if (row_elems == 0 || src_off == dst_off) return TI_OK;
  const int64_t chunks = row_elems / 8;
  const unsigned bx = (unsigned)((chunks + 255) / 256 < 64 ? (chunks + 255) / 256 : 64);
  hipLaunchKernelGGL(kv_copy_kernel, dim3(bx, rows, n_tab), dim3(256), 0, (hipStream_t)stream, tab, src_off, dst_off,
                     row_pitch, chunks);
  TI_LAUNCH_CHECK("kv_copy_kernel");
  return TI_OK;
}

// Same-run HBM calibration for bench lines: the read rate of a `bytes` buffer
// streamed by 4 waves per CU x 2 rounds, and hipMemcpyAsync device-to-device (read + write bytes),
// each the best of `reps` timed passes after one warm pass.  Allocates and frees its buffers.
extern "C" int ti_hbm_calibrate(size_t bytes, int reps, double* read_gbps, double* copy_gbps, ti_stream_t stream) {
  if (!read_gbps || !copy_gbps || bytes < (1u << 20) || reps < 1) return ti_set_error(TI_ERR_ARG, "ti_hbm_calibrate: bad arguments");
  hipStream_t s = (hipStream_t)stream;
  void *a = nullptr, *b = nullptr, *sink = nullptr;
  int dev = 0, cus = 0;
  TI_HIP_CHECK(hipGetDevice(&dev), "hipGetDevice");
  TI_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev), "hipDeviceGetAttribute");
  bytes &= ~(size_t)15;
  hipError_t e = hipMalloc(&a, bytes);
  if (e == hipSuccess) e = hipMalloc(&b, bytes);
  if (e == hipSuccess) e = hipMalloc(&sink, 4096 * 4);
  if (e == hipSuccess) e = hipMemsetAsync(a, 1, bytes, s);
  hipEvent_t e0 = nullptr, e1 = nullptr;
  if (e == hipSuccess) e = hipEventCreate(&e0);
  if (e == hipSuccess) e = hipEventCreate(&e1);
  double best_r = 0.0, best_c = 0.0;
  const int grid = 2 * (cus > 0 ? cus : 256);
  for (int r = 0; r <= reps && e == hipSuccess; ++r) {
    float ms = 0.0f;
    e = hipEventRecord(e0, s);
    if (e == hipSuccess) {
      hipLaunchKernelGGL(ti::hbm_read_kernel, dim3(grid), dim3(512), 0, s, (const ti::hbm_u32x4*)a, bytes / 16, (uint32_t*)sink);
      e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipEventRecord(e1, s);
    if (e == hipSuccess) e = hipEventSynchronize(e1);
    if (e == hipSuccess) e = hipEventElapsedTime(&ms, e0, e1);
    if (e == hipSuccess && r > 0 && ms > 0.0f) best_r = std::max(best_r, (double)bytes / (ms * 1e-3) / 1e9);
    if (e == hipSuccess) e = hipEventRecord(e0, s);
    if (e == hipSuccess) e = hipMemcpyAsync(b, a, bytes, hipMemcpyDeviceToDevice, s);
    if (e == hipSuccess) e = hipEventRecord(e1, s);
    if (e == hipSuccess) e = hipEventSynchronize(e1);
    if (e == hipSuccess) e = hipEventElapsedTime(&ms, e0, e1);
    if (e == hipSuccess && r > 0 && ms > 0.0f) best_c = std::max(best_c, 2.0 * (double)bytes / (ms * 1e-3) / 1e9);
  }
  if (e0) hipEventDestroy(e0);
  if (e1) hipEventDestroy(e1);
  if (a) hipFree(a);
  if (b) hipFree(b);
  if (sink) hipFree(sink);
  TI_HIP_CHECK(e, "ti_hbm_calibrate");
  *read_gbps = best_r;
  *copy_gbps = best_c;
  return TI_OK;
}

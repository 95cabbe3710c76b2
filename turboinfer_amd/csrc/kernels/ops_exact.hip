// ops_exact.hip -- fp32 op-level kernels behind core::TensorEngine on the GPU.
//
// Compiled with -ffp-contract=off: each kernel reproduces the reference CPU build's
// rounding sequence (where the reference fuses, an explicit fmaf is written), so
// matmul, rms_norm, apply_rope (given the host cos/sin table), add, multiply, relu and
// softmax for rows whose length is a multiple of 8 are bit-identical to the compiled
// reference (tests/test_gpu_ops.py).  silu / the attention's exp use the device expf.
#include <math.h>

#include "common.hpp"

namespace ti {

// matmul_3d_2d (tensor_engine.cpp:620-633): sum = 0; for k ascending sum = fma(a, b, sum).
__global__ __launch_bounds__(256) void matmul_f32_kernel(const float* a, const float* b, float* y,
                                                         const float* resid, int rows, int K, int N, int mode) {
  const int j = blockIdx.x * 256 + threadIdx.x, r = blockIdx.y;
  if (j >= N) return;
  const float* ar = a + (size_t)r * K;
  float s = 0.0f;
  int k = 0;
  for (; k + 4 <= K; k += 4) {
    const float b0 = b[(size_t)k * N + j], b1 = b[(size_t)(k + 1) * N + j];
    const float b2 = b[(size_t)(k + 2) * N + j], b3 = b[(size_t)(k + 3) * N + j];
    s = fmaf(ar[k], b0, s);
    s = fmaf(ar[k + 1], b1, s);
    s = fmaf(ar[k + 2], b2, s);
    s = fmaf(ar[k + 3], b3, s);
  }
  for (; k < K; ++k) s = fmaf(ar[k], b[(size_t)k * N + j], s);
  if (mode == 1) s = (0.0f < s) ? s : 0.0f;                       // relu (:846-866)
  if (mode == 2) s = resid[(size_t)r * N + j] + s;                // add(residual, y)
  y[(size_t)r * N + j] = s;
}

// rms_norm (tensor_engine.cpp:1488-1505) with the reference build's summation order:
// products of the 8-wide main loop and one 4-wide epilogue step rounded, added in
// order; the last n%4 terms fused (see dot_ordered in oracle/ti_oracle.c).
__global__ __launch_bounds__(256) void rms_norm_f32_kernel(const float* x, const float* w, float* y, int n,
                                                           float eps) {
  __shared__ float s_rms;
  const float* xr = x + (size_t)blockIdx.x * n;
  if (threadIdx.x == 0) {
    float s = 0.0f;
    int i = 0;
    for (; i + 8 <= n; i += 8)
      for (int l = 0; l < 8; ++l) s = s + xr[i + l] * xr[i + l];
    if (i + 4 <= n) {
      for (int l = 0; l < 4; ++l) s = s + xr[i + l] * xr[i + l];
      i += 4;
    }
    for (; i < n; ++i) s = fmaf(xr[i], xr[i], s);
    s_rms = sqrtf(s / (float)n + eps);
  }
  __syncthreads();
  const float rms = s_rms;
  for (int i = threadIdx.x; i < n; i += 256) y[(size_t)blockIdx.x * n + i] = (xr[i] / rms) * w[i];
}

// apply_rope rotation (tensor_engine.cpp:1602-1612), reference contraction pattern.
__global__ void rope_f32_kernel(const float* x, float* y, const float* cs, int B, int heads, int S, int D,
                                int pos_2d) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int half = D >> 1;
  const int64_t total = (int64_t)B * heads * S * half;
  if (t >= total) return;
  const int i = (int)(t % half);
  const int64_t row = t / half;                 // ((b*heads + h)*S + s)
  const int s = (int)(row % S);
  const int b = (int)(row / ((int64_t)heads * S));
  const int csrow = pos_2d ? b * S + s : s;
  const float c = cs[((size_t)csrow * half + i) * 2], sn = cs[((size_t)csrow * half + i) * 2 + 1];
  const float xe = x[row * D + 2 * i], xo = x[row * D + 2 * i + 1];
  y[row * D + 2 * i] = fmaf(-xo, sn, xe * c);
  y[row * D + 2 * i + 1] = fmaf(xo, c, xe * sn);
}

__global__ void eltwise_kernel(const float* a, const float* b, float* y, int64_t n, int op) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float v = a[i];
    float r;
    switch (op) {
      case 0: r = v / (1.0f + expf(-v)); break;      // silu (:913-917)
      case 1: r = (0.0f < v) ? v : 0.0f; break;       // relu
      case 2: r = v + b[i]; break;                    // add
      default: r = v * b[i]; break;                   // multiply
    }
    y[i] = r;
  }
}

// fast_exp_avx2 (tensor_engine.cpp:262-302), one lane, same rounding sequence.
__device__ __forceinline__ float fast_exp_ref(float x) {
  x = (x < 88.0f) ? x : 88.0f;
  x = (x > -88.0f) ? x : -88.0f;
  const float xl = x * 1.44269504f;
  const float fx = floorf(xl);
  const float frac = xl - fx;
  const int fi = (int)fx;
  const float e = __builtin_bit_cast(float, (uint32_t)(fi + 127) << 23);
  const float xf = frac * 0.69314718f;
  float p = 1.0f;
  p = fmaf(xf, 0.69314718f, p);
  const float x2 = xf * xf;
  p = fmaf(x2, 0.24022651f, p);
  const float x3 = x2 * xf;
  p = fmaf(x3, 0.05550410f, p);
  const float x4 = x3 * xf;
  p = fmaf(x4, 0.00961812f, p);
  return e * p;
}

// softmax (tensor_engine.cpp:943-1037): 8 interleaved lane partials (max, then sum of
// fast_exp) reduced sequentially, std::exp tail, division by the sum.  One block per row.
__global__ __launch_bounds__(256) void softmax_f32_kernel(const float* x, float* y, int n, float T) {
  __shared__ float s_lane[8];
  __shared__ float s_m, s_s;
  const float* in = x + (size_t)blockIdx.x * n;
  float* out = y + (size_t)blockIdx.x * n;
  const int tid = threadIdx.x;
  if (n >= 16) {
    const int se = (n / 8) * 8;
    if (tid < 8) {
      float m = -INFINITY;
      for (int i = tid; i < se; i += 8) m = (m > in[i]) ? m : in[i];
      s_lane[tid] = m;
    }
    __syncthreads();
    if (tid == 0) {
      float m = -INFINITY;
      for (int l = 0; l < 8; ++l) m = (m < s_lane[l]) ? s_lane[l] : m;
      for (int i = se; i < n; ++i) m = (m < in[i]) ? in[i] : m;
      s_m = m;
    }
    __syncthreads();
    const float m = s_m;
    for (int i = tid; i < se; i += 256) out[i] = fast_exp_ref((in[i] - m) / T);
    __syncthreads();
    if (tid < 8) {
      float s = 0.0f;
      for (int i = tid; i < se; i += 8) s = s + out[i];
      s_lane[tid] = s;
    }
    __syncthreads();
    if (tid == 0) {
      float s = 0.0f;
      for (int l = 0; l < 8; ++l) s += s_lane[l];
      for (int i = se; i < n; ++i) {
        const float e = expf((in[i] - m) / T);
        out[i] = e;
        s += e;
      }
      s_s = s;
    }
    __syncthreads();
    const float s = s_s;
    for (int i = tid; i < n; i += 256) out[i] = out[i] / s;
  } else {
    if (tid == 0) {
      float m = in[0];
      for (int i = 1; i < n; ++i) m = (m < in[i]) ? in[i] : m;
      float s = 0.0f;
      for (int i = 0; i < n; ++i) {
        out[i] = expf((in[i] - m) / T);
        s += out[i];
      }
      for (int i = 0; i < n; ++i) out[i] /= s;
    }
  }
}

__global__ __launch_bounds__(256) void argmax_f32_kernel(const float* x, int32_t* out, int n) {
  __shared__ float s_v[4];
  __shared__ int s_i[4];
  const float* in = x + (size_t)blockIdx.x * n;
  float bv = -INFINITY;
  int bi = 0x7fffffff;
  for (int i = threadIdx.x; i < n; i += 256) {
    const float v = in[i];
    if (v > bv || (v == bv && i < bi)) { bv = v; bi = i; }
  }
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(bv, o, kWave);
    const int oi = __shfl_xor(bi, o, kWave);
    if (ov > bv || (ov == bv && oi < bi)) { bv = ov; bi = oi; }
  }
  if ((threadIdx.x & 63) == 0) { s_v[threadIdx.x >> 6] = bv; s_i[threadIdx.x >> 6] = bi; }
  __syncthreads();
  if (threadIdx.x == 0) {
    bv = s_v[0];
    bi = s_i[0];
    for (int w = 1; w < 4; ++w)
      if (s_v[w] > bv || (s_v[w] == bv && s_i[w] < bi)) { bv = s_v[w]; bi = s_i[w]; }
    out[blockIdx.x] = bi == 0x7fffffff ? 0 : bi;
  }
}

}  // namespace ti

// attention_fast_incremental (tensor_engine.cpp:1254-1388) for one (batch row, head) per
// block, heads addressed with strides so multi_head_attention's slicing (:1149-1252) needs
// no copies.  Scores: 8 lane partial fmas over the 8-aligned prefix, lanes added in
// order, then the ordered tail (as the reference's AVX2 loop + scalar remainder); softmax
// with max / exp / sequential sum / divide; output: 8 lane partial fmas over the 8-aligned
// key prefix, lanes added in order, fused tail.  exp is the device expf (glibc's expf may
// differ by an ulp), so results match within rounding, not bitwise.
__global__ __launch_bounds__(256) void attention_f32_kernel(const float* q, const float* k, const float* v,
                                                            float* out, float* scratch, int S, int D, int heads,
                                                            int64_t ldq, int64_t ldkv, int64_t ldo) {
  const int b = blockIdx.x, h = blockIdx.y;
  const float* qb = q + (size_t)b * ldq + (size_t)h * D;
  const float* kb = k + (size_t)b * S * ldkv + (size_t)h * D;
  const float* vb = v + (size_t)b * S * ldkv + (size_t)h * D;
  float* sc = scratch + ((size_t)b * heads + h) * S;
  const float scale = 1.0f / sqrtf((float)D);
  const int de = (D / 8) * 8;
  for (int j = threadIdx.x; j < S; j += 256) {
    const float* kr = kb + (size_t)j * ldkv;
    float lane[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int i = 0; i < de; i += 8)
      for (int l = 0; l < 8; ++l) lane[l] = fmaf(qb[i + l], kr[i + l], lane[l]);
    float s = 0.0f;
    for (int l = 0; l < 8; ++l) s = s + lane[l];
    int i = de;
    for (; i + 4 <= D; i += 4)
      for (int l = 0; l < 4; ++l) s = s + qb[i + l] * kr[i + l];
    for (; i < D; ++i) s = fmaf(qb[i], kr[i], s);
    sc[j] = s * scale;
  }
  __syncthreads();
  __shared__ float s_sum;
  if (threadIdx.x == 0) {
    float mx = sc[0];
    for (int j = 1; j < S; ++j) mx = (mx < sc[j]) ? sc[j] : mx;
    float se = 0.0f;
    for (int j = 0; j < S; ++j) {
      sc[j] = expf(sc[j] - mx);
      se = se + sc[j];
    }
    s_sum = se;
  }
  __syncthreads();
  const float se = s_sum;
  for (int j = threadIdx.x; j < S; j += 256) sc[j] = sc[j] / se;
  __syncthreads();
  const int ke = (S / 8) * 8;
  for (int d = threadIdx.x; d < D; d += 256) {
    float lane[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int j = 0; j < ke; j += 8)
      for (int l = 0; l < 8; ++l) lane[l] = fmaf(sc[j + l], vb[(size_t)(j + l) * ldkv + d], lane[l]);
    float o = 0.0f;
    for (int l = 0; l < 8; ++l) o = o + lane[l];
    for (int j = ke; j < S; ++j) o = fmaf(sc[j], vb[(size_t)j * ldkv + d], o);
    out[(size_t)b * ldo + (size_t)h * D + d] = o;
  }
}

static unsigned grid_for(int64_t n) {
  const int64_t b = (n + 255) / 256;
  return (unsigned)(b < 65536 ? (b > 0 ? b : 1) : 65536);
}

extern "C" int ti_matmul_f32(const float* a, const float* b, float* y, const float* resid, int rows, int K, int N,
                             int mode, ti_stream_t s) {
  if (!a || !b || !y || rows < 1 || K < 1 || N < 1 || mode < 0 || mode > 2 || (mode == 2 && !resid))
    return ti_set_error(TI_ERR_ARG, "ti_matmul_f32: bad arguments");
  if (rows > 65535) return ti_set_error(TI_ERR_UNSUPPORTED, "ti_matmul_f32: rows > 65535");
  hipLaunchKernelGGL(ti::matmul_f32_kernel, dim3((N + 255) / 256, rows), dim3(256), 0, (hipStream_t)s, a, b, y,
                     resid, rows, K, N, mode);
  TI_LAUNCH_CHECK("matmul_f32_kernel");
  return TI_OK;
}

extern "C" int ti_rms_norm_f32(const float* x, const float* w, float* y, int rows, int n, float eps, ti_stream_t s) {
  if (!x || !w || !y || rows < 1 || n < 1) return ti_set_error(TI_ERR_ARG, "ti_rms_norm_f32: bad arguments");
  hipLaunchKernelGGL(ti::rms_norm_f32_kernel, dim3(rows), dim3(256), 0, (hipStream_t)s, x, w, y, n, eps);
  TI_LAUNCH_CHECK("rms_norm_f32_kernel");
  return TI_OK;
}

extern "C" int ti_rope_f32(const float* x, float* y, const float* cs, int B, int heads, int S, int D, int pos_2d,
                           ti_stream_t s) {
  if (!x || !y || !cs || B < 1 || heads < 1 || S < 1 || D < 2 || (D & 1))
    return ti_set_error(TI_ERR_ARG, "ti_rope_f32: bad arguments");
  const int64_t total = (int64_t)B * heads * S * (D / 2);
  hipLaunchKernelGGL(ti::rope_f32_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)s, x, y,
                     cs, B, heads, S, D, pos_2d);
  TI_LAUNCH_CHECK("rope_f32_kernel");
  return TI_OK;
}

static int eltwise(const float* a, const float* b, float* y, int64_t n, int op, ti_stream_t s, const char* name) {
  if (!a || !y || n < 0 || (op >= 2 && !b)) return ti_set_error(TI_ERR_ARG, "%s: bad arguments", name);
  if (n == 0) return TI_OK;
  hipLaunchKernelGGL(ti::eltwise_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)s, a, b, y, n, op);
  TI_LAUNCH_CHECK(name);
  return TI_OK;
}
extern "C" int ti_silu_f32(const float* x, float* y, int64_t n, ti_stream_t s) { return eltwise(x, nullptr, y, n, 0, s, "ti_silu_f32"); }
extern "C" int ti_relu_f32(const float* x, float* y, int64_t n, ti_stream_t s) { return eltwise(x, nullptr, y, n, 1, s, "ti_relu_f32"); }
extern "C" int ti_add_f32(const float* a, const float* b, float* y, int64_t n, ti_stream_t s) { return eltwise(a, b, y, n, 2, s, "ti_add_f32"); }
extern "C" int ti_mul_f32(const float* a, const float* b, float* y, int64_t n, ti_stream_t s) { return eltwise(a, b, y, n, 3, s, "ti_mul_f32"); }

extern "C" int ti_softmax_f32(const float* x, float* y, int rows, int n, float temperature, ti_stream_t s) {
  if (!x || !y || rows < 1 || n < 1) return ti_set_error(TI_ERR_ARG, "ti_softmax_f32: bad arguments");
  hipLaunchKernelGGL(ti::softmax_f32_kernel, dim3(rows), dim3(256), 0, (hipStream_t)s, x, y, n, temperature);
  TI_LAUNCH_CHECK("softmax_f32_kernel");
  return TI_OK;
}

extern "C" int ti_attention_f32(const float* q, const float* k, const float* v, float* out, float* scratch, int B,
                                int S, int H, int heads, ti_stream_t s) {
  using namespace ti;
  if (!q || !k || !v || !out || !scratch || B < 1 || S < 1 || heads < 1 || H < heads || H % heads)
    return ti_set_error(TI_ERR_ARG, "ti_attention_f32: bad arguments B=%d S=%d H=%d heads=%d", B, S, H, heads);
  hipLaunchKernelGGL(attention_f32_kernel, dim3(B, heads), dim3(256), 0, (hipStream_t)s, q, k, v, out, scratch, S,
                     H / heads, heads, (int64_t)H, (int64_t)H, (int64_t)H);
  TI_LAUNCH_CHECK("attention_f32_kernel");
  return TI_OK;
}

extern "C" int ti_argmax_f32(const float* x, int32_t* out, int rows, int n, ti_stream_t s) {
  if (!x || !out || rows < 1 || n < 1) return ti_set_error(TI_ERR_ARG, "ti_argmax_f32: bad arguments");
  hipLaunchKernelGGL(ti::argmax_f32_kernel, dim3(rows), dim3(256), 0, (hipStream_t)s, x, out, n);
  TI_LAUNCH_CHECK("argmax_f32_kernel");
  return TI_OK;
}

// Fused cross-entropy for gfx950: log-softmax + NLL forward, the gradient (softmax - onehot)
// written in the same launch, and the eval metrics (argmax) - one kernel instead of ATen's
// log_softmax / nll_loss / softmax_backward / argmax / eq / sum chain
// (reference: nn.CrossEntropyLoss at R/my_ray_module.py:141,156,167; argmax at :170).
//
// One 256-thread block per row.  Pass 1: per-thread online (max, sum-exp, argmax) over
// 16-B vector loads, block-combined.  Pass 2 (when a gradient buffer is given): re-reads the
// row (L2-resident: one 100 KB GPT-2 row per block) and writes scale*(softmax - onehot);
// padded vocabulary columns [V, ld) get exactly 0.  Rows whose target is ignore_index get a
// zero loss and zero gradient.
#include "gemm_common.h"

#include <cstdlib>

namespace rtdc {

template <typename T>
__device__ __forceinline__ float ldv(const T* p, long long i);
template <>
__device__ __forceinline__ float ldv<float>(const float* p, long long i) { return p[i]; }
template <>
__device__ __forceinline__ float ldv<bf16_t>(const bf16_t* p, long long i) { return bf2f(p[i]); }
template <typename T>
__device__ __forceinline__ void stv(T* p, long long i, float v);
template <>
__device__ __forceinline__ void stv<float>(float* p, long long i, float v) { p[i] = v; }
template <>
__device__ __forceinline__ void stv<bf16_t>(bf16_t* p, long long i, float v) { p[i] = f2bf(v); }

template <typename T>
__device__ __forceinline__ void ldvec(const T* p, float* v);  // 16 B
template <>
__device__ __forceinline__ void ldvec<float>(const float* p, float* v) {
  f32x4 x = *(const f32x4*)p;
  v[0] = x[0]; v[1] = x[1]; v[2] = x[2]; v[3] = x[3];
}
template <>
__device__ __forceinline__ void ldvec<bf16_t>(const bf16_t* p, float* v) {
  uint4 x = *(const uint4*)p;
  uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[2 * i] = __uint_as_float(w[i] << 16);
    v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}
template <typename T>
__device__ __forceinline__ void stvec(T* p, const float* v);
template <>
__device__ __forceinline__ void stvec<float>(float* p, const float* v) {
  *(f32x4*)p = f32x4{v[0], v[1], v[2], v[3]};
}
template <>
__device__ __forceinline__ void stvec<bf16_t>(bf16_t* p, const float* v) {
  *(uint4*)p = make_uint4(pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3]), pack_bf2(v[4], v[5]),
                          pack_bf2(v[6], v[7]));
}

struct OnlineMax {
  float m, s;
  int arg;
};

__device__ __forceinline__ void om_push(OnlineMax& o, float x, int j) {
  if (x > o.m) {
    o.s = o.s * __expf(o.m - x) + 1.f;
    o.m = x;
    o.arg = j;
  } else {
    o.s += __expf(x - o.m);
  }
}
__device__ __forceinline__ OnlineMax om_merge(OnlineMax a, OnlineMax b) {
  if (b.m > a.m || (b.m == a.m && b.arg < a.arg)) {
    OnlineMax t = a;
    a = b;
    b = t;
  }
  // a.m >= b.m
  if (b.m == -INFINITY) return a;
  a.s += b.s * __expf(b.m - a.m);
  return a;
}

template <typename T, bool VEC>
__global__ __launch_bounds__(256) void xent_kernel(const T* logits, T* dlogits,
                                                  const int64_t* __restrict__ target, float* __restrict__ loss,
                                                  float* __restrict__ lse_out, int64_t* __restrict__ argmax,
                                                  int M, int V, int ld, float grad_scale,
                                                  int ignore_index) {
  __shared__ float sm[4], ss[4];
  __shared__ int sa[4];
  const int row = blockIdx.x;
  if (row >= M) return;
  const T* x = logits + (long long)row * ld;
  OnlineMax o{-INFINITY, 0.f, 0x7fffffff};
  if constexpr (VEC) {
    // 8 elements per 16-B load (bf16) / 4 (fp32); U loads in flight per thread, and the running
    // max is rescaled once per 16-B chunk (chunk max first) instead of a data-dependent branch
    // per element
    constexpr int E = 16 / sizeof(T), U = 4;
    for (int c0 = threadIdx.x * E; c0 < ld; c0 += 256 * E * U) {
      float v[U][E];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int c = c0 + u * 256 * E;
        if (c < ld) ldvec<T>(x + c, v[u]);
#pragma unroll
        for (int e = 0; e < E; ++e)
          if (c >= ld || c + e >= V) v[u][e] = -INFINITY;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int c = c0 + u * 256 * E;
        float cm = v[u][0];
        int ca = c;
#pragma unroll
        for (int e = 1; e < E; ++e)
          if (v[u][e] > cm) {
            cm = v[u][e];
            ca = c + e;
          }
        if (cm > o.m) {  // first occurrence wins ties: later chunks only replace on a strict max
          o.s *= __expf(o.m - cm);
          o.m = cm;
          o.arg = ca;
        }
        if (o.m != -INFINITY) {
#pragma unroll
          for (int e = 0; e < E; ++e) o.s += __expf(v[u][e] - o.m);
        }
      }
    }
  } else {
    for (int j = threadIdx.x; j < V; j += 256) om_push(o, ldv<T>(x, j), j);
  }
  // wave combine
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    OnlineMax p;
    p.m = __shfl_xor(o.m, off, 64);
    p.s = __shfl_xor(o.s, off, 64);
    p.arg = __shfl_xor(o.arg, off, 64);
    o = om_merge(o, p);
  }
  const int w = threadIdx.x >> 6;
  // target logit read BEFORE the barrier: pass 2 may overwrite the row in place
  const int64_t tgt = target ? target[row] : -1;
  const bool valid = target && tgt != ignore_index && tgt >= 0 && tgt < V;
  const float xt = (threadIdx.x == 0 && valid) ? ldv<T>(x, tgt) : 0.f;
  if ((threadIdx.x & 63) == 0) {
    sm[w] = o.m;
    ss[w] = o.s;
    sa[w] = o.arg;
  }
  __syncthreads();
  OnlineMax r{sm[0], ss[0], sa[0]};
#pragma unroll
  for (int i = 1; i < 4; ++i) r = om_merge(r, OnlineMax{sm[i], ss[i], sa[i]});
  const float lse = r.m + __logf(r.s);
  if (threadIdx.x == 0) {
    if (loss) loss[row] = valid ? lse - xt : 0.f;
    if (lse_out) lse_out[row] = lse;
    if (argmax) argmax[row] = r.arg;
  }
  if (!dlogits) return;
  T* dx = dlogits + (long long)row * ld;
  const float sc = valid ? grad_scale : 0.f;
  // every thread has read its own elements already; reads of other threads' elements happen
  // only through their own (same-thread) indices below, so dlogits may alias logits.
  if constexpr (VEC) {
    constexpr int E = 16 / sizeof(T);
    for (int c = threadIdx.x * E; c < ld; c += 256 * E) {
      float v[E], gv[E];
      ldvec<T>(x + c, v);
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const int j = c + e;
        gv[e] = j < V ? sc * (__expf(v[e] - lse) - (j == tgt ? 1.f : 0.f)) : 0.f;
      }
      stvec<T>(dx + c, gv);
    }
  } else {
    for (int j = threadIdx.x; j < ld; j += 256) {
      float gv = 0.f;
      if (j < V) gv = sc * (__expf(ldv<T>(x, j) - lse) - (j == tgt ? 1.f : 0.f));
      stv<T>(dx, j, gv);
    }
  }
}

// Register-resident variant for bf16 training rows that fit in the block's registers
// (GPT-2: 50304 columns = 25 x 16 B per thread at 256 threads): the row is loaded ONCE,
// max / argmax and sum-exp are two exact block reductions over the registers, and the
// gradient is written from the same registers - one HBM read + one write of the logits
// instead of read, re-read (L2 misses at 16 K rows of 100 KB in flight), write.
template <int NT>
__device__ __forceinline__ float block_max_arg(float m, int& arg, float* sred, int* sarg) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const float om = __shfl_xor(m, off, 64);
    const int oa = __shfl_xor(arg, off, 64);
    if (om > m || (om == m && oa < arg)) {
      m = om;
      arg = oa;
    }
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    sred[w] = m;
    sarg[w] = arg;
  }
  __syncthreads();
  m = sred[0];
  arg = sarg[0];
#pragma unroll
  for (int i = 1; i < NT / 64; ++i)
    if (sred[i] > m || (sred[i] == m && sarg[i] < arg)) {
      m = sred[i];
      arg = sarg[i];
    }
  return m;
}

template <int NT>
__device__ __forceinline__ float block_sum2(float s, float* sred) {
  s = wave_sum(s);
  const int w = threadIdx.x >> 6;
  __syncthreads();  // sred reuse after block_max_arg
  if ((threadIdx.x & 63) == 0) sred[w] = s;
  __syncthreads();
  float r = 0.f;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) r += sred[i];
  return r;
}

__device__ __forceinline__ float bf_lo(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float bf_hi(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }

// Keep the row as packed bf16: without this the compiler keeps the 8 unpacked floats of every
// chunk alive from the max pass to the sum / gradient passes (4x the registers, 1 wave/SIMD).
template <int NCH>
__device__ __forceinline__ void opaque(uint32_t (&v)[NCH][4]) {
#pragma unroll
  for (int c = 0; c < NCH; ++c)
#pragma unroll
    for (int i = 0; i < 4; ++i) asm volatile("" : "+v"(v[c][i]));
}

template <int NT, int NCH, bool ARG>
__global__ __launch_bounds__(NT) void xent_reg_kernel(const bf16_t* logits, bf16_t* dlogits,
                                                     const int64_t* __restrict__ target, float* __restrict__ loss,
                                                     float* __restrict__ lse_out, int64_t* __restrict__ argmax,
                                                     int M, int V, int ld, float grad_scale, int ignore_index) {
  __shared__ float sred[NT / 64];
  __shared__ int sarg[NT / 64];
  const int row = blockIdx.x;
  const bf16_t* x = logits + (long long)row * ld;
  const int tid = threadIdx.x;
  // target logit read before any write of this row (dlogits may alias logits)
  const int64_t tgt = target ? target[row] : -1;
  const bool valid = target && tgt != ignore_index && tgt >= 0 && tgt < V;
  const float xt = (tid == 0 && valid) ? bf2f(x[tgt]) : 0.f;
  // the row, 8 bf16 per 16-B chunk, chunk c of thread t at column (c*NT + t)*8; columns >= V
  // (vocabulary padding, and chunks past the row) become -inf, so exp() zeroes them below
  // buffer loads: one VGPR offset (tid * 16) + a scalar per-chunk offset; chunks past the row
  // read 0 through the descriptor's range check and are masked below like the padding
  const auto rx = make_rsrc(x, 0, (long long)ld * 2);
  uint32_t v[NCH][4];
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int col = (c * NT + tid) * 8;
    const u32x4 q = __builtin_amdgcn_raw_buffer_load_b128(rx, tid * 16, c * NT * 16, 0);
    v[c][0] = q[0];
    v[c][1] = q[1];
    v[c][2] = q[2];
    v[c][3] = q[3];
    if (col + 8 > V) {
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (col + e >= V) v[c][e >> 1] = e & 1 ? (v[c][e >> 1] & 0x0000ffffu) | 0xff800000u
                                               : (v[c][e >> 1] & 0xffff0000u) | 0x0000ff80u;
    }
  }
  float m = -INFINITY;
#pragma unroll
  for (int c = 0; c < NCH; ++c)
#pragma unroll
    for (int i = 0; i < 4; ++i) m = fmaxf(m, fmaxf(bf_lo(v[c][i]), bf_hi(v[c][i])));
  int arg = 0x7fffffff;
  if constexpr (ARG) {  // first column holding the maximum (per thread columns ascend with c, e)
    const float mt = m;
#pragma unroll
    for (int c = NCH - 1; c >= 0; --c)
#pragma unroll
      for (int e = 7; e >= 0; --e) {
        const float f = e & 1 ? bf_hi(v[c][e >> 1]) : bf_lo(v[c][e >> 1]);
        if (f == mt) arg = (c * NT + tid) * 8 + e;
      }
  }
  m = block_max_arg<NT>(m, arg, sred, sarg);
  opaque(v);
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < NCH; ++c)
#pragma unroll
    for (int i = 0; i < 4; ++i) s += __expf(bf_lo(v[c][i]) - m) + __expf(bf_hi(v[c][i]) - m);
  s = block_sum2<NT>(s, sred);
  const float lse = m + __logf(s);
  if (tid == 0) {
    if (loss) loss[row] = valid ? lse - xt : 0.f;
    if (lse_out) lse_out[row] = lse;
    if (argmax) argmax[row] = arg;
  }
  if (!dlogits) return;
  __syncthreads();  // every thread's reads of the row precede any overwrite (in-place dlogits)
  opaque(v);
  const auto rd = make_rsrc(dlogits + (long long)row * ld, 0, (long long)ld * 2);
  const float sc = valid ? grad_scale : 0.f;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int col = (c * NT + tid) * 8;
    {
      float g[8];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        g[2 * i] = sc * __expf(bf_lo(v[c][i]) - lse);
        g[2 * i + 1] = sc * __expf(bf_hi(v[c][i]) - lse);
      }
      const int o = (int)(tgt - col);
      if (valid && (unsigned)o < 8u) {
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (e == o) g[e] -= sc;
      }
      // stores past the row are dropped by the descriptor's range check
      __builtin_amdgcn_raw_buffer_store_b128(pack8bf(g), rd, tid * 16, c * NT * 16, 0);
    }
  }
}

}  // namespace rtdc

using namespace rtdc;

// register-resident launch for bf16 rows of at most NT*NCH*8 columns (returns false if none fits)
static bool launch_xent_reg(const void* logits, void* dlogits, const int64_t* target, float* loss, float* lse,
                            int64_t* argmax, int M, int V, int ld, float grad_scale, int ignore_index,
                            hipStream_t st) {
  if (ld % 8 != 0 || getenv("RTDC_XENT_TWO_PASS")) return false;
#define XR(NT, NCH)                                                                                          \
  if (ld <= NT * NCH * 8) {                                                                                 \
    if (argmax)                                                                                              \
      hipLaunchKernelGGL((xent_reg_kernel<NT, NCH, true>), dim3(M), dim3(NT), 0, st, (const bf16_t*)logits,  \
                         (bf16_t*)dlogits, target, loss, lse, argmax, M, V, ld, grad_scale, ignore_index);  \
    else                                                                                                     \
      hipLaunchKernelGGL((xent_reg_kernel<NT, NCH, false>), dim3(M), dim3(NT), 0, st, (const bf16_t*)logits, \
                         (bf16_t*)dlogits, target, loss, lse, argmax, M, V, ld, grad_scale, ignore_index);  \
    return true;                                                                                             \
  }
  // NT x NCH x 8 columns; one wave per SIMD per block so several blocks share a CU and one
  // block's write phase overlaps the next block's loads (GPT-2: 256 x 25)
  XR(256, 4)
  XR(256, 8)
  XR(256, 16)
  XR(256, 25)
  XR(512, 16)
  XR(1024, 16)
#undef XR
  return false;
}

extern "C" int rtdc_xent(const void* logits, void* dlogits, const int64_t* target, float* loss,
                         float* lse, int64_t* argmax, int M, int V, int ld, float grad_scale,
                         int ignore_index, int is_bf16, hipStream_t st) {
  dim3 grid(M), block(256);
  const bool vec = (ld % 8 == 0);
  if (is_bf16 && launch_xent_reg(logits, dlogits, target, loss, lse, argmax, M, V, ld, grad_scale, ignore_index,
                                 st))
    return hipGetLastError() == hipSuccess ? 0 : 2;
  if (is_bf16) {
    if (vec)
      hipLaunchKernelGGL((xent_kernel<bf16_t, true>), grid, block, 0, st, (const bf16_t*)logits,
                         (bf16_t*)dlogits, target, loss, lse, argmax, M, V, ld, grad_scale, ignore_index);
    else
      hipLaunchKernelGGL((xent_kernel<bf16_t, false>), grid, block, 0, st, (const bf16_t*)logits,
                         (bf16_t*)dlogits, target, loss, lse, argmax, M, V, ld, grad_scale, ignore_index);
  } else {
    if (vec)
      hipLaunchKernelGGL((xent_kernel<float, true>), grid, block, 0, st, (const float*)logits,
                         (float*)dlogits, target, loss, lse, argmax, M, V, ld, grad_scale, ignore_index);
    else
      hipLaunchKernelGGL((xent_kernel<float, false>), grid, block, 0, st, (const float*)logits,
                         (float*)dlogits, target, loss, lse, argmax, M, V, ld, grad_scale, ignore_index);
  }
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

// ---- loss finalisation without ATen reductions: one block sums the per-row losses and counts
// the non-ignored targets in a fixed order; out[0] = mean loss, out[1] = divisor (count clamped
// to >= 1, or the caller's fixed divisor when target is null).
namespace rtdc {
__global__ __launch_bounds__(1024) void xent_finalize_kernel(const float* __restrict__ loss,
                                                            const int64_t* __restrict__ target, int M, float fixed_n,
                                                            int ignore, float* __restrict__ out) {
  __shared__ float red[16];
  float s = 0.f, c = 0.f;
  for (int i = threadIdx.x; i < M; i += 1024) {
    s += loss[i];
    if (target) c += target[i] != ignore ? 1.f : 0.f;
  }
  s = block_sum<1024>(s, red);
  c = block_sum<1024>(c, red);
  if (threadIdx.x == 0) {
    const float n = target ? fmaxf(c, 1.f) : fixed_n;
    out[0] = s / n;
    out[1] = n;
  }
}

// out[0] = g[0] / den[0]: the upstream loss gradient over the divisor, as a device alpha
__global__ void xent_alpha_kernel(const float* __restrict__ g, const float* __restrict__ den, float* __restrict__ out) {
  if (threadIdx.x == 0 && blockIdx.x == 0) out[0] = g[0] / den[0];
}

// y = x * (g[0] / den[0]) (bf16 or fp32 x, 8 elements per thread)
template <typename T>
__global__ __launch_bounds__(256) void scale_dev_kernel(const T* __restrict__ x, T* __restrict__ y, long long n,
                                                       const float* __restrict__ g, const float* __restrict__ den) {
  const float a = g[0] / den[0];
  const long long n8 = n / 8;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n8; i += (long long)gridDim.x * 256) {
    if constexpr (sizeof(T) == 2) {
      const uint4 q = ((const uint4*)x)[i];
      const uint32_t w[4] = {q.x, q.y, q.z, q.w};
      uint32_t o[4];
#pragma unroll
      for (int e = 0; e < 4; ++e)
        o[e] = pack_bf2(__uint_as_float(w[e] << 16) * a, __uint_as_float(w[e] & 0xffff0000u) * a);
      ((uint4*)y)[i] = make_uint4(o[0], o[1], o[2], o[3]);
    } else {
      const float4 p = ((const float4*)x)[2 * i], q = ((const float4*)x)[2 * i + 1];
      ((float4*)y)[2 * i] = make_float4(p.x * a, p.y * a, p.z * a, p.w * a);
      ((float4*)y)[2 * i + 1] = make_float4(q.x * a, q.y * a, q.z * a, q.w * a);
    }
  }
  // tail (n % 8)
  for (long long i = n8 * 8 + blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    if constexpr (sizeof(T) == 2) y[i] = f2bf(bf2f(x[i]) * a);
    else y[i] = x[i] * a;
  }
}
}  // namespace rtdc

extern "C" int rtdc_xent_finalize(const float* loss, const int64_t* target, int M, float fixed_n, int ignore, float* out,
                                  hipStream_t st) {
  hipLaunchKernelGGL(rtdc::xent_finalize_kernel, dim3(1), dim3(1024), 0, st, loss, target, M, fixed_n, ignore, out);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

extern "C" int rtdc_xent_alpha(const float* g, const float* den, float* out, hipStream_t st) {
  hipLaunchKernelGGL(rtdc::xent_alpha_kernel, dim3(1), dim3(64), 0, st, g, den, out);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

extern "C" int rtdc_scale_dev(const void* x, void* y, long long n, int is_bf16, const float* g, const float* den,
                              hipStream_t st) {
  long long blocks = (n / 8 + 255) / 256;
  blocks = blocks < 1 ? 1 : (blocks > 4096 ? 4096 : blocks);
  if (is_bf16)
    hipLaunchKernelGGL(rtdc::scale_dev_kernel<bf16_t>, dim3((unsigned)blocks), dim3(256), 0, st, (const bf16_t*)x,
                       (bf16_t*)y, n, g, den);
  else
    hipLaunchKernelGGL(rtdc::scale_dev_kernel<float>, dim3((unsigned)blocks), dim3(256), 0, st, (const float*)x,
                       (float*)y, n, g, den);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

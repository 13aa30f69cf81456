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
#include "common.h"

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

}  // namespace rtdc

using namespace rtdc;

extern "C" int rtdc_xent(const void* logits, void* dlogits, const int64_t* target, float* loss,
                         float* lse, int64_t* argmax, int M, int V, int ld, float grad_scale,
                         int ignore_index, int is_bf16, hipStream_t st) {
  dim3 grid(M), block(256);
  const bool vec = (ld % 8 == 0);
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

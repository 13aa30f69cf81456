// Embedding, dropout (Philox, regenerated in backward) and small fused elementwise ops (gfx950).
// All bf16 traffic moves 16 B per lane (cdna_hip_programming.md §6 Guideline 13).
#include "common.h"

namespace rtdc {

__device__ __forceinline__ void ld8e(const bf16_t* p, float* v) {
  uint4 x = *(const uint4*)p;
  uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[2 * i] = __uint_as_float(w[i] << 16);
    v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}
__device__ __forceinline__ void st8e(bf16_t* p, const float* v) {
  *(uint4*)p = make_uint4(pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3]), pack_bf2(v[4], v[5]),
                          pack_bf2(v[6], v[7]));
}

// out[t, :] = wte[idx[t], :] + (wpe ? wpe[t % T, :] : 0); one wave per token.
__global__ __launch_bounds__(256) void embed_fwd_kernel(const int64_t* __restrict__ idx, const bf16_t* __restrict__ wte,
                                                       const bf16_t* __restrict__ wpe, bf16_t* __restrict__ out,
                                                       int ntok, int T, int D) {
  const int lane = threadIdx.x & 63;
  const int t = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (t >= ntok) return;
  const long long row = idx[t];
  const int pos = t % T;
  for (int c = lane * 8; c < D; c += 512) {
    float a[8], b[8];
    ld8e(wte + row * D + c, a);
    if (wpe) {
      ld8e(wpe + (long long)pos * D + c, b);
#pragma unroll
      for (int e = 0; e < 8; ++e) a[e] += b[e];
    }
    st8e(out + (long long)t * D + c, a);
  }
}

// dwte[v, :] = sum over tokens t with idx[t] == v of dout[t, :], deterministic: the tokens
// arrive stably sorted by id (sidx = sorted ids, perm = their original positions), one wave per
// sorted position; only the wave at the start of a run of equal ids works, summing the run in
// original token order and writing the row once.  No float atomics (bitwise reproducible).
__global__ __launch_bounds__(256) void embed_bwd_wte_kernel(const int64_t* __restrict__ sidx,
                                                           const int64_t* __restrict__ perm,
                                                           const bf16_t* __restrict__ dout,
                                                           float* __restrict__ dwte, int ntok, int D,
                                                           int accumulate) {
  const int lane = threadIdx.x & 63;
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= ntok) return;
  const int64_t row = sidx[i];
  if (i > 0 && sidx[i - 1] == row) return;
  int e = i + 1;
  while (e < ntok && sidx[e] == row) ++e;
  for (int c = lane * 8; c < D; c += 512) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int j = i; j < e; ++j) {
      float g[8];
      ld8e(dout + perm[j] * D + c, g);
#pragma unroll
      for (int q = 0; q < 8; ++q) acc[q] += g[q];
    }
    float* o = dwte + row * D + c;
    if (accumulate) {  // second use of a tied table: add into the gradient already there
      const float4 a0 = *(const float4*)o, a1 = *(const float4*)(o + 4);
      acc[0] += a0.x; acc[1] += a0.y; acc[2] += a0.z; acc[3] += a0.w;
      acc[4] += a1.x; acc[5] += a1.y; acc[6] += a1.z; acc[7] += a1.w;
    }
    *(float4*)o = make_float4(acc[0], acc[1], acc[2], acc[3]);
    *(float4*)(o + 4) = make_float4(acc[4], acc[5], acc[6], acc[7]);
  }
}

// x[0, n) = v with 16-B stores (the embedding-gradient reset: a 2.1 GB fp32 table per Llama-3-8B
// step, which ATen's FillFunctor did before; grid-stride, ~2 blocks per CU keep HBM busy)
__global__ __launch_bounds__(256) void fill_f32_kernel(float* __restrict__ x, long long n, float v) {
  const long long n4 = n >> 2;
  const float4 q = make_float4(v, v, v, v);
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n4; i += (long long)gridDim.x * 256) ((float4*)x)[i] = q;
  if (blockIdx.x == 0 && threadIdx.x < (n & 3)) x[(n4 << 2) + threadIdx.x] = v;
}

// dwpe[p, d] (+)= sum_b dout[b*T + p, d]   deterministic (fixed b order)
__global__ __launch_bounds__(256) void embed_bwd_wpe_kernel(const bf16_t* __restrict__ dout, float* __restrict__ dwpe,
                                                           int B, int T, int D, int accumulate) {
  const int d = blockIdx.y * 256 + threadIdx.x;
  const int p = blockIdx.x;
  if (d >= D) return;
  float s = 0.f;
  for (int b = 0; b < B; ++b) s += bf2f(dout[((long long)b * T + p) * D + d]);
  const long long o = (long long)p * D + d;
  dwpe[o] = accumulate ? dwpe[o] + s : s;
}

// Dropout with a counter-based Philox stream: element e uses counter (offset + e/4), lane e%4.
// keep = u >= p ; y = keep ? x/(1-p) : 0.  Same (seed, offset) regenerates the mask.
template <typename T>
__device__ __forceinline__ float ldx(const T* p, long long i);
template <> __device__ __forceinline__ float ldx<float>(const float* p, long long i) { return p[i]; }
template <> __device__ __forceinline__ float ldx<bf16_t>(const bf16_t* p, long long i) { return bf2f(p[i]); }
template <typename T>
__device__ __forceinline__ void stx(T* p, long long i, float v);
template <> __device__ __forceinline__ void stx<float>(float* p, long long i, float v) { p[i] = v; }
template <> __device__ __forceinline__ void stx<bf16_t>(bf16_t* p, long long i, float v) { p[i] = f2bf(v); }

template <typename T>
__global__ __launch_bounds__(256) void dropout_kernel(const T* __restrict__ x, T* __restrict__ y, long long n, float p,
                                                     unsigned long long seed, unsigned long long offset,
                                                     const long long* __restrict__ off_dev) {
  const float scale = 1.f / (1.f - p);
  if (off_dev) offset += (unsigned long long)*off_dev;  // graph replay: per-step base on device
  for (long long q = blockIdx.x * 256LL + threadIdx.x; q * 4 < n; q += gridDim.x * 256LL) {
    uint4 r = Philox::gen(seed, 0, offset + q);
    uint32_t rr[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const long long i = q * 4 + e;
      if (i < n) {
        const bool keep = u32_to_unit(rr[e]) >= p;
        stx<T>(y, i, keep ? ldx<T>(x, i) * scale : 0.f);
      }
    }
  }
}

// y = relu(x) then dropout (toy MLP hidden activation, R/my_ray_module.py:100-104), and its
// backward dx = dy * keep/(1-p) * (h > 0) with h the saved pre-activation.
template <typename T>
__global__ __launch_bounds__(256) void relu_dropout_kernel(const T* __restrict__ h, T* __restrict__ y,
                                                          const T* __restrict__ dy, T* __restrict__ dx, long long n,
                                                          float p, unsigned long long seed,
                                                          unsigned long long offset, int backward) {
  // backward == 2: the mask is read off the saved OUTPUT h = relu(x) * keep / (1 - p) (h > 0
  // iff kept and positive) - no RNG, right under graph replay too (fused GEMM dropout)
  const float scale = p > 0.f ? 1.f / (1.f - p) : 1.f;
  for (long long q = blockIdx.x * 256LL + threadIdx.x; q * 4 < n; q += gridDim.x * 256LL) {
    uint32_t rr[4] = {0u, 0u, 0u, 0u};
    if (p > 0.f && backward != 2) {
      uint4 r = Philox::gen(seed, 0, offset + q);
      rr[0] = r.x; rr[1] = r.y; rr[2] = r.z; rr[3] = r.w;
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const long long i = q * 4 + e;
      if (i < n) {
        const bool keep = (p > 0.f && backward != 2) ? (u32_to_unit(rr[e]) >= p) : true;
        const float hv = ldx<T>(h, i);
        const float m = (keep && hv > 0.f) ? scale : 0.f;
        if (backward) stx<T>(dx, i, ldx<T>(dy, i) * m);
        else stx<T>(y, i, hv * m);
      }
    }
  }
}

}  // namespace rtdc

using namespace rtdc;

static inline unsigned ew_grid(long long n_quads) {
  long long b = (n_quads + 255) / 256;
  if (b > 8192) b = 8192;
  if (b < 1) b = 1;
  return (unsigned)b;
}

extern "C" int rtdc_embed_fwd(const int64_t* idx, const void* wte, const void* wpe, void* out, int ntok,
                              int T, int D, hipStream_t st) {
  if (D % 8 != 0) return 1;
  hipLaunchKernelGGL(embed_fwd_kernel, dim3((ntok + 3) / 4), dim3(256), 0, st, idx, (const bf16_t*)wte,
                     (const bf16_t*)wpe, (bf16_t*)out, ntok, T, D);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

// sidx/perm: token ids stably sorted and their original positions (dwte rows that no token
// uses are left untouched: the caller zero-fills).
extern "C" int rtdc_embed_bwd(const int64_t* sidx, const int64_t* perm, const void* dout, float* dwte, float* dwpe,
                              int B, int T, int D, int accumulate_wpe, int accumulate_wte, hipStream_t st) {
  if (D % 8 != 0) return 1;
  const int ntok = B * T;
  hipLaunchKernelGGL(embed_bwd_wte_kernel, dim3((ntok + 3) / 4), dim3(256), 0, st, sidx, perm, (const bf16_t*)dout,
                     dwte, ntok, D, accumulate_wte);
  if (dwpe)
    hipLaunchKernelGGL(embed_bwd_wpe_kernel, dim3(T, (D + 255) / 256), dim3(256), 0, st, (const bf16_t*)dout,
                       dwpe, B, T, D, accumulate_wpe);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

extern "C" int rtdc_fill_f32(float* x, long long n, float v, hipStream_t st) {
  if (n <= 0) return 0;
  if (((uintptr_t)x & 15) != 0) return 1;
  long long blocks = (n / 4 + 255) / 256;
  blocks = blocks < 1 ? 1 : (blocks > 2048 ? 2048 : blocks);
  hipLaunchKernelGGL(fill_f32_kernel, dim3((unsigned)blocks), dim3(256), 0, st, x, n, v);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

// off_dev (optional): device-resident counter base added to `offset` (hipGraph replays)
extern "C" int rtdc_dropout(const void* x, void* y, long long n, float p, unsigned long long seed,
                            unsigned long long offset, const long long* off_dev, int is_bf16, hipStream_t st) {
  const unsigned g = ew_grid((n + 3) / 4);
  if (is_bf16)
    hipLaunchKernelGGL((dropout_kernel<bf16_t>), dim3(g), dim3(256), 0, st, (const bf16_t*)x, (bf16_t*)y, n, p,
                       seed, offset, off_dev);
  else
    hipLaunchKernelGGL((dropout_kernel<float>), dim3(g), dim3(256), 0, st, (const float*)x, (float*)y, n, p,
                       seed, offset, off_dev);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

extern "C" int rtdc_relu_dropout(const void* h, void* y, const void* dy, void* dx, long long n, float p,
                                 unsigned long long seed, unsigned long long offset, int backward, int is_bf16,
                                 hipStream_t st) {
  const unsigned g = ew_grid((n + 3) / 4);
  if (is_bf16)
    hipLaunchKernelGGL((relu_dropout_kernel<bf16_t>), dim3(g), dim3(256), 0, st, (const bf16_t*)h, (bf16_t*)y,
                       (const bf16_t*)dy, (bf16_t*)dx, n, p, seed, offset, backward);
  else
    hipLaunchKernelGGL((relu_dropout_kernel<float>), dim3(g), dim3(256), 0, st, (const float*)h, (float*)y,
                       (const float*)dy, (float*)dx, n, p, seed, offset, backward);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

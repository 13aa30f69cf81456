// Causal softmax forward/backward over materialised attention scores (gfx950).
//
// Used by the GEMM-composed attention path (S = alpha*Q K^T by the MFMA GEMM with tiles above
// the diagonal skipped; O = P V; backward dS = P*(dP - rowsum(P*dP))).  One wave64 per row,
// the row held in registers (T <= 4096), 16-B vector loads.  Entries above the diagonal are
// never read (the GEMM did not write them) and are written as exact zeros so the following
// P*V / P^T*dO products may read whole diagonal tiles.
#include "common.h"

namespace rtdc {

__device__ __forceinline__ void ld8f(const bf16_t* p, float* v) {
  uint4 x = *(const uint4*)p;
  uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[2 * i] = __uint_as_float(w[i] << 16);
    v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}
__device__ __forceinline__ void st8f(bf16_t* p, const float* v) {
  *(uint4*)p = make_uint4(pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3]), pack_bf2(v[4], v[5]),
                          pack_bf2(v[6], v[7]));
}

// rows = BH*T; row r -> query index i = r % T; valid columns [0, i] when causal.
template <int CPL>
__global__ __launch_bounds__(256) void softmax_fwd_kernel(const bf16_t* __restrict__ S, bf16_t* __restrict__ P,
                                                         float* __restrict__ lse_out, long long rows, int T,
                                                         int causal) {
  const int lane = threadIdx.x & 63;
  const long long r = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= rows) return;
  const int i = (int)(r % T);
  const int ncols = causal ? i + 1 : T;
  const bf16_t* s = S + r * T;
  bf16_t* p = P + r * T;
  float v[CPL][8];
  float mx = -INFINITY;
#pragma unroll
  for (int c = 0; c < CPL; ++c) {
    const int j0 = (lane + 64 * c) * 8;
    if (j0 < ncols) {
      ld8f(s + j0, v[c]);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        if (j0 + e >= ncols) v[c][e] = -INFINITY;
        mx = fmaxf(mx, v[c][e]);
      }
    }
  }
  mx = wave_max(mx);
  float sum = 0.f;
#pragma unroll
  for (int c = 0; c < CPL; ++c) {
    const int j0 = (lane + 64 * c) * 8;
    if (j0 < ncols) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        v[c][e] = (j0 + e < ncols) ? __expf(v[c][e] - mx) : 0.f;
        sum += v[c][e];
      }
    }
  }
  sum = wave_sum(sum);
  const float inv = 1.f / sum;
  if (lane == 0 && lse_out) lse_out[r] = mx + __logf(sum);
#pragma unroll
  for (int c = 0; c < CPL; ++c) {
    const int j0 = (lane + 64 * c) * 8;
    if (j0 < T) {
      float o[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = (j0 < ncols) ? v[c][e] * inv : 0.f;
      st8f(p + j0, o);
    }
  }
}

// dS = P * (dP - sum_j P*dP); dS may alias dP.
template <int CPL>
__global__ __launch_bounds__(256) void softmax_bwd_kernel(const bf16_t* __restrict__ P, const bf16_t* dP,
                                                         bf16_t* dS, long long rows, int T, int causal) {
  const int lane = threadIdx.x & 63;
  const long long r = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= rows) return;
  const int i = (int)(r % T);
  const int ncols = causal ? i + 1 : T;
  const bf16_t* p = P + r * T;
  const bf16_t* dp = dP + r * T;
  float pv[CPL][8], dv[CPL][8];
  float dot = 0.f;
#pragma unroll
  for (int c = 0; c < CPL; ++c) {
    const int j0 = (lane + 64 * c) * 8;
    if (j0 < ncols) {
      ld8f(p + j0, pv[c]);
      ld8f(dp + j0, dv[c]);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        if (j0 + e >= ncols) { pv[c][e] = 0.f; dv[c][e] = 0.f; }
        dot += pv[c][e] * dv[c][e];
      }
    }
  }
  dot = wave_sum(dot);
  bf16_t* ds = dS + r * T;
#pragma unroll
  for (int c = 0; c < CPL; ++c) {
    const int j0 = (lane + 64 * c) * 8;
    if (j0 < T) {
      float o[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = (j0 < ncols) ? pv[c][e] * (dv[c][e] - dot) : 0.f;
      st8f(ds + j0, o);
    }
  }
}

}  // namespace rtdc

using namespace rtdc;

extern "C" int rtdc_softmax_fwd(const void* S, void* P, float* lse, long long rows, int T, int causal,
                                hipStream_t st) {
  if (T % 8 != 0) return 1;
  const int cpl = (T / 8 + 63) / 64;
  dim3 grid((unsigned)((rows + 3) / 4)), block(256);
#define L(C) hipLaunchKernelGGL((softmax_fwd_kernel<C>), grid, block, 0, st, (const bf16_t*)S, (bf16_t*)P, lse, rows, T, causal)
  if (cpl <= 1) L(1);
  else if (cpl <= 2) L(2);
  else if (cpl <= 4) L(4);
  else if (cpl <= 8) L(8);
  else return 1;
#undef L
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

extern "C" int rtdc_softmax_bwd(const void* P, const void* dP, void* dS, long long rows, int T, int causal,
                                hipStream_t st) {
  if (T % 8 != 0) return 1;
  const int cpl = (T / 8 + 63) / 64;
  dim3 grid((unsigned)((rows + 3) / 4)), block(256);
#define L(C) hipLaunchKernelGGL((softmax_bwd_kernel<C>), grid, block, 0, st, (const bf16_t*)P, (const bf16_t*)dP, (bf16_t*)dS, rows, T, causal)
  if (cpl <= 1) L(1);
  else if (cpl <= 2) L(2);
  else if (cpl <= 4) L(4);
  else if (cpl <= 8) L(8);
  else return 1;
#undef L
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

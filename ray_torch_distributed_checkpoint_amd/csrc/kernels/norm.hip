// LayerNorm / RMSNorm forward + backward for bf16 activations (gfx950).
//
// One wave64 per row; each lane owns CPL 16-B chunks (8 bf16) of the row, so the row lives in
// registers between the statistics pass and the normalisation pass (one HBM read, one write).
// Backward fuses the residual-gradient add (dx = dres + LN'(dy)) and writes per-wave partial
// dgamma/dbeta rows to a workspace that a second kernel reduces in a fixed order, so the
// parameter gradients are bitwise reproducible (no float atomics, MI355X_MICROARCH.md §Global
// float atomics).
#include "gemm_common.h"

#include <cstdlib>

namespace rtdc {

__device__ __forceinline__ void ld8(const bf16_t* p, float* v) {
  uint4 x = *(const uint4*)p;
  uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[2 * i] = __uint_as_float(w[i] << 16);
    v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}
__device__ __forceinline__ void st8(bf16_t* p, const float* v) {
  uint4 x = make_uint4(pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3]), pack_bf2(v[4], v[5]),
                       pack_bf2(v[6], v[7]));
  *(uint4*)p = x;
}

// red4[q] = (add ? red4[q] + v : v) for the 4 floats v (per-block partial-sum combine in LDS)
__device__ __forceinline__ void red_acc4(float* red, int q, const float* v, int add) {
  f32x4* p = (f32x4*)red + q;
  f32x4 a = {v[0], v[1], v[2], v[3]};
  if (add) a = *p + a;
  *p = a;
}

template <int CPL, bool RMS>
__global__ __launch_bounds__(256) void norm_fwd_kernel(const bf16_t* __restrict__ x,
                                                      const bf16_t* __restrict__ g,
                                                      const bf16_t* __restrict__ b,
                                                      bf16_t* __restrict__ y, float* __restrict__ mean_out,
                                                      float* __restrict__ rstd_out, int M, int D, float eps) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const int nch = D >> 3;
  const bf16_t* xr = x + (long long)row * D;
  float v[CPL][8];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < CPL; ++i) {
    const int c = lane + 64 * i;
    if (c < nch) {
      ld8(xr + c * 8, v[i]);
#pragma unroll
      for (int e = 0; e < 8; ++e) s += v[i][e];
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[i][e] = 0.f;
    }
  }
  float mean = 0.f;
  if (!RMS) mean = wave_sum(s) / D;
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < CPL; ++i) {
    const int c = lane + 64 * i;
    if (c < nch) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float d = v[i][e] - mean;
        ss += d * d;
      }
    }
  }
  const float rstd = rsqrtf(wave_sum(ss) / D + eps);
  if (lane == 0) {
    if (mean_out) mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
  bf16_t* yr = y + (long long)row * D;
#pragma unroll
  for (int i = 0; i < CPL; ++i) {
    const int c = lane + 64 * i;
    if (c < nch) {
      float gg[8], bb[8], o[8];
      ld8(g + c * 8, gg);
      if (!RMS) ld8(b + c * 8, bb);
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = (v[i][e] - mean) * rstd * gg[e] + (RMS ? 0.f : bb[e]);
      st8(yr + c * 8, o);
    }
  }
}

// Two rows per wave with full 16-B lanes where one row's D / 8 chunks are 64k + 32 (GPT-2's
// D = 768: 96 chunks, so the one-row form leaves half the lanes idle on its second load): the
// 2 (64k + 32) chunks of a row pair are NPL = 2k + 1 per lane, chunk q = lane + 64 i of the pair
// belongs to row q / nch.  Same per-row math as norm_fwd_kernel; the second row's chunks sit
// on other lanes, so its wave reductions add the partials in another order (last-bit
// differences in mean / rstd).
template <int NPL, bool RMS>
__global__ __launch_bounds__(256) void norm_fwd2r_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ g,
                                                         const bf16_t* __restrict__ b, bf16_t* __restrict__ y,
                                                         float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                         int M, int D, float eps) {
  const int lane = threadIdx.x & 63;
  const int r0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * 2;  // rows r0, r0 + 1
  if (r0 >= M) return;
  const int nch = D >> 3;
  const bool two = r0 + 1 < M;
  const bf16_t* xr = x + (long long)r0 * D;  // the pair is contiguous: chunk q at xr + 8 q
  float v[NPL][8];
  float s[2] = {0.f, 0.f};
#pragma unroll
  for (int i = 0; i < NPL; ++i) {
    const int q = lane + 64 * i;
    const int rr = q >= nch ? 1 : 0;
    if (rr == 0 || two) {
      ld8(xr + q * 8, v[i]);
      float t = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) t += v[i][e];
      s[rr] += t;
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[i][e] = 0.f;
    }
  }
  float mean[2] = {0.f, 0.f};
  if (!RMS) {
    mean[0] = wave_sum(s[0]) / D;
    mean[1] = wave_sum(s[1]) / D;
  }
  float ss[2] = {0.f, 0.f};
#pragma unroll
  for (int i = 0; i < NPL; ++i) {
    const int q = lane + 64 * i;
    const int rr = q >= nch ? 1 : 0;
    float t = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float d = v[i][e] - mean[rr];
      t += d * d;
    }
    ss[rr] += t;
  }
  const float rstd[2] = {rsqrtf(wave_sum(ss[0]) / D + eps), rsqrtf(wave_sum(ss[1]) / D + eps)};
  if (lane == 0) {
    if (mean_out) mean_out[r0] = mean[0];
    rstd_out[r0] = rstd[0];
    if (two) {
      if (mean_out) mean_out[r0 + 1] = mean[1];
      rstd_out[r0 + 1] = rstd[1];
    }
  }
  bf16_t* yr = y + (long long)r0 * D;
#pragma unroll
  for (int i = 0; i < NPL; ++i) {
    const int q = lane + 64 * i;
    const int rr = q >= nch ? 1 : 0;
    if (rr == 1 && !two) continue;
    const int c = q - rr * nch;
    float gg[8], bb[8], o[8];
    ld8(g + c * 8, gg);
    if (!RMS) ld8(b + c * 8, bb);
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = (v[i][e] - mean[rr]) * rstd[rr] * gg[e] + (RMS ? 0.f : bb[e]);
    st8(yr + q * 8, o);
  }
}

// dxhat = dy*g ; dx = rstd * (dxhat - mean(dxhat) - xhat * mean(dxhat*xhat))   (LayerNorm)
// dx = rstd * (dxhat - xhat * mean(dxhat*xhat))                                  (RMSNorm)
// CS: also the column sums of dx itself (the residual-stream gradient this kernel produces is
// the output gradient of the block's residual projection, whose bias gradient is exactly that
// colsum - computed here on the way out instead of re-reading dx in a separate reduction).
// Partial rows per block: ws_dg [nblk][D], ws_db = ws_dg + nblk*D, ws_cs = ws_db + nblk*D.
template <int CPL, bool RMS, bool CS>
__global__ __launch_bounds__(256) void norm_bwd_kernel(
    const bf16_t* __restrict__ dy, const bf16_t* __restrict__ x, const bf16_t* __restrict__ g,
    const float* __restrict__ mean_in, const float* __restrict__ rstd_in,
    const bf16_t* __restrict__ dres, bf16_t* __restrict__ dx, float* __restrict__ ws_dg,
    float* __restrict__ ws_db, float* __restrict__ ws_cs, int M, int D) {
  const int lane = threadIdx.x & 63;
  const int gw = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int nw = gridDim.x * 4;
  const int nch = D >> 3;
  float adg[CPL][8], adb[CPL][8], acs[CS ? CPL : 1][8];
#pragma unroll
  for (int i = 0; i < CPL; ++i)
#pragma unroll
    for (int e = 0; e < 8; ++e) adg[i][e] = adb[i][e] = 0.f;
#pragma unroll
  for (int i = 0; i < (CS ? CPL : 1); ++i)
#pragma unroll
    for (int e = 0; e < 8; ++e) acs[i][e] = 0.f;

  float gg[CPL][8];
#pragma unroll
  for (int i = 0; i < CPL; ++i) {
    const int c = lane + 64 * i;
    if (c < nch) ld8(g + c * 8, gg[i]);
  }

  // rows are software-pipelined: the next row's x / dy / dres (and its statistics) are in
  // flight while this row is reduced and written (a wave owns M/nw rows in sequence)
  uint4 px[CPL], pd[CPL], pr[CPL];
  float pmean = 0.f, prstd = 0.f;
  auto fetch = [&](int r) {
#pragma unroll
    for (int i = 0; i < CPL; ++i) {
      const int c = lane + 64 * i;
      if (c < nch) {
        px[i] = *(const uint4*)(x + (long long)r * D + c * 8);
        pd[i] = *(const uint4*)(dy + (long long)r * D + c * 8);
        if (dres) pr[i] = *(const uint4*)(dres + (long long)r * D + c * 8);
      }
    }
    pmean = RMS ? 0.f : mean_in[r];
    prstd = rstd_in[r];
  };
  if (gw < M) fetch(gw);
  for (int row = gw; row < M; row += nw) {
    const float mean = pmean;
    const float rstd = prstd;
    uint4 cx[CPL], cd[CPL], rraw[CPL];
#pragma unroll
    for (int i = 0; i < CPL; ++i) {
      cx[i] = px[i];
      cd[i] = pd[i];
      rraw[i] = pr[i];
    }
    if (row + nw < M) fetch(row + nw);
    float xh[CPL][8], dxh[CPL][8];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < CPL; ++i) {
      const int c = lane + 64 * i;
      if (c < nch) {
        float xv[8], dv[8];
        unpack8bf(u32x4{cx[i].x, cx[i].y, cx[i].z, cx[i].w}, xv);
        unpack8bf(u32x4{cd[i].x, cd[i].y, cd[i].z, cd[i].w}, dv);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          xh[i][e] = (xv[e] - mean) * rstd;
          dxh[i][e] = dv[e] * gg[i][e];
          s1 += dxh[i][e];
          s2 += dxh[i][e] * xh[i][e];
          adg[i][e] += dv[e] * xh[i][e];
          adb[i][e] += dv[e];
        }
      }
    }
    const float m1 = RMS ? 0.f : wave_sum(s1) / D;
    const float m2 = wave_sum(s2) / D;
    bf16_t* dxr = dx + (long long)row * D;
#pragma unroll
    for (int i = 0; i < CPL; ++i) {
      const int c = lane + 64 * i;
      if (c < nch) {
        float o[8], r[8];
        if (dres) {
          const uint32_t w[4] = {rraw[i].x, rraw[i].y, rraw[i].z, rraw[i].w};
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            r[2 * k] = __uint_as_float(w[k] << 16);
            r[2 * k + 1] = __uint_as_float(w[k] & 0xffff0000u);
          }
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          o[e] = rstd * (dxh[i][e] - m1 - xh[i][e] * m2);
          if (dres) o[e] += r[e];
          if constexpr (CS) acs[i][e] += o[e];
        }
        st8(dxr + c * 8, o);
      }
    }
  }
  // combine the block's 4 waves in LDS (fixed wave order), one partial row per block
  extern __shared__ float red[];  // [D] dgamma (+ [D] dbeta) (+ [D] colsum(dx))
  constexpr int KCS = RMS ? 1 : 2;
  const int wv = threadIdx.x >> 6;
  for (int w = 0; w < 4; ++w) {
    if (wv == w) {
#pragma unroll
      for (int i = 0; i < CPL; ++i) {
        const int c = lane + 64 * i;
        if (c < nch) {
          // 16-B LDS accesses (scalar ones at a 32-B lane stride were 8-way bank conflicts)
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            red_acc4(red, c * 2 + h, adg[i] + 4 * h, w);
            if (!RMS) red_acc4(red, D / 4 + c * 2 + h, adb[i] + 4 * h, w);
            if constexpr (CS) red_acc4(red, KCS * D / 4 + c * 2 + h, acs[i] + 4 * h, w);
          }
        }
      }
    }
    __syncthreads();
  }
  for (int d = threadIdx.x; d < D; d += 256) {
    ws_dg[(long long)blockIdx.x * D + d] = red[d];
    if (!RMS) ws_db[(long long)blockIdx.x * D + d] = red[D + d];
    if constexpr (CS) ws_cs[(long long)blockIdx.x * D + d] = red[KCS * D + d];
  }
}

// The same backward with 8-B (4-element) lane chunks, for widths whose 16-B chunk count is not
// a multiple of 64 (GPT-2: D = 768 -> 96 chunks of 8, so the 16-B form leaves half the lanes
// idle in its second chunk and carries [2][8] accumulators; here 192 chunks of 4 = 3 per lane,
// every lane busy, [3][4] accumulators: fewer VGPRs, more waves per SIMD for this latency-bound
// stream).  Same math, same per-block partial rows.
__device__ __forceinline__ void ld4b(const bf16_t* p, float* v) {
  const uint2 q = *(const uint2*)p;
  v[0] = __uint_as_float(q.x << 16);
  v[1] = __uint_as_float(q.x & 0xffff0000u);
  v[2] = __uint_as_float(q.y << 16);
  v[3] = __uint_as_float(q.y & 0xffff0000u);
}
__device__ __forceinline__ void unpack4(uint2 q, float* v) {
  v[0] = __uint_as_float(q.x << 16);
  v[1] = __uint_as_float(q.x & 0xffff0000u);
  v[2] = __uint_as_float(q.y << 16);
  v[3] = __uint_as_float(q.y & 0xffff0000u);
}

// Forward with 8-B lane chunks for widths whose 16-B chunk count is not a multiple of 64
// (GPT-2: D = 768 -> 192 chunks of 4 = 3 per lane, every lane busy; the 16-B form idles half
// the lanes in its second chunk).  A wave owns rows gw, gw + nw, ...: gamma / beta are loaded
// into registers once per wave instead of once per row, and the next row's x is in flight
// while this row is reduced and written (the rows are a pure HBM stream: 1 read + 1 write).
template <int CPL, bool RMS>
__global__ __launch_bounds__(256) void norm_fwd4_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ g,
                                                       const bf16_t* __restrict__ b, bf16_t* __restrict__ y,
                                                       float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                       int M, int D, float eps) {
  const int lane = threadIdx.x & 63;
  const int gw = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int nw = gridDim.x * 4;
  const int nch = D >> 2;
  float gg[CPL][4], bb[CPL][4];
#pragma unroll
  for (int i = 0; i < CPL; ++i) {
    const int c = lane + 64 * i;
    if (c < nch) {
      ld4b(g + c * 4, gg[i]);
      if (!RMS) ld4b(b + c * 4, bb[i]);
    }
  }
  uint2 px[CPL];
  auto fetch = [&](int r) {
#pragma unroll
    for (int i = 0; i < CPL; ++i) {
      const int c = lane + 64 * i;
      if (c < nch) {
        const unsigned long long q =
            __builtin_nontemporal_load((const unsigned long long*)(x + (long long)r * D + c * 4));
        px[i] = make_uint2((uint32_t)q, (uint32_t)(q >> 32));
      }
    }
  };
  if (gw < M) fetch(gw);
  for (int row = gw; row < M; row += nw) {
    float v[CPL][4];
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < CPL; ++i) {
      const int c = lane + 64 * i;
      if (c < nch) {
        unpack4(px[i], v[i]);
#pragma unroll
        for (int e = 0; e < 4; ++e) s += v[i][e];
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[i][e] = 0.f;
      }
    }
    if (row + nw < M) fetch(row + nw);
    const float mean = RMS ? 0.f : wave_sum(s) / D;
    float ss = 0.f;
#pragma unroll
    for (int i = 0; i < CPL; ++i) {
      const int c = lane + 64 * i;
      if (c < nch) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float d = v[i][e] - mean;
          ss += d * d;
        }
      }
    }
    const float rstd = rsqrtf(wave_sum(ss) / D + eps);
    if (lane == 0) {
      if (mean_out) mean_out[row] = mean;
      rstd_out[row] = rstd;
    }
    bf16_t* yr = y + (long long)row * D;
#pragma unroll
    for (int i = 0; i < CPL; ++i) {
      const int c = lane + 64 * i;
      if (c < nch) {
        float o[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = (v[i][e] - mean) * rstd * gg[i][e] + (RMS ? 0.f : bb[i][e]);
        *(uint2*)(yr + c * 4) = make_uint2(pack_bf2(o[0], o[1]), pack_bf2(o[2], o[3]));
      }
    }
  }
}

template <int CPL, bool RMS, bool CS>
__global__ __launch_bounds__(256) void norm_bwd4_kernel(
    const bf16_t* __restrict__ dy, const bf16_t* __restrict__ x, const bf16_t* __restrict__ g,
    const float* __restrict__ mean_in, const float* __restrict__ rstd_in,
    const bf16_t* __restrict__ dres, bf16_t* __restrict__ dx, float* __restrict__ ws_dg,
    float* __restrict__ ws_db, float* __restrict__ ws_cs, int M, int D) {
  const int lane = threadIdx.x & 63;
  const int gw = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int nw = gridDim.x * 4;
  const int nch = D >> 2;
  float adg[CPL][4], adb[CPL][4], acs[CS ? CPL : 1][4];
#pragma unroll
  for (int i = 0; i < CPL; ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) adg[i][e] = adb[i][e] = 0.f;
#pragma unroll
  for (int i = 0; i < (CS ? CPL : 1); ++i)
#pragma unroll
    for (int e = 0; e < 4; ++e) acs[i][e] = 0.f;

  float gg[CPL][4];
#pragma unroll
  for (int i = 0; i < CPL; ++i) {
    const int c = lane + 64 * i;
    if (c < nch) ld4b(g + c * 4, gg[i]);
  }
  uint2 px[CPL], pd[CPL], pr[CPL];
  float pmean = 0.f, prstd = 0.f;
  auto fetch = [&](int r) {
#pragma unroll
    for (int i = 0; i < CPL; ++i) {
      const int c = lane + 64 * i;
      if (c < nch) {
        px[i] = *(const uint2*)(x + (long long)r * D + c * 4);
        pd[i] = *(const uint2*)(dy + (long long)r * D + c * 4);
        if (dres) pr[i] = *(const uint2*)(dres + (long long)r * D + c * 4);
      }
    }
    pmean = RMS ? 0.f : mean_in[r];
    prstd = rstd_in[r];
  };
  if (gw < M) fetch(gw);
  for (int row = gw; row < M; row += nw) {
    const float mean = pmean;
    const float rstd = prstd;
    uint2 cx[CPL], cd[CPL], rraw[CPL];
#pragma unroll
    for (int i = 0; i < CPL; ++i) {
      cx[i] = px[i];
      cd[i] = pd[i];
      rraw[i] = pr[i];
    }
    if (row + nw < M) fetch(row + nw);
    float xh[CPL][4], dxh[CPL][4];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < CPL; ++i) {
      const int c = lane + 64 * i;
      if (c < nch) {
        float xv[4], dv[4];
        unpack4(cx[i], xv);
        unpack4(cd[i], dv);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          xh[i][e] = (xv[e] - mean) * rstd;
          dxh[i][e] = dv[e] * gg[i][e];
          s1 += dxh[i][e];
          s2 += dxh[i][e] * xh[i][e];
          adg[i][e] += dv[e] * xh[i][e];
          adb[i][e] += dv[e];
        }
      }
    }
    const float m1 = RMS ? 0.f : wave_sum(s1) / D;
    const float m2 = wave_sum(s2) / D;
    bf16_t* dxr = dx + (long long)row * D;
#pragma unroll
    for (int i = 0; i < CPL; ++i) {
      const int c = lane + 64 * i;
      if (c < nch) {
        float o[4], r[4];
        if (dres) unpack4(rraw[i], r);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          o[e] = rstd * (dxh[i][e] - m1 - xh[i][e] * m2);
          if (dres) o[e] += r[e];
          if constexpr (CS) acs[i][e] += o[e];
        }
        *(uint2*)(dxr + c * 4) = make_uint2(pack_bf2(o[0], o[1]), pack_bf2(o[2], o[3]));
      }
    }
  }
  extern __shared__ float red[];
  constexpr int KCS = RMS ? 1 : 2;
  const int wv = threadIdx.x >> 6;
  for (int w = 0; w < 4; ++w) {
    if (wv == w) {
#pragma unroll
      for (int i = 0; i < CPL; ++i) {
        const int c = lane + 64 * i;
        if (c < nch) {
          // 16-B LDS accesses (scalar ones at a 16-B lane stride were 4-way bank conflicts)
          red_acc4(red, c, adg[i], w);
          if (!RMS) red_acc4(red, D / 4 + c, adb[i], w);
          if constexpr (CS) red_acc4(red, KCS * D / 4 + c, acs[i], w);
        }
      }
    }
    __syncthreads();
  }
  for (int d = threadIdx.x; d < D; d += 256) {
    ws_dg[(long long)blockIdx.x * D + d] = red[d];
    if (!RMS) ws_db[(long long)blockIdx.x * D + d] = red[D + d];
    if constexpr (CS) ws_cs[(long long)blockIdx.x * D + d] = red[KCS * D + d];
  }
}

// out[d] (+)= sum_w ws[w][d], fixed summation order.  A block owns 64 columns; its 4 waves
// stride over the W partial rows (coalesced 256-B rows per wave) and combine through LDS,
// so a 1024 x 768 workspace is 12 blocks x 256 loads per lane instead of 768 serial chains.
// Sum W partial rows of ws [W][D] -> out[S][D] where block (x, y) reduces rows
// [y*R, (y+1)*R) of 64 columns; 4 waves stride the rows, combined in LDS in fixed order.
// Run twice (W -> S -> 1) so every thread keeps only a few independent loads in flight and
// the reduction order is fixed (deterministic).
struct OutPtrs {
  float* p[4];
};
// out: tmp + z * out_z when tmp is set (first of two stages), else outs.p[z]
__global__ __launch_bounds__(256) void colsum_ws_kernel(const float* __restrict__ ws, float* __restrict__ tmp,
                                                       OutPtrs outs, int W, int D, int R, int accumulate,
                                                       long long ws_z, long long out_z) {
  __shared__ float part[4][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  ws += blockIdx.z * ws_z;  // z = independent reductions batched into one launch
  float* out = tmp ? tmp + blockIdx.z * out_z : outs.p[blockIdx.z];
  const int d = blockIdx.x * 64 + lane;
  const int r0 = blockIdx.y * R, r1 = min(W, r0 + R);
  float s0 = 0.f, s1 = 0.f;
  if (d < D) {
    int w = r0 + wv;
    for (; w + 4 < r1; w += 8) {
      s0 += ws[(long long)w * D + d];
      s1 += ws[(long long)(w + 4) * D + d];
    }
    if (w < r1) s0 += ws[(long long)w * D + d];
  }
  part[wv][lane] = s0 + s1;
  __syncthreads();
  if (wv == 0 && d < D) {
    const float t = (part[0][lane] + part[1][lane]) + (part[2][lane] + part[3][lane]);
    float* o = out + (long long)blockIdx.y * D + d;
    *o = (accumulate && gridDim.y == 1) ? *o + t : t;
  }
}

// One launch for up to kWideMaxRows partial rows: a 1024-thread block owns 64 columns; its 16
// waves stride the rows (wave w: rows w, w+16, ...) with kWideU loads in flight per lane, and
// the 16 wave partials are added in wave order in LDS - a fixed order for a given W
// (bitwise reproducible).  The two-launch form (W -> W/32 -> 1) paid a second launch and a
// kernel-boundary drain per reduction (~50 per GPT-2 step).
constexpr int kWideU = 12, kWideMaxRows = 4096;
__global__ __launch_bounds__(1024) void colsum_wide_kernel(const float* __restrict__ ws, OutPtrs outs, int W, int D,
                                                          int accumulate, long long ws_z) {
  __shared__ float part[16][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  ws += blockIdx.z * ws_z;
  const int d = blockIdx.x * 64 + lane;
  float acc = 0.f;
  if (d < D) {
    for (int w0 = wv; w0 < W; w0 += 16 * kWideU) {
      float v[kWideU];
#pragma unroll
      for (int u = 0; u < kWideU; ++u) {
        const int w = w0 + 16 * u;
        v[u] = w < W ? ws[(long long)w * D + d] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < kWideU; ++u) acc += v[u];
    }
  }
  part[wv][lane] = acc;
  __syncthreads();
  if (wv == 0 && d < D) {
    float t = part[0][lane];
#pragma unroll
    for (int i = 1; i < 16; ++i) t += part[i][lane];
    float* o = outs.p[blockIdx.z] + d;
    *o = accumulate ? *o + t : t;
  }
}

// Deferred column-sum reductions of one backward window in ONE launch (ops/gemm.py: the bias /
// LayerNorm-parameter gradients of two layers flushed with their grouped weight gradients):
// job j = ws_j [W_j][D_j] partial rows -> out_j [D_j]; block b works on 64 columns of the job
// whose block range holds b.  Per job the body, and so the summation order, is
// colsum_wide_kernel's: the result is bitwise the non-deferred one.
constexpr int kMultiJobs = 32;
struct ColsumJobs {
  const float* ws[kMultiJobs];
  float* out[kMultiJobs];
  int W[kMultiJobs];
  int D[kMultiJobs];
  int start[kMultiJobs + 1];
  int accumulate;  // bit j: out_j += sum
  int n;
};
static_assert(sizeof(ColsumJobs) <= 4096, "kernel argument segment");

__global__ __launch_bounds__(1024) void colsum_multi_kernel(ColsumJobs jobs) {
  __shared__ float part[16][64];
  const int b = blockIdx.x;
  int j = 0;
#pragma unroll
  for (int i = 1; i < kMultiJobs; ++i) j += (i < jobs.n && b >= jobs.start[i]) ? 1 : 0;
  j = __builtin_amdgcn_readfirstlane(j);
  const float* __restrict__ ws = jobs.ws[j];
  const int W = jobs.W[j], D = jobs.D[j];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int d = (b - jobs.start[j]) * 64 + lane;
  float acc = 0.f;
  if (d < D) {
    for (int w0 = wv; w0 < W; w0 += 16 * kWideU) {
      float v[kWideU];
#pragma unroll
      for (int u = 0; u < kWideU; ++u) {
        const int w = w0 + 16 * u;
        v[u] = w < W ? ws[(long long)w * D + d] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < kWideU; ++u) acc += v[u];
    }
  }
  part[wv][lane] = acc;
  __syncthreads();
  if (wv == 0 && d < D) {
    float t = part[0][lane];
#pragma unroll
    for (int i = 1; i < 16; ++i) t += part[i][lane];
    float* o = jobs.out[j] + d;
    *o = ((jobs.accumulate >> j) & 1) ? *o + t : t;
  }
}

static bool colsum_wide_enabled() {
  static int v = -1;  // RTDC_COLSUM_WIDE=0: the two-launch form (A/B)
  if (v < 0) {
    const char* e = getenv("RTDC_COLSUM_WIDE");
    v = (e && e[0] == '0') ? 0 : 1;
  }
  return v == 1;
}

// nz <= 4 independent reductions ws + z*ws_z [W][D] (W partial rows) -> outs.p[z] [D];
// tmp holds nz x S intermediate rows (nz * 64 * D floats).
static void colsum_ws_reduce(const float* ws, int W, int D, float* tmp, OutPtrs outs, int accumulate,
                             hipStream_t st, int nz = 1, long long ws_z = 0) {
  int S = W / 32;
  S = S < 1 ? 1 : (S > 64 ? 64 : S);
  // every W the wide kernel takes goes through it - also a handful of rows: the deferred form
  // (colsum_multi_kernel) sums in its order, so a reduction's bits must not depend on whether
  // its target was a deferrable gradient slot
  if (W <= kWideMaxRows && colsum_wide_enabled()) {
    hipLaunchKernelGGL(colsum_wide_kernel, dim3((D + 63) / 64, 1, nz), dim3(1024), 0, st, ws, outs, W, D, accumulate,
                       ws_z);
  } else if (S > 1 && tmp) {
    const int R = (W + S - 1) / S;
    hipLaunchKernelGGL(colsum_ws_kernel, dim3((D + 63) / 64, S, nz), dim3(256), 0, st, ws, tmp, outs, W, D, R, 0,
                       ws_z, 64LL * D);
    hipLaunchKernelGGL(colsum_ws_kernel, dim3((D + 63) / 64, 1, nz), dim3(256), 0, st, (const float*)tmp,
                       (float*)nullptr, outs, S, D, S, accumulate, 64LL * D, 0LL);
  } else {
    hipLaunchKernelGGL(colsum_ws_kernel, dim3((D + 63) / 64, 1, nz), dim3(256), 0, st, ws, (float*)nullptr, outs, W,
                       D, W, accumulate, ws_z, 0LL);
  }
}
static OutPtrs outs1(float* a, float* b = nullptr, float* c = nullptr) { return OutPtrs{{a, b, c, nullptr}}; }

// Column sums of a [M][N] matrix (bias gradient), stage 1: block (x, y) reduces rows
// [x*R, (x+1)*R) of columns [y*512, y*512+512): lane = 8 columns (16-B loads for bf16), the 4
// waves stride the rows and are combined in LDS -> ws[x][N].  Stage 2 = colsum_ws_reduce.
__device__ __forceinline__ float as_f(bf16_t v) { return bf2f(v); }
__device__ __forceinline__ float as_f(float v) { return v; }
template <typename T>
__device__ __forceinline__ void ld8c(const T* p, float* v);
template <>
__device__ __forceinline__ void ld8c<bf16_t>(const bf16_t* p, float* v) { ld8(p, v); }
template <>
__device__ __forceinline__ void ld8c<float>(const float* p, float* v) {
  const float4 a = *(const float4*)p, b = *(const float4*)(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}
template <typename T, bool VEC>
__global__ __launch_bounds__(256) void colsum_partial_kernel(const T* __restrict__ X, int M, int N, int ld,
                                                            int rows_per_block, float* __restrict__ ws) {
  __shared__ float part[4][512];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int c = blockIdx.y * 512 + lane * 8;
  const int r0 = blockIdx.x * rows_per_block;
  const int r1 = min(M, r0 + rows_per_block);
  float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (c < N) {
    for (int r = r0 + wv; r < r1; r += 4) {
      float v[8];
      if constexpr (VEC) {
        ld8c<T>(X + (long long)r * ld + c, v);
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = c + e < N ? as_f(X[(long long)r * ld + c + e]) : 0.f;
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) a[e] += v[e];
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) part[wv][lane * 8 + e] = a[e];
  __syncthreads();
  for (int j = threadIdx.x; j < 512; j += 256) {
    const int n = blockIdx.y * 512 + j;
    if (n < N) ws[(long long)blockIdx.x * N + n] = (part[0][j] + part[1][j]) + (part[2][j] + part[3][j]);
  }
}

}  // namespace rtdc

using namespace rtdc;

template <bool RMS>
static int launch_norm_fwd(const void* x, const void* g, const void* b, void* y, float* mean,
                           float* rstd, int M, int D, float eps, hipStream_t st) {
  if (D % 8 != 0) return 1;
  const int cpl = (D / 8 + 63) / 64;
  // RTDC_NORM_FWD4=1: 8-B chunks, rows looped per wave (norm_fwd4_kernel) where they fill every
  // lane and 16-B ones would not (GPT-2's D = 768); RTDC_NORM_FWD_BPC: its resident 256-thread
  // blocks per CU (default 4).  Opt-in: measured 12.9-15.0 us against 12.8 us for the one-row-
  // per-wave form at 16384 x 768 (profiles/layernorm_fwd4_ab_r5.txt) - a 50 MB, ~13 us kernel
  // sits at its launch/ramp-bound ~4 TB/s either way.
  static int fwd4 = -1, bpc = 4, cus = 0;
  if (fwd4 < 0) {
    const char* e = getenv("RTDC_NORM_FWD4");
    fwd4 = (e && e[0] == '1') ? 1 : 0;
    const char* c = getenv("RTDC_NORM_FWD_BPC");
    if (c && atoi(c) > 0) bpc = atoi(c);
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      cus = 256;
  }
  const int cpl4 = (D / 4) / 64;
  if (fwd4 && (D / 8) % 64 != 0 && (D / 4) % 64 == 0 && cpl4 >= 1 && cpl4 <= 4) {
    int nb = (M + 3) / 4;
    if (nb > cus * bpc) nb = cus * bpc;
    dim3 grid4(nb), block4(256);
#define L4(C)                                                                                 \
  hipLaunchKernelGGL((norm_fwd4_kernel<C, RMS>), grid4, block4, 0, st, (const bf16_t*)x,       \
                     (const bf16_t*)g, (const bf16_t*)b, (bf16_t*)y, mean, rstd, M, D, eps)
    if (cpl4 == 1) L4(1);
    else if (cpl4 == 2) L4(2);
    else if (cpl4 == 3) L4(3);
    else L4(4);
#undef L4
    return hipGetLastError() == hipSuccess ? 0 : 2;
  }
  // RTDC_NORM_FWD2R=1: two rows per wave where a row's 16-B chunks are 64k + 32 (A/B)
  static int fwd2r = -1;
  if (fwd2r < 0) {
    const char* e = getenv("RTDC_NORM_FWD2R");
    fwd2r = (e && e[0] == '1') ? 1 : 0;
  }
  if (fwd2r && (D / 8) % 64 == 32 && (D / 8) <= 224) {
    const int npl = (2 * (D / 8)) / 64;
    dim3 grid2((M + 7) / 8), block2(256);
#define L2(C)                                                                                 \
  hipLaunchKernelGGL((norm_fwd2r_kernel<C, RMS>), grid2, block2, 0, st, (const bf16_t*)x,      \
                     (const bf16_t*)g, (const bf16_t*)b, (bf16_t*)y, mean, rstd, M, D, eps)
    if (npl == 1) L2(1);
    else if (npl == 3) L2(3);
    else if (npl == 5) L2(5);
    else L2(7);
#undef L2
    return hipGetLastError() == hipSuccess ? 0 : 2;
  }
  dim3 grid((M + 3) / 4), block(256);
#define L(C)                                                                                  \
  hipLaunchKernelGGL((norm_fwd_kernel<C, RMS>), grid, block, 0, st, (const bf16_t*)x,         \
                     (const bf16_t*)g, (const bf16_t*)b, (bf16_t*)y, mean, rstd, M, D, eps)
  if (cpl <= 1) L(1);
  else if (cpl <= 2) L(2);
  else if (cpl <= 4) L(4);
  else if (cpl <= 8) L(8);
  else if (cpl <= 16) L(16);
  else return 1;
#undef L
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

// ws layout: [nz][nblk][D] partials (dgamma | dbeta | colsum(dx)) | nz x [64][D] level-2 rows,
// nz = (RMS ? 1 : 2) + (dxsum != nullptr).  dxsum is always written (never accumulated).
// resident 256-thread blocks of a norm_bwd_kernel variant on this device (cached per variant)
template <int C, bool RMS, bool CS>
static int resident_blocks(size_t lds) {
  static int cus = 0, occ = 0;
  static size_t occ_lds = ~(size_t)0;
  if (cus == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      cus = 256;
  }
  if (lds != occ_lds) {
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, norm_bwd_kernel<C, RMS, CS>, 256, lds) != hipSuccess ||
        occ <= 0)
      occ = 1;
    occ_lds = lds;
  }
  return cus * occ;
}

template <bool RMS, bool CS>
static int resident_blocks4(size_t lds, int cpl4) {
  static int cus = 0;
  static int occ[5] = {0, 0, 0, 0, 0};
  static size_t occ_lds[5] = {~(size_t)0, ~(size_t)0, ~(size_t)0, ~(size_t)0, ~(size_t)0};
  if (cus == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      cus = 256;
  }
  if (cpl4 < 1 || cpl4 > 4) return cus;
  if (lds != occ_lds[cpl4]) {
    hipError_t e = hipErrorInvalidValue;
    int o = 0;
    if (cpl4 == 1) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, norm_bwd4_kernel<1, RMS, CS>, 256, lds);
    if (cpl4 == 2) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, norm_bwd4_kernel<2, RMS, CS>, 256, lds);
    if (cpl4 == 3) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, norm_bwd4_kernel<3, RMS, CS>, 256, lds);
    if (cpl4 == 4) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, norm_bwd4_kernel<4, RMS, CS>, 256, lds);
    occ[cpl4] = (e != hipSuccess || o <= 0) ? 1 : o;
    occ_lds[cpl4] = lds;
  }
  return cus * occ[cpl4];
}

template <bool RMS>
static int launch_norm_bwd(const void* dy, const void* x, const void* g, const float* mean,
                           const float* rstd, const void* dres, void* dx, float* ws, float* dg,
                           float* db, float* dxsum, int M, int D, int nwaves, int accumulate, hipStream_t st,
                           int* nblk_out = nullptr) {
  if (D % 8 != 0 || nwaves % 4 != 0) return 1;
  const int cpl = (D / 8 + 63) / 64;
  const bool cs = dxsum != nullptr;
  const int nz = (RMS ? 1 : 2) + (cs ? 1 : 0);
  const size_t lds = (size_t)nz * D * sizeof(float);
  if (lds > 160 * 1024) return 1;
  static int vw4_env = -1;
  if (vw4_env < 0) {
    const char* e = getenv("RTDC_NORM_BWD_VW4");
    vw4_env = (e && e[0] == '0') ? 0 : 1;
  }
  // 8-B chunks when they fill every lane (D/4 a multiple of 64) and 16-B ones would not
  const bool vw4 = vw4_env && (D / 8) % 64 != 0 && (D / 4) % 64 == 0 && D / 4 <= 64 * 4;
  // one wave of blocks: a grid past the resident block slots leaves a partial second wave
  // (GPT-2: 1024 blocks on 768 slots ran 0.94 ms/step of LayerNorm backward, 768 blocks 0.67)
#define RB(C) (cs ? resident_blocks<C, RMS, true>(lds) : resident_blocks<C, RMS, false>(lds))
  const int cpl4 = (D / 4) / 64;
  const int slots = vw4 ? (cs ? resident_blocks4<RMS, true>(lds, cpl4) : resident_blocks4<RMS, false>(lds, cpl4))
                        : cpl <= 1 ? RB(1) : cpl <= 2 ? RB(2) : cpl <= 4 ? RB(4) : RB(8);
#undef RB
  const int nblk = nwaves / 4 < slots ? nwaves / 4 : slots;
  dim3 grid(nblk), block(256);
  const long long part = (long long)nblk * D;
  float* ws_dg = ws;
  float* ws_db = ws + part;
  float* ws_cs = ws + (RMS ? 1 : 2) * part;
  float* tmp = ws + nz * part;
#define L(C, CS)                                                                              \
  hipLaunchKernelGGL((norm_bwd_kernel<C, RMS, CS>), grid, block, lds, st, (const bf16_t*)dy,   \
                     (const bf16_t*)x, (const bf16_t*)g, mean, rstd, (const bf16_t*)dres,     \
                     (bf16_t*)dx, ws_dg, ws_db, ws_cs, M, D)
#define LC(C) \
  if (cs) L(C, true); else L(C, false)
#define L4(C, CS)                                                                             \
  hipLaunchKernelGGL((norm_bwd4_kernel<C, RMS, CS>), grid, block, lds, st, (const bf16_t*)dy,  \
                     (const bf16_t*)x, (const bf16_t*)g, mean, rstd, (const bf16_t*)dres,     \
                     (bf16_t*)dx, ws_dg, ws_db, ws_cs, M, D)
  if (vw4) {
    if (cpl4 == 1) { if (cs) L4(1, true); else L4(1, false); }
    else if (cpl4 == 2) { if (cs) L4(2, true); else L4(2, false); }
    else if (cpl4 == 3) { if (cs) L4(3, true); else L4(3, false); }
    else { if (cs) L4(4, true); else L4(4, false); }
  } else if (cpl <= 1) { LC(1); }
  else if (cpl <= 2) { LC(2); }
  else if (cpl <= 4) { LC(4); }
  else if (cpl <= 8) { LC(8); }
  else return 1;
#undef LC
#undef L
#undef L4
  if (nblk_out) {  // deferred: the caller reduces the [nz][nblk][D] partials (rtdc_colsum_multi)
    *nblk_out = nblk;
    return hipGetLastError() == hipSuccess ? 0 : 2;
  }
  // one reduction launch pair for all of them; the colsum of dx is never accumulated, so it
  // gets its own pair when dgamma/dbeta accumulate
  if (!cs || !accumulate) {
    OutPtrs o = RMS ? outs1(dg, cs ? dxsum : nullptr) : outs1(dg, db, cs ? dxsum : nullptr);
    colsum_ws_reduce(ws, nblk, D, tmp, o, accumulate, st, nz, part);
  } else {
    colsum_ws_reduce(ws, nblk, D, tmp, RMS ? outs1(dg) : outs1(dg, db), accumulate, st, nz - 1, part);
    colsum_ws_reduce(ws_cs, nblk, D, tmp, outs1(dxsum), 0, st, 1, part);
  }
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

extern "C" int rtdc_layernorm_fwd(const void* x, const void* g, const void* b, void* y, float* mean,
                                  float* rstd, int M, int D, float eps, hipStream_t st) {
  return launch_norm_fwd<false>(x, g, b, y, mean, rstd, M, D, eps, st);
}
extern "C" int rtdc_rmsnorm_fwd(const void* x, const void* g, void* y, float* rstd, int M, int D,
                                float eps, hipStream_t st) {
  return launch_norm_fwd<true>(x, g, nullptr, y, nullptr, rstd, M, D, eps, st);
}
extern "C" int rtdc_layernorm_bwd(const void* dy, const void* x, const void* g, const float* mean,
                                  const float* rstd, const void* dres, void* dx, float* ws,
                                  float* dg, float* db, float* dxsum, int M, int D, int nwaves,
                                  int accumulate, hipStream_t st, int* nblk_out) {
  return launch_norm_bwd<false>(dy, x, g, mean, rstd, dres, dx, ws, dg, db, dxsum, M, D, nwaves,
                                accumulate, st, nblk_out);
}
extern "C" int rtdc_rmsnorm_bwd(const void* dy, const void* x, const void* g, const float* rstd,
                                const void* dres, void* dx, float* ws, float* dg, float* dxsum, int M,
                                int D, int nwaves, int accumulate, hipStream_t st) {
  return launch_norm_bwd<true>(dy, x, g, nullptr, rstd, dres, dx, ws, dg, nullptr, dxsum, M, D, nwaves,
                               accumulate, st);
}
// out[D] (+)= sum of W partial rows ws[W][D] (tmp: 64 * D floats of scratch)
extern "C" int rtdc_colsum_rows(const float* ws, int W, int D, float* tmp, float* out, int accumulate,
                                hipStream_t st) {
  colsum_ws_reduce(ws, W, D, tmp, outs1(out), accumulate, st);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
// n <= 32 deferred reductions (see colsum_multi_kernel); every W_j <= kWideMaxRows
extern "C" int rtdc_colsum_multi(const float* const* ws, float* const* out, const int* W, const int* D,
                                 const int* accumulate, int n, hipStream_t st) {
  if (n < 1 || n > kMultiJobs) return 1;
  ColsumJobs jobs{};
  int blocks = 0;
  for (int i = 0; i < n; ++i) {
    if (W[i] < 1 || W[i] > kWideMaxRows || D[i] < 1) return 1;
    jobs.ws[i] = ws[i];
    jobs.out[i] = out[i];
    jobs.W[i] = W[i];
    jobs.D[i] = D[i];
    jobs.start[i] = blocks;
    if (accumulate[i]) jobs.accumulate |= 1 << i;
    blocks += (D[i] + 63) / 64;
  }
  jobs.start[n] = blocks;
  jobs.n = n;
  hipLaunchKernelGGL(colsum_multi_kernel, dim3((unsigned)blocks), dim3(1024), 0, st, jobs);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

// stage 1 only (the partial rows ws [nblk][N]); the reduction is deferred to rtdc_colsum_multi
extern "C" int rtdc_colsum_partial(const void* X, int M, int N, int ld, float* ws, int nblk, int is_bf16,
                                   hipStream_t st) {
  const bool vec = N % 8 == 0 && ld % 8 == 0;
  const int rpb = (M + nblk - 1) / nblk;
  dim3 grid(nblk, (N + 511) / 512), block(256);
#define CS(T, V) hipLaunchKernelGGL((colsum_partial_kernel<T, V>), grid, block, 0, st, (const T*)X, M, N, ld, rpb, ws)
  if (is_bf16) {
    if (vec) CS(bf16_t, true); else CS(bf16_t, false);
  } else {
    if (vec) CS(float, true); else CS(float, false);
  }
#undef CS
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

extern "C" int rtdc_colsum(const void* X, int M, int N, int ld, float* ws, int nblk, float* out,
                           int accumulate, int is_bf16, hipStream_t st) {
  // ws: [nblk][N] partials followed by [64][N] level-2 rows
  const bool vec = N % 8 == 0 && ld % 8 == 0;
  const int rpb = (M + nblk - 1) / nblk;
  dim3 grid(nblk, (N + 511) / 512), block(256);
#define CS(T, V) hipLaunchKernelGGL((colsum_partial_kernel<T, V>), grid, block, 0, st, (const T*)X, M, N, ld, rpb, ws)
  if (is_bf16) {
    if (vec) CS(bf16_t, true); else CS(bf16_t, false);
  } else {
    if (vec) CS(float, true); else CS(float, false);
  }
#undef CS
  colsum_ws_reduce(ws, nblk, N, ws + (long long)nblk * N, outs1(out), accumulate, st);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

// Convolution support (NHWC, bf16) for gfx950: im2col / col2im around the MFMA GEMM, fused
// BatchNorm(+residual)(+ReLU) forward/backward with deterministic two-stage channel
// reductions, max-pool 3x3/s2 and global average pool.  ResNet-18 (BASELINE config 2).
//
// Channels-last puts the GEMM reduction dimension (kh, kw, c) contiguous, so a convolution is
// Y[B*Ho*Wo, Cout] = cols[B*Ho*Wo, K] . Wmat[Cout, K]^T on the K-major x K-major GEMM, its
// weight gradient the MN x MN GEMM (split-K: K-reduction over B*Ho*Wo) and its input gradient
// dcols = dY . Wmat followed by a col2im GATHER (each input element sums the <= KH*KW columns
// that read it: no atomics, bitwise reproducible).
#include "common.h"

namespace rtdc {

struct ConvGeom {
  int B, H, W, C, Ho, Wo, KH, KW, stride, pad, K, Kp;
};

// All element/chunk counts handled below are < 2^31 (checked by the launchers), so index
// arithmetic is 32-bit: 64-bit integer division is a long software sequence on CDNA.

// cols[(b,ho,wo)][k], k = (kh*KW + kw)*C + c ; zero for k >= K and for padding taps.
__global__ __launch_bounds__(256) void im2col_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ cols,
                                                    ConvGeom g, int vec) {
  const int rows = g.B * g.Ho * g.Wo;
  const int per_row = vec ? g.Kp / 8 : g.Kp;
  const int total = rows * per_row;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < total; i += gridDim.x * 256) {
    const int r = i / per_row;
    const int kk = (i - r * per_row) * (vec ? 8 : 1);
    const int q = r / g.Wo, wo = r - q * g.Wo;
    const int b = q / g.Ho, ho = q - b * g.Ho;
    bf16_t* dst = cols + (size_t)r * g.Kp + kk;
    if (vec) {
      uint4 v = make_uint4(0u, 0u, 0u, 0u);
      if (kk < g.K) {
        const int tap = kk / g.C, c = kk - tap * g.C, kh = tap / g.KW, kw = tap - kh * g.KW;
        const int h = ho * g.stride - g.pad + kh, w = wo * g.stride - g.pad + kw;
        if ((unsigned)h < (unsigned)g.H && (unsigned)w < (unsigned)g.W)
          v = *(const uint4*)(x + ((size_t)(b * g.H + h) * g.W + w) * g.C + c);
      }
      *(uint4*)dst = v;
    } else {
      bf16_t v = 0;
      if (kk < g.K) {
        const int tap = kk / g.C, c = kk - tap * g.C, kh = tap / g.KW, kw = tap - kh * g.KW;
        const int h = ho * g.stride - g.pad + kh, w = wo * g.stride - g.pad + kw;
        if ((unsigned)h < (unsigned)g.H && (unsigned)w < (unsigned)g.W) v = x[((size_t)(b * g.H + h) * g.W + w) * g.C + c];
      }
      *dst = v;
    }
  }
}

// Small-channel stem (C = 3, 7x7): one thread per 8-element (16-B) chunk of a column row;
// the (tap, c) decomposition divides by compile-time constants, stores are full 16 B.
template <int C, int KW>
__global__ __launch_bounds__(256) void im2col_small_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ cols,
                                                          ConvGeom g) {
  const int per_row = g.Kp / 8;
  const int total = g.B * g.Ho * g.Wo * per_row;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < total; i += gridDim.x * 256) {
    const int r = i / per_row;
    const int k0 = (i - r * per_row) * 8;
    const int q = r / g.Wo, wo = r - q * g.Wo;
    const int b = q / g.Ho, ho = q - b * g.Ho;
    const int hb = ho * g.stride - g.pad, wb = wo * g.stride - g.pad;
    const bf16_t* xb = x + (size_t)b * g.H * g.W * C;
    uint32_t u[4];
#pragma unroll
    for (int e2 = 0; e2 < 4; ++e2) {
      uint32_t pair = 0;
#pragma unroll
      for (int h2 = 0; h2 < 2; ++h2) {
        const int k = k0 + 2 * e2 + h2;
        uint32_t v = 0;
        if (k < g.K) {
          const int tap = k / C, c = k - tap * C, kh = tap / KW, kw = tap - kh * KW;
          const int h = hb + kh, w = wb + kw;
          if ((unsigned)h < (unsigned)g.H && (unsigned)w < (unsigned)g.W) v = xb[(h * g.W + w) * C + c];
        }
        pair |= v << (16 * h2);
      }
      u[e2] = pair;
    }
    *(uint4*)(cols + (size_t)r * g.Kp + k0) = make_uint4(u[0], u[1], u[2], u[3]);
  }
}

// Stem im2col (C = 3, 7x7, stride 2) through LDS: one block per output row (b, ho).  The 7
// input rows it needs are staged with aligned 16-B loads into zero-padded LDS rows (16 leading
// + 16 trailing elements cover pad = 3 pixels), then every 16-B column chunk is assembled from
// LDS with 2-B reads: for a tap row kh the 21 (kw, c) values of a pixel are contiguous, at
// kh*ROW + 16 + (2*wo - 3)*3 + (k - 21*kh).  Global traffic: the input once per block (from
// L2) and the column matrix once, all 16-B - the old per-element gathers were load-bound.
template <int W, int Kp>
__global__ __launch_bounds__(256) void im2col_stem_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ cols,
                                                         int H, int Ho, int Wo) {
  constexpr int C = 3, KH = 7, KW = 7, S = 2, PAD = 3, K = KH * KW * C;
  constexpr int ROW = 16 + W * C + 16;  // elements per staged row
  constexpr int NCH = W * C / 8;        // 16-B chunks per input row
  static_assert((W * C) % 8 == 0, "row must be whole 16-B chunks");
  __shared__ __attribute__((aligned(16))) bf16_t rows[KH * ROW];
  const int bo = blockIdx.x;  // b * Ho + ho
  const int b = bo / Ho, ho = bo - b * Ho;
  const int h0 = ho * S - PAD;
  for (int i = threadIdx.x; i < KH * (ROW / 8); i += 256) {
    const int kh = i / (ROW / 8), c8 = i - kh * (ROW / 8);  // 16-B chunk c8 of staged row kh
    const int h = h0 + kh;
    uint4 v = make_uint4(0, 0, 0, 0);
    const int src = c8 - 2;  // the data starts 16 elements (2 chunks) into the row
    if (src >= 0 && src < NCH && (unsigned)h < (unsigned)H)
      v = *(const uint4*)(x + (((size_t)b * H + h) * W) * C + src * 8);
    *(uint4*)(rows + kh * ROW + c8 * 8) = v;
  }
  __syncthreads();
  constexpr int PER = Kp / 8;
  bf16_t* out = cols + (size_t)bo * Wo * Kp;
  for (int i = threadIdx.x; i < Wo * PER; i += 256) {
    const int wo = i / PER, k0 = (i - wo * PER) * 8;
    const int base = 16 + (wo * S - PAD) * C;
    uint32_t u[4];
#pragma unroll
    for (int e2 = 0; e2 < 4; ++e2) {
      uint32_t pair = 0;
#pragma unroll
      for (int h2 = 0; h2 < 2; ++h2) {
        const int k = k0 + 2 * e2 + h2;
        uint32_t v = 0;
        if (k < K) {
          const int kh = k / (KW * C);
          v = rows[kh * ROW + base + (k - kh * KW * C)];
        }
        pair |= v << (16 * h2);
      }
      u[e2] = pair;
    }
    *(uint4*)(out + (size_t)wo * Kp + k0) = make_uint4(u[0], u[1], u[2], u[3]);
  }
}

__device__ __forceinline__ void acc8(float* acc, uint4 v) {
  uint32_t u[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    acc[2 * e] += __uint_as_float(u[e] << 16);
    acc[2 * e + 1] += __uint_as_float(u[e] & 0xffff0000u);
  }
}
__device__ __forceinline__ uint4 pack8(const float* o) {
  return make_uint4(pack_bf2(o[0], o[1]), pack_bf2(o[2], o[3]), pack_bf2(o[4], o[5]), pack_bf2(o[6], o[7]));
}

// dx[b,h,w,c] = sum_{kh,kw} dcols[(b,ho,wo)][(kh,kw,c)] over taps with ho*s - p + kh = h.
// 8 channels per thread (C % 8 == 0).
// addend (nullable, same layout as dx): the input's gradient from another consumer, summed in.
__global__ __launch_bounds__(256) void col2im_kernel(const bf16_t* __restrict__ dcols, bf16_t* __restrict__ dx,
                                                    const bf16_t* __restrict__ addend, ConvGeom g) {
  const int cg = g.C / 8;
  const int total = g.B * g.H * g.W * cg;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < total; i += gridDim.x * 256) {
    const int pix = i / cg, c = (i - pix * cg) * 8;
    const int q = pix / g.W, w = pix - q * g.W;
    const int b = q / g.H, h = q - b * g.H;
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (addend) acc8(acc, *(const uint4*)(addend + (size_t)pix * g.C + c));
    for (int kh = 0; kh < g.KH; ++kh) {
      const int hs = h + g.pad - kh;
      if (hs < 0) break;
      if (hs % g.stride) continue;
      const int ho = hs / g.stride;
      if (ho >= g.Ho) continue;
      for (int kw = 0; kw < g.KW; ++kw) {
        const int ws = w + g.pad - kw;
        if (ws < 0) break;
        if (ws % g.stride) continue;
        const int wo = ws / g.stride;
        if (wo >= g.Wo) continue;
        const int r = (b * g.Ho + ho) * g.Wo + wo;
        acc8(acc, *(const uint4*)(dcols + (size_t)r * g.Kp + (kh * g.KW + kw) * g.C + c));
      }
    }
    *(uint4*)(dx + (size_t)pix * g.C + c) = pack8(acc);
  }
}

// ---- BatchNorm: per-channel statistics over rows of a [N][C] (NHWC-flattened) bf16 tensor.
// Stage 1: block b owns rows [b*R, (b+1)*R).  Thread = (row lane, 8-channel group): 16-B loads,
// a wave covers 64 groups x 16 B of consecutive memory.  Sums are taken about a per-block pivot
// (the block's first row) so sum/sum-of-squares do not cancel; lanes are combined in LDS in a
// fixed order.  Stage 2 merges the block partials in fixed order (Chan) -> mean, rstd, running
// stats.  No atomics anywhere: statistics are bitwise reproducible run to run.
__device__ __forceinline__ void unpack8(const uint4& q, float* v) {
  const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[2 * i] = __uint_as_float(w[i] << 16);
    v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}
__device__ __forceinline__ void ld8f(const bf16_t* p, float* v) {
  uint4 x = *(const uint4*)p;
  uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[2 * i] = __uint_as_float(w[i] << 16);
    v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}

// mode 0 (forward): a = x            -> out0 = pivot + s1/n (block mean), out1 = M2
// mode 1 (backward): a = dy, b = y (relu mask, may be null), c = x -> out0 = sum g, out1 = sum g*xhat
//   with gamma/beta set (ReLU without a residual): the mask is recomputed from x as the forward
//   computed it, t = fma(x, rstd*gamma, beta - mean*rstd*gamma) > 0 - no pass over y
__global__ __launch_bounds__(256) void bn_reduce_kernel(const bf16_t* __restrict__ a, const bf16_t* __restrict__ yb,
                                                       const bf16_t* __restrict__ xb, const float* __restrict__ mean,
                                                       const float* __restrict__ rstd, long long N, int C, int R,
                                                       int mode, float* __restrict__ out0, float* __restrict__ out1,
                                                       const float* __restrict__ gamma = nullptr,
                                                       const float* __restrict__ beta = nullptr) {
  const bool mx = gamma != nullptr;  // relu mask from x
  // channel-major partials: red[k][e][thread] - consecutive threads hit consecutive banks on both
  // the stores and the reduction's reads (a [thread][8] layout made the reads 8-way conflicted:
  // 4.3 conflict cycles per LDS instruction, round-5 ResNet PMC)
  __shared__ float red[2][8][256];
  const long long r0 = (long long)blockIdx.x * R;
  const long long r1 = min(N, r0 + R);
  const int n = (int)max(0LL, r1 - r0);
  const int cg = C / 8;
  for (int gbase = 0; gbase < cg; gbase += 256) {
    const int chunk = min(256, cg - gbase);
    const int rl = 256 / chunk;
    const int t = threadIdx.x;
    const int lane = t / chunk, gi = t % chunk;
    const int c = (gbase + gi) * 8;
    float s1[8] = {0, 0, 0, 0, 0, 0, 0, 0}, s2[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    float piv[8], m8[8], r8[8], ka[8], kb[8];
    if (lane < rl && n > 0) {
      if (mode == 0) {
        ld8f(a + r0 * C + c, piv);
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          m8[e] = mean[c + e];
          r8[e] = rstd[c + e];
          if (mx) {
            ka[e] = rstd[c + e] * gamma[c + e];
            kb[e] = beta[c + e] - mean[c + e] * ka[e];
          }
        }
      }
      // U rows per iteration with every load issued before any use: 3U 16-B loads in flight
      // per thread instead of 3 (the reduction was latency-bound at half the HBM rate)
      constexpr int U = 4;
      long long r = r0 + lane;
      for (; r + (U - 1) * rl < r1; r += U * rl) {
        uint4 va[U], vx[U], vy[U];
#pragma unroll
        for (int u = 0; u < U; ++u) va[u] = *(const uint4*)(a + (r + u * rl) * C + c);
        if (mode != 0) {
#pragma unroll
          for (int u = 0; u < U; ++u) vx[u] = *(const uint4*)(xb + (r + u * rl) * C + c);
          if (yb) {
#pragma unroll
            for (int u = 0; u < U; ++u) vy[u] = *(const uint4*)(yb + (r + u * rl) * C + c);
          }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          float v[8];
          unpack8(va[u], v);
          if (mode == 0) {
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const float d = v[e] - piv[e];
              s1[e] += d;
              s2[e] += d * d;
            }
          } else {
            float xv[8];
            unpack8(vx[u], xv);
            if (yb) {
              float yv[8];
              unpack8(vy[u], yv);
#pragma unroll
              for (int e = 0; e < 8; ++e) v[e] = yv[e] > 0.f ? v[e] : 0.f;
            } else if (mx) {
#pragma unroll
              for (int e = 0; e < 8; ++e) v[e] = fmaf(xv[e], ka[e], kb[e]) > 0.f ? v[e] : 0.f;
            }
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              s1[e] += v[e];
              s2[e] += v[e] * (xv[e] - m8[e]) * r8[e];
            }
          }
        }
      }
      for (; r < r1; r += rl) {
        float v[8];
        ld8f(a + r * C + c, v);
        if (mode == 0) {
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float d = v[e] - piv[e];
            s1[e] += d;
            s2[e] += d * d;
          }
        } else {
          float xv[8];
          ld8f(xb + r * C + c, xv);
          if (yb) {
            float yv[8];
            ld8f(yb + r * C + c, yv);
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = yv[e] > 0.f ? v[e] : 0.f;
          } else if (mx) {
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = fmaf(xv[e], ka[e], kb[e]) > 0.f ? v[e] : 0.f;
          }
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            s1[e] += v[e];
            s2[e] += v[e] * (xv[e] - m8[e]) * r8[e];
          }
        }
      }
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      red[0][e][t] = s1[e];
      red[1][e][t] = s2[e];
    }
    __syncthreads();
    // one thread per output channel (8 x chunk of them, not one thread per 8-channel group):
    // each sums its rl row-lane partials in lane order, the order of the loop it replaces
    for (int o = t; o < 8 * chunk; o += 256) {
      const int e = o / chunk, go = o - e * chunk;
      float A = 0.f, Bq = 0.f;
      for (int l = 0; l < rl; ++l) {
        A += red[0][e][l * chunk + go];
        Bq += red[1][e][l * chunk + go];
      }
      const int ce = (gbase + go) * 8 + e;
      float o0 = A, o1 = Bq;
      if (mode == 0) {
        const float p = n > 0 ? bf2f(a[r0 * C + ce]) : 0.f;
        o0 = n > 0 ? p + A / n : 0.f;
        o1 = n > 0 ? fmaxf(Bq - A * A / n, 0.f) : 0.f;
      }
      out0[(long long)blockIdx.x * C + ce] = o0;
      out1[(long long)blockIdx.x * C + ce] = o1;
    }
    __syncthreads();
  }
}

// one wave per channel: lanes merge block partials b = lane, lane+64, ... (Chan), then a fixed
// xor-shuffle tree merges the 64 lane states.
// Merge the per-tile (mean, M2) partials of one channel (block = channel, 256 threads): with
// the grand mean known the merge is two plain sums - mean = sum(n_b m_b) / n, then
// M2 = sum(M2_b + n_b (m_b - mean)^2) - so the loops carry no division chain (the serial
// Welford merge over ~6k GEMM-tile partials ran 13 us per BatchNorm).  Fixed reduction order.
__device__ __forceinline__ float block_sum256(float v, float* red) {
  v = wave_sum(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  return (red[0] + red[1]) + (red[2] + red[3]);
}

__global__ __launch_bounds__(256) void bn_finalize_kernel(const float* __restrict__ pmean, const float* __restrict__ pm2,
                                                         int nblk, long long N, int R, int C, float eps, float momentum,
                                                         float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                         float* running_mean, float* running_var,
                                                         long long* __restrict__ num_batches_tracked) {
  __shared__ float red[4];
  const int c = blockIdx.x, l = threadIdx.x;
  // BatchNorm2d.num_batches_tracked += 1 (one thread of the grid, no separate ATen add)
  if (num_batches_tracked && c == 0 && l == 0) *num_batches_tracked += 1;
  float snm = 0.f;
  for (int b = l; b < nblk; b += 256) {
    const float nb = (float)max(0LL, min((long long)R, N - (long long)b * R));
    snm += nb * pmean[(long long)b * C + c];
  }
  const float n = (float)N;
  const float mean = block_sum256(snm, red) / n;
  float sm2 = 0.f;
  for (int b = l; b < nblk; b += 256) {
    const float nb = (float)max(0LL, min((long long)R, N - (long long)b * R));
    const float d = pmean[(long long)b * C + c] - mean;
    sm2 += pm2[(long long)b * C + c] + nb * d * d;
  }
  const float m2 = block_sum256(sm2, red);
  if (l == 0) {
    const float var = m2 / n;
    mean_out[c] = mean;
    rstd_out[c] = rsqrtf(var + eps);
    if (running_mean) {
      running_mean[c] = (1.f - momentum) * running_mean[c] + momentum * mean;
      running_var[c] = (1.f - momentum) * running_var[c] + momentum * (n > 1.f ? m2 / (n - 1.f) : var);
    }
  }
}

// Split merge, stage 1: block (x, s) merges the per-row-block (mean, M2) partials of row-blocks
// [s*per, min(nblk, (s+1)*per)) for channels 64x + lane.  Lanes run along the channels, so every
// wave load is 256 coalesced bytes (bn_finalize_kernel alone - a block per channel whose loads
// stride C floats - ran ~10 us per BatchNorm over the ~6k GEMM-tile partials of a 56x56 layer on
// 64..512 blocks).  Same two-sum form as bn_finalize_kernel; the 4 waves' sums are added in wave
// order (fixed).  Stage 2 is bn_finalize_kernel over the splits: split s is a row-block of
// per*R rows.
__global__ __launch_bounds__(256) void bn_merge_split_kernel(const float* __restrict__ pmean,
                                                            const float* __restrict__ pm2, int nblk, long long N,
                                                            int R, int C, int per, float* __restrict__ omean,
                                                            float* __restrict__ om2) {
  __shared__ float red[4][64];
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + l, s = blockIdx.y;
  const int b0 = s * per, b1 = min(nblk, b0 + per);
  const float ns = (float)max(0LL, min((long long)per * R, N - (long long)b0 * R));
  float snm = 0.f;
  if (c < C)
    for (int b = b0 + w; b < b1; b += 4) {
      const float nb = (float)max(0LL, min((long long)R, N - (long long)b * R));
      snm += nb * pmean[(long long)b * C + c];
    }
  red[w][l] = snm;
  __syncthreads();
  const float mean = ns > 0.f ? ((red[0][l] + red[1][l]) + (red[2][l] + red[3][l])) / ns : 0.f;
  __syncthreads();
  float sm2 = 0.f;
  if (c < C)
    for (int b = b0 + w; b < b1; b += 4) {
      const float nb = (float)max(0LL, min((long long)R, N - (long long)b * R));
      const float d = pmean[(long long)b * C + c] - mean;
      sm2 += pm2[(long long)b * C + c] + nb * d * d;
    }
  red[w][l] = sm2;
  __syncthreads();
  if (w == 0 && c < C) {
    omean[(long long)s * C + c] = mean;
    om2[(long long)s * C + c] = (red[0][l] + red[1][l]) + (red[2][l] + red[3][l]);
  }
}

// y = act((x - mean) * rstd * gamma + beta (+ res)); 8 channels per thread (C % 8 == 0).
// The grid stride (gridDim.x * 256 threads) is a multiple of C/8 whenever 256 % (C/8) == 0, so
// each thread keeps ONE group of 8 channels for its whole grid-stride loop: the per-channel
// affine coefficients are computed once per thread (not 32 scalar parameter loads per 16-B
// group), and two rows are processed per iteration so two loads are in flight per stream.
__global__ __launch_bounds__(256) void bn_apply_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ res,
                                                      bf16_t* __restrict__ y, const float* __restrict__ mean,
                                                      const float* __restrict__ rstd, const float* __restrict__ gamma,
                                                      const float* __restrict__ beta, long long N, int C, int relu) {
  const int cg = C / 8;
  const long long total = N * cg;
  const long long i0 = (long long)blockIdx.x * 256 + threadIdx.x, stride = (long long)gridDim.x * 256;
  if (stride % cg == 0) {
    const int c = (int)(i0 % cg) * 8;
    float ka[8], kb[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      ka[e] = rstd[c + e] * gamma[c + e];
      kb[e] = beta[c + e] - mean[c + e] * ka[e];
    }
    for (long long i = i0; i < total; i += 2 * stride) {
      const bool two = i + stride < total;
      const uint4 v0 = *(const uint4*)(x + i * 8);
      uint4 v1 = v0, q0 = v0, q1 = v0;
      if (two) v1 = *(const uint4*)(x + (i + stride) * 8);
      if (res) {
        q0 = *(const uint4*)(res + i * 8);
        if (two) q1 = *(const uint4*)(res + (i + stride) * 8);
      }
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        if (h == 1 && !two) break;
        float xv[8], rr[8], o[8];
        unpack8(h ? v1 : v0, xv);
        if (res) unpack8(h ? q1 : q0, rr);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          float t = fmaf(xv[e], ka[e], kb[e]);
          if (res) t += rr[e];
          if (relu) t = fmaxf(t, 0.f);
          o[e] = t;
        }
        *(uint4*)(y + (i + h * stride) * 8) =
            make_uint4(pack_bf2(o[0], o[1]), pack_bf2(o[2], o[3]), pack_bf2(o[4], o[5]), pack_bf2(o[6], o[7]));
      }
    }
    return;
  }
  for (long long i = i0; i < total; i += stride) {
    const long long row = i / cg;
    const int c = (int)(i - row * cg) * 8;
    const size_t off = (size_t)row * C + c;
    float xv[8], rr[8], o[8];
    unpack8(*(const uint4*)(x + off), xv);
    if (res) unpack8(*(const uint4*)(res + off), rr);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      // the fast path's coefficients exactly (a backward may recompute the ReLU mask from x)
      const float ka = rstd[c + e] * gamma[c + e], kb = beta[c + e] - mean[c + e] * ka;
      float t = fmaf(xv[e], ka, kb);
      if (res) t += rr[e];
      if (relu) t = fmaxf(t, 0.f);
      o[e] = t;
    }
    *(uint4*)(y + off) = make_uint4(pack_bf2(o[0], o[1]), pack_bf2(o[2], o[3]), pack_bf2(o[4], o[5]), pack_bf2(o[6], o[7]));
  }
}

__global__ __launch_bounds__(64) void bn_bwd_finalize_kernel(const float* __restrict__ psum, const float* __restrict__ psumx,
                                                            int nblk, int C, float* __restrict__ dbeta,
                                                            float* __restrict__ dgamma) {
  const int c = blockIdx.x, l = threadIdx.x;
  float s = 0.f, sx = 0.f;
  for (int b = l; b < nblk; b += 64) {
    s += psum[(long long)b * C + c];
    sx += psumx[(long long)b * C + c];
  }
  s = wave_sum(s);
  sx = wave_sum(sx);
  if (l == 0) {
    dbeta[c] = s;
    dgamma[c] = sx;
  }
}

// dx = gamma*rstd/N * (N*g - sum(g) - xhat*sum(g*xhat)); dres = g (when res given). 8 ch/thread.
// dx = gamma*rstd*(g - dbeta/N - xhat*dgamma/N) = A*g + B*x + D per channel (g: dy masked by
// y > 0 when the forward fused a ReLU); dres = g.  Coefficients hoisted per thread as in
// bn_apply_kernel.
template <int RELU>
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ y,
                                                          const bf16_t* __restrict__ x, const float* __restrict__ mean,
                                                          const float* __restrict__ rstd, const float* __restrict__ gamma,
                                                          const float* __restrict__ dbeta, const float* __restrict__ dgamma,
                                                          bf16_t* __restrict__ dx, bf16_t* __restrict__ dres, long long N,
                                                          int C, const float* __restrict__ beta) {
  // RELU: 0 none, 1 mask y > 0 (y read), 2 mask recomputed from x (ReLU without a residual:
  // t = fma(x, rstd*gamma, beta - mean*rstd*gamma) as bn_apply_kernel computed it; y not read).
  // A compile-time mode: with a runtime one hipcc re-loaded the per-channel coefficients inside
  // the loop (3-6x slower).
  const int cg = C / 8;
  const long long total = N * cg;
  const float invN = 1.f / (float)N;
  const long long i0 = (long long)blockIdx.x * 256 + threadIdx.x, stride = (long long)gridDim.x * 256;
  const bool hoist = stride % cg == 0;
  float kA[8], kB[8], kD[8], ka[8], kb[8];
  auto coef = [&](int c) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float r = rstd[c + e], gr = gamma[c + e] * r;
      kA[e] = gr;
      kB[e] = -gr * r * dgamma[c + e] * invN;
      kD[e] = -gr * dbeta[c + e] * invN - kB[e] * mean[c + e];
      if constexpr (RELU == 2) {
        ka[e] = rstd[c + e] * gamma[c + e];
        kb[e] = beta[c + e] - mean[c + e] * ka[e];
      }
    }
  };
  if (hoist) coef((int)(i0 % cg) * 8);
  for (long long i = i0; i < total; i += stride) {
    if (!hoist) coef((int)(i % cg) * 8);
    const size_t off = (size_t)i * 8;
    const uint4 g4 = *(const uint4*)(dy + off), x4 = *(const uint4*)(x + off);
    uint4 y4 = g4;
    if constexpr (RELU == 1) y4 = *(const uint4*)(y + off);
    float gv[8], xv[8], o[8];
    unpack8(g4, gv);
    unpack8(x4, xv);
    if constexpr (RELU == 1) {
      float yv[8];
      unpack8(y4, yv);
#pragma unroll
      for (int e = 0; e < 8; ++e) gv[e] = yv[e] > 0.f ? gv[e] : 0.f;
    } else if constexpr (RELU == 2) {
#pragma unroll
      for (int e = 0; e < 8; ++e) gv[e] = fmaf(xv[e], ka[e], kb[e]) > 0.f ? gv[e] : 0.f;
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = fmaf(kA[e], gv[e], fmaf(kB[e], xv[e], kD[e]));
    *(uint4*)(dx + off) = make_uint4(pack_bf2(o[0], o[1]), pack_bf2(o[2], o[3]), pack_bf2(o[4], o[5]), pack_bf2(o[6], o[7]));
    if (dres)
      *(uint4*)(dres + off) =
          make_uint4(pack_bf2(gv[0], gv[1]), pack_bf2(gv[2], gv[3]), pack_bf2(gv[4], gv[5]), pack_bf2(gv[6], gv[7]));
  }
}

// max pool (KxK, stride s, pad p), NHWC, 8 channels per thread; the argmax tap index (uint8)
// is kept for the backward gather.  Ties keep the first tap in (kh, kw) order (= PyTorch).
__global__ __launch_bounds__(256) void maxpool_fwd_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y,
                                                         uint8_t* __restrict__ arg, int B, int H, int W, int C, int Ho,
                                                         int Wo, int K, int s, int p) {
  const int cg = C / 8;
  const int total = B * Ho * Wo * cg;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < total; i += gridDim.x * 256) {
    const int pix = i / cg, c = (i - pix * cg) * 8;
    const int q = pix / Wo, wo = pix - q * Wo;
    const int b = q / Ho, ho = q - b * Ho;
    float best[8];
    uint32_t bi[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      best[e] = -INFINITY;
      bi[e] = 0;
    }
    for (int kh = 0; kh < K; ++kh) {
      const int h = ho * s - p + kh;
      if ((unsigned)h >= (unsigned)H) continue;
      for (int kw = 0; kw < K; ++kw) {
        const int w = wo * s - p + kw;
        if ((unsigned)w >= (unsigned)W) continue;
        float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        acc8(v, *(const uint4*)(x + ((size_t)(b * H + h) * W + w) * C + c));
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (v[e] > best[e]) {
            best[e] = v[e];
            bi[e] = kh * K + kw;
          }
      }
    }
    const size_t o = (size_t)pix * C + c;
    *(uint4*)(y + o) = pack8(best);
    *(uint2*)(arg + o) = make_uint2(bi[0] | bi[1] << 8 | bi[2] << 16 | bi[3] << 24,
                                    bi[4] | bi[5] << 8 | bi[6] << 16 | bi[7] << 24);
  }
}

// ResNet stem: y = maxpool_KxK/s(relu(BN(x))) with the per-tap argmax, straight from the
// convolution output x - the full-resolution BN output (4x the pooled size) is never stored.
// Each window element is rounded to bf16 exactly as bn_apply_kernel stores it and compared as
// maxpool_fwd_kernel compares it (first strict maximum in (kh, kw) order), so y and arg are
// bitwise those of the unfused pair; the backward recomputes the ReLU mask from x.
// A thread keeps one 8-channel group for the whole grid-stride loop (stride % (C/8) == 0,
// checked by the launcher), so the BN coefficients are computed once per thread.
__global__ __launch_bounds__(256) void bn_relu_maxpool_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y,
                                                             uint8_t* __restrict__ arg, const float* __restrict__ mean,
                                                             const float* __restrict__ rstd,
                                                             const float* __restrict__ gamma,
                                                             const float* __restrict__ beta, int B, int H, int W, int C,
                                                             int Ho, int Wo, int K, int s, int p) {
  const int cg = C / 8;
  const int total = B * Ho * Wo * cg;
  const int i0 = blockIdx.x * 256 + threadIdx.x, stride = gridDim.x * 256;
  const int c = (i0 % cg) * 8;
  float ka[8], kb[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    ka[e] = rstd[c + e] * gamma[c + e];
    kb[e] = beta[c + e] - mean[c + e] * ka[e];
  }
  for (int i = i0; i < total; i += stride) {
    const int pix = i / cg;
    const int q = pix / Wo, wo = pix - q * Wo;
    const int b = q / Ho, ho = q - b * Ho;
    float best[8];
    uint32_t bi[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      best[e] = -INFINITY;
      bi[e] = 0;
    }
    for (int kh = 0; kh < K; ++kh) {
      const int h = ho * s - p + kh;
      if ((unsigned)h >= (unsigned)H) continue;
      for (int kw = 0; kw < K; ++kw) {
        const int w = wo * s - p + kw;
        if ((unsigned)w >= (unsigned)W) continue;
        float v[8];
        unpack8(*(const uint4*)(x + ((size_t)(b * H + h) * W + w) * C + c), v);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float t = bf2f(f2bf(fmaxf(fmaf(v[e], ka[e], kb[e]), 0.f)));
          if (t > best[e]) {
            best[e] = t;
            bi[e] = kh * K + kw;
          }
        }
      }
    }
    const size_t o = (size_t)pix * C + c;
    *(uint4*)(y + o) = pack8(best);
    *(uint2*)(arg + o) = make_uint2(bi[0] | bi[1] << 8 | bi[2] << 16 | bi[3] << 24,
                                    bi[4] | bi[5] << 8 | bi[6] << 16 | bi[7] << 24);
  }
}

__global__ __launch_bounds__(256) void maxpool_bwd_kernel(const bf16_t* __restrict__ dy, const uint8_t* __restrict__ arg,
                                                         bf16_t* __restrict__ dx, int B, int H, int W, int C, int Ho,
                                                         int Wo, int K, int s, int p) {
  const int cg = C / 8;
  const int total = B * H * W * cg;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < total; i += gridDim.x * 256) {
    const int pix = i / cg, c = (i - pix * cg) * 8;
    const int q = pix / W, w = pix - q * W;
    const int b = q / H, h = q - b * H;
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int kh = 0; kh < K; ++kh) {
      const int hs = h + p - kh;
      if (hs < 0) break;
      if (hs % s) continue;
      const int ho = hs / s;
      if (ho >= Ho) continue;
      for (int kw = 0; kw < K; ++kw) {
        const int ws = w + p - kw;
        if (ws < 0) break;
        if (ws % s) continue;
        const int wo = ws / s;
        if (wo >= Wo) continue;
        const size_t o = ((size_t)(b * Ho + ho) * Wo + wo) * C + c;
        const uint2 a8 = *(const uint2*)(arg + o);
        float g[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        acc8(g, *(const uint4*)(dy + o));
        const uint32_t tap = kh * K + kw;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const uint32_t ae = ((e < 4 ? a8.x : a8.y) >> (8 * (e & 3))) & 0xffu;
          if (ae == tap) acc[e] += g[e];
        }
      }
    }
    *(uint4*)(dx + (size_t)pix * C + c) = pack8(acc);
  }
}

// 3x3 / stride 2 / pad 1 (the ResNet stem pool) backward, gather form with the window algebra
// resolved at compile time: input row h is covered by output row h/2 (tap 1) when h is even,
// by rows (h+1)/2 (tap 0) and (h-1)/2 (tap 2) when odd - same for columns - so a thread visits
// its 1, 2 or 4 windows directly instead of testing 9 taps with runtime divisions.
template <int C>
__global__ __launch_bounds__(256) void maxpool3s2_bwd_kernel(const bf16_t* __restrict__ dy,
                                                            const uint8_t* __restrict__ arg, bf16_t* __restrict__ dx,
                                                            int B, int H, int W, int Ho, int Wo) {
  constexpr int CG = C / 8;
  const int total = B * H * W * CG;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < total; i += gridDim.x * 256) {
    const int pix = i / CG, c = (i - pix * CG) * 8;
    const int q = pix / W, w = pix - q * W;
    const int b = q / H, h = q - b * H;
    int hos[2], khs[2], nh = 0, wos[2], kws[2], nw = 0;
    if (h & 1) {
      if ((h + 1) / 2 < Ho) { hos[nh] = (h + 1) / 2; khs[nh++] = 0; }
      hos[nh] = (h - 1) / 2; khs[nh++] = 2;
    } else {
      if (h / 2 < Ho) { hos[nh] = h / 2; khs[nh++] = 1; }
    }
    if (w & 1) {
      if ((w + 1) / 2 < Wo) { wos[nw] = (w + 1) / 2; kws[nw++] = 0; }
      wos[nw] = (w - 1) / 2; kws[nw++] = 2;
    } else {
      if (w / 2 < Wo) { wos[nw] = w / 2; kws[nw++] = 1; }
    }
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int a = 0; a < nh; ++a)
      for (int bb = 0; bb < nw; ++bb) {
        const size_t o = ((size_t)(b * Ho + hos[a]) * Wo + wos[bb]) * C + c;
        const uint2 a8 = *(const uint2*)(arg + o);
        const uint4 g4 = *(const uint4*)(dy + o);
        const uint32_t tap = khs[a] * 3 + kws[bb];
        const uint32_t gw[4] = {g4.x, g4.y, g4.z, g4.w};
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const uint32_t ae = ((e < 4 ? a8.x : a8.y) >> (8 * (e & 3))) & 0xffu;
          const float g = __uint_as_float((e & 1) ? (gw[e >> 1] & 0xffff0000u) : (gw[e >> 1] << 16));
          if (ae == tap) acc[e] += g;
        }
      }
    *(uint4*)(dx + (size_t)pix * C + c) = pack8(acc);
  }
}

// ResNet stem backward, maxpool(relu(BN(x))) with the pool's input gradient never stored:
// pass 1 gathers g = maxpool'(dy) at every BN-output position (rounded to bf16 exactly as
// maxpool3s2_bwd_kernel stores it), masks it by the ReLU recomputed from x and reduces
// (sum g, sum g * xhat) per channel into per-block partial rows (bn_reduce_kernel's mode 1
// format, merged by bn_bwd_finalize_kernel); pass 2 gathers g again and writes
// dx = A g + B x + D (bn_bwd_apply_kernel<2>'s arithmetic).  Against maxpool backward + BN
// reduce + BN apply this drops the full-resolution gradient's write and its two re-reads
// (3 x B*H*W*C bf16).  A thread keeps one 8-channel group (grid stride % (C/8) == 0).
template <int C>
__device__ __forceinline__ void pool3s2_gather(const bf16_t* __restrict__ dy, const uint8_t* __restrict__ arg, int b,
                                               int h, int w, int c, int Ho, int Wo, float* g) {
  // branch-free: input row h is covered by output row a = h >> 1 (tap 1 if h even, tap 2 if odd)
  // and, for odd h, by a + 1 (tap 0) when it exists; same for columns.  All four candidate
  // windows are loaded unconditionally (an absent one re-reads window (a, a') and is masked
  // out), so every load of a thread is independent and issued together.
  const int ah = h >> 1, aw = w >> 1;
  const bool h1 = (h & 1) && ah + 1 < Ho, w1 = (w & 1) && aw + 1 < Wo;
  const uint32_t th0 = (h & 1) ? 2u : 1u, tw0 = (w & 1) ? 2u : 1u;
  const int hh[2] = {ah, h1 ? ah + 1 : ah}, ww[2] = {aw, w1 ? aw + 1 : aw};
  const uint32_t th[2] = {th0, 0u}, tw[2] = {tw0, 0u};
  const bool okh[2] = {true, h1}, okw[2] = {true, w1};
  uint2 a8[4];
  uint4 g4[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const size_t o = ((size_t)(b * Ho + hh[k >> 1]) * Wo + ww[k & 1]) * C + c;
    a8[k] = *(const uint2*)(arg + o);
    g4[k] = *(const uint4*)(dy + o);
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) g[e] = 0.f;
  // summed in maxpool3s2_bwd_kernel's window order (row a+1 before a, column a'+1 before a')
#pragma unroll
  for (int k = 3; k >= 0; --k) {
    const bool ok = okh[k >> 1] && okw[k & 1];
    const uint32_t tap = ok ? th[k >> 1] * 3 + tw[k & 1] : 0xffu;  // 0xff: never an argmax tap
    const uint32_t gw[4] = {g4[k].x, g4[k].y, g4[k].z, g4[k].w};
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const uint32_t ae = ((e < 4 ? a8[k].x : a8[k].y) >> (8 * (e & 3))) & 0xffu;
      const float v = __uint_as_float((e & 1) ? (gw[e >> 1] & 0xffff0000u) : (gw[e >> 1] << 16));
      g[e] += ae == tap ? v : 0.f;
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) g[e] = bf2f(f2bf(g[e]));  // the stored bf16 gradient
}

template <int C>
__global__ __launch_bounds__(256) void pool_bn_bwd_reduce_kernel(const bf16_t* __restrict__ dy,
                                                                const uint8_t* __restrict__ arg,
                                                                const bf16_t* __restrict__ x,
                                                                const float* __restrict__ mean,
                                                                const float* __restrict__ rstd,
                                                                const float* __restrict__ gamma,
                                                                const float* __restrict__ beta, int B, int H, int W,
                                                                int Ho, int Wo, float* __restrict__ out0,
                                                                float* __restrict__ out1) {
  constexpr int CG = C / 8;
  __shared__ float red[2][8][256];  // channel-major (conflict-free, as bn_reduce_kernel)
  const int total = B * H * W * CG;
  const int i0 = blockIdx.x * 256 + threadIdx.x, stride = gridDim.x * 256;
  const int c = (i0 % CG) * 8;
  float ka[8], kb[8], m8[8], r8[8], s1[8], s2[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    m8[e] = mean[c + e];
    r8[e] = rstd[c + e];
    ka[e] = r8[e] * gamma[c + e];
    kb[e] = beta[c + e] - m8[e] * ka[e];
    s1[e] = s2[e] = 0.f;
  }
#pragma unroll 2
  for (int i = i0; i < total; i += stride) {
    const int pix = i / CG;
    const int q = pix / W, w = pix - q * W;
    const int b = q / H, h = q - b * H;
    float g[8], xv[8];
    unpack8(*(const uint4*)(x + (size_t)pix * C + c), xv);
    pool3s2_gather<C>(dy, arg, b, h, w, c, Ho, Wo, g);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float gm = fmaf(xv[e], ka[e], kb[e]) > 0.f ? g[e] : 0.f;
      s1[e] += gm;
      s2[e] += gm * (xv[e] - m8[e]) * r8[e];
    }
  }
  const int t = threadIdx.x;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    red[0][e][t] = s1[e];
    red[1][e][t] = s2[e];
  }
  __syncthreads();
  // one thread per output channel: threads go, go + CG, go + 2 CG, ... of this block share channel
  // group go (summed in that fixed order)
  for (int o = t; o < 8 * CG; o += 256) {
    const int e = o / CG, go = o - e * CG;
    float A = 0.f, Bq = 0.f;
    for (int l = go; l < 256; l += CG) {
      A += red[0][e][l];
      Bq += red[1][e][l];
    }
    out0[(long long)blockIdx.x * C + go * 8 + e] = A;
    out1[(long long)blockIdx.x * C + go * 8 + e] = Bq;
  }
}

template <int C>
__global__ __launch_bounds__(256) void pool_bn_bwd_apply_kernel(const bf16_t* __restrict__ dy,
                                                               const uint8_t* __restrict__ arg,
                                                               const bf16_t* __restrict__ x,
                                                               const float* __restrict__ mean,
                                                               const float* __restrict__ rstd,
                                                               const float* __restrict__ gamma,
                                                               const float* __restrict__ beta,
                                                               const float* __restrict__ dbeta,
                                                               const float* __restrict__ dgamma,
                                                               bf16_t* __restrict__ dx, int B, int H, int W, int Ho,
                                                               int Wo) {
  constexpr int CG = C / 8;
  const int total = B * H * W * CG;
  const float invN = 1.f / ((float)B * H * W);
  const int i0 = blockIdx.x * 256 + threadIdx.x, stride = gridDim.x * 256;
  const int c = (i0 % CG) * 8;
  float kA[8], kB[8], kD[8], ka[8], kb[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const float r = rstd[c + e], gr = gamma[c + e] * r;
    kA[e] = gr;
    kB[e] = -gr * r * dgamma[c + e] * invN;
    kD[e] = -gr * dbeta[c + e] * invN - kB[e] * mean[c + e];
    ka[e] = rstd[c + e] * gamma[c + e];
    kb[e] = beta[c + e] - mean[c + e] * ka[e];
  }
#pragma unroll 2
  for (int i = i0; i < total; i += stride) {
    const int pix = i / CG;
    const int q = pix / W, w = pix - q * W;
    const int b = q / H, h = q - b * H;
    float g[8], xv[8], o[8];
    unpack8(*(const uint4*)(x + (size_t)pix * C + c), xv);
    pool3s2_gather<C>(dy, arg, b, h, w, c, Ho, Wo, g);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float gm = fmaf(xv[e], ka[e], kb[e]) > 0.f ? g[e] : 0.f;
      o[e] = fmaf(kA[e], gm, fmaf(kB[e], xv[e], kD[e]));
    }
    *(uint4*)(dx + (size_t)pix * C + c) = pack8(o);
  }
}

// Network input NCHW fp32 -> NHWC bf16 in one pass (the permute + cast + contiguous of ATen
// are three): a thread takes 8 consecutive pixels of one image - 2 x 16-B loads per channel,
// C x 16-B stores of the interleaved row (HW % 8 == 0).
template <int C>
__global__ __launch_bounds__(256) void nchw_to_nhwc_bf16_kernel(const float* __restrict__ x, bf16_t* __restrict__ y,
                                                               int B, long long HW) {
  const long long per = HW / 8, groups = (long long)B * per;
  for (long long gi = blockIdx.x * 256LL + threadIdx.x; gi < groups; gi += (long long)gridDim.x * 256) {
    const long long b = gi / per, p0 = (gi - b * per) * 8;
    float v[C][8];
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const float4* src = (const float4*)(x + (b * C + c) * HW + p0);
      const float4 a = src[0], d = src[1];
      v[c][0] = a.x; v[c][1] = a.y; v[c][2] = a.z; v[c][3] = a.w;
      v[c][4] = d.x; v[c][5] = d.y; v[c][6] = d.z; v[c][7] = d.w;
    }
    uint32_t o[4 * C];
#pragma unroll
    for (int j = 0; j < 4 * C; ++j) {
      const int e0 = 2 * j, e1 = 2 * j + 1;  // interleaved index p * C + c
      o[j] = pack_bf2(v[e0 % C][e0 / C], v[e1 % C][e1 / C]);
    }
    uint4* dst = (uint4*)(y + (b * HW + p0) * C);
#pragma unroll
    for (int q = 0; q < C; ++q) dst[q] = make_uint4(o[4 * q], o[4 * q + 1], o[4 * q + 2], o[4 * q + 3]);
  }
}

// ---- ResNet stem as a space-to-depth convolution -------------------------------------------
// The 7x7 / stride-2 / pad-3 convolution of a 3-channel image equals a 4x4 / stride-1 / pad-2
// convolution (Ho x Wo = H/2 x W/2) of its 2x2 space-to-depth image
//     X'[b][i][j][q] = X[b][2i+di][2j+dj][c],   q = (2*di + dj)*3 + c  (q < 12; 12..15 zero)
// with  W'[co][a][bb][q] = W[co][2a+di-1][2bb+dj-1][c]  (zero where 2a+di-1 or 2bb+dj-1 is -1):
// output pixel (ho, wo) reads input rows 2(ho-2+a)+di = 2ho-3+kh for kh = 2a+di-1.  K becomes
// 16 taps x 16 channels = 256 = four 64-deep k tiles of 4 taps each - an implicit GEMM on the
// MFMA kernel (ConvStagerK, C = 16) with no column matrix, instead of a 147(->192)-deep im2col
// that was written once and read twice per step.
__global__ __launch_bounds__(256) void nchw_to_s2d_bf16_kernel(const float* __restrict__ x, bf16_t* __restrict__ y,
                                                              int B, int H, int W) {
  const int Ho = H / 2, Wo = W / 2;
  const long long total = (long long)B * Ho * Wo;
  const long long HW = (long long)H * W;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const long long q = i / Wo;
    const int j = (int)(i - q * Wo);
    const long long b = q / Ho;
    const int r = (int)(q - b * Ho);
    float v[16];
#pragma unroll
    for (int di = 0; di < 2; ++di)
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const float2 t = *(const float2*)(x + (b * 3 + c) * HW + (long long)(2 * r + di) * W + 2 * j);
        v[(2 * di + 0) * 3 + c] = t.x;
        v[(2 * di + 1) * 3 + c] = t.y;
      }
#pragma unroll
    for (int e = 12; e < 16; ++e) v[e] = 0.f;
    uint4* dst = (uint4*)(y + i * 16);
    dst[0] = pack8(v);
    dst[1] = pack8(v + 8);
  }
}

// W' [Cout][256] (k = (a*4 + bb)*16 + q) from the channels-last bf16 weight [Cout][7][7][3]
__global__ __launch_bounds__(256) void stem_w_to_s2d_kernel(const bf16_t* __restrict__ w, bf16_t* __restrict__ wp,
                                                           int Cout) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= Cout * 256) return;
  const int co = i >> 8, k = i & 255;
  const int a = k >> 6, bb = (k >> 4) & 3, q = k & 15;
  bf16_t v = 0;
  if (q < 12) {
    const int di = q / 6, dj = (q / 3) & 1, c = q % 3;
    const int kh = 2 * a + di - 1, kw = 2 * bb + dj - 1;
    if (kh >= 0 && kw >= 0) v = w[co * 147 + (kh * 7 + kw) * 3 + c];
  }
  wp[i] = v;
}

// dW [Cout][7][7][3] (fp32, channels-last gradient slot) = the matching entries of dW' [Cout][256]
__global__ __launch_bounds__(256) void stem_dw_from_s2d_kernel(const float* __restrict__ dwp, float* __restrict__ dw,
                                                              int Cout) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= Cout * 147) return;
  const int co = i / 147, r = i - co * 147;
  const int kh = r / 21, kw = (r / 3) % 7, c = r % 3;
  const int a = (kh + 1) >> 1, di = (kh + 1) & 1, bb = (kw + 1) >> 1, dj = (kw + 1) & 1;
  dw[i] = dwp[co * 256 + (a * 4 + bb) * 16 + (2 * di + dj) * 3 + c];
}

// global average pool [B][HW][C] -> [B][C] (fp32 accumulate, bf16 out)
__global__ __launch_bounds__(256) void avgpool_fwd_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y, int B,
                                                         int HW, int C) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= B * C) return;
  const int b = i / C, c = i - b * C;
  float s = 0.f;
  for (int j = 0; j < HW; ++j) s += bf2f(x[((size_t)b * HW + j) * C + c]);
  y[i] = f2bf(s / HW);
}

__global__ __launch_bounds__(256) void avgpool_bwd_kernel(const bf16_t* __restrict__ dy, bf16_t* __restrict__ dx, int B,
                                                         int HW, int C) {
  const int total = B * HW * C;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < total; i += gridDim.x * 256) {
    const int c = i % C;
    const int b = i / (HW * C);
    dx[i] = f2bf(bf2f(dy[b * C + c]) / HW);
  }
}

}  // namespace rtdc

using namespace rtdc;

static inline unsigned gsz(long long work) {
  long long b = (work + 255) / 256;
  if (b > 16384) b = 16384;
  if (b < 1) b = 1;
  return (unsigned)b;
}

extern "C" int rtdc_im2col(const void* x, void* cols, int B, int H, int W, int C, int Ho, int Wo, int KH, int KW,
                           int stride, int pad, int K, int Kp, hipStream_t st) {
  ConvGeom g{B, H, W, C, Ho, Wo, KH, KW, stride, pad, K, Kp};
  const int vec = (C % 8 == 0 && Kp % 8 == 0) ? 1 : 0;
  const long long work = (long long)B * Ho * Wo * (vec ? Kp / 8 : Kp);
  if (work >= (1LL << 31) || (long long)B * H * W * C >= (1LL << 31)) return 1;
  if (C == 3 && KH == 7 && KW == 7 && stride == 2 && pad == 3 && W == 224 && Kp == 192 && Wo == 112) {
    hipLaunchKernelGGL((im2col_stem_kernel<224, 192>), dim3(B * Ho), dim3(256), 0, st, (const bf16_t*)x,
                       (bf16_t*)cols, H, Ho, Wo);
    return hipGetLastError() == hipSuccess ? 0 : 2;
  }
  if (C == 3 && KW == 7 && Kp % 8 == 0) {
    hipLaunchKernelGGL((im2col_small_kernel<3, 7>), dim3(gsz((long long)B * Ho * Wo * (Kp / 8))), dim3(256), 0, st,
                       (const bf16_t*)x, (bf16_t*)cols, g);
    return hipGetLastError() == hipSuccess ? 0 : 2;
  }
  hipLaunchKernelGGL(im2col_kernel, dim3(gsz(work)), dim3(256), 0, st, (const bf16_t*)x, (bf16_t*)cols, g, vec);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

extern "C" int rtdc_col2im(const void* dcols, void* dx, const void* addend, int B, int H, int W, int C, int Ho,
                           int Wo, int KH, int KW, int stride, int pad, int K, int Kp, hipStream_t st) {
  if (C % 8 != 0 || (long long)B * Ho * Wo * Kp >= (1LL << 31) || (long long)B * H * W * C >= (1LL << 31)) return 1;
  ConvGeom g{B, H, W, C, Ho, Wo, KH, KW, stride, pad, K, Kp};
  hipLaunchKernelGGL(col2im_kernel, dim3(gsz((long long)B * H * W * (C / 8))), dim3(256), 0, st,
                     (const bf16_t*)dcols, (bf16_t*)dx, (const bf16_t*)addend, g);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

static bool split_finalize_enabled() {
  static int v = -1;  // RTDC_BN_SPLIT_FINALIZE=0: one block per channel over all partials (A/B)
  if (v < 0) {
    const char* e = getenv("RTDC_BN_SPLIT_FINALIZE");
    v = (e && e[0] == '0') ? 0 : 1;
  }
  return v == 1;
}

// pmean/pm2 (optional): per-row-block statistics already computed by the producer (the
// convolution GEMM epilogue, blocks of pR rows): the statistics pass over x is skipped.
extern "C" int rtdc_bn_fwd(const void* x, const void* res, void* y, float* mean, float* rstd, const float* gamma,
                           const float* beta, float* running_mean, float* running_var, long long N, int C, float eps,
                           float momentum, int training, int relu, float* ws, int nblk, const float* pmean,
                           const float* pm2, int p_nblk, int p_R, long long* nbt, hipStream_t st) {
  if (C % 8 != 0 || N * C >= (1LL << 31)) return 1;
  if (training && pmean) {
    // many producer partials: merged in splits over ~512 coalesced blocks first (ws holds the
    // 2 x S split rows; S <= nblk, the caller's ws capacity), then finalized per channel
    const int cg = (C + 63) / 64;
    int S = std::min(std::min((512 + cg - 1) / cg, (p_nblk + 7) / 8), nblk);
    if (S >= 4 && ws && split_finalize_enabled()) {
      const int per = (p_nblk + S - 1) / S;
      S = (p_nblk + per - 1) / per;
      hipLaunchKernelGGL(bn_merge_split_kernel, dim3(cg, S), dim3(256), 0, st, pmean, pm2, p_nblk, N, p_R, C, per, ws,
                         ws + (long long)S * C);
      hipLaunchKernelGGL(bn_finalize_kernel, dim3(C), dim3(256), 0, st, (const float*)ws,
                         (const float*)(ws + (long long)S * C), S, N, per * p_R, C, eps, momentum, mean, rstd,
                         running_mean, running_var, nbt);
    } else {
      hipLaunchKernelGGL(bn_finalize_kernel, dim3(C), dim3(256), 0, st, pmean, pm2, p_nblk, N, p_R, C, eps, momentum,
                         mean, rstd, running_mean, running_var, nbt);
    }
  } else if (training) {
    const int R = (int)((N + nblk - 1) / nblk);
    hipLaunchKernelGGL(bn_reduce_kernel, dim3(nblk), dim3(256), 0, st, (const bf16_t*)x, (const bf16_t*)nullptr,
                       (const bf16_t*)nullptr, (const float*)nullptr, (const float*)nullptr, N, C, R, 0, ws,
                       ws + (long long)nblk * C);
    hipLaunchKernelGGL(bn_finalize_kernel, dim3(C), dim3(256), 0, st, (const float*)ws,
                       (const float*)(ws + (long long)nblk * C), nblk, N, R, C, eps, momentum, mean, rstd, running_mean,
                       running_var, nbt);
  }
  if (y)  // (y null: statistics only - the consumer applies the normalisation itself)
    hipLaunchKernelGGL(bn_apply_kernel, dim3(gsz(N * (C / 8))), dim3(256), 0, st, (const bf16_t*)x,
                       (const bf16_t*)res, (bf16_t*)y, (const float*)mean, (const float*)rstd, gamma, beta, N, C, relu);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

extern "C" int rtdc_bn_relu_maxpool(const void* x, void* y, void* arg, const float* mean, const float* rstd,
                                    const float* gamma, const float* beta, int B, int H, int W, int C, int Ho, int Wo,
                                    int K, int s, int p, hipStream_t st) {
  const int cg = C / 8;
  if (C % 8 != 0 || 256 % cg != 0 || K * K > 255 || (long long)B * H * W * C >= (1LL << 31)) return 1;
  hipLaunchKernelGGL(bn_relu_maxpool_kernel, dim3(gsz((long long)B * Ho * Wo * cg)), dim3(256), 0, st,
                     (const bf16_t*)x, (bf16_t*)y, (uint8_t*)arg, mean, rstd, gamma, beta, B, H, W, C, Ho, Wo, K, s, p);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

// relu: 0 none, 1 mask from y, 2 mask recomputed from x (needs beta; y unused)
// psum / psumx (optional, p_nblk rows each): the (sum g, sum g*xhat) partials already reduced by
// the producer of dy (conv_gemm_bnb: the dgrad GEMM epilogue) - the statistics pass is skipped
extern "C" int rtdc_bn_bwd(const void* dy, const void* y, const void* x, const float* mean, const float* rstd,
                           const float* gamma, const float* beta, void* dx, void* dres, float* dgamma, float* dbeta,
                           long long N, int C, int relu, float* ws, int nblk, const float* psum, const float* psumx,
                           int p_nblk, hipStream_t st) {
  const int R = (int)((N + nblk - 1) / nblk);
  if (C % 8 != 0 || N * C >= (1LL << 31) || relu < 0 || relu > 2 || (relu == 2 && !beta)) return 1;
  if (psum) {
    hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3(C), dim3(64), 0, st, psum, psumx, p_nblk, C, dbeta, dgamma);
  } else {
    hipLaunchKernelGGL(bn_reduce_kernel, dim3(nblk), dim3(256), 0, st, (const bf16_t*)dy,
                       (const bf16_t*)(relu == 1 ? y : nullptr), (const bf16_t*)x, mean, rstd, N, C, R, 1, ws,
                       ws + (long long)nblk * C, relu == 2 ? gamma : (const float*)nullptr,
                       relu == 2 ? beta : (const float*)nullptr);
    hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3(C), dim3(64), 0, st, (const float*)ws,
                       (const float*)(ws + (long long)nblk * C), nblk, C, dbeta, dgamma);
  }
#define BWA(R)                                                                                          \
  hipLaunchKernelGGL(bn_bwd_apply_kernel<R>, dim3(gsz(N * (C / 8))), dim3(256), 0, st, (const bf16_t*)dy, \
                     (const bf16_t*)y, (const bf16_t*)x, mean, rstd, gamma, (const float*)dbeta,           \
                     (const float*)dgamma, (bf16_t*)dx, (bf16_t*)dres, N, C, beta)
  if (relu == 2) BWA(2);
  else if (relu == 1) BWA(1);
  else BWA(0);
#undef BWA
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

// dgrad operand of a stride-1 convolution: W'[c][kh'][kw'][co] = W[co][KH-1-kh'][KW-1-kw'][c]
// from the forward's bf16 [Cout][KH][KW][Cin] matrix (one launch instead of ATen's flip +
// permute + contiguous copy per conv per step).  Output-linear indexing: coalesced writes.
// out[c][kh][kw][co] = w[co][KH-1-kh][KW-1-kw][c] (stride-1 dgrad operand): for each (kh, kw) a
// [Cout][C] -> [C][Cout] transpose in 64x64 tiles through LDS, coalesced 128-B wave rows on both
// sides and 32-bit index math (the element-wise form with 64-bit div/mod per element ran ~7 us
// per ResNet conv).
__global__ __launch_bounds__(256) void conv_w_flip_t_kernel(const bf16_t* __restrict__ w, bf16_t* __restrict__ out,
                                                           int Cout, int KH, int KW, int C) {
  __shared__ bf16_t tile[64][66];  // +2: the column reads hit distinct banks
  const int c0 = blockIdx.x * 64, co0 = blockIdx.y * 64, khw = blockIdx.z;
  const int kh = khw / KW, kw = khw - kh * KW;
  const int src = (KH - 1 - kh) * KW + (KW - 1 - kw), taps = KH * KW;
  const int l = threadIdx.x & 63, r0 = threadIdx.x >> 6;
#pragma unroll 4
  for (int i = 0; i < 16; ++i) {
    const int r = r0 + 4 * i, co = co0 + r, c = c0 + l;
    if (co < Cout && c < C) tile[r][l] = w[(co * taps + src) * C + c];
  }
  __syncthreads();
#pragma unroll 4
  for (int i = 0; i < 16; ++i) {
    const int r = r0 + 4 * i, c = c0 + r, co = co0 + l;
    if (c < C && co < Cout) out[(c * taps + khw) * Cout + co] = tile[l][r];
  }
}

extern "C" int rtdc_conv_w_flip_t(const void* w, void* out, int Cout, int KH, int KW, int C, hipStream_t st) {
  if (Cout < 1 || C < 1 || KH < 1 || KW < 1 || (long long)Cout * KH * KW * C >= (1LL << 31)) return 1;
  hipLaunchKernelGGL(conv_w_flip_t_kernel, dim3((C + 63) / 64, (Cout + 63) / 64, KH * KW), dim3(256), 0, st,
                     (const bf16_t*)w, (bf16_t*)out, Cout, KH, KW, C);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

extern "C" int rtdc_maxpool(const void* x, void* y, void* arg, const void* dy, void* dx, int B, int H, int W, int C,
                            int Ho, int Wo, int K, int s, int p, int backward, hipStream_t st) {
  if (C % 8 != 0 || K * K > 255 || (long long)B * H * W * C >= (1LL << 31)) return 1;
  if (!backward)
    hipLaunchKernelGGL(maxpool_fwd_kernel, dim3(gsz((long long)B * Ho * Wo * C / 8)), dim3(256), 0, st, (const bf16_t*)x,
                       (bf16_t*)y, (uint8_t*)arg, B, H, W, C, Ho, Wo, K, s, p);
  else if (K == 3 && s == 2 && p == 1 && C == 64 && Ho == (H - 1) / 2 + 1 && Wo == (W - 1) / 2 + 1)
    hipLaunchKernelGGL(maxpool3s2_bwd_kernel<64>, dim3(gsz((long long)B * H * W * C / 8)), dim3(256), 0, st,
                       (const bf16_t*)dy, (const uint8_t*)arg, (bf16_t*)dx, B, H, W, Ho, Wo);
  else
    hipLaunchKernelGGL(maxpool_bwd_kernel, dim3(gsz((long long)B * H * W * C / 8)), dim3(256), 0, st, (const bf16_t*)dy,
                       (const uint8_t*)arg, (bf16_t*)dx, B, H, W, C, Ho, Wo, K, s, p);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

// Stem backward of maxpool3s2(relu(BN(x))) (pool_bn_bwd_*_kernel): dy [B][Ho][Wo][C] + argmax ->
// dx [B][H][W][C], dgamma, dbeta.  ws: 2 * nblk * C floats.  Returns 1 for an unsupported shape.
extern "C" int rtdc_pool_bn_bwd(const void* dy, const void* arg, const void* x, const float* mean, const float* rstd,
                                const float* gamma, const float* beta, void* dx, float* dgamma, float* dbeta, float* ws,
                                int nblk, int B, int H, int W, int C, int Ho, int Wo, hipStream_t st) {
  if (C != 64 || Ho != (H - 1) / 2 + 1 || Wo != (W - 1) / 2 + 1 || (long long)B * H * W * C >= (1LL << 31) ||
      nblk < 1)
    return 1;
  hipLaunchKernelGGL(pool_bn_bwd_reduce_kernel<64>, dim3(nblk), dim3(256), 0, st, (const bf16_t*)dy,
                     (const uint8_t*)arg, (const bf16_t*)x, mean, rstd, gamma, beta, B, H, W, Ho, Wo, ws,
                     ws + (long long)nblk * C);
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3(C), dim3(64), 0, st, (const float*)ws,
                     (const float*)(ws + (long long)nblk * C), nblk, C, dbeta, dgamma);
  hipLaunchKernelGGL(pool_bn_bwd_apply_kernel<64>, dim3(gsz((long long)B * H * W * C / 8)), dim3(256), 0, st,
                     (const bf16_t*)dy, (const uint8_t*)arg, (const bf16_t*)x, mean, rstd, gamma, beta,
                     (const float*)dbeta, (const float*)dgamma, (bf16_t*)dx, B, H, W, Ho, Wo);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

extern "C" int rtdc_avgpool(const void* x, void* y, int B, int HW, int C, int backward, hipStream_t st) {
  if ((long long)B * HW * C >= (1LL << 31)) return 1;
  if (!backward)
    hipLaunchKernelGGL(avgpool_fwd_kernel, dim3((B * C + 255) / 256), dim3(256), 0, st, (const bf16_t*)x, (bf16_t*)y, B,
                       HW, C);
  else
    hipLaunchKernelGGL(avgpool_bwd_kernel, dim3(gsz((long long)B * HW * C)), dim3(256), 0, st, (const bf16_t*)x,
                       (bf16_t*)y, B, HW, C);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

extern "C" int rtdc_nchw_to_nhwc_bf16(const float* x, void* y, int B, int C, long long HW, hipStream_t st) {
  if (HW % 8 != 0 || C != 3) return 1;
  const long long groups = (long long)B * HW / 8;
  hipLaunchKernelGGL(nchw_to_nhwc_bf16_kernel<3>, dim3(gsz(groups)), dim3(256), 0, st, x, (bf16_t*)y, B, HW);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

extern "C" int rtdc_stem_s2d(const float* x, void* y, int B, int H, int W, hipStream_t st) {
  if (H % 2 || W % 2 || W % 4) return 1;
  hipLaunchKernelGGL(nchw_to_s2d_bf16_kernel, dim3(gsz((long long)B * (H / 2) * (W / 2))), dim3(256), 0, st, x,
                     (bf16_t*)y, B, H, W);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
extern "C" int rtdc_stem_w_s2d(const void* w, void* wp, int Cout, hipStream_t st) {
  hipLaunchKernelGGL(stem_w_to_s2d_kernel, dim3((Cout * 256 + 255) / 256), dim3(256), 0, st, (const bf16_t*)w,
                     (bf16_t*)wp, Cout);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
extern "C" int rtdc_stem_dw_s2d(const float* dwp, float* dw, int Cout, hipStream_t st) {
  hipLaunchKernelGGL(stem_dw_from_s2d_kernel, dim3((Cout * 147 + 255) / 256), dim3(256), 0, st, dwp, dw, Cout);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

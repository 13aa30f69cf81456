// 256x256 bf16 GEMM, 8 waves (128x64 outputs per wave), ONE block barrier per 64-deep K-tile
// (tile_cfg 13; gfx950).  The schedule of gemm4b.hip (two steps of MFMAs per K-tile, the
// second k-slice's fragments read during step A, a single vmcnt(0) + lgkmcnt(0) + s_barrier,
// then the next K-tile's first k-slice and the DMA of the K-tile after it during step B) on the
// 8-wave wave layout of gemm8_kernel (gemm_8ph.h): two waves per SIMD, so a wave's LDS latency
// and its partner's MFMAs also overlap, at 1.5x the LDS bytes per MFMA of the 4-wave tile.
// Per wave and k-slice: 8 A + 4 B fragments (12 ds_read_b128) and 8 groups of 4 MFMAs; per
// K-tile: 8 DMA pieces of 1 KiB.  K-major A and B only.
#include "gemm_8ph.h"

namespace rtdc {
namespace g8 {

// 4 MFMAs into four separate accumulators: c_k += b_k (x) a, accumulators pinned to AGPRs
__device__ __forceinline__ void mfma4x_agpr(f32x4& c0, f32x4& c1, f32x4& c2, f32x4& c3, const bf16x8& a,
                                            const bf16x8& b0, const bf16x8& b1, const bf16x8& b2,
                                            const bf16x8& b3) {
  asm volatile(
      "s_nop 1\n\t"
      "v_mfma_f32_16x16x32_bf16 %0, %5, %4, %0\n\t"
      "v_mfma_f32_16x16x32_bf16 %1, %6, %4, %1\n\t"
      "v_mfma_f32_16x16x32_bf16 %2, %7, %4, %2\n\t"
      "v_mfma_f32_16x16x32_bf16 %3, %8, %4, %3\n\t"
      : "+a"(c0), "+a"(c1), "+a"(c2), "+a"(c3)
      : "v"(a), "v"(b0), "v"(b1), "v"(b2), "v"(b3));
}

// MFMA D -> any other reader: 12+ wait states (8-pass XDL); naming the accumulators keeps the
// epilogue's reads below the nops
__device__ __forceinline__ void mfma_drain8(f32x4 (&c)[4][2]) {
  asm volatile("s_nop 15" : "+a"(c[0][0]), "+a"(c[0][1]), "+a"(c[1][0]), "+a"(c[1][1]), "+a"(c[2][0]), "+a"(c[2][1]),
               "+a"(c[3][0]), "+a"(c[3][1]));
}

template <typename OutT>
__global__ __launch_bounds__(512, 1) void gemm8b_kernel(GemmArgs a) {
  constexpr int BN = 256, BH = 128, SA = 64, SB = 32, TMQ = 4, TNQ = 2;
  constexpr int BUF = 4 * HALF;  // [A-lo, A-hi, B-lo, B-hi] of one K-tile
  __shared__ __attribute__((aligned(16))) char smem[2 * BUF];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wa = wave % 2, wb = wave / 2;

  const int tiles_m = (a.M + BM - 1) / BM, tiles_n = (a.N + BN - 1) / BN;
  int tm, tn;
  tile_coords(blockIdx.x, tiles_m, tiles_n, tm, tn);
  const int m0 = tm * BM, n0 = tn * BN;

  int kb = 0, ke = a.K;
  if (a.splitk > 1) {
    const int ktiles = a.K / gemm::BK;
    const int per = (ktiles + a.splitk - 1) / a.splitk;
    kb = blockIdx.y * per * gemm::BK;
    ke = min(a.K, kb + per * gemm::BK);
  }
  const int nt = ke > kb ? (ke - kb) / gemm::BK : 0;

  Stager<true, 128, 8> st[4];  // A-lo, A-hi, B-lo, B-hi (2 pieces per wave each)
  st[0].init(a.A, a.lda, a.M, m0, wave, lane);
  st[1].init(a.A, a.lda, a.M, m0 + 128, wave, lane);
  st[2].init(a.B, a.ldb, a.N, n0, wave, lane);
  st[3].init(a.B, a.ldb, a.N, n0 + BH, wave, lane);
  // DMA piece p (0..7: half p >> 1, piece p & 1) of K-tile j into its stage
  auto dma = [&](int j, int p) {
    const int h = p >> 1;
    st[h].issue_one(kb + j * gemm::BK, smem + (j & 1) * BUF + h * HALF, wave, p & 1);
  };

  f32x4 acc[2][2][TMQ][TNQ];
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y)
#pragma unroll
      for (int i = 0; i < TMQ; ++i)
#pragma unroll
        for (int j = 0; j < TNQ; ++j) acc[x][y][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // fragments of one k-slice: A [half][block i] (rows SA*wa + 16 i), B [half][block j]
  // (columns SB*wb + 16 j)
  bf16x8 fa0[2][TMQ], fb0[2][TNQ], fa1[2][TMQ], fb1[2][TNQ];
  // read r (0..11): r < 8 -> A (half r >> 2, block r & 3), else B (half (r-8) >> 1, block (r-8) & 1)
  auto read = [&](bf16x8 (&fa)[2][TMQ], bf16x8 (&fb)[2][TNQ], const char* stage, int ks, int r) {
    if (r < 8) {
      const int qa = r >> 2, i = r & 3;
      fa[qa][i] = load_frag<true, 128>(stage + qa * HALF, SA * wa + 16 * i, ks, lane);
    } else {
      const int qb = (r - 8) >> 1, j = (r - 8) & 1;
      fb[qb][j] = load_frag<true, 128>(stage + (2 + qb) * HALF, SB * wb + 16 * j, ks, lane);
    }
  };
  // group g (0..7) = (half qa = g >> 2, A block i = g & 3) x every B fragment: 4 MFMAs
  auto mma = [&](int g, bf16x8 (&fa)[2][TMQ], bf16x8 (&fb)[2][TNQ]) {
    const int qa = g >> 2, i = g & 3;
    mfma4x_agpr(acc[qa][0][i][0], acc[qa][0][i][1], acc[qa][1][i][0], acc[qa][1][i][1], fa[qa][i], fb[0][0],
                fb[0][1], fb[1][0], fb[1][1]);
  };

  if (nt > 0) {
#pragma unroll
    for (int p = 0; p < 8; ++p) dma(0, p);
    if (nt > 1) {
#pragma unroll
      for (int p = 0; p < 8; ++p) dma(1, p);
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // tile 0 (this wave's pieces)
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
#pragma unroll
    for (int r = 0; r < 12; ++r) read(fa0, fb0, smem, 0, r);
  }

  auto ktile = [&](int t, auto MORE, auto MORE2) {
    constexpr bool more = decltype(MORE)::value, more2 = decltype(MORE2)::value;
    const char* cur = smem + (t & 1) * BUF;
    const char* nxt = smem + ((t + 1) & 1) * BUF;
    // ---- step A: k-slice 0 MFMAs; k-slice 1 fragments of this tile (2 reads per group, 0-5)
#pragma unroll
    for (int g = 0; g < 8; ++g) {
      mma(g, fa0, fb0);
      __builtin_amdgcn_sched_barrier(0);
      if (g < 6) {
        read(fa1, fb1, cur, 1, 2 * g);
        read(fa1, fb1, cur, 1, 2 * g + 1);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    if constexpr (more) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // tile t+1 landed (my pieces)
    lgkm0();                                                              // my reads of stage t retired
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    // ---- step B: k-slice 1 MFMAs; k-slice 0 fragments of tile t+1; DMA of tile t+2
#pragma unroll
    for (int g = 0; g < 8; ++g) {
      mma(g, fa1, fb1);
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (more) {
        if (g < 6) {
          read(fa0, fb0, nxt, 0, 2 * g);
          read(fa0, fb0, nxt, 0, 2 * g + 1);
        }
      }
      if constexpr (more2) dma(t + 2, g);
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  using T_ = std::true_type;
  using F_ = std::false_type;
  for (int t = 0; t + 2 < nt; ++t) ktile(t, T_{}, T_{});
  if (nt >= 2) ktile(nt - 2, T_{}, F_{});
  if (nt >= 1) ktile(nt - 1, F_{}, F_{});
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y) mfma_drain8(acc[x][y]);

  const float alpha = a.alpha_dev ? a.alpha * *a.alpha_dev : a.alpha;
  if (a.splitk > 1) {
    float* Wp = a.ws + (long long)blockIdx.y * a.M * a.N;
#pragma unroll
    for (int qa = 0; qa < 2; ++qa)
#pragma unroll
      for (int qb = 0; qb < 2; ++qb)
#pragma unroll
        for (int i = 0; i < TMQ; ++i) {
          const int m = m0 + 128 * qa + SA * wa + 16 * i + (lane & 15);
          if (m >= a.M) continue;
#pragma unroll
          for (int j = 0; j < TNQ; ++j) {
            const int n = n0 + BH * qb + SB * wb + 16 * j + 4 * (lane >> 4);
            if (n >= a.N) continue;
            float v[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = acc[qa][qb][i][j][r] * alpha;
            store4<float>(Wp + (long long)m * a.N + n, v);
          }
        }
    return;
  }
  tile_epilogue<OutT, TMQ, TNQ, SA, SB, BH, false>(a, acc, m0, n0, wa, wb, lane, alpha);
}

}  // namespace g8
}  // namespace rtdc

using namespace rtdc;

// K-major A and B only (returns 1 otherwise); a->splitk honoured.
extern "C" int rtdc_gemm8b_launch(const GemmArgs* args, int a_kmajor, int b_kmajor, int out_fp32, hipStream_t st) {
  const GemmArgs& a = *args;
  if (!a_kmajor || !b_kmajor) return 1;
  const unsigned tiles = (unsigned)(((a.M + 255) / 256) * ((a.N + 255) / 256));
  dim3 grid(tiles, a.splitk > 1 ? a.splitk : 1, 1), block(512);
  if (out_fp32) hipLaunchKernelGGL((g8::gemm8b_kernel<float>), grid, block, 0, st, a);
  else hipLaunchKernelGGL((g8::gemm8b_kernel<bf16_t>), grid, block, 0, st, a);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

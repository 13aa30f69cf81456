// 256x256 bf16 GEMM, 4 waves (128x128 outputs per wave, fp32 accumulators in AGPRs), ONE block
// barrier per 64-deep K-tile (tile_cfg 12; gfx950).
//
// Why another 4-wave kernel: the counters of profiles/gemm_pmc_4wave_vs_8wave_r4.txt put both
// existing 256x256 kernels at 28-38 % of wave cycles parked in s_barrier / s_waitcnt (hipBLASLt's
// 256x256x64 kernel: 12 %).  gemm4_kernel (gemm_8ph.h) has 4 barriers per K-tile - one per
// quadrant phase, because each half-tile is restaged as soon as its region is free - and with a
// single wave per SIMD the matrix pipe idles at every one of them.  Here a K-tile is two steps
// of 64 MFMAs (one per 32-deep k-slice), and the only barrier sits between them:
//
//   step A (k-slice 0 of tile t):  MFMAs on F0 = frags(t, ks 0)
//                                  interleaved: ds_reads frags(t, ks 1) -> F1
//   vmcnt(0) (tile t+1's DMA, issued a step earlier) + lgkmcnt(0) (my reads of stage t) + barrier
//   step B (k-slice 1 of tile t):  MFMAs on F1
//                                  interleaved: ds_reads frags(t+1, ks 0) -> F0 (stage t+1: landed
//                                  and visible after the barrier), DMA of tile t+2 -> stage t
//                                  (every wave finished reading stage t before the barrier)
//
// The fragment reads ride on the first 8 of the 16 4-MFMA groups of a step (two ds_read_b128 per
// 64 cycles of matrix work) so they have landed when the step ends; every group of step B also
// carries one 1-KiB global_load_lds piece; the order is pinned with sched_barrier(0) around the asm MFMA groups
// (accumulators "+a": hipcc's own allocation of 256 accumulators beside the fragments shuffles them
// through v_accvgpr moves).  Tile t+2's DMA has ~1.5 steps to land before the wait that needs it.
// All four operand layouts (MN-major operands through the transposing LDS read, retired by an
// explicit lgkmcnt(0) at the end of each step); LDS images, swizzles, stagers and the epilogue are
// those of the 8-wave kernels.  Per-tile launch only: a persistent form (next tile's DMA under the
// epilogue) measured 8-17 % slower at K = 768 (profiles/gemm_4wave_one_barrier_r4.txt).
#include "gemm_8ph.h"

namespace rtdc {
namespace g8 {

template <bool AK, bool BKM, typename OutT>
__global__ __launch_bounds__(256, 1) void gemm4b_kernel(GemmArgs a) {
  // MN-major operands read through the asm transposing read (TrPair): retired by an explicit
  // lgkm0() before the MFMAs that take them (compiler-tracked K-major reads need none)
  constexpr bool TR = !AK || !BKM;
  constexpr int BN = 256, BH = 128, SA = 64, SB = 64, TMQ = 4, TNQ = 4;
  constexpr int BUF = 4 * HALF;  // [A-lo, A-hi, B-lo, B-hi] of one K-tile
  __shared__ __attribute__((aligned(16))) char smem[2 * BUF];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wa = wave & 1, wb = wave >> 1;

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

  Stager<AK, 128, 4> sta[2];   // A-lo, A-hi (4 pieces per wave each)
  Stager<BKM, 128, 4> stb[2];  // B-lo, B-hi
  sta[0].init(a.A, a.lda, a.M, m0, wave, lane);
  sta[1].init(a.A, a.lda, a.M, m0 + 128, wave, lane);
  stb[0].init(a.B, a.ldb, a.N, n0, wave, lane);
  stb[1].init(a.B, a.ldb, a.N, n0 + BH, wave, lane);
  // DMA piece p (0..15: half p >> 2 = A-lo, A-hi, B-lo, B-hi; piece p & 3) of K-tile j into its stage
  auto dma = [&](int j, int p) {
    const int h = p >> 2;
    char* dst = smem + (j & 1) * BUF + h * HALF;
    if (h < 2) sta[h].issue_one(kb + j * gemm::BK, dst, wave, p & 3);
    else stb[h - 2].issue_one(kb + j * gemm::BK, dst, wave, p & 3);
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

  // fragments: [half][block] of one k-slice (A: rows SA*wa + 16 i of half qa; B: columns
  // SB*wb + 16 j of half qb)
  using FA = typename Frag<AK>::T;
  using FB = typename Frag<BKM>::T;
  FA fa0[2][TMQ], fa1[2][TMQ];
  FB fb0[2][TNQ], fb1[2][TNQ];
  // MN-major images: the lane part of a transposing fragment read's LDS offset (k-rows
  // 8g + q (+4), chunk (R0/8 + p/2) ^ swizzle, half chunk p & 1; gemm_common.h load_frag_tr) does
  // not depend on the k-slice (an immediate, 32 k-rows = 8 KiB) - only on the 16-row block, so
  // it is computed once per block here instead of per read (which cost ~200 VALU per K-tile)
  uint32_t toffA[TMQ], toffB[TNQ];
  {
    const int idx = lane & 15, q = idx >> 2, p = idx & 3, g = lane >> 4;
    const int swz = (q | ((g & 1) << 2)) << 1;  // mnmaj_swz<128>(k-row), the same for all reads
#pragma unroll
    for (int i = 0; i < TMQ; ++i)
      toffA[i] = (8 * g + q) * 256 + ((((SA * wa + 16 * i) >> 3) + (p >> 1)) ^ swz) * 16 + (p & 1) * 8;
#pragma unroll
    for (int j = 0; j < TNQ; ++j)
      toffB[j] = (8 * g + q) * 256 + ((((SB * wb + 16 * j) >> 3) + (p >> 1)) ^ swz) * 16 + (p & 1) * 8;
  }
  auto read_tr = [&](const char* half, uint32_t lofs, int ks) {
    const uint32_t addr = lds_addr_of(half) + lofs;
    TrPair f;
    if (ks == 0) {
      f.lo = ds_tr16_imm<0>(addr);
      f.hi = ds_tr16_imm<1024>(addr);
    } else {
      f.lo = ds_tr16_imm<8192>(addr);
      f.hi = ds_tr16_imm<8192 + 1024>(addr);
    }
    return f;
  };
  // fragment read r (0..15) of k-slice ks of the tile in `stage`: r < 8 -> A, else B
  auto read = [&](FA (&fa)[2][TMQ], FB (&fb)[2][TNQ], const char* stage, int ks, int r) {
    if (r < 8) {
      const int qa = r >> 2, i = r & 3;
      if constexpr (AK) fa[qa][i] = load_frag<true, 128>(stage + qa * HALF, SA * wa + 16 * i, ks, lane);
      else fa[qa][i] = read_tr(stage + qa * HALF, toffA[i], ks);
    } else {
      const int qb = (r - 8) >> 2, j = (r - 8) & 3;
      if constexpr (BKM) fb[qb][j] = load_frag<true, 128>(stage + (2 + qb) * HALF, SB * wb + 16 * j, ks, lane);
      else fb[qb][j] = read_tr(stage + (2 + qb) * HALF, toffB[j], ks);
    }
  };
  // 4 MFMAs: acc[qa][qb][i][0..3] += fb[qb][0..3] (x) fa[qa][i]
  auto mma = [&](int qa, int qb, int i, FA (&fa)[2][TMQ], FB (&fb)[2][TNQ]) {
    const bf16x8 av = fval(fa[qa][i]);
    const bf16x8 bv[4] = {fval(fb[qb][0]), fval(fb[qb][1]), fval(fb[qb][2]), fval(fb[qb][3])};
    mfma4_agpr(acc[qa][qb][i], av, bv);
  };

  if (nt > 0) {
#pragma unroll
    for (int p = 0; p < 16; ++p) dma(0, p);
    if (nt > 1) {
#pragma unroll
      for (int p = 0; p < 16; ++p) dma(1, p);
      asm volatile("s_waitcnt vmcnt(16)" ::: "memory");  // tile 0 (this wave's pieces)
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
#pragma unroll
    for (int r = 0; r < 16; ++r) read(fa0, fb0, smem, 0, r);
    if constexpr (TR) lgkm0();
  }

  // one K-tile; MORE / MORE2 (compile-time): tile t+1 / t+2 exist.  The last two K-tiles are
  // peeled so the steady-state body carries no per-group branches.
  auto ktile = [&](int t, auto MORE, auto MORE2) {
    constexpr bool more = decltype(MORE)::value, more2 = decltype(MORE2)::value;
    const char* cur = smem + (t & 1) * BUF;
    const char* nxt = smem + ((t + 1) & 1) * BUF;
    // ---- step A: k-slice 0 MFMAs; k-slice 1 fragments of this tile
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      const int qa = g >> 3, qb = (g >> 2) & 1, i = g & 3;
      mma(qa, qb, i, fa0, fb0);
      __builtin_amdgcn_sched_barrier(0);
      // reads front-loaded (2 per group in the first half of the step): the last one then has
      // 8 groups of MFMA work to land before the lgkmcnt(0) ahead of the barrier
      if (g < 8) {
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
    for (int g = 0; g < 16; ++g) {
      const int qa = g >> 3, qb = (g >> 2) & 1, i = g & 3;
      mma(qa, qb, i, fa1, fb1);
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (more) {
        if (g < 8) {
          read(fa0, fb0, nxt, 0, 2 * g);
          read(fa0, fb0, nxt, 0, 2 * g + 1);
        }
      }
      if constexpr (more2) dma(t + 2, g);
      __builtin_amdgcn_sched_barrier(0);
    }
    if constexpr (TR && more) lgkm0();  // the next K-tile's k-slice 0 (asm reads) retired
  };
  using T_ = std::true_type;
  using F_ = std::false_type;
  for (int t = 0; t + 2 < nt; ++t) ktile(t, T_{}, T_{});
  if (nt >= 2) ktile(nt - 2, T_{}, F_{});
  if (nt >= 1) ktile(nt - 1, F_{}, F_{});
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y) mfma_drain(acc[x][y]);

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

// All four operand layouts; a->splitk honoured.
extern "C" int rtdc_gemm4b_launch(const GemmArgs* args, int a_kmajor, int b_kmajor, int out_fp32, hipStream_t st) {
  const GemmArgs& a = *args;
  const unsigned tiles = (unsigned)(((a.M + 255) / 256) * ((a.N + 255) / 256));
  dim3 grid(tiles, a.splitk > 1 ? a.splitk : 1, 1), block(256);
#define G4B(AK, BKM, T) hipLaunchKernelGGL((g8::gemm4b_kernel<AK, BKM, T>), grid, block, 0, st, a)
  if (out_fp32) {
    if (a_kmajor && b_kmajor) G4B(true, true, float);
    else if (a_kmajor) G4B(true, false, float);
    else if (!b_kmajor) G4B(false, false, float);
    else G4B(false, true, float);
  } else {
    if (a_kmajor && b_kmajor) G4B(true, true, bf16_t);
    else if (a_kmajor) G4B(true, false, bf16_t);
    else if (!b_kmajor) G4B(false, false, bf16_t);
    else G4B(false, true, bf16_t);
  }
#undef G4B
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

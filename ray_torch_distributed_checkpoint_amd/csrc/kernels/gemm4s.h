// Persistent, stream-K 256x256 bf16 GEMM: 4 waves (128x128 outputs per wave, fp32 accumulators in
// AGPRs), one block barrier per 64-deep K-tile, one block per CU for the whole product
// (tile_cfg 14; gfx950).
//
// Why: the one-barrier 4-wave main loop (gemm4b.hip) has hipBLASLt's LDS-read ratio (0.25 LDS
// instructions per MFMA) but pays a prologue (two K-tiles of DMA latency) and an exposed epilogue
// per 256x256 tile - at K = 768 that is 12 K-tiles of work against ~2 K-tiles of bubble - and
// its one-tile-per-block grid quantises badly onto 256 CUs (Llama-3-8B's o / down projections at
// 2048 tokens: 128 tiles, half the chip idle; gate|up: 896 tiles = 3.5 rounds).  Here:
//
// * Persistent: block b works through a list of SEGMENTS (tile, K-range) with ONE continuous
//   K-tile stream - the DMA of K-tile g+2 is issued in step B of K-tile g whatever segment it
//   belongs to, so the next tile's first two K-tiles land under this tile's last MFMAs and under
//   its epilogue; the epilogue's stores drain under the next tile's first K-tile (the wait that
//   needs K-tile g+2 counts past them: vmcnt(32), every bf16 epilogue issues >= 32 stores).
// * Stream-K (hybrid): with T tiles on G blocks and T % G != 0, the first (T / G - 1) rounds are
//   whole tiles (data-parallel), and the remaining T_sk = T - d*G tiles' K-iterations are split
//   EVENLY over the G blocks (P each), so every block does the same number of K-tiles.  A tile
//   split over several blocks is finished by its LAST arriver (no block ever waits for another:
//   deadlock-free at any residency): a block that ends a partial segment first peeks at the
//   tile's arrival counter - if every other contributor already published, it finishes without
//   writing; otherwise it writes its fp32 partial (a lane-linear register image, 256 KiB),
//   releases it (agent-scope fence) and takes a ticket; the ticket's previous value tells whether
//   it came last.  The finisher acquires, sums the contributors' partials in contributor order
//   (fixed: bitwise identical whichever block finishes), runs the fused epilogue and resets the
//   counter for the next launch (cdna_hip_programming.md §5 "Projection GEMM" item 2, §6 G16).
// * XCD-aware: virtual block vb = (b % 8) * (G / 8) + b / 8, so the blocks of one XCD work on a
//   contiguous run of tiles (GROUP_M-ordered: they share A/B panels in that XCD's L2) and a split
//   tile's contributors are neighbours on the same XCD.
//
// The K-tile body is gemm4b's: step A = 64 MFMAs on k-slice 0 with the k-slice 1 fragments read
// under them, one vmcnt + lgkmcnt + barrier, step B = 64 MFMAs on k-slice 1 with the next K-tile's
// k-slice 0 fragments read and the K-tile after it DMA'd (one 1-KiB piece per 4-MFMA group).  The
// body is branch-free: past the end of the block's work the DMA pieces re-read the last K-tile
// into a dead stage, so every wave issues the same counted instruction stream.
#pragma once
#include "gemm_8ph.h"

// Timing-only builds (results are wrong; never shipped): bit 1 drops the main loop's DMA wait,
// bit 2 its block barrier (scripts/build_variant.sh g4sdiag "-DRTDC_G4S_DIAG=1")
#ifndef RTDC_G4S_DIAG
#define RTDC_G4S_DIAG 0
#endif

namespace rtdc {
namespace g8 {

struct SkArgs {
  int G;        // blocks (a multiple of 8)
  int tiles;    // output tiles
  int nt;       // K-tiles per tile
  int d;        // data-parallel tiles per block
  int P;        // stream-K iterations per block
  int I_sk;     // stream-K iterations in all = (tiles - d * G) * nt
  int tiles_m, tiles_n;
  int* cnt;     // [tiles - d * G] arrival counters (zero at launch; each finisher resets its own)
  float* part;  // [2 * G][256 * 256] fp32 partial images
};

// GROUP_M-ordered tile l -> (tm, tn): 8 consecutive row tiles per column sweep
__device__ __forceinline__ void sk_tile_mn(int l, int tiles_m, int tiles_n, int& tm, int& tn) {
  constexpr int GROUP_M = 8;
  const int group = l / (GROUP_M * tiles_n);
  const int first_m = group * GROUP_M;
  const int gsize = min(tiles_m - first_m, GROUP_M);
  const int r = l - group * (GROUP_M * tiles_n);
  tm = first_m + r % gsize;
  tn = r / gsize;
}

struct SkSeg {
  int tile, kb, ke, j;  // j: stream-K tile index (tile - d * G), -1 for a data-parallel tile
};

struct SkPlan {
  int d, nt, G, vb, T_dp, sk_lo, sk_hi, nseg;
  __device__ __forceinline__ SkSeg seg(int s) const {
    SkSeg r;
    if (s < d) {
      r.tile = s * G + vb;
      r.kb = 0;
      r.ke = nt;
      r.j = -1;
      return r;
    }
    const int j0 = sk_lo / nt, j = j0 + (s - d);
    r.tile = T_dp + j;
    r.kb = s == d ? sk_lo - j0 * nt : 0;
    r.ke = min(nt, sk_hi - j * nt);
    r.j = j;
    return r;
  }
};

// One operand's DMA through a buffer descriptor (buffer_load_dwordx4 ... lds): the per-lane part
// of every piece's byte offset is one of two VGPRs (the LDS swizzle alternates with the piece
// index), the tile origin, K-tile and piece row go to the scalar offset.  Switching the stream to
// another tile is scalar arithmetic (no per-lane address rebuild in the loop), and rows / columns
// past the operand's end read as zero (descriptor range) instead of needing clamped addresses:
// they only feed output rows / columns the epilogue never stores.
template <bool KMAJOR>
struct BufOperand {
  __amdgpu_buffer_rsrc_t rs;
  uint32_t vo[2];
  uint32_t pitch;  // bytes per row (K-major) / per k-row (MN-major)
  __device__ __forceinline__ void init(const bf16_t* X, long long bytes, int ld, int lane) {
    rs = make_rsrc(X, 0, bytes);
    pitch = (uint32_t)ld * 2u;
#pragma unroll
    for (int v = 0; v < 2; ++v) {
      if constexpr (KMAJOR) {  // piece p: rows 8p + lane / 8; chunk swizzle by ((row >> 1) & 7)
        const int lchunk = (lane & 7) ^ ((4 * v + (lane >> 4)) & 7);  // v = p & 1
        vo[v] = (uint32_t)(lane >> 3) * pitch + lchunk * 16;
      } else {  // piece p: k-rows 4p + lane / 16; chunk swizzle mnmaj_swz<128>(k-row)
        const int kr = lane >> 4;  // (+ 4p)
        const int swz = ((kr & 3) | (v << 2)) << 1;  // v = (p >> 1) & 1
        vo[v] = (uint32_t)kr * pitch + ((lane & 15) ^ swz) * 16;
      }
    }
  }
  // piece p (0..15) of the 128-row half at row / column r0, K-tile at k0, into lds_half + p KiB
  __device__ __forceinline__ void issue(int r0, int k0, int p, char* lds_half) const {
    uint32_t so;
    int v;
    if constexpr (KMAJOR) {
      so = (uint32_t)(r0 + 8 * p) * pitch + (uint32_t)k0 * 2u;
      v = p & 1;
    } else {
      so = (uint32_t)(k0 + 4 * p) * pitch + (uint32_t)r0 * 2u;
      v = (p >> 1) & 1;
    }
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, LDS_PTR(lds_half + p * 1024), 16, vo[v],
                                             __builtin_amdgcn_readfirstlane(so), 0, 0);
  }
};

// 4 MFMAs that START an accumulation (C = 0): the first K-tile of a segment overwrites the
// previous tile's accumulators, so nothing ever re-zeroes them ("=a": the old values are dead)
__device__ __forceinline__ void mfma4_agpr_z(f32x4 (&c)[4], const bf16x8& a, const bf16x8 (&b)[4]) {
  asm volatile(
      "s_nop 1\n\t"
      "v_mfma_f32_16x16x32_bf16 %0, %5, %4, 0\n\t"
      "v_mfma_f32_16x16x32_bf16 %1, %6, %4, 0\n\t"
      "v_mfma_f32_16x16x32_bf16 %2, %7, %4, 0\n\t"
      "v_mfma_f32_16x16x32_bf16 %3, %8, %4, 0\n\t"
      : "=&a"(c[0]), "=&a"(c[1]), "=&a"(c[2]), "=&a"(c[3])
      : "v"(a), "v"(b[0]), "v"(b[1]), "v"(b[2]), "v"(b[3]));
}

// one accumulator element, read where it stands (AGPR) at this point of the instruction stream:
// the epilogue then holds a few accumulators in VGPRs at a time instead of hipcc copying all 256
// out of the AGPRs at once (which, with the persistent loop's live state, spilled)
__device__ __forceinline__ float agpr_rd(float x) {
  float v;
  asm volatile("v_accvgpr_read_b32 %0, %1" : "=v"(v) : "a"(x));
  return v;
}
__device__ __forceinline__ f32x4 agpr_rd4(const f32x4& x) {
  return f32x4{agpr_rd(x[0]), agpr_rd(x[1]), agpr_rd(x[2]), agpr_rd(x[3])};
}

// tile_epilogue_bf16 (gemm_8ph.h) for the 4-wave 256x256 tile (TMQ = TNQ = 4, SA = SB = 64):
// same per-element arithmetic, column runs, buffer-descriptor bounds and partial column-sum
// rows; accumulators read through agpr_rd (see above) and not re-zeroed.
template <int ACT>
__device__ __forceinline__ void epi4s(const GemmArgs& a, f32x4 (&acc)[2][2][4][4], int m0, int n0, int wa, int wb,
                                      int lane, float alpha) {
  constexpr int TMQ = 4, TNQ = 4, SA = 64, SB = 64, BH = 128;
  constexpr bool ACT_IN = ACT == 3 || ACT == 4 || ACT == 6;
  const long long tile_off = (long long)m0 * a.ldc * 2, rows_bytes = (long long)(a.M - m0) * a.ldc * 2;
  const auto rC = make_rsrc(a.C, tile_off, rows_bytes);
  const bool has_cin = a.Cin && a.beta != 0.f;
  const auto rIn = make_rsrc(ACT_IN ? (const void*)a.aux_in : a.Cin, tile_off, (ACT_IN || has_cin) ? rows_bytes : 0);
  const auto rCin = make_rsrc(a.Cin, tile_off, (ACT_IN && has_cin) ? rows_bytes : 0);
  const auto rAux = make_rsrc(a.aux_out, tile_off, (ACT == 2 || ACT == 5) ? rows_bytes : 0);
  const int bias_elt = a.bias_type == 2 ? 4 : 2;
  const auto rBias = make_rsrc(a.bias, 0, a.bias_type ? (long long)a.N * bias_elt : 0);
  const int g = lane >> 4;
  const int nrun = n0 + SB * wb + 16 * (g & 1) + 8 * (g >> 1);
  auto cno = [&](int c) { return BH * (c >> 1) + 32 * (c & 1); };
  const int rrow = SA * wa + (lane & 15);
  constexpr int NP = 2 * TMQ * TNQ, W = 2;
  const int lbase = rrow * a.ldc + nrun, rows_left = a.M - m0;
  auto poff = [&](int P) -> uint32_t {
    const int ro = 128 * (P / (TMQ * TNQ)) + 16 * ((P / TNQ) % TMQ), no = cno(P % TNQ);
    return (rrow + ro < rows_left && nrun + no < a.N) ? (uint32_t)(lbase + ro * a.ldc + no) * 2u : BUF_OOB;
  };
  float bb[TNQ][8];
#pragma unroll
  for (int c = 0; c < TNQ; ++c) {
    const int n = nrun + cno(c);
    if (a.bias_type == 2) {
      const uint32_t o = n < a.N ? (uint32_t)n * 4u : BUF_OOB;
      const u32x4 x = buf_load16(rBias, o), y = buf_load16(rBias, o + 16u);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        bb[c][r] = __uint_as_float(x[r]);
        bb[c][4 + r] = __uint_as_float(y[r]);
      }
    } else {
      unpack8bf(buf_load16(rBias, n < a.N ? (uint32_t)n * 2u : BUF_OOB), bb[c]);
    }
  }
  constexpr bool CSUM = ACT == 3 || ACT == 6;
  const bool do_cs = CSUM && a.cs_ws != nullptr;
  float cs[CSUM ? TNQ : 1][8];
  if constexpr (CSUM) {
#pragma unroll
    for (int c = 0; c < TNQ; ++c)
#pragma unroll
      for (int r = 0; r < 8; ++r) cs[c][r] = 0.f;
  }
  u32x4 xin[NP];
  const bool load_in = ACT_IN || has_cin;
#pragma unroll
  for (int P = 0; P < W; ++P)
    if (load_in) xin[P] = buf_load16(rIn, poff(P));
#pragma unroll
  for (int P = 0; P < NP; ++P) {
    const int qa = P / (TMQ * TNQ), i = (P / TNQ) % TMQ, c = P % TNQ;
    if (load_in && P + W < NP) xin[P + W] = buf_load16(rIn, poff(P + W));
    const uint32_t off = poff(P);
    const f32x4 x0 = agpr_rd4(acc[qa][c >> 1][i][2 * (c & 1)]);
    const f32x4 x1 = agpr_rd4(acc[qa][c >> 1][i][2 * (c & 1) + 1]);
    float v[8];
    pair_frags(x0, x1, alpha, v);
#pragma unroll
    for (int r = 0; r < 8; ++r) v[r] += bb[c][r];
    float x[8];
    if constexpr (ACT_IN) {
      unpack8bf(xin[P], x);
      if (has_cin) {
        float cc[8];
        unpack8bf(buf_load16(rCin, off), cc);
#pragma unroll
        for (int r = 0; r < 8; ++r) v[r] += a.beta * cc[r];
      }
    } else if (has_cin) {
      unpack8bf(xin[P], x);
#pragma unroll
      for (int r = 0; r < 8; ++r) v[r] += a.beta * x[r];
    }
    if constexpr (ACT == 1) {
#pragma unroll
      for (int r = 0; r < 8; ++r) v[r] = fmaxf(v[r], 0.f);
    } else if constexpr (ACT == 2) {
      buf_store16(rAux, off, pack8bf(v));
#pragma unroll
      for (int r = 0; r < 8; ++r) v[r] = gelu_tanh(v[r]);
    } else if constexpr (ACT == 5) {
      float gg[8];
#pragma unroll
      for (int r = 0; r < 8; ++r) v[r] = gelu_tanh_and_grad(v[r], gg[r]);
      buf_store16(rAux, off, pack8bf(gg));
    } else if constexpr (ACT == 3 || ACT == 6) {
#pragma unroll
      for (int r = 0; r < 8; ++r) v[r] *= ACT == 6 ? x[r] : gelu_tanh_grad(x[r]);
      if (do_cs && off != BUF_OOB) {
#pragma unroll
        for (int r = 0; r < 8; ++r) cs[c][r] += v[r];
      }
    } else if constexpr (ACT == 4) {
#pragma unroll
      for (int r = 0; r < 8; ++r) v[r] = x[r] > 0.f ? v[r] : 0.f;
    }
    buf_store16(rC, off, pack8bf(v));
  }
  if constexpr (CSUM) {
    if (do_cs) {
      float* dst = a.cs_ws + (long long)((m0 / 256) * 2 + wa) * a.N;
#pragma unroll
      for (int c = 0; c < TNQ; ++c) {
#pragma unroll
        for (int r = 0; r < 8; ++r) cs[c][r] = row16_sum(cs[c][r]);
        const int n = nrun + cno(c);
        if ((lane & 15) == 0 && n < a.N) {
          *(f32x4*)(dst + n) = f32x4{cs[c][0], cs[c][1], cs[c][2], cs[c][3]};
          *(f32x4*)(dst + n + 4) = f32x4{cs[c][4], cs[c][5], cs[c][6], cs[c][7]};
        }
      }
    }
  }
}

// ACT: the fused epilogue (0 plain / residual, 2 bias + GELU, 3 GELU' + column sums); SKT: the
// launch splits tiles (stream-K fix-up code compiled in).
template <bool AK, bool BKM, int ACT, bool SKT>
__global__ __launch_bounds__(256, 1) void gemm4s_kernel(GemmArgs a, SkArgs sk) {
  constexpr bool TR = !AK || !BKM;
  constexpr int BH = 128, SA = 64, SB = 64, TMQ = 4, TNQ = 4;
  constexpr int BUF = 4 * HALF;  // [A-lo, A-hi, B-lo, B-hi] of one K-tile
  // 2 stages + the stream-K finisher's broadcast word
  __shared__ __attribute__((aligned(16))) char smem[2 * BUF + 16];
  int* const bword = (int*)(smem + 2 * BUF);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wa = wave & 1, wb = wave >> 1;
  const int b = blockIdx.x;

  SkPlan pl;
  pl.d = sk.d;
  pl.nt = sk.nt;
  pl.G = sk.G;
  pl.vb = (b & 7) * (sk.G >> 3) + (b >> 3);
  pl.T_dp = sk.d * sk.G;
  pl.sk_lo = min(pl.vb * sk.P, sk.I_sk);
  pl.sk_hi = min(pl.sk_lo + sk.P, sk.I_sk);
  const int nsk = pl.sk_hi > pl.sk_lo ? (pl.sk_hi - 1) / sk.nt - pl.sk_lo / sk.nt + 1 : 0;
  pl.nseg = sk.d + nsk;
  const int total = sk.d * sk.nt + (pl.sk_hi - pl.sk_lo);
  if (total == 0) return;

  BufOperand<AK> opA;
  BufOperand<BKM> opB;
  {
    // exact extents (element (r, k) of a K-major operand at r * ld + k; (k, c) of an MN-major one
    // at k * ld + c): the descriptor range ends at the last element
    const long long ea = AK ? (long long)(a.M - 1) * a.lda + a.K : (long long)(a.K - 1) * a.lda + a.M;
    const long long eb = BKM ? (long long)(a.N - 1) * a.ldb + a.K : (long long)(a.K - 1) * a.ldb + a.N;
    opA.init(a.A, ea * 2, a.lda, lane);
    opB.init(a.B, eb * 2, a.ldb, lane);
  }
  int dm0 = 0, dn0 = 0;  // origin of the DMA cursor's tile
  auto stage_seg = [&](const SkSeg& s) {
    int tm, tn;
    sk_tile_mn(s.tile, sk.tiles_m, sk.tiles_n, tm, tn);
    dm0 = tm * BM;
    dn0 = tn * 256;
  };
  // DMA cursor: the K-tile whose pieces are issued next (stagers point at its segment's tile)
  int ds = 0, dk;
  SkSeg dseg = pl.seg(0);
  dk = dseg.kb;
  stage_seg(dseg);
  int dg = 0;  // global index of the DMA cursor's K-tile
  auto dma_advance = [&]() {
    if (dg + 1 >= total) {  // no further K-tile: stay on the last one (re-read into a dead stage)
      ++dg;
      return;
    }
    ++dg;
    if (++dk == dseg.ke) {
      dseg = pl.seg(++ds);
      dk = dseg.kb;
      stage_seg(dseg);
    }
  };
  // piece p (0..15: half p >> 2 = A-lo, A-hi, B-lo, B-hi; piece p & 3) of the cursor's K-tile
  // into stage (dg & 1).  Past the end of the work the cursor stays on the last K-tile and the
  // pieces re-read it into a stage no later read depends on (K-tile g+2 >= total is issued in
  // step B of g into stage g & 1, whose reads were retired before that step's barrier)
  auto dma = [&](int p) {
    const int h = p >> 2, piece = 4 * wave + (p & 3);
    char* dst = smem + (dg & 1) * BUF + h * HALF;
    if (h < 2) opA.issue(dm0 + 128 * h, dk * gemm::BK, piece, dst);
    else opB.issue(dn0 + 128 * (h - 2), dk * gemm::BK, piece, dst);
  };

  f32x4 acc[2][2][TMQ][TNQ];  // (every segment's first K-tile starts them: C = 0)

  using FA = typename Frag<AK>::T;
  using FB = typename Frag<BKM>::T;
  FA fa0[2][TMQ], fa1[2][TMQ];
  FB fb0[2][TNQ], fb1[2][TNQ];
  uint32_t toffA[TMQ], toffB[TNQ];
  {
    const int idx = lane & 15, q = idx >> 2, p = idx & 3, g = lane >> 4;
    const int swz = (q | ((g & 1) << 2)) << 1;  // mnmaj_swz<128>(k-row)
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
  // 4 MFMAs: acc[qa][qb][i][0..3] (+)= fb[qb][0..3] (x) fa[qa][i]; Z: start the accumulation
  auto mma = [&](int qa, int qb, int i, FA (&fa)[2][TMQ], FB (&fb)[2][TNQ], auto Z) {
    const bf16x8 av = fval(fa[qa][i]);
    const bf16x8 bv[4] = {fval(fb[qb][0]), fval(fb[qb][1]), fval(fb[qb][2]), fval(fb[qb][3])};
    if constexpr (decltype(Z)::value) mfma4_agpr_z(acc[qa][qb][i], av, bv);
    else mfma4_agpr(acc[qa][qb][i], av, bv);
  };

  // prologue: K-tiles 0 and 1 in flight, k-slice 0 fragments of K-tile 0 in registers
#pragma unroll
  for (int p = 0; p < 16; ++p) dma(p);
  dma_advance();
#pragma unroll
  for (int p = 0; p < 16; ++p) dma(p);
  dma_advance();
  asm volatile("s_waitcnt vmcnt(16)" ::: "memory");  // K-tile 0 (this wave's pieces)
  __builtin_amdgcn_s_barrier();
#pragma unroll
  for (int r = 0; r < 16; ++r) read(fa0, fb0, smem, 0, r);
  if constexpr (TR) lgkm0();

  const float alpha = a.alpha_dev ? a.alpha * *a.alpha_dev : a.alpha;
  // partial image of (virtual block, stream-K tile j): slot 0 = the block's first stream-K
  // segment, 1 = its last; lane-linear per wave: [wave][fragment f][lane] x 16 B
  auto part_of = [&](int v, int j) -> float* {
    const int first_j = min(v * sk.P, sk.I_sk) / sk.nt;
    const int slot = 2 * v + (j == first_j ? 0 : 1);
    return sk.part + (size_t)slot * (256 * 256) + (size_t)wave * (64 * 64 * 4) + lane * 4;
  };
  // end of a stream-K segment of tile j: true when this block finishes the tile (acc = full sum)
  auto sk_finish = [&](int j) -> bool {
    const int c0 = (j * sk.nt) / sk.P;
    const int c1 = min(((j + 1) * sk.nt - 1) / sk.P, sk.G - 1);
    if (c0 == c1) return true;
    const int nc = c1 - c0 + 1;
    // every wave is past its reads of bword from an earlier tile end before lane 0 rewrites it
    __builtin_amdgcn_s_barrier();
    if (tid == 0) *bword = __hip_atomic_load(&sk.cnt[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    bool last = *bword == nc - 1;  // every other contributor has published: finish unwritten
    if (!last) {
      float* dst = part_of(pl.vb, j);
#pragma unroll
      for (int qa = 0; qa < 2; ++qa)
#pragma unroll
        for (int qb = 0; qb < 2; ++qb)
#pragma unroll
          for (int i = 0; i < TMQ; ++i)
#pragma unroll
            for (int jj = 0; jj < TNQ; ++jj) {
              const int f = ((qa * 2 + qb) * TMQ + i) * TNQ + jj;
              *(f32x4*)(dst + f * 256) = agpr_rd4(acc[qa][qb][i][jj]);
            }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's partial stores complete
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();                     // ... and every other wave's (and bword read)
      if (tid == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        *bword = __hip_atomic_fetch_add(&sk.cnt[j], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      last = *bword == nc - 1;
    }
    if (!last) return false;  // (the next segment's first K-tile overwrites acc)
    // finisher: acquire the others' partials, then sum in contributor order c0..c1 with this
    // block's own partial taken from its registers (the same order whoever finishes)
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      __hip_atomic_store(&sk.cnt[j], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
#pragma unroll
    for (int qa = 0; qa < 2; ++qa)
#pragma unroll
      for (int qb = 0; qb < 2; ++qb)
#pragma unroll
        for (int i = 0; i < TMQ; ++i) {
          f32x4 S[TNQ];
          for (int c = c0; c <= c1; ++c) {
            f32x4 v[TNQ];
            if (c == pl.vb) {
#pragma unroll
              for (int jj = 0; jj < TNQ; ++jj) v[jj] = agpr_rd4(acc[qa][qb][i][jj]);
            } else {
              const float* src = part_of(c, j);
#pragma unroll
              for (int jj = 0; jj < TNQ; ++jj) {
                const int f = ((qa * 2 + qb) * TMQ + i) * TNQ + jj;
                v[jj] = *(const f32x4*)(src + f * 256);
              }
            }
#pragma unroll
            for (int jj = 0; jj < TNQ; ++jj) S[jj] = c == c0 ? v[jj] : S[jj] + v[jj];
          }
#pragma unroll
          for (int jj = 0; jj < TNQ; ++jj) acc[qa][qb][i][jj] = S[jj];
        }
    return true;
  };

  // One K-tile.  FIRST: step A starts the accumulation (C = 0).  LAST: step B reads no
  // fragments (the next K-tile's k-slice 0 is read after the epilogue, so none is live across it).
  bool after_epi = false;
  auto ktile = [&](int g, auto FIRST, auto LAST) {
    constexpr bool last = decltype(LAST)::value;
    const char* cur = smem + (g & 1) * BUF;
    const char* nxt = smem + ((g + 1) & 1) * BUF;
    // ---- step A: k-slice 0 MFMAs; k-slice 1 fragments of this K-tile
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      mma(q >> 3, (q >> 2) & 1, q & 3, fa0, fb0, FIRST);
      __builtin_amdgcn_sched_barrier(0);
      if (q < 8) {
        read(fa1, fb1, cur, 1, 2 * q);
        read(fa1, fb1, cur, 1, 2 * q + 1);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    // K-tile g+1 landed (this wave's pieces; after an epilogue its >= 32 stores may still drain)
#if RTDC_G4S_DIAG & 1
    asm volatile("s_waitcnt vmcnt(63)" ::: "memory");  // timing-only build: results are wrong
#else
    if (after_epi) asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
    lgkm0();
    asm volatile("" ::: "memory");
#if !(RTDC_G4S_DIAG & 2)
    __builtin_amdgcn_s_barrier();
#endif
    after_epi = false;
    // ---- step B: k-slice 1 MFMAs; k-slice 0 fragments of K-tile g+1; DMA of K-tile g+2 into
    // the stage every wave has just left
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      mma(q >> 3, (q >> 2) & 1, q & 3, fa1, fb1, std::false_type{});
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (!last) {
        if (q < 8) {
          read(fa0, fb0, nxt, 0, 2 * q);
          read(fa0, fb0, nxt, 0, 2 * q + 1);
        }
      }
      dma(q);
      __builtin_amdgcn_sched_barrier(0);
    }
    dma_advance();
    if constexpr (TR && !last) lgkm0();
  };
  using T_ = std::true_type;
  using F_ = std::false_type;
  int g = 0;
  for (int s = 0; s < pl.nseg; ++s) {
    const SkSeg cseg = pl.seg(s);
    if (cseg.ke - cseg.kb == 1) {
      ktile(g, T_{}, T_{});
    } else {
      ktile(g++, T_{}, F_{});
      for (int k = cseg.kb + 1; k + 1 < cseg.ke; ++k) ktile(g++, F_{}, F_{});
      ktile(g, F_{}, T_{});
    }
    // ---- end of the segment: epilogue (whole tile) or stream-K hand-off
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int y = 0; y < 2; ++y) mfma_drain(acc[x][y]);
    bool fin = true;
    if constexpr (SKT) {
      if (cseg.j >= 0) fin = sk_finish(cseg.j);
    }
    if (fin) {
      int tm, tn;
      sk_tile_mn(cseg.tile, sk.tiles_m, sk.tiles_n, tm, tn);
      epi4s<ACT>(a, acc, tm * BM, tn * 256, wa, wb, lane, alpha);
      after_epi = true;
    }
    ++g;
    if (g < total) {
      // the next K-tile's k-slice 0 fragments (its stage landed before the last barrier); the
      // memory clobber keeps hipcc from hoisting these LDS reads above the epilogue's global
      // stores, which would keep 64 fragment VGPRs live across it
      asm volatile("" ::: "memory");
      const char* nxt = smem + (g & 1) * BUF;
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int r = 0; r < 16; ++r) read(fa0, fb0, nxt, 0, r);
      if constexpr (TR) lgkm0();
    }
  }
  // no LDS-DMA may still be landing when the workgroup's LDS is handed to the next one
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

}  // namespace g8
}  // namespace rtdc


namespace rtdc {
namespace g8 {
// launch helpers, one translation unit per epilogue (gemm4s_a<ACT>.hip)
template <int ACT>
int gemm4s_launch_act(const GemmArgs& a, const SkArgs& s, int a_kmajor, int b_kmajor, hipStream_t st) {
  if (!a_kmajor) return 1;  // (MN-major A: the weight gradients, fp32 outputs - not this kernel)
  dim3 grid(s.G), block(256);
  const bool sk = s.I_sk > 0;
  if (b_kmajor) {
    if (sk) hipLaunchKernelGGL((gemm4s_kernel<true, true, ACT, true>), grid, block, 0, st, a, s);
    else hipLaunchKernelGGL((gemm4s_kernel<true, true, ACT, false>), grid, block, 0, st, a, s);
  } else {
    if (sk) hipLaunchKernelGGL((gemm4s_kernel<true, false, ACT, true>), grid, block, 0, st, a, s);
    else hipLaunchKernelGGL((gemm4s_kernel<true, false, ACT, false>), grid, block, 0, st, a, s);
  }
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
int gemm4s_launch_a0(const GemmArgs& a, const SkArgs& s, int a_kmajor, int b_kmajor, hipStream_t st);
int gemm4s_launch_a2(const GemmArgs& a, const SkArgs& s, int a_kmajor, int b_kmajor, hipStream_t st);
int gemm4s_launch_a3(const GemmArgs& a, const SkArgs& s, int a_kmajor, int b_kmajor, hipStream_t st);
}  // namespace g8
}  // namespace rtdc

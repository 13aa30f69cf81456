// 256x256 bf16 MFMA GEMM, 8 waves, counted-vmcnt phase pipeline (gfx950).
//
// Same contract, operand layouts (K-major / MN-major), fused epilogues and split-K slabs as
// gemm_bf16.hip, for large outputs.  What is different is the schedule
// (cdna_hip_programming.md §5 "The 256² 8-phase template", T3+T4):
//
// * The 256x64 A and B K-tiles are staged as HALF tiles (128 rows x 64 k, 16 KiB, two
//   global_load_lds_dwordx4 per thread) into 2 LDS buffers (2 x 4 halves = 128 KiB).
// * Wave w owns a 128x64 output made of four 64x32 quadrants, one per (A half, B half)
//   pair: rows 64*(w&1) of each A half, columns 32*(w>>1) of each B half.  A K-tile is
//   4 phases, one quadrant each, in the order (lo,lo) (lo,hi) (hi,lo) (hi,hi) - 16 MFMA
//   16x16x32 per phase.  A-lo is therefore dead after phase 2, B-lo after phase 3 (its
//   fragments stay in registers for phase 3), and each half of the NEXT tiles can be
//   restaged early: one half-tile is issued per phase -
//       p1: B-lo(t+1)   p2: B-hi(t+1)   p3: A-hi(t+1)   p4: A-lo(t+2)
//   so every half-tile load has 4-5 phases (>= one K-tile of MFMA work) to land, with three
//   half-tiles (6 loads) in flight across every barrier: s_waitcnt vmcnt(6), never 0 in
//   the steady state, and raw s_barrier (a __syncthreads() would drain the DMA queue).
// * RAW: a half is read one phase after the wait that retires it; WAR: a half is restaged
//   >= 3 phases after its last ds_read (the reads were retired by lgkmcnt(0) before the
//   barrier in between).  All LDS lives in ONE __shared__ array (a second object makes
//   hipcc drain vmcnt before every ds_read).
#pragma once
#include "gemm_common.h"

namespace rtdc {
namespace g8 {

constexpr int BM = 256, HALF = 16384;

// ---- B half-tiles of 96 rows (256x192 tiles: N = 768 -> 4 column tiles, 64 x 4 = 256 tiles =
// one wave of the chip at M = 16384; a 256x256 tile leaves 64 of 256 CUs idle there).
// A 96-row half is 12 KiB = 12 one-KiB glds pieces; with 8 waves x 2 pieces, pieces 12..15
// are dummies aimed at a junk LDS slot so every wave issues exactly two loads per half-tile
// (the counted vmcnt schedule assumes uniform counts).
// K-major image: plain 128-B rows with the kmaj_off swizzle.  MN-major image: 64 k-rows of
// 192 B (12 chunks); chunk c of k-row kr lives in slot (c + 2*((kr >> 3) & 1)) % 12, which
// makes the ds_read_b64_tr_b16 fragment reads bank-conflict-free (row bases kr*48 mod 64
// banks are {0,48,32,16} for the 4 rows of a lane group; the rotation moves the group 8 rows
// later by 8 banks).
__device__ __forceinline__ int rot96(int kr) { return 2 * ((kr >> 3) & 1); }

template <bool KMAJOR>
struct Half96Stager {
  const bf16_t* src[2];
  int dst[2];  // byte offset inside the half image, or -1 for a dummy piece
  long long kmul;

  __device__ __forceinline__ void init(const bf16_t* X, int ld, int rows, int r0, int wave, int lane) {
#pragma unroll
    for (int ii = 0; ii < 2; ++ii) {
      const int piece = wave * 2 + ii;
      const int pc = piece < 12 ? piece : 0;  // dummies re-read a real piece
      dst[ii] = piece < 12 ? piece * 1024 : -1;
      if constexpr (KMAJOR) {
        const int row = pc * 8 + (lane >> 3);
        const int lchunk = (lane & 7) ^ ((row >> 1) & 7);
        int gr = r0 + row;
        gr = gr < rows ? gr : rows - 1;
        src[ii] = X + (long long)gr * ld + lchunk * 8;
      } else {
        const int G = pc * 64 + lane;  // 16-B slot index in the image
        const int kr = G / 12, slot = G % 12;
        const int c = (slot - rot96(kr) + 12) % 12;
        int gc = r0 + c * 8;
        gc = gc < rows ? gc : rows - 8;
        src[ii] = X + (long long)kr * ld + gc;
      }
    }
    kmul = KMAJOR ? 1 : ld;
  }

  __device__ __forceinline__ void issue(int k0, char* lds_half, char* junk) const {
    const long long koff = (long long)k0 * kmul;
#pragma unroll
    for (int ii = 0; ii < 2; ++ii) {
      char* d = dst[ii] >= 0 ? lds_half + dst[ii] : junk;
      __builtin_amdgcn_global_load_lds((const void*)(src[ii] + koff), LDS_PTR(d), 16, 0, 0);
    }
  }
};

// fragment of a 96-row half: rows (= n) R0..R0+15, k-slice ks (same lane contract as
// load_fragx: MN-major through the asm transposing read)
template <bool KMAJOR>
__device__ __forceinline__ typename Frag<KMAJOR>::T load_frag96(const char* tile, int R0, int ks, int lane) {
  if constexpr (KMAJOR) {
    return load_frag<true, 96>(tile, R0, ks, lane);
  } else {
    const int idx = lane & 15, q = idx >> 2, p = idx & 3, g = lane >> 4;
    const int c = (R0 >> 3) + (p >> 1);
    const int kr0 = ks * 32 + 8 * g + q, kr1 = kr0 + 4;
    TrPair f;
    f.lo = ds_tr16(tile + kr0 * 192 + (((c + rot96(kr0)) % 12) << 4) + ((p & 1) << 3));
    f.hi = ds_tr16(tile + kr1 * 192 + (((c + rot96(kr1)) % 12) << 4) + ((p & 1) << 3));
    return f;
  }
}

// ---- tile epilogue: lane holds C[m][n..n+3] of every (quadrant, i, j) fragment.
// bf16 outputs (the launcher guarantees 16-B-aligned operands): two fragments of the same rows
// are regrouped by pair_frags so that each lane owns 8 consecutive columns and every global
// access is 16 B - half the memory instructions of the 4-wide form (c_fc forward stores the
// GELU output AND the pre-activation).  With an even TNQ the pair is (j, j+1) of one column
// half, so one store instruction writes 32 consecutive columns (64 B) of each of its 16 rows;
// otherwise (256x192 tiles) it is the same j of the two halves.  All epilogue traffic goes
// through buffer descriptors whose range check replaces the per-lane bounds branches (with
// branches hipcc's wait insertion falls back to vmcnt(0) at every join).  The residual /
// activation input of a fragment pair is loaded W pairs ahead of its use: a load issued right
// behind stores waits for them too (vmcnt counts both), which would serialise the store
// stream behind each load.  One specialisation per
// activation keeps the per-element code branch-free.
// residual / activation-input pairs loaded ahead of their use in the bf16 epilogue (A/B builds:
// -DRTDC_EPI_W=N)
#ifndef RTDC_EPI_W
#define RTDC_EPI_W 2
#endif

// s_waitcnt vmcnt(0) lgkmcnt(0) as the builtin, which the compiler's wait insertion reads (asm
// waits it cannot).  hipcc treats a global_load_lds (a FLAT instruction, counted in vmcnt AND
// lgkmcnt) as pending until a wait it sees clears both counters, and while one is pending every
// wait it inserts is vmcnt(0): each activation-input read of the epilogue waited for all the
// stores issued before it (small-kernel check: after a glds, the builtin vmcnt(0) alone keeps
// later waits at 0; vmcnt(0) lgkmcnt(0) makes them counted; profiles/r6/gemm_epilogue_counted_waits_ab_r6.txt).
__device__ __forceinline__ void vm_drained() { __builtin_amdgcn_s_waitcnt(0x0070); }

template <int ACT, int TMQ, int TNQ, int SA, int SB, int BH, bool ZERO>
__device__ __forceinline__ void tile_epilogue_bf16(const GemmArgs& a, f32x4 (&acc)[2][2][TMQ][TNQ], int m0, int n0,
                                                   int wa, int wb, int lane, float alpha) {
  constexpr bool ACT_IN = ACT == 3 || ACT == 4 || ACT == 6;
  // descriptors over this tile's rows m0.. (tile-relative 32-bit offsets: the launcher keeps
  // 256 rows x ldc x 2 B under 2 GiB)
  const long long tile_off = (long long)m0 * a.ldc * 2, rows_bytes = (long long)(a.M - m0) * a.ldc * 2;
  const auto rC = make_rsrc(a.C, tile_off, rows_bytes);
  // (an input-gradient activation takes no residual here: the launcher routes that combination
  // to the general kernel, so the ACT_IN epilogue has no conditional load)
  const bool has_cin = !ACT_IN && a.Cin && a.beta != 0.f;
  const auto rIn = make_rsrc(ACT_IN ? (const void*)a.aux_in : a.Cin, tile_off, (ACT_IN || has_cin) ? rows_bytes : 0);
  const auto rAux = make_rsrc(a.aux_out, tile_off, (ACT == 2 || ACT == 5) ? rows_bytes : 0);
  const int bias_elt = a.bias_type == 2 ? 4 : 2;
  const auto rBias = make_rsrc(a.bias, 0, a.bias_type ? (long long)a.N * bias_elt : 0);

  // column runs c < TNQ: pair (qb, 2jp), (qb, 2jp + 1) for c = qb * TNQ/2 + jp (PJ), or
  // (0, c), (1, c) (PQ); the lane's 8 columns are nrun + cno(c)
  constexpr bool PJ = TNQ % 2 == 0;
  const int g = lane >> 4;
  const int nrun = n0 + SB * wb + (PJ ? 16 * (g & 1) : BH * (g & 1)) + 8 * (g >> 1);
  auto cno = [&](int c) { return PJ ? BH * (c / (TNQ / 2)) + 32 * (c % (TNQ / 2)) : 16 * c; };
  const int rrow = SA * wa + (lane & 15);  // + 128 qa + 16 i (tile-relative)
  // fragment pairs in order P = (qa * TMQ + i) * TNQ + c: consecutive stores complete a row's
  // run of SB columns (a column-run-outer order left each 128-B line half written for half
  // the epilogue; with outputs that miss the caches, c_fc forward took 159 instead of 124 us)
  constexpr int NP = 2 * TMQ * TNQ, W = RTDC_EPI_W < NP ? RTDC_EPI_W : NP;
  // (the lane part of the offset is one register; the per-pair parts are wave-uniform, so
  // nothing per pair is loop-invariant across the persistent kernel's tiles)
  const int lbase = rrow * a.ldc + nrun, rows_left = a.M - m0;
  auto poff = [&](int P) -> uint32_t {
    const int ro = 128 * (P / (TMQ * TNQ)) + 16 * ((P / TNQ) % TMQ), no = cno(P % TNQ);
    return (rrow + ro < rows_left && nrun + no < a.N) ? (uint32_t)(lbase + ro * a.ldc + no) * 2u : BUF_OOB;
  };
  float bb[TNQ][8];  // bias of each column run
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
    } else {  // bf16 bias, or none (zero records: loads return 0)
      unpack8bf(buf_load16(rBias, n < a.N ? (uint32_t)n * 2u : BUF_OOB), bb[c]);
    }
  }
  // column sums of the gelu-backward output (the c_fc bias gradient): per lane over its pairs,
  // then over the 16 lanes of a row group, one partial row per (row tile, wave row) in cs_ws
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
    float v[8];
    f32x4& x0 = PJ ? acc[qa][c / (TNQ / 2)][i][2 * (c % (TNQ / 2))] : acc[qa][0][i][c];
    f32x4& x1 = PJ ? acc[qa][c / (TNQ / 2)][i][2 * (c % (TNQ / 2)) + 1] : acc[qa][1][i][c];
    pair_frags(x0, x1, alpha, v);
    if constexpr (ZERO) {
      x0 = f32x4{0.f, 0.f, 0.f, 0.f};
      x1 = f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int r = 0; r < 8; ++r) v[r] += bb[c][r];
    float x[8];
    if constexpr (ACT_IN) {
      unpack8bf(xin[P], x);
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
      float g[8];
#pragma unroll
      for (int r = 0; r < 8; ++r) v[r] = gelu_tanh_and_grad(v[r], g[r]);
      buf_store16(rAux, off, pack8bf(g));
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
      constexpr int WA = 128 / SA;
      float* dst = a.cs_ws + (long long)((m0 / 256) * WA + wa) * a.N;
#pragma unroll
      for (int c = 0; c < TNQ; ++c) {
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          cs[c][r] = row16_sum(cs[c][r]);
        }
        const int n = nrun + cno(c);
        if ((lane & 15) == 0 && n < a.N) {
          *(f32x4*)(dst + n) = f32x4{cs[c][0], cs[c][1], cs[c][2], cs[c][3]};
          *(f32x4*)(dst + n + 4) = f32x4{cs[c][4], cs[c][5], cs[c][6], cs[c][7]};
        }
      }
    }
  }
}

template <typename OutT, int TMQ, int TNQ, int SA, int SB, int BH, bool ZERO>
__device__ __forceinline__ void tile_epilogue(const GemmArgs& a, f32x4 (&acc)[2][2][TMQ][TNQ], int m0, int n0,
                                              int wa, int wb, int lane, float alpha) {
  // this block's operand DMA has landed (non-persistent: the last K-tile's asm waits;
  // persistent: A-lo(g+2) is still in flight and this retires it, as the epilogue's first load
  // wait would - vmcnt is in order) - said in a wait hipcc sees
  vm_drained();
  if constexpr (std::is_same_v<OutT, bf16_t>) {
    switch (a.act) {
      case 1: tile_epilogue_bf16<1, TMQ, TNQ, SA, SB, BH, ZERO>(a, acc, m0, n0, wa, wb, lane, alpha); break;
      case 2: tile_epilogue_bf16<2, TMQ, TNQ, SA, SB, BH, ZERO>(a, acc, m0, n0, wa, wb, lane, alpha); break;
      case 3: tile_epilogue_bf16<3, TMQ, TNQ, SA, SB, BH, ZERO>(a, acc, m0, n0, wa, wb, lane, alpha); break;
      case 4: tile_epilogue_bf16<4, TMQ, TNQ, SA, SB, BH, ZERO>(a, acc, m0, n0, wa, wb, lane, alpha); break;
      case 5: tile_epilogue_bf16<5, TMQ, TNQ, SA, SB, BH, ZERO>(a, acc, m0, n0, wa, wb, lane, alpha); break;
      case 6: tile_epilogue_bf16<6, TMQ, TNQ, SA, SB, BH, ZERO>(a, acc, m0, n0, wa, wb, lane, alpha); break;
      default: tile_epilogue_bf16<0, TMQ, TNQ, SA, SB, BH, ZERO>(a, acc, m0, n0, wa, wb, lane, alpha); break;
    }
  } else {
    OutT* C = (OutT*)a.C;
    const OutT* Cin = (const OutT*)a.Cin;
#pragma unroll
    for (int qa = 0; qa < 2; ++qa)
#pragma unroll
      for (int qb = 0; qb < 2; ++qb)
#pragma unroll
        for (int i = 0; i < TMQ; ++i) {
          const int m = m0 + 128 * qa + SA * wa + 16 * i + (lane & 15);
#pragma unroll
          for (int j = 0; j < TNQ; ++j) {
            const int n = n0 + BH * qb + SB * wb + 16 * j + 4 * (lane >> 4);
            if (m < a.M && n < a.N) {
              float v[4];
#pragma unroll
              for (int r = 0; r < 4; ++r) v[r] = acc[qa][qb][i][j][r] * alpha;
              epilogue4<OutT>(a, C, Cin, m, n, v);
            }
            if constexpr (ZERO) acc[qa][qb][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
          }
        }
  }
}

// Timing-only builds (results are wrong; never shipped): bit 1 drops the main loop's vmcnt
// waits, bit 2 reads LDS fragments in the first K-tile only, bit 4 drops the loop barriers.
#ifndef RTDC_G8_DIAG
#define RTDC_G8_DIAG 0
#endif

// outstanding glds instructions allowed (wave-uniform): counted waits are immediates
__device__ __forceinline__ void wait_vm(int allowed) {
  if (allowed >= 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else if (allowed == 5) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
  else if (allowed == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if (allowed == 3) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
  else if (allowed == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  else if (allowed == 1) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// glds instructions per wave of events first..last (event kinds e & 3: 0 A-lo, 1 B-lo, 2 B-hi,
// 3 A-hi): an A half is 16 KiB = 2 per wave, a B half CB (64-row halves of the 256x128 tile: 1)
template <int CB>
__device__ __forceinline__ int ev_loads(int first, int last) {
  int n = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int x = first + i;
    if (x <= last) n += ((x & 3) == 1 || (x & 3) == 2) ? CB : 2;
  }
  return n;
}

// The kernel body over one (tile, K-slice): `bid` = the product's flat tile id, `ks` = the split-K
// slice.  gemm8_kernel runs one product (bid = blockIdx.x, ks = blockIdx.y); gemm8g_kernel a
// group of independent products in one launch.
template <bool AK, bool BKM, typename OutT, int BN>
__device__ __forceinline__ void gemm8_body(const GemmArgs& a, const int bid, const int ks) {
  // BN = 256: waves 2 (A) x 4 (B), quadrant 64x32; BN = 192: waves 4 x 2, quadrant 32x48;
  // BN = 128: waves 4 x 2, quadrant 32x32 (M = 2048 products with N = 4096: 8 x 32 = 256
  // tiles, one full round of the chip where 256x256 tiles leave half of it idle)
  constexpr int BH = BN / 2, WA = BN == 256 ? 2 : 4, WB = 8 / WA;
  constexpr int CB = BN == 128 ? 1 : 2;  // glds per wave of one B half
  constexpr int SA = 128 / WA, SB = BH / WB, TMQ = SA / 16, TNQ = SB / 16;
  constexpr int BHALF = BH * 128, BUF = 2 * HALF + 2 * BHALF;
  __shared__ __attribute__((aligned(16))) char smem[2 * BUF + 1024];  // [buf][A-lo, A-hi, B-lo, B-hi] + junk
  char* junk = smem + 2 * BUF;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wa = wave % WA, wb = wave / WA;

  const int tiles_m = (a.M + BM - 1) / BM, tiles_n = (a.N + BN - 1) / BN;
  int tm, tn;
  tile_coords(bid, tiles_m, tiles_n, tm, tn);
  const int m0 = tm * BM, n0 = tn * BN;

  int kb = 0, ke = a.K;
  if (a.splitk > 1) {
    const int ktiles = a.K / gemm::BK;
    const int per = (ktiles + a.splitk - 1) / a.splitk;
    kb = ks * per * gemm::BK;
    ke = min(a.K, kb + per * gemm::BK);
  }
  const int nt = ke > kb ? (ke - kb) / gemm::BK : 0;
  const int total_ev = 4 * nt;

  Stager<AK, 128, 8> sa0, sa1;
  using SBT = std::conditional_t<BN == 192, Half96Stager<BKM>, Stager<BKM, BH, 8>>;
  SBT sb0, sb1;
  sa0.init(a.A, a.lda, a.M, m0, wave, lane);
  sa1.init(a.A, a.lda, a.M, m0 + 128, wave, lane);
  sb0.init(a.B, a.ldb, a.N, n0, wave, lane);
  sb1.init(a.B, a.ldb, a.N, n0 + BH, wave, lane);

  // event e = 4*tile + kind, kind 0: A-lo, 1: B-lo, 2: B-hi, 3: A-hi (issue order = e order)
  auto issue = [&](int e) {
    if (e >= total_ev) return;
    const int j = e >> 2, kind = e & 3;
    const int k0 = kb + j * gemm::BK;
    char* base = smem + (j & 1) * BUF;
    if (kind == 0) sa0.issue(k0, base, wave);
    else if (kind == 3) sa1.issue(k0, base + HALF, wave);
    else if constexpr (BN != 192) {
      if (kind == 1) sb0.issue(k0, base + 2 * HALF, wave);
      else sb1.issue(k0, base + 2 * HALF + BHALF, wave);
    } else {
      if (kind == 1) sb0.issue(k0, base + 2 * HALF, junk);
      else sb1.issue(k0, base + 2 * HALF + BHALF, junk);
    }
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

  if (nt > 0) {
    // prologue: A-lo(0) B-lo(0) B-hi(0) A-hi(0) A-lo(1); phase (0,1) needs events 0 and 1
#pragma unroll
    for (int e = 0; e < 5; ++e) issue(e);
    wait_vm(ev_loads<CB>(2, min(4, total_ev - 1)));
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }

  bf16x8 fa[TMQ][2], fbl[TNQ][2], fbh[TNQ][2];
  for (int t = 0; t < nt; ++t) {
    const char* buf = smem + (t & 1) * BUF;
#pragma unroll
    for (int p = 1; p <= 4; ++p) {
      // 1. fragments for this phase's quadrant (data retired by an earlier wait + barrier)
      // fragments of this phase (MN-major ones as asm TrPair halves, turned into MFMA operands
      // after the lgkmcnt wait below)
      typename Frag<AK>::T ra[TMQ][2];
      typename Frag<BKM>::T rb[TNQ][2];
      const bool rd = !(RTDC_G8_DIAG & 2) || t == 0;
      if ((p == 1 || p == 3) && rd) {
        const char* ah = buf + (p == 1 ? 0 : HALF);
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
          for (int i = 0; i < TMQ; ++i) ra[i][ks] = load_fragx<AK, 128>(ah, SA * wa + 16 * i, ks, lane);
      }
      if ((p == 1 || p == 2) && rd) {
        const char* bh = buf + 2 * HALF + (p == 1 ? 0 : BHALF);
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
          for (int j = 0; j < TNQ; ++j) {
            if constexpr (BN != 192) rb[j][ks] = load_fragx<BKM, BH>(bh, SB * wb + 16 * j, ks, lane);
            else rb[j][ks] = load_frag96<BKM>(bh, SB * wb + 16 * j, ks, lane);
          }
      }
      // 2. restage one half-tile of a later K-tile
      const int e = p < 4 ? 4 * t + 4 + p : 4 * t + 8;
      issue(e);
      // 3. retire what the next phase reads (p3 -> p4 reads nothing new)
      if (p != 3 && (p != 4 || t + 1 < nt) && !(RTDC_G8_DIAG & 1)) {
        const int need = p == 1 ? 4 * t + 2 : (p == 2 ? 4 * t + 3 : 4 * t + 5);
        wait_vm(ev_loads<CB>(need + 1, min(e, total_ev - 1)));
      }
      asm volatile("" ::: "memory");
      if (!(RTDC_G8_DIAG & 4)) __builtin_amdgcn_s_barrier();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if ((p == 1 || p == 3) && rd) {
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
          for (int i = 0; i < TMQ; ++i) fa[i][ks] = fval(ra[i][ks]);
      }
      if ((p == 1 || p == 2) && rd) {
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
          for (int j = 0; j < TNQ; ++j) {
            if (p == 1) fbl[j][ks] = fval(rb[j][ks]);
            else fbh[j][ks] = fval(rb[j][ks]);
          }
      }
      // 4. one quadrant x K=64
      const int qa = (p - 1) >> 1, qb = (p - 1) & 1;
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int i = 0; i < TMQ; ++i)
#pragma unroll
          for (int j = 0; j < TNQ; ++j) {
            if (qb == 0)
              acc[qa][0][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fbl[j][ks], fa[i][ks], acc[qa][0][i][j], 0, 0, 0);
            else
              acc[qa][1][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fbh[j][ks], fa[i][ks], acc[qa][1][i][j], 0, 0, 0);
          }
      __builtin_amdgcn_s_setprio(0);
    }
  }

  if (RTDC_G8_DIAG) asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
  // ---- epilogue: lane holds C[m][n..n+3] of every (quadrant, i, j) fragment ----
  const float alpha = a.alpha_dev ? a.alpha * *a.alpha_dev : a.alpha;
  if (a.splitk > 1) {
    float* Wp = a.ws + (long long)ks * a.M * a.N;
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

template <bool AK, bool BKM, typename OutT, int BN = 256>
__global__ __launch_bounds__(512, 1) void gemm8_kernel(GemmArgs a) {
  gemm8_body<AK, BKM, OutT, BN>(a, blockIdx.x, blockIdx.y);
}

// ---- grouped launch: independent products (same layouts, 256x256 tiles, no split-K) in one
// grid - block b works on tile b - start[p] of product p.  The weight gradients of GPT-2's
// linears are 9..36 tiles each with K = 16384: alone each one needs split-K slabs + a reduce
// kernel to fill the chip; two layers' eight products together are 216 full-K tiles, one
// round, with no slab traffic (ops/gemm.py WgradGroup).
constexpr int G8_MAX_GROUP = 10;  // (10 x GemmArgs: the kernel argument stays < 4 KiB)
struct GemmGroup {
  GemmArgs g[G8_MAX_GROUP];
  int start[G8_MAX_GROUP + 1];
  int n;
};
static_assert(sizeof(GemmGroup) <= 4096, "kernel argument segment");

template <bool AK, bool BKM, typename OutT>
__global__ __launch_bounds__(512, 1) void gemm8g_kernel(GemmGroup gg) {
  const int b = blockIdx.x;
  int p = 0;
#pragma unroll
  for (int i = 1; i < G8_MAX_GROUP; ++i) p += (i < gg.n && b >= gg.start[i]) ? 1 : 0;
  p = __builtin_amdgcn_readfirstlane(p);
  gemm8_body<AK, BKM, OutT, 256>(gg.g[p], b - gg.start[p], 0);
}

// ---- persistent variant: one block per CU walks its tiles; the K-tile event stream runs on
// across tile boundaries, so the next tile's first half-tiles are in flight while this tile
// finishes, and its epilogue stores drain under the next tile's first MFMA phases.
//
// Block b owns tiles b, b + G, b + 2G, ... (G = gridDim.x, a multiple of 8 when the grid is
// persistent, so all of a block's tiles stay on its XCD under tile_coords' XCD remap).  Global
// K-tile index g = s*nt + t (s = the block's tile sequence number); event e = 4g + kind; LDS
// buffer g & 1: gemm8_kernel's steady-state schedule, unchanged, over one long K loop.  What
// changes at a tile boundary (g = the last K-tile of tile s):
//   * the stagers switch to tile s+1 right before phase 4 of K-tile g-1 (the first issue of an
//     event of the next tile: A-lo(g+1));
//   * phase 4 of g retires through A-hi(g+1) (vmcnt(2) instead of vmcnt(6)): everything the
//     next tile's phases 1-3 read is in LDS before the epilogue, so phases 1 and 2 of K-tile
//     g+1 need no wait, and the stores issued in between are first waited on in phase 4 of
//     g+1, three phases of MFMA work later.  No load/store completion order is assumed: every
//     wait counts only the loads issued after the one it needs, so outstanding stores can
//     make a wait longer, never let it pass early (CDNA4 vmcnt counts stores too);
//   * accumulators are re-zeroed after the epilogue.
template <bool AK, bool BKM, typename OutT, int BN = 256>
__global__ __launch_bounds__(512, 1) void gemm8p_kernel(GemmArgs a) {
  constexpr int BH = BN / 2, WA = BN == 256 ? 2 : 4, WB = 8 / WA;
  constexpr int SA = 128 / WA, SB = BH / WB, TMQ = SA / 16, TNQ = SB / 16;
  constexpr int BHALF = BH * 128, BUF = 2 * HALF + 2 * BHALF;
  __shared__ __attribute__((aligned(16))) char smem[2 * BUF + 1024];
  char* junk = smem + 2 * BUF;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wa = wave % WA, wb = wave / WA;

  const int tiles_m = (a.M + BM - 1) / BM, tiles_n = (a.N + BN - 1) / BN;
  const int ntiles = tiles_m * tiles_n;
  const int G = gridDim.x, b = blockIdx.x;
  const int my_tiles = b < ntiles ? (ntiles - b + G - 1) / G : 0;
  const int nt = a.K / gemm::BK;  // >= 2 (host-checked)
  const int total_kt = my_tiles * nt;
  const int total_ev = 4 * total_kt;
  if (total_kt == 0) return;

  Stager<AK, 128, 8> sa0, sa1;
  using SBT = std::conditional_t<BN == 192, Half96Stager<BKM>, Stager<BKM, BH, 8>>;
  SBT sb0, sb1;
  auto stage_tile = [&](int s) {
    int tm, tn;
    tile_coords(b + s * G, tiles_m, tiles_n, tm, tn);
    sa0.init(a.A, a.lda, a.M, tm * BM, wave, lane);
    sa1.init(a.A, a.lda, a.M, tm * BM + 128, wave, lane);
    sb0.init(a.B, a.ldb, a.N, tn * BN, wave, lane);
    sb1.init(a.B, a.ldb, a.N, tn * BN + BH, wave, lane);
  };
  // issue event e whose K-tile index inside its own tile is j (stagers point at that tile)
  auto issue = [&](int e, int j) {
    if (e >= total_ev) return;
    const int kind = e & 3;
    const int k0 = j * gemm::BK;
    char* base = smem + ((e >> 2) & 1) * BUF;
    if (kind == 0) sa0.issue(k0, base, wave);
    else if (kind == 3) sa1.issue(k0, base + HALF, wave);
    else if constexpr (BN != 192) {
      if (kind == 1) sb0.issue(k0, base + 2 * HALF, wave);
      else sb1.issue(k0, base + 2 * HALF + BHALF, wave);
    } else {
      if (kind == 1) sb0.issue(k0, base + 2 * HALF, junk);
      else sb1.issue(k0, base + 2 * HALF + BHALF, junk);
    }
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

  stage_tile(0);
  // prologue: A-lo(0) B-lo(0) B-hi(0) A-hi(0) A-lo(1) of the first tile (nt >= 2)
  issue(0, 0);
  issue(1, 0);
  issue(2, 0);
  issue(3, 0);
  issue(4, 1);
  wait_vm(6);
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();

  const float alpha = a.alpha_dev ? a.alpha * *a.alpha_dev : a.alpha;

  bf16x8 fa[TMQ][2], fbl[TNQ][2], fbh[TNQ][2];
  for (int s = 0; s < my_tiles; ++s) {
    int tm, tn;
    tile_coords(b + s * G, tiles_m, tiles_n, tm, tn);
    const int m0 = tm * BM, n0 = tn * BN;
    const bool more = s + 1 < my_tiles;
    for (int t = 0; t < nt; ++t) {
      const int g = s * nt + t;
      const char* buf = smem + (g & 1) * BUF;
      const bool first = t == 0 && s > 0;  // its phase 1-2 data was retired before the epilogue
      const bool last = t == nt - 1;
#pragma unroll
      for (int p = 1; p <= 4; ++p) {
        // fragments of this phase (MN-major ones as asm TrPair halves, turned into MFMA operands
        // after the lgkmcnt wait below)
        typename Frag<AK>::T ra[TMQ][2];
        typename Frag<BKM>::T rb[TNQ][2];
        if (p == 1 || p == 3) {
          const char* ah = buf + (p == 1 ? 0 : HALF);
#pragma unroll
          for (int ks = 0; ks < 2; ++ks)
#pragma unroll
            for (int i = 0; i < TMQ; ++i) ra[i][ks] = load_fragx<AK, 128>(ah, SA * wa + 16 * i, ks, lane);
        }
        if (p == 1 || p == 2) {
          const char* bh = buf + 2 * HALF + (p == 1 ? 0 : BHALF);
#pragma unroll
          for (int ks = 0; ks < 2; ++ks)
#pragma unroll
            for (int j = 0; j < TNQ; ++j) {
              if constexpr (BN == 256) rb[j][ks] = load_fragx<BKM, 128>(bh, SB * wb + 16 * j, ks, lane);
              else rb[j][ks] = load_frag96<BKM>(bh, SB * wb + 16 * j, ks, lane);
            }
        }
        // restage: p1-p3 -> K-tile t+1 (the next tile's K-tile 0 when t is the last),
        //          p4    -> A-lo of K-tile t+2
        if (p == 4 && t == nt - 2 && more) stage_tile(s + 1);
        if (p < 4) issue(4 * g + 4 + p, last ? 0 : t + 1);
        else issue(4 * g + 8, t + 2 < nt ? t + 2 : t + 2 - nt);
        // retire what later phases read
        if (p == 1 || p == 2) {
          if (!first) {
            const int e = 4 * g + 4 + p, need = 4 * g + 1 + p;
            wait_vm(2 * (min(e + 1, total_ev) - 1 - need));
          }
        } else if (p == 4 && g + 1 < total_kt) {
          const int e = 4 * g + 8;
          const int need = last ? 4 * g + 7 : 4 * g + 5;  // A-hi(g+1) ahead of an epilogue
          wait_vm(2 * (min(e + 1, total_ev) - 1 - need));
        }
        asm volatile("" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (p == 1 || p == 3) {
#pragma unroll
          for (int ks = 0; ks < 2; ++ks)
#pragma unroll
            for (int i = 0; i < TMQ; ++i) fa[i][ks] = fval(ra[i][ks]);
        }
        if (p == 1 || p == 2) {
#pragma unroll
          for (int ks = 0; ks < 2; ++ks)
#pragma unroll
            for (int j = 0; j < TNQ; ++j) {
              if (p == 1) fbl[j][ks] = fval(rb[j][ks]);
              else fbh[j][ks] = fval(rb[j][ks]);
            }
        }
        const int qa = (p - 1) >> 1, qb = (p - 1) & 1;
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
          for (int i = 0; i < TMQ; ++i)
#pragma unroll
            for (int j = 0; j < TNQ; ++j) {
              if (qb == 0)
                acc[qa][0][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fbl[j][ks], fa[i][ks], acc[qa][0][i][j], 0, 0, 0);
              else
                acc[qa][1][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fbh[j][ks], fa[i][ks], acc[qa][1][i][j], 0, 0, 0);
            }
        __builtin_amdgcn_s_setprio(0);
      }
    }
    // ---- epilogue of tile s (its stores drain under tile s+1's first phases); re-zeroes acc
    tile_epilogue<OutT, TMQ, TNQ, SA, SB, BH, true>(a, acc, m0, n0, wa, wb, lane, alpha);
  }
}

// ---- plain fp32 tile store through a buffer descriptor (no bias / Cin / activation: the
// grouped weight-gradient form).  Out-of-range rows / columns get BUF_OOB offsets instead of
// per-lane branches, so no wait on the next tile's in-flight loads is inserted at a join;
// re-zeroes the accumulators.
template <int TMQ, int TNQ, int SA, int SB, int BH>
__device__ __forceinline__ void tile_store_f32(const GemmArgs& a, f32x4 (&acc)[2][2][TMQ][TNQ], int m0, int n0,
                                               int wa, int wb, int lane, float alpha) {
  const long long tile_off = (long long)m0 * a.ldc * 4, rows_bytes = (long long)(a.M - m0) * a.ldc * 4;
  const auto rC = make_rsrc(a.C, tile_off, rows_bytes);
  const int rows_left = a.M - m0;
#pragma unroll
  for (int qa = 0; qa < 2; ++qa)
#pragma unroll
    for (int qb = 0; qb < 2; ++qb)
#pragma unroll
      for (int i = 0; i < TMQ; ++i) {
        const int r = 128 * qa + SA * wa + 16 * i + (lane & 15);
#pragma unroll
        for (int j = 0; j < TNQ; ++j) {
          const int n = n0 + BH * qb + SB * wb + 16 * j + 4 * (lane >> 4);
          const uint32_t off = (r < rows_left && n < a.N) ? (uint32_t)(r * a.ldc + n) * 4u : BUF_OOB;
          const f32x4 x = acc[qa][qb][i][j];
          buf_store16(rC, off, u32x4{__float_as_uint(x[0] * alpha), __float_as_uint(x[1] * alpha),
                                     __float_as_uint(x[2] * alpha), __float_as_uint(x[3] * alpha)});
          acc[qa][qb][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
      }
}

// ---- grouped persistent variant (gemm8gp_kernel): gemm8p_kernel's cross-tile pipeline over
// the tiles of a GROUP of independent products with the same K (a layer's weight gradients:
// K = tokens).  Global tile T indexes the products' tiles back to back (gg.start); the XCD
// remap runs over the global list, so each XCD walks a contiguous run of tiles - consecutive
// GROUP_M-ordered tiles of one product, sharing operand panels in that XCD's L2 - and the
// stagers switch product where the run crosses a product boundary.  Against the one-block-per-
// tile gemm8g_kernel this overlaps each tile's fp32 epilogue (256 KiB of stores) and the next
// tile's prologue with MFMA work: with K = 2048 (Llama-3-8B, 32 K-tiles per tile) those were
// ~25 % of a tile's time.
__device__ __forceinline__ void group_tile(const GemmGroup& gg, int T, int total, int& p, int& tm, int& tn) {
  int wgid = T;
  if (total > 8) {
    const int xcd = T & 7, q = total >> 3, r = total & 7;
    wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (T >> 3);
  }
  int pp = 0;
#pragma unroll
  for (int i = 1; i < G8_MAX_GROUP; ++i) pp += (i < gg.n && wgid >= gg.start[i]) ? 1 : 0;
  p = __builtin_amdgcn_readfirstlane(pp);
  const int local = wgid - gg.start[p];
  const int tiles_m = (gg.g[p].M + BM - 1) / BM, tiles_n = (gg.g[p].N + 255) / 256;
  constexpr int GROUP_M = 8;
  const int group = local / (GROUP_M * tiles_n);
  const int first_m = group * GROUP_M;
  const int gsize = min(tiles_m - first_m, GROUP_M);
  tm = first_m + (local % (GROUP_M * tiles_n)) % gsize;
  tn = (local % (GROUP_M * tiles_n)) / gsize;
}

template <bool AK, bool BKM>
__global__ __launch_bounds__(512, 1) void gemm8gp_kernel(GemmGroup gg) {
  constexpr int BN = 256, BH = BN / 2, WA = 2, WB = 8 / WA;
  constexpr int SA = 128 / WA, SB = BH / WB, TMQ = SA / 16, TNQ = SB / 16;
  constexpr int BHALF = BH * 128, BUF = 2 * HALF + 2 * BHALF;
  __shared__ __attribute__((aligned(16))) char smem[2 * BUF + 1024];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wa = wave % WA, wb = wave / WA;

  const int ntiles = gg.start[gg.n];
  const int G = gridDim.x, b = blockIdx.x;
  const int my_tiles = b < ntiles ? (ntiles - b + G - 1) / G : 0;
  const int nt = gg.g[0].K / gemm::BK;  // same K for every product, >= 2 (host-checked)
  const int total_kt = my_tiles * nt;
  const int total_ev = 4 * total_kt;
  if (total_kt == 0) return;

  Stager<AK, 128, 8> sa0, sa1;
  Stager<BKM, BH, 8> sb0, sb1;
  auto stage_tile = [&](int s) {
    int p, tm, tn;
    group_tile(gg, b + s * G, ntiles, p, tm, tn);
    const GemmArgs& a = gg.g[p];
    sa0.init(a.A, a.lda, a.M, tm * BM, wave, lane);
    sa1.init(a.A, a.lda, a.M, tm * BM + 128, wave, lane);
    sb0.init(a.B, a.ldb, a.N, tn * BN, wave, lane);
    sb1.init(a.B, a.ldb, a.N, tn * BN + BH, wave, lane);
  };
  auto issue = [&](int e, int j) {
    if (e >= total_ev) return;
    const int kind = e & 3;
    const int k0 = j * gemm::BK;
    char* base = smem + ((e >> 2) & 1) * BUF;
    if (kind == 0) sa0.issue(k0, base, wave);
    else if (kind == 3) sa1.issue(k0, base + HALF, wave);
    else if (kind == 1) sb0.issue(k0, base + 2 * HALF, wave);
    else sb1.issue(k0, base + 2 * HALF + BHALF, wave);
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

  stage_tile(0);
  issue(0, 0);
  issue(1, 0);
  issue(2, 0);
  issue(3, 0);
  issue(4, 1);
  wait_vm(6);
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();

  bf16x8 fa[TMQ][2], fbl[TNQ][2], fbh[TNQ][2];
  for (int s = 0; s < my_tiles; ++s) {
    int p, tm, tn;
    group_tile(gg, b + s * G, ntiles, p, tm, tn);
    const int m0 = tm * BM, n0 = tn * BN;
    const bool more = s + 1 < my_tiles;
    for (int t = 0; t < nt; ++t) {
      const int g = s * nt + t;
      const char* buf = smem + (g & 1) * BUF;
      const bool first = t == 0 && s > 0;
      const bool last = t == nt - 1;
#pragma unroll
      for (int ph = 1; ph <= 4; ++ph) {
        typename Frag<AK>::T ra[TMQ][2];
        typename Frag<BKM>::T rb[TNQ][2];
        if (ph == 1 || ph == 3) {
          const char* ah = buf + (ph == 1 ? 0 : HALF);
#pragma unroll
          for (int ks = 0; ks < 2; ++ks)
#pragma unroll
            for (int i = 0; i < TMQ; ++i) ra[i][ks] = load_fragx<AK, 128>(ah, SA * wa + 16 * i, ks, lane);
        }
        if (ph == 1 || ph == 2) {
          const char* bh = buf + 2 * HALF + (ph == 1 ? 0 : BHALF);
#pragma unroll
          for (int ks = 0; ks < 2; ++ks)
#pragma unroll
            for (int j = 0; j < TNQ; ++j) rb[j][ks] = load_fragx<BKM, 128>(bh, SB * wb + 16 * j, ks, lane);
        }
        if (ph == 4 && t == nt - 2 && more) stage_tile(s + 1);
        if (ph < 4) issue(4 * g + 4 + ph, last ? 0 : t + 1);
        else issue(4 * g + 8, t + 2 < nt ? t + 2 : t + 2 - nt);
        if (ph == 1 || ph == 2) {
          if (!first) {
            const int e = 4 * g + 4 + ph, need = 4 * g + 1 + ph;
            wait_vm(2 * (min(e + 1, total_ev) - 1 - need));
          }
        } else if (ph == 4 && g + 1 < total_kt) {
          const int e = 4 * g + 8;
          const int need = last ? 4 * g + 7 : 4 * g + 5;
          wait_vm(2 * (min(e + 1, total_ev) - 1 - need));
        }
        asm volatile("" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (ph == 1 || ph == 3) {
#pragma unroll
          for (int ks = 0; ks < 2; ++ks)
#pragma unroll
            for (int i = 0; i < TMQ; ++i) fa[i][ks] = fval(ra[i][ks]);
        }
        if (ph == 1 || ph == 2) {
#pragma unroll
          for (int ks = 0; ks < 2; ++ks)
#pragma unroll
            for (int j = 0; j < TNQ; ++j) {
              if (ph == 1) fbl[j][ks] = fval(rb[j][ks]);
              else fbh[j][ks] = fval(rb[j][ks]);
            }
        }
        const int qa = (ph - 1) >> 1, qb = (ph - 1) & 1;
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
          for (int i = 0; i < TMQ; ++i)
#pragma unroll
            for (int j = 0; j < TNQ; ++j) {
              if (qb == 0)
                acc[qa][0][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fbl[j][ks], fa[i][ks], acc[qa][0][i][j], 0, 0, 0);
              else
                acc[qa][1][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fbh[j][ks], fa[i][ks], acc[qa][1][i][j], 0, 0, 0);
            }
        __builtin_amdgcn_s_setprio(0);
      }
    }
    const GemmArgs& a = gg.g[p];
    tile_store_f32<TMQ, TNQ, SA, SB, BH>(a, acc, m0, n0, wa, wb, lane, a.alpha);
  }
}

// ---- 4-wave 256x256 kernel: a 128x128 output per wave (accumulators in AGPRs) ----------
//
// Why: the 8-wave kernel's per-wave 128x64 tile reads (128 + 64) x 64 x 2 B of LDS fragments per
// 2 x 128 x 64 x 64 FLOP: 384 B per 16x16x32 MFMA, ~96 B/clk per CU at the MFMA peak against an
// LDS port that delivers ~64 B/clk for swizzled ds_read_b128 - the fragment reads, not MFMA issue,
// bound its main loop (profiles/gemm_mfma_shape_diag.txt).  A 128x128 per-wave tile reads
// 256 B per MFMA (-33 %).  Its 256 fp32 accumulators live in AGPRs (one wave per SIMD: 512
// registers per lane), the fragments in VGPRs.
//
// With one wave per SIMD nothing else hides a wave's own LDS latency, so fragments are
// PREFETCHED one phase ahead - the ds_reads of phase p+1 are issued at the top of phase p and
// run under phase p's 32 MFMAs:
//     phase   MFMA quadrant (A half, B half)   reads issued (for later phases)
//       p1      (lo, lo)  fa0 fbl              B-hi(t)   -> fbh
//       p2      (lo, hi)  fa0 fbh              A-hi(t)   -> fa1
//       p3      (hi, lo)  fa1 fbl              -
//       p4      (hi, hi)  fa1 fbh              A-lo(t+1) -> fa0, B-lo(t+1) -> fbl
// Half-tile DMA (event e = 4 * K-tile + kind, kind 0 A-lo, 1 B-lo, 2 B-hi, 3 A-hi; 4 glds
// per thread each) is issued as soon as the region's previous occupant (same half, K-tile
// t - 2, same LDS buffer) has been read: p1 issues A-lo(t+2), B-lo(t+2); p2 B-hi(t+2); p3
// A-hi(t+2).  Every load then has ~6 phases (~190 MFMAs per SIMD) to land, with up to 6
// half-tiles (24 glds) in flight per wave across each raw s_barrier (counted vmcnt, never 0
// in the steady state).
// RAW: a half is read in the phase after the barrier that follows its retiring wait;
// WAR: a half is restaged only after the barrier that follows the lgkmcnt(0) retiring its
// last read.
__device__ __forceinline__ void wait_vm4(int allowed_events) {
  // allowed outstanding glds = 4 per event
  switch (allowed_events < 0 ? 0 : (allowed_events > 6 ? 6 : allowed_events)) {
    case 6: asm volatile("s_waitcnt vmcnt(24)" ::: "memory"); break;
    case 5: asm volatile("s_waitcnt vmcnt(20)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(16)" ::: "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(12)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}

// 16 MFMAs of one k-slice, c[i][j] += b[j] (x) a[i], with the accumulators pinned to AGPRs
// ("+a"): hipcc's own allocation of 256 accumulators beside 128+ fragment VGPRs rotated them
// through a[4:7] with 4 v_accvgpr_mov per MFMA (and spilled VGPRs into AGPRs).  Hazards
// (cdna_hip_programming.md §5.7 item 2): the leading s_nop 1 covers a VALU write of an operand
// right before the statement; consecutive statements chain accumulators whole (0 states); the
// reader after the last statement is fenced by mfma_drain().
__device__ __forceinline__ void mfma16_agpr(f32x4 (&c)[4][4], const bf16x8 (&a)[4], const bf16x8 (&b)[4]) {
  asm volatile(
      "s_nop 1\n\t"
      "v_mfma_f32_16x16x32_bf16 %0, %20, %16, %0\n\t"
      "v_mfma_f32_16x16x32_bf16 %1, %21, %16, %1\n\t"
      "v_mfma_f32_16x16x32_bf16 %2, %22, %16, %2\n\t"
      "v_mfma_f32_16x16x32_bf16 %3, %23, %16, %3\n\t"
      "v_mfma_f32_16x16x32_bf16 %4, %20, %17, %4\n\t"
      "v_mfma_f32_16x16x32_bf16 %5, %21, %17, %5\n\t"
      "v_mfma_f32_16x16x32_bf16 %6, %22, %17, %6\n\t"
      "v_mfma_f32_16x16x32_bf16 %7, %23, %17, %7\n\t"
      "v_mfma_f32_16x16x32_bf16 %8, %20, %18, %8\n\t"
      "v_mfma_f32_16x16x32_bf16 %9, %21, %18, %9\n\t"
      "v_mfma_f32_16x16x32_bf16 %10, %22, %18, %10\n\t"
      "v_mfma_f32_16x16x32_bf16 %11, %23, %18, %11\n\t"
      "v_mfma_f32_16x16x32_bf16 %12, %20, %19, %12\n\t"
      "v_mfma_f32_16x16x32_bf16 %13, %21, %19, %13\n\t"
      "v_mfma_f32_16x16x32_bf16 %14, %22, %19, %14\n\t"
      "v_mfma_f32_16x16x32_bf16 %15, %23, %19, %15\n\t"
      : "+a"(c[0][0]), "+a"(c[0][1]), "+a"(c[0][2]), "+a"(c[0][3]), "+a"(c[1][0]), "+a"(c[1][1]), "+a"(c[1][2]), "+a"(c[1][3]), "+a"(c[2][0]), "+a"(c[2][1]), "+a"(c[2][2]), "+a"(c[2][3]), "+a"(c[3][0]), "+a"(c[3][1]), "+a"(c[3][2]), "+a"(c[3][3])
      : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(b[0]), "v"(b[1]), "v"(b[2]), "v"(b[3]));
}

// MFMA D -> any other reader needs 12 wait states (8-pass XDL): naming every accumulator keeps
// the compiler's reads below the nops
__device__ __forceinline__ void mfma_drain(f32x4 (&c)[4][4]) {
  asm volatile("s_nop 15" : "+a"(c[0][0]), "+a"(c[0][1]), "+a"(c[0][2]), "+a"(c[0][3]), "+a"(c[1][0]), "+a"(c[1][1]), "+a"(c[1][2]), "+a"(c[1][3]), "+a"(c[2][0]), "+a"(c[2][1]), "+a"(c[2][2]), "+a"(c[2][3]), "+a"(c[3][0]), "+a"(c[3][1]), "+a"(c[3][2]), "+a"(c[3][3]));
}

// 4 MFMAs (one A fragment x 4 B fragments of one k-slice), accumulators pinned to AGPRs; the
// unit the interleaved schedule places loads between.  s_nop 1: a VALU write of an operand
// right before the statement (hazard, cdna_hip_programming.md §5.7 item 2).
__device__ __forceinline__ void mfma4_agpr(f32x4 (&c)[4], const bf16x8& a, const bf16x8 (&b)[4]) {
  asm volatile(
      "s_nop 1\n\t"
      "v_mfma_f32_16x16x32_bf16 %0, %5, %4, %0\n\t"
      "v_mfma_f32_16x16x32_bf16 %1, %6, %4, %1\n\t"
      "v_mfma_f32_16x16x32_bf16 %2, %7, %4, %2\n\t"
      "v_mfma_f32_16x16x32_bf16 %3, %8, %4, %3\n\t"
      : "+a"(c[0]), "+a"(c[1]), "+a"(c[2]), "+a"(c[3])
      : "v"(a), "v"(b[0]), "v"(b[1]), "v"(b[2]), "v"(b[3]));
}

// all LDS reads retired, stated through the builtin so hipcc's wait bookkeeping knows it (an
// asm wait is invisible to it: it then re-waits lgkmcnt(0) before the first use of data it
// still thinks is in flight - after the next phase's prefetch reads were issued, which
// serialised them with the MFMAs).  vmcnt / expcnt fields at their maxima (no wait).
__device__ __forceinline__ void lgkm0() { __builtin_amdgcn_s_waitcnt(0xC07F); }

__device__ __forceinline__ uint32_t lds_addr_of(const char* p) {
  return (uint32_t)(uintptr_t)((const __attribute__((address_space(3))) char*)p);
}
// ds_read_b64_tr_b16 with an immediate byte offset (common.h ds_tr16 protocol: retire with an
// lgkmcnt wait, then tr_use)
template <int OFF>
__device__ __forceinline__ bf16x4 ds_tr16_imm(uint32_t addr) {
  bf16x4 r;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "i"(OFF) : "memory");
  return r;
}

template <bool AK, bool BKM, typename OutT>
__global__ __launch_bounds__(256, 1) void gemm4_kernel(GemmArgs a) {
  constexpr int BN = 256, BH = 128, SA = 64, SB = 64, TMQ = 4, TNQ = 4;
  constexpr int BUF = 4 * HALF;  // [A-lo, A-hi, B-lo, B-hi]
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
  const int tev = 4 * nt;

  Stager<AK, 128, 4> sa0, sa1;
  Stager<BKM, 128, 4> sb0, sb1;
  sa0.init(a.A, a.lda, a.M, m0, wave, lane);
  sa1.init(a.A, a.lda, a.M, m0 + 128, wave, lane);
  sb0.init(a.B, a.ldb, a.N, n0, wave, lane);
  sb1.init(a.B, a.ldb, a.N, n0 + BH, wave, lane);

  auto issue = [&](int e) {
    if (e >= tev) return;
    const int j = e >> 2, kind = e & 3;
    const int k0 = kb + j * gemm::BK;
    char* base = smem + (j & 1) * BUF;
    if (kind == 0) sa0.issue(k0, base, wave);
    else if (kind == 1) sb0.issue(k0, base + 2 * HALF, wave);
    else if (kind == 2) sb1.issue(k0, base + 3 * HALF, wave);
    else sa1.issue(k0, base + HALF, wave);
  };
  // wait until event `need` has landed, given that events up to `last` were issued
  auto retire = [&](int need, int last) { wait_vm4(min(last, tev - 1) - need); };

  f32x4 acc[2][2][TMQ][TNQ];
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y)
#pragma unroll
      for (int i = 0; i < TMQ; ++i)
#pragma unroll
        for (int j = 0; j < TNQ; ++j) acc[x][y][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // fragments [k-slice][row / column block]
  bf16x8 fa0[2][TMQ], fa1[2][TMQ], fbl[2][TNQ], fbh[2][TNQ];
  auto load_a = [&](typename Frag<AK>::T (&r)[2][TMQ], const char* half) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < TMQ; ++i) r[ks][i] = load_fragx<AK, 128>(half, SA * wa + 16 * i, ks, lane);
  };
  auto load_b = [&](typename Frag<BKM>::T (&r)[2][TNQ], const char* half) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int j = 0; j < TNQ; ++j) r[ks][j] = load_fragx<BKM, 128>(half, SB * wb + 16 * j, ks, lane);
  };
  auto take_a = [&](bf16x8 (&f)[2][TMQ], typename Frag<AK>::T (&r)[2][TMQ]) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < TMQ; ++i) f[ks][i] = fval(r[ks][i]);
  };
  auto take_b = [&](bf16x8 (&f)[2][TNQ], typename Frag<BKM>::T (&r)[2][TNQ]) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int j = 0; j < TNQ; ++j) f[ks][j] = fval(r[ks][j]);
  };

  if (nt > 0) {
    // prologue: K-tiles 0 and 1 in flight; A-lo(0), B-lo(0) into registers (B-hi(0) landed too)
#pragma unroll
    for (int e = 0; e < 8; ++e) issue(e);
    retire(2, 7);
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    typename Frag<AK>::T ra[2][TMQ];
    typename Frag<BKM>::T rb[2][TNQ];
    load_a(ra, smem);
    load_b(rb, smem + 2 * HALF);
    lgkm0();
    __builtin_amdgcn_s_barrier();  // WAR: nobody restages A-lo/B-lo(0)'s buffer before all read it
    take_a(fa0, ra);
    take_b(fbl, rb);
  }

  // one phase: 8 groups of 4 MFMAs (k-slice ks = g / 4, A block i = g % 4) of quadrant
  // (qa, qb); after group g, fill(g) places loads - fragment reads for a later phase and DMA
  // pieces - so they issue while the matrix core works (one wave per SIMD: nothing else
  // would cover their issue cost)
  auto phase = [&](int qa, int qb, bf16x8 (&fa)[2][TMQ], bf16x8 (&fb)[2][TNQ], auto&& fill) {
#pragma unroll
    for (int g = 0; g < 8; ++g) {
      mfma4_agpr(acc[qa][qb][g & 3], fa[g >> 2][g & 3], fb[g >> 2]);
      __builtin_amdgcn_sched_barrier(0);
      fill(g);
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  // DMA piece ii of half-tile event e (kind = e & 3)
  auto dma = [&](int e, int ii) {
    if (e >= tev) return;
    const int j = e >> 2, kind = e & 3;
    const int k0 = kb + j * gemm::BK;
    char* base = smem + (j & 1) * BUF;
    if (kind == 0) sa0.issue_one(k0, base, wave, ii);
    else if (kind == 1) sb0.issue_one(k0, base + 2 * HALF, wave, ii);
    else if (kind == 2) sb1.issue_one(k0, base + 3 * HALF, wave, ii);
    else sa1.issue_one(k0, base + HALF, wave, ii);
  };

  for (int t = 0; t < nt; ++t) {
    const char* buf = smem + (t & 1) * BUF;
    const char* nbuf = smem + ((t + 1) & 1) * BUF;
    const bool more = t + 1 < nt;
    const int e2 = 4 * (t + 2);  // events of K-tile t + 2
    // ---- p1: (lo, lo); reads B-hi(t) (2 per group, groups 0-3); DMA A-lo, B-lo(t+2) (groups 4-7)
    {
      typename Frag<BKM>::T rb[2][TNQ];
      phase(0, 0, fa0, fbl, [&](int g) {
        if (g < 4) {
          rb[g >> 1][2 * (g & 1)] = load_fragx<BKM, 128>(buf + 3 * HALF, SB * wb + 32 * (g & 1), g >> 1, lane);
          rb[g >> 1][2 * (g & 1) + 1] = load_fragx<BKM, 128>(buf + 3 * HALF, SB * wb + 32 * (g & 1) + 16, g >> 1, lane);
        } else {
          dma(e2 + 0, g - 4);
          dma(e2 + 1, g - 4);
        }
      });
      retire(4 * t + 3, 4 * t + 9);  // A-hi(t) for p2's reads
      lgkm0();
      asm volatile("" ::: "memory");
      __builtin_amdgcn_s_barrier();
      take_b(fbh, rb);
    }
    // ---- p2: (lo, hi); reads A-hi(t) (groups 0-3); DMA B-hi(t+2) (groups 4-7)
    {
      typename Frag<AK>::T ra[2][TMQ];
      phase(0, 1, fa0, fbh, [&](int g) {
        if (g < 4) {
          ra[g >> 1][2 * (g & 1)] = load_fragx<AK, 128>(buf + HALF, SA * wa + 32 * (g & 1), g >> 1, lane);
          ra[g >> 1][2 * (g & 1) + 1] = load_fragx<AK, 128>(buf + HALF, SA * wa + 32 * (g & 1) + 16, g >> 1, lane);
        } else {
          dma(e2 + 2, g - 4);
        }
      });
      lgkm0();
      asm volatile("" ::: "memory");
      __builtin_amdgcn_s_barrier();
      take_a(fa1, ra);
    }
    // ---- p3: (hi, lo); no reads; DMA A-hi(t+2) (groups 4-7)
    phase(1, 0, fa1, fbl, [&](int g) {
      if (g >= 4) dma(e2 + 3, g - 4);
    });
    if (more) retire(4 * t + 5, 4 * t + 11);  // A-lo(t+1), B-lo(t+1) for p4's reads
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    // ---- p4: (hi, hi); reads A-lo(t+1) (groups 0-3), B-lo(t+1) (groups 4-7)
    {
      typename Frag<AK>::T ra[2][TMQ];
      typename Frag<BKM>::T rb[2][TNQ];
      phase(1, 1, fa1, fbh, [&](int g) {
        if (!more) return;
        const int h = g & 3;
        if (g < 4) {
          ra[h >> 1][2 * (h & 1)] = load_fragx<AK, 128>(nbuf, SA * wa + 32 * (h & 1), h >> 1, lane);
          ra[h >> 1][2 * (h & 1) + 1] = load_fragx<AK, 128>(nbuf, SA * wa + 32 * (h & 1) + 16, h >> 1, lane);
        } else {
          rb[h >> 1][2 * (h & 1)] = load_fragx<BKM, 128>(nbuf + 2 * HALF, SB * wb + 32 * (h & 1), h >> 1, lane);
          rb[h >> 1][2 * (h & 1) + 1] =
              load_fragx<BKM, 128>(nbuf + 2 * HALF, SB * wb + 32 * (h & 1) + 16, h >> 1, lane);
        }
      });
      if (more) {
        retire(4 * t + 6, 4 * t + 11);  // B-hi(t+1) for the next p1's reads
        lgkm0();
        asm volatile("" ::: "memory");
        __builtin_amdgcn_s_barrier();
        take_a(fa0, ra);
        take_b(fbl, rb);
      }
    }
  }
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

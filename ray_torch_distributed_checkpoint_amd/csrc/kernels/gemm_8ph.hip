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

// fragment of a 96-row half: rows (= n) R0..R0+15, k-slice ks (same lane contract as load_frag)
template <bool KMAJOR>
__device__ __forceinline__ bf16x8 load_frag96(const char* tile, int R0, int ks, int lane) {
  if constexpr (KMAJOR) {
    return load_frag<true, 96>(tile, R0, ks, lane);
  } else {
    const int idx = lane & 15, q = idx >> 2, p = idx & 3, g = lane >> 4;
    const int c = (R0 >> 3) + (p >> 1);
    bf16x4 v[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int kr = ks * 32 + 8 * g + 4 * h + q;
      const int off = kr * 192 + (((c + rot96(kr)) % 12) << 4) + ((p & 1) << 3);
      v[h] = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) bf16x4*)(tile + off));
    }
    bf16x8 r;
    r[0] = v[0][0]; r[1] = v[0][1]; r[2] = v[0][2]; r[3] = v[0][3];
    r[4] = v[1][0]; r[5] = v[1][1]; r[6] = v[1][2]; r[7] = v[1][3];
    return r;
  }
}

// outstanding glds instructions allowed (wave-uniform): counted waits are immediates
__device__ __forceinline__ void wait_vm(int allowed) {
  if (allowed >= 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else if (allowed >= 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if (allowed >= 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <bool AK, bool BKM, typename OutT, int BN = 256>
__global__ __launch_bounds__(512, 1) void gemm8_kernel(GemmArgs a) {
  // BN = 256: waves 2 (A) x 4 (B), quadrant 64x32; BN = 192: waves 4 x 2, quadrant 32x48
  constexpr int BH = BN / 2, WA = BN == 256 ? 2 : 4, WB = 8 / WA;
  constexpr int SA = 128 / WA, SB = BH / WB, TMQ = SA / 16, TNQ = SB / 16;
  constexpr int BHALF = BH * 128, BUF = 2 * HALF + 2 * BHALF;
  __shared__ __attribute__((aligned(16))) char smem[2 * BUF + 1024];  // [buf][A-lo, A-hi, B-lo, B-hi] + junk
  char* junk = smem + 2 * BUF;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wa = wave % WA, wb = wave / WA;

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
  const int total_ev = 4 * nt;

  Stager<AK, 128, 8> sa0, sa1;
  using SBT = std::conditional_t<BN == 256, Stager<BKM, 128, 8>, Half96Stager<BKM>>;
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
    else if constexpr (BN == 256) {
      if (kind == 1) sb0.issue(k0, base + 2 * HALF, wave);
      else sb1.issue(k0, base + 3 * HALF, wave);
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
    wait_vm(2 * (min(5, total_ev) - 2));
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }

  bf16x8 fa[TMQ][2], fbl[TNQ][2], fbh[TNQ][2];
  for (int t = 0; t < nt; ++t) {
    const char* buf = smem + (t & 1) * BUF;
#pragma unroll
    for (int p = 1; p <= 4; ++p) {
      // 1. fragments for this phase's quadrant (data retired by an earlier wait + barrier)
      if (p == 1 || p == 3) {
        const char* ah = buf + (p == 1 ? 0 : HALF);
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
          for (int i = 0; i < TMQ; ++i) fa[i][ks] = load_frag<AK, 128>(ah, SA * wa + 16 * i, ks, lane);
      }
      if (p == 1 || p == 2) {
        const char* bh = buf + 2 * HALF + (p == 1 ? 0 : BHALF);
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
          for (int j = 0; j < TNQ; ++j) {
            bf16x8 f;
            if constexpr (BN == 256) f = load_frag<BKM, 128>(bh, SB * wb + 16 * j, ks, lane);
            else f = load_frag96<BKM>(bh, SB * wb + 16 * j, ks, lane);
            if (p == 1) fbl[j][ks] = f;
            else fbh[j][ks] = f;
          }
      }
      // 2. restage one half-tile of a later K-tile
      const int e = p < 4 ? 4 * t + 4 + p : 4 * t + 8;
      issue(e);
      // 3. retire what the next phase reads (p3 -> p4 reads nothing new)
      if (p != 3 && (p != 4 || t + 1 < nt)) {
        const int need = p == 1 ? 4 * t + 2 : (p == 2 ? 4 * t + 3 : 4 * t + 5);
        wait_vm(2 * (min(e + 1, total_ev) - 1 - need));
      }
      asm volatile("" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
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

  // ---- epilogue: lane holds C[m][n..n+3] of every (quadrant, i, j) fragment ----
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
  OutT* C = (OutT*)a.C;
  const OutT* Cin = (const OutT*)a.Cin;
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
          epilogue4<OutT>(a, C, Cin, m, n, v);
        }
      }
}

}  // namespace g8
}  // namespace rtdc

using namespace rtdc;

// Launch the 8-phase kernel (batch 1, no causal modes).  a->splitk is honoured as set.
// bn: 256 or 192 (output tile columns)
extern "C" int rtdc_gemm8_launch(const GemmArgs* args, int a_kmajor, int b_kmajor, int out_fp32, int bn,
                                 hipStream_t st) {
  const GemmArgs& a = *args;
  const unsigned tiles = (unsigned)(((a.M + 255) / 256) * ((a.N + bn - 1) / bn));
  dim3 grid(tiles, a.splitk > 1 ? a.splitk : 1, 1), block(512);
#define G8(AK, BKM, T)                                                                      \
  do {                                                                                      \
    if (bn == 192) hipLaunchKernelGGL((g8::gemm8_kernel<AK, BKM, T, 192>), grid, block, 0, st, a); \
    else hipLaunchKernelGGL((g8::gemm8_kernel<AK, BKM, T, 256>), grid, block, 0, st, a);           \
  } while (0)
  if (out_fp32) {
    if (a_kmajor && b_kmajor) G8(true, true, float);
    else if (a_kmajor) G8(true, false, float);
    else if (!b_kmajor) G8(false, false, float);
    else G8(false, true, float);
  } else {
    if (a_kmajor && b_kmajor) G8(true, true, bf16_t);
    else if (a_kmajor) G8(true, false, bf16_t);
    else if (!b_kmajor) G8(false, false, bf16_t);
    else G8(false, true, bf16_t);
  }
#undef G8
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

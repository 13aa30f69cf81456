// bf16 MFMA GEMM for gfx950 with fused epilogues.
//
//   C[z](m, n) = epilogue( alpha * sum_k A[z](m, k) * B[z](k, n) )
//
// Each operand is either K-major (A stored [M][lda] with k contiguous; B stored [N][ldb] with
// k contiguous) or MN-major (A stored [K][lda] with m contiguous; B stored [K][ldb] with n
// contiguous).  nn.Linear needs all three combinations:
//   forward  Y  = X  W^T : A = X  (K-major), B = W (K-major)
//   dgrad    dX = dY W   : A = dY (K-major), B = W (MN-major)
//   wgrad    dW = dY^T X : A = dY (MN-major), B = X (MN-major)
// so the MN-major form is not a transpose kernel in front of the GEMM: tiles are staged into
// LDS exactly as they sit in HBM (coalesced 16-B global_load_lds) and the k-strided MFMA
// fragments are read back with the gfx950 transposing LDS read ds_read_b64_tr_b16.
//
// Tile configurations (BM x BN, waves WM x WN; BK = 64; v_mfma_f32_16x16x32_bf16):
//   0: 128x128, 2x2 waves (256 threads), 64 KiB LDS, 2 blocks/CU    - small / batched GEMMs
//   1: 256x128, 4x2 waves (512 threads), 96 KiB LDS                  - tall GEMMs
//   2: 128x256, 2x4 waves (512 threads), 96 KiB LDS                  - wide GEMMs
//   3: 256x256, 2x4 waves (512 threads), 128 KiB LDS, 128x64 / wave  - large GEMMs
// chosen per shape by the launcher so the grid fills the 256 CUs in whole waves (a GEMM with
// 192 tiles leaves 25% of the chip idle) while keeping the MFMA:LDS-byte ratio high.
// Staging: global_load_lds_dwordx4 (1 KiB per wave-instruction, LDS image lane-linear), the
// bank-conflict swizzle applied on the SOURCE address and on the read (cdna_hip_programming.md
// §5.4 rule 21); per-lane source pointers are computed once and advanced by k per stage.
// The MFMA is issued with the operands swapped (B-data as MFMA "A") so each lane's
// accumulator holds 4 consecutive n of one output row: 8-16 B vector stores.
//
// Split-K (wgrad: output 768x768..3072x768 but K = B*T = 16384 -> only 36..144 tiles): the
// K range is cut into `splitk` slices over blockIdx.y, each writing an fp32 partial slab; a
// second kernel sums the slabs in a fixed order (bitwise reproducible, no float atomics).
//
// Batching (attention) uses blockIdx.z with a two-level (outer, inner) stride per operand;
// causal modes skip/limit work for the triangular attention products.
#include "gemm_common.h"

#include <cstdlib>

namespace rtdc {


// Per-column (mean, M2) of this block's output tile - the BatchNorm statistics of a
// convolution output computed in the GEMM epilogue instead of by a separate pass over the
// activation (values rounded to bf16 exactly as stored).  Each lane sums v and v^2 over its
// TM rows, an xor-shuffle tree sums the 16 lanes that share a column, the WM waves that
// share a column are added in LDS in fixed order, and the tile's (mean, M2) = (S/n,
// Q - S^2/n) (a 128/256-row tile keeps the one-pass cancellation small; tiles are then
// merged with Chan's formula by the BatchNorm finalize kernel).  Deterministic.
template <class CFG>
__device__ __forceinline__ void conv_tile_stats(const GemmArgs& a, const f32x4 (&acc)[CFG::TM][CFG::TN], float alpha,
                                                int m0, int n0, int wm, int wn, int lane, char* smem) {
  constexpr int TM = CFG::TM, TN = CFG::TN, WM = CFG::WM, BN = CFG::BN, BM = CFG::BM;
  float* sh = (float*)smem;  // [WM][BN][2]
  __syncthreads();          // staging buffers are free (the k-loop ended with a barrier)
  float s1[TN][4], s2[TN][4];
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) s1[j][r] = s2[j][r] = 0.f;
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int m = m0 + wm * (TM * 16) + i * 16 + (lane & 15);
    if (m >= a.M) continue;
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float v = bf2f(f2bf(acc[i][j][r] * alpha));
        s1[j][r] += v;
        s2[j][r] += v * v;
      }
  }
  // the 16 lanes of a column group: DPP row reduction (VALU only; the __shfl_xor tree was 128
  // ds_bpermute LDS round trips per lane per tile)
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      s1[j][r] = row16_sum(s1[j][r]);
      s2[j][r] = row16_sum(s2[j][r]);
    }
  if ((lane & 15) == 0) {
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int col = wn * (TN * 16) + j * 16 + 4 * (lane >> 4) + r;
        sh[(wm * BN + col) * 2] = s1[j][r];
        sh[(wm * BN + col) * 2 + 1] = s2[j][r];
      }
  }
  __syncthreads();
  const int tile = m0 / BM;
  const float n = (float)min(BM, a.M - m0);
  for (int col = threadIdx.x; col < BN; col += CFG::NT) {
    const int nn = n0 + col;
    if (nn >= a.N) continue;
    float S = 0.f, Q = 0.f;
    for (int w = 0; w < WM; ++w) {
      S += sh[(w * BN + col) * 2];
      Q += sh[(w * BN + col) * 2 + 1];
    }
    const float mean = S / n;
    a.stats_mean[(long long)tile * a.N + nn] = mean;
    a.stats_m2[(long long)tile * a.N + nn] = fmaxf(Q - S * mean, 0.f);
  }
}

// Per-column BatchNorm-backward partials of this block's output tile (GM 4), in a pass after
// the epilogue: each lane re-reads the bf16 gradient values it just stored (L2-hot), x (and
// y), one 16-column block at a time (`unroll 1`: the per-column constants and sums stay ~30
// registers - kept in registers across the epilogue they cost the 8-wave tiles a wave per SIMD,
// +0.9 ms on ResNet-18); the 16 lanes sharing a column and then the WM waves are added in fixed
// order -> stats_mean[tile][n] = sum g*mask, stats_m2 = sum g*mask*xhat.
template <class CFG, typename OutT>
__device__ __forceinline__ void bnb_tile_stats(const GemmArgs& a, const OutT* C, int m0, int n0, int wm, int wn,
                                               int lane, char* smem) {
  constexpr int TM = CFG::TM, TN = CFG::TN, WM = CFG::WM, BN = CFG::BN, BM = CFG::BM;
  float* sh = (float*)smem;  // [WM][BN][2]
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this lane's C stores are complete
  __syncthreads();                                  // staging buffers are free
#pragma unroll 1
  for (int j = 0; j < TN; ++j) {
    const int n = n0 + wn * (TN * 16) + j * 16 + 4 * (lane >> 4);
    float s1[4] = {0.f, 0.f, 0.f, 0.f}, s2[4] = {0.f, 0.f, 0.f, 0.f};
    if (n < a.N) {  // (N % 8 == 0: the lane's 4 columns are all in range)
      float mu[4], rs[4], ka[4], kb[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        mu[r] = a.bnb_mean[n + r];
        rs[r] = a.bnb_rstd[n + r];
        // the forward's ReLU argument t = fma(x, rstd*gamma, beta - mean*rstd*gamma) (bn_apply_kernel)
        ka[r] = rs[r] * a.bnb_gamma[n + r];
        kb[r] = a.bnb_beta[n + r] - mu[r] * ka[r];
      }
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int m = m0 + wm * (TM * 16) + i * 16 + (lane & 15);
        if (m >= a.M) continue;
        const long long off = (long long)m * a.ldc + n;
        float gv[4], xv[4], yv[4];
        load4<OutT>(C + off, gv);  // as stored (bf16)
        load4<bf16_t>((const bf16_t*)a.bnb_x + off, xv);
        if (a.bnb_y) load4<bf16_t>((const bf16_t*)a.bnb_y + off, yv);  // (wave-uniform)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const bool on = a.bnb_y ? yv[r] > 0.f : fmaf(xv[r], ka[r], kb[r]) > 0.f;
          const float gm = on ? gv[r] : 0.f;
          s1[r] += gm;
          s2[r] += gm * (xv[r] - mu[r]) * rs[r];
        }
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      s1[r] = row16_sum(s1[r]);
      s2[r] = row16_sum(s2[r]);
    }
    if ((lane & 15) == 0) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int col = wn * (TN * 16) + j * 16 + 4 * (lane >> 4) + r;
        sh[(wm * BN + col) * 2] = s1[r];
        sh[(wm * BN + col) * 2 + 1] = s2[r];
      }
    }
  }
  __syncthreads();
  const int tile = m0 / BM;
  for (int col = threadIdx.x; col < BN; col += CFG::NT) {
    const int nn = n0 + col;
    if (nn >= a.N) continue;
    float S = 0.f, Q = 0.f;
    for (int w = 0; w < WM; ++w) {
      S += sh[(w * BN + col) * 2];
      Q += sh[(w * BN + col) * 2 + 1];
    }
    a.stats_mean[(long long)tile * a.N + nn] = S;
    a.stats_m2[(long long)tile * a.N + nn] = Q;
  }
}

// outstanding glds allowed at an NS-stage wait: `ahead` later stages of LPS loads each
// (wave-uniform; immediates only)
template <int LPS>
__device__ __forceinline__ void wait_stages(int ahead) {
  if (ahead >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * LPS) : "memory");
  else if (ahead == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(LPS) : "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// NS = 2: two LDS stages, every k-step ends with vmcnt(0) + __syncthreads() (two blocks/CU).
// NS = 3 / 4 (the implicit-GEMM convolutions' thin tiles, one block/CU): NS-1 k-tiles in flight
// across each barrier - at step t the wait retires only tile t (counted vmcnt, never 0 before
// the last steps), a raw s_barrier publishes it, then tile t+NS-1 is issued into the stage that
// step t-1 read (every wave passed the barrier after consuming its fragments: WAR-safe).  With
// 9-18 k-tiles per tile and 128-256 x 64 outputs the 2-stage loop exposed one global-load
// latency per k-step (the N = 64 convolutions ran at 300-430 TF).
template <class CFG, bool AK, bool BKM, typename OutT, int GM = 0, int NS = 2>
__global__ __launch_bounds__(CFG::NT, NS == 2 ? 2 : 1) void gemm_bf16_kernel(GemmArgs a) {
  using namespace gemm;
  constexpr int BM = CFG::BM, BN = CFG::BN, TM = CFG::TM, TN = CFG::TN, WN = CFG::WN, NW = CFG::NW;
  static_assert(NS >= 2 && NS <= 4, "2..4 LDS stages");
  __shared__ __attribute__((aligned(16))) char smem[NS * CFG::STAGE];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;

  // XCD-aware, bijective remap of the flat tile id (cdna_hip_programming.md §5, T1) followed
  // by GROUP_M super-rows so consecutive tiles on one XCD share A row-panels in its L2.
  const int tiles_m = (a.M + BM - 1) / BM, tiles_n = (a.N + BN - 1) / BN;
  const int nwg = tiles_m * tiles_n;
  const int bid = blockIdx.x;
  int wgid = bid;
  if (nwg > 8) {
    const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  }
  constexpr int GROUP_M = 8;
  const int group = wgid / (GROUP_M * tiles_n);
  const int first_m = group * GROUP_M;
  const int gsize = min(tiles_m - first_m, GROUP_M);
  const int tm = first_m + (wgid % (GROUP_M * tiles_n)) % gsize;
  const int tn = (wgid % (GROUP_M * tiles_n)) / gsize;
  const int m0 = tm * BM, n0 = tn * BN;

  if (a.causal == 1 && n0 > m0 + BM - 1) return;  // tile entirely above the diagonal

  const int z = blockIdx.z;
  const int zo = z / a.batch_inner, zi = z % a.batch_inner;
  const bf16_t* A = a.A + zo * a.sA0 + zi * a.sA1;
  const bf16_t* B = a.B + zo * a.sB0 + zi * a.sB1;
  const long long coff = zo * a.sC0 + zi * a.sC1;

  int kb = 0, ke = a.K;
  if (a.causal == 2) ke = min(a.K, m0 + BM);
  if (a.causal == 3) kb = (m0 / BK) * BK;
  if (a.splitk > 1) {
    const int ktiles = (ke - kb) / BK;
    const int per = (ktiles + a.splitk - 1) / a.splitk;
    const int s = blockIdx.y;
    const int k_lo = kb + s * per * BK;
    ke = min(ke, k_lo + per * BK);
    kb = k_lo;
  }
  const int nt = ke > kb ? (ke - kb) / BK : 0;

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // GM 1: gathered A (implicit-GEMM convolution); 3: the same plus fused BatchNorm statistics;
  // 4: gathered A plus fused BatchNorm-backward statistics of the output (bnb_*)
  constexpr bool GATHER_A = GM == 1 || GM == 3 || GM == 4;
  using SA = std::conditional_t<GATHER_A, ConvStagerK<BM, NW>, Stager<AK, BM, NW>>;
  using SB = std::conditional_t<GM == 2, ConvStagerMN<BN, NW>, Stager<BKM, BN, NW>>;
  SA sa;
  SB sb;
  if constexpr (GATHER_A) sa.init(a, A, a.M, m0, wave, lane);
  else sa.init(A, a.lda, a.M, m0, wave, lane);
  if constexpr (GM == 2) sb.init(a, B, a.N, n0, wave, lane);
  else sb.init(B, a.ldb, a.N, n0, wave, lane);

  // stage s: A tile at smem + s*STAGE, B tile right after it
#define BUF_A(s) (smem + (s) * CFG::STAGE)
#define BUF_B(s) (smem + (s) * CFG::STAGE + CFG::A_BYTES)

  if constexpr (NS == 2) {
    if (nt > 0) {
      sa.issue(kb, BUF_A(0), wave);
      sb.issue(kb, BUF_B(0), wave);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
  } else {
#pragma unroll
    for (int s = 0; s < NS - 1; ++s)
      if (s < nt) {
        sa.issue(kb + s * BK, BUF_A(s), wave);
        sb.issue(kb + s * BK, BUF_B(s), wave);
      }
  }
  for (int t = 0; t < nt; ++t) {
    int cur;
    if constexpr (NS == 2) {
      cur = t & 1;
      if (t + 1 < nt) {
        sa.issue(kb + (t + 1) * BK, BUF_A(cur ^ 1), wave);
        sb.issue(kb + (t + 1) * BK, BUF_B(cur ^ 1), wave);
      }
    } else {
      constexpr int LPS = (BM / 8) / NW + (BN / 8) / NW;  // glds per thread per stage
      cur = t % NS;
      wait_stages<LPS>(min(NS - 2, nt - 1 - t));
      asm volatile("" ::: "memory");
      __builtin_amdgcn_s_barrier();
      if (t + NS - 1 < nt) {
        const int st = (t + NS - 1) % NS;
        sa.issue(kb + (t + NS - 1) * BK, BUF_A(st), wave);
        sb.issue(kb + (t + NS - 1) * BK, BUF_B(st), wave);
      }
    }
    const char* tA = BUF_A(cur);
    const char* tB = BUF_B(cur);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      typename Frag<AK>::T fa[TM];
      typename Frag<BKM>::T fb[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) fa[i] = load_fragx<AK, BM>(tA, wm * (TM * 16) + i * 16, ks, lane);
#pragma unroll
      for (int j = 0; j < TN; ++j) fb[j] = load_fragx<BKM, BN>(tB, wn * (TN * 16) + j * 16, ks, lane);
      if constexpr (!AK || !BKM) lgkm_wait0();  // asm transposing reads (gemm_common.h)
      bf16x8 va[TM], vb[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) va[i] = fval(fa[i]);
#pragma unroll
      for (int j = 0; j < TN; ++j) vb[j] = fval(fb[j]);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vb[j], va[i], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
    if constexpr (NS == 2) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
  }
#undef BUF_A
#undef BUF_B
  const float alpha = a.alpha_dev ? a.alpha * *a.alpha_dev : a.alpha;

  if (a.splitk > 1) {
    // raw fp32 partial slab (alpha applied); epilogue happens in the reduce kernel
    float* W = a.ws + (long long)blockIdx.y * a.M * a.N;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int m = m0 + wm * (TM * 16) + i * 16 + (lane & 15);
      if (m >= a.M) continue;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int n = n0 + wn * (TN * 16) + j * 16 + 4 * (lane >> 4);
        if (n >= a.N) continue;
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = acc[i][j][r] * alpha;
        store4<float>(W + (long long)m * a.N + n, v);
      }
    }
    return;
  }

  // ---- epilogue: lane holds C[m][n..n+3] ----
  OutT* C = (OutT*)a.C + coff;
  const OutT* Cin = a.Cin ? (const OutT*)a.Cin + coff : nullptr;
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int m = m0 + wm * (TM * 16) + i * 16 + (lane & 15);
    if (m >= a.M) continue;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = n0 + wn * (TN * 16) + j * 16 + 4 * (lane >> 4);
      if (n >= a.N) continue;
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = acc[i][j][r] * alpha;
      if (a.bias_type == 1) {
        float bb[4];
        load4<bf16_t>((const bf16_t*)a.bias + n, bb);
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] += bb[r];
      } else if (a.bias_type == 2) {
        float bb[4];
        load4<float>((const float*)a.bias + n, bb);
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] += bb[r];
      }
      const long long off = (long long)m * a.ldc + n;
      if (Cin && a.beta != 0.f) {
        float c[4];
        load4<OutT>(Cin + off, c);
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] += a.beta * c[r];
      }
      if (a.act == 1) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = fmaxf(v[r], 0.f);
      } else if (a.act == 2) {
        store4<bf16_t>(a.aux_out + off, v);
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = gelu_tanh(v[r]);
      } else if (a.act == 5) {
        float g[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = gelu_tanh_and_grad(v[r], g[r]);
        store4<bf16_t>(a.aux_out + off, g);
      } else if (a.act == 3 || a.act == 4 || a.act == 6) {
        float h[4];
        load4<bf16_t>(a.aux_in + off, h);
#pragma unroll
        for (int r = 0; r < 4; ++r)
          v[r] *= (a.act == 6) ? h[r] : (a.act == 3) ? gelu_tanh_grad(h[r]) : (h[r] > 0.f ? 1.f : 0.f);
      }
      store4<OutT>(C + off, v);
    }
  }
  if constexpr (GM == 3) conv_tile_stats<CFG>(a, acc, alpha, m0, n0, wm, wn, lane, smem);
  if constexpr (GM == 4) bnb_tile_stats<CFG>(a, C, m0, n0, wm, wn, lane, smem);
}

// out[m][n] = sum_s ws[s][m][n] (+ beta * Cin[m][n]).  A block owns 64 float4 column groups
// and W = min(16, S) waves: wave w sums slices w, w+W, w+2W, ... (four loads in flight), and the
// W partials are added in wave order - a fixed order for a given S, so the result is bitwise
// reproducible.  (One thread summing all S slices serially was latency-bound at S = 170-512:
// the single-tile weight gradients of the 64-channel convolutions.)
template <typename OutT>
__global__ __launch_bounds__(1024) void splitk_reduce_kernel(const float* __restrict__ ws, int S, int M, int N,
                                                            OutT* C, const OutT* Cin, int ldc, float beta) {
  __shared__ f32x4 part[16][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, W = blockDim.x >> 6;
  const long long total4 = (long long)M * N / 4;
  const long long q = (long long)blockIdx.x * 64 + lane;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  if (q < total4) {
    const long long MN = (long long)M * N;
    const float* p = ws + q * 4;
    int s = w;
    for (; s + 3 * W < S; s += 4 * W) {
      const f32x4 x0 = *(const f32x4*)(p + (long long)s * MN);
      const f32x4 x1 = *(const f32x4*)(p + (long long)(s + W) * MN);
      const f32x4 x2 = *(const f32x4*)(p + (long long)(s + 2 * W) * MN);
      const f32x4 x3 = *(const f32x4*)(p + (long long)(s + 3 * W) * MN);
      acc += x0;
      acc += x1;
      acc += x2;
      acc += x3;
    }
    for (; s < S; s += W) acc += *(const f32x4*)(p + (long long)s * MN);
  }
  part[w][lane] = acc;
  __syncthreads();
  if (w != 0 || q >= total4) return;
  f32x4 v4 = part[0][lane];
  for (int i = 1; i < W; ++i) v4 += part[i][lane];
  const long long e = q * 4;
  const int m = (int)(e / N), n = (int)(e % N);
  float v[4] = {v4[0], v4[1], v4[2], v4[3]};
  const long long off = (long long)m * ldc + n;
  if (Cin && beta != 0.f) {
    float c[4];
    load4<OutT>(Cin + off, c);
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] += beta * c[r];
  }
  store4<OutT>(C + off, v);
}

template <typename OutT>
static void launch_splitk_reduce(const GemmArgs& a, hipStream_t st) {
  const long long total4 = (long long)a.M * a.N / 4;
  const int W = a.splitk < 16 ? a.splitk : 16;
  hipLaunchKernelGGL(splitk_reduce_kernel<OutT>, dim3((unsigned)((total4 + 63) / 64)), dim3(64 * W), 0, st, a.ws,
                     a.splitk, a.M, a.N, (OutT*)a.C, (const OutT*)a.Cin, a.ldc, a.beta);
}

using Cfg128x128 = TileCfg<128, 128, 2, 2>;
using Cfg256x128 = TileCfg<256, 128, 4, 2>;
using Cfg128x256 = TileCfg<128, 256, 2, 4>;
using Cfg256x256 = TileCfg<256, 256, 2, 4>;
using Cfg256x64 = TileCfg<256, 64, 4, 1>;   // narrow outputs (Cout = 64 convolutions)
using Cfg64x256 = TileCfg<64, 256, 1, 4>;   // short outputs (Cout = 64 weight gradients)
using Cfg256x64w8 = TileCfg<256, 64, 8, 1>; // narrow outputs, 8 waves of 32x64 (RTDC_CONV64_W8)
using Cfg128x128w8 = TileCfg<128, 128, 4, 2>; // 8 waves of 32x64 (RTDC_CONV128_W8)
using Cfg64x256w8 = TileCfg<64, 256, 1, 8>;   // 8 waves of 64x32 (RTDC_CONV64WG_W8)

template <class CFG>
static inline long long ntiles(const GemmArgs& a) {
  return (long long)((a.M + CFG::BM - 1) / CFG::BM) * ((a.N + CFG::BN - 1) / CFG::BN);
}

template <class CFG, bool AK, bool BKM, typename OutT, int GM = 0, int NS = 2>
static void launch_cfg(const GemmArgs& a, int batch, hipStream_t st) {
  dim3 grid((unsigned)ntiles<CFG>(a), a.splitk > 1 ? a.splitk : 1, batch), block(CFG::NT);
  hipLaunchKernelGGL((gemm_bf16_kernel<CFG, AK, BKM, OutT, GM, NS>), grid, block, 0, st, a);
}

// LDS stages of the implicit-GEMM convolution kernels (RTDC_CONV_NS=2|3|4; see the NS note at
// gemm_bf16_kernel)
// The N <= 64 implicit-GEMM convolutions (ResNet stem / layer1) on 256x64 tiles of 8 waves
// (32x64 each: 97-102 VGPRs, four waves per SIMD with two blocks per CU) instead of 4 waves of
// 64x64 (169 registers, two waves per SIMD): ResNet-18 8.74 vs 8.88 ms/step
// (profiles/conv_w8_ab_r3.txt).  RTDC_CONV64_W8=0 restores the 4-wave tiles.
static bool conv64_w8() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("RTDC_CONV64_W8");
    v = (e && e[0] == '0') ? 0 : 1;
  }
  return v == 1;
}
// The N > 64 implicit-GEMM convolutions (forward, dgrad, weight gradient) on 128x128 tiles of 8
// waves (32x64 each) instead of 4 (64x64): ResNet-18 8.56 vs 8.71 ms/step
// (profiles/conv_w8_ab_r3.txt).  RTDC_CONV128_W8=0 restores the 4-wave tiles.
static bool conv128_w8() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("RTDC_CONV128_W8");
    v = (e && e[0] == '0') ? 0 : 1;
  }
  return v == 1;
}
// RTDC_CONV64WG_W8=1: the Cout = 64 weight gradients on 64x256 tiles of 8 waves (64x32 each)
static bool conv64wg_w8() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("RTDC_CONV64WG_W8");
    v = (e && e[0] == '1') ? 1 : 0;
  }
  return v == 1;
}

static int conv_stages() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("RTDC_CONV_NS");
    v = (e && e[0] >= '2' && e[0] <= '4') ? e[0] - '0' : 2;
  }
  return v;
}
template <class CFG, bool AK, bool BKM, typename OutT, int GM>
static void launch_conv(const GemmArgs& a, hipStream_t st) {
  switch (conv_stages()) {
    case 3: launch_cfg<CFG, AK, BKM, OutT, GM, 3>(a, 1, st); break;
    case 4: launch_cfg<CFG, AK, BKM, OutT, GM, 4>(a, 1, st); break;
    default: launch_cfg<CFG, AK, BKM, OutT, GM, 2>(a, 1, st); break;
  }
}

template <bool AK, bool BKM, typename OutT>
static void launch_layout(const GemmArgs& a, int cfg, int batch, hipStream_t st) {
  switch (cfg) {
    case 1: launch_cfg<Cfg256x128, AK, BKM, OutT>(a, batch, st); break;
    case 2: launch_cfg<Cfg128x256, AK, BKM, OutT>(a, batch, st); break;
    case 3: launch_cfg<Cfg256x256, AK, BKM, OutT>(a, batch, st); break;
    case 4: launch_cfg<Cfg256x64, AK, BKM, OutT>(a, batch, st); break;
    case 5: launch_cfg<Cfg64x256, AK, BKM, OutT>(a, batch, st); break;
    default: launch_cfg<Cfg128x128, AK, BKM, OutT>(a, batch, st); break;
  }
}

}  // namespace rtdc

using namespace rtdc;

// Choose the tile configuration.  Measured on MI355X (benchmarks/gemm_bench.py --sweep,
// random operands, GPT-2 / Llama shapes, profiles/gemm_bench_8ph.jsonl): the 256x256
// 8-wave counted-vmcnt kernel (cfg 6) beats the 128x128 2-stage kernel on every MN-major-B
// product (dgrad +13..39 %, wgrad +10..18 % once >= 24 output tiles exist for split-K), and
// on forward products when the grid quantises well onto 256 CUs or K is long (fc 887 vs 808,
// mlp_proj 1020 vs 934, lm_head 872 vs 768 TF); at 2.25 waves and K = 768 (qkv) the 128x128
// tile with 2 blocks/CU still wins (764 vs 703).
static int pick_cfg(const GemmArgs& a, int batch, bool a_kmajor, bool b_kmajor) {
  if (a.tile_cfg >= 0) return a.tile_cfg;
  if (batch == 1 && a.causal == 0) {
    // 64-wide outputs (Cout = 64 convolutions): a 128x128 tile would idle half its MFMAs
    if (a.N <= 64 && a.M >= 256) return 4;
    if (a.M <= 64 && a.N >= 128) return 5;
    if (a.M >= 256 && a.N >= 192) {
      // 8-wave counted-vmcnt kernel, 256x256 (cfg 6) or 256x192 (cfg 7) tiles: the 192-wide
      // tile when it quantises onto the 256 CUs clearly better (N = 768: 256 vs 192 tiles)
      auto eff_of = [](long long t) { return (double)t / (double)(((t + 255) / 256) * 256); };
      const long long t6 = (long long)((a.M + 255) / 256) * ((a.N + 255) / 256);
      const long long t7 = (long long)((a.M + 255) / 256) * ((a.N + 191) / 192);
      // measured (profiles/gemm_bench_v4_256x192.jsonl): the 192-wide tile wins for forward
      // products with one wave of tiles or long K (mlp_proj 1132 vs 983 TF, attn_proj 700 vs
      // 654), for short-K dgrads (+2..4 %); it loses on long-K dgrad (LM head 943 vs 1059)
      // and qkv forward (737 vs 778 for 128x128), where per-tile efficiency outweighs the
      // better wave quantisation
      const bool better7 = eff_of(t7) > eff_of(t6) + 0.05;
      // (re-measured with the asm transposing reads and the persistent form,
      // profiles/gemm_bench_v5_asm_tr_persist.jsonl: qkv forward 840 TF at 256x192 vs 728 at
      // 128x128 - the better-quantised 192-wide tile now wins for every forward product)
      const bool use7 = better7 && ((a_kmajor && b_kmajor) || (a_kmajor && !b_kmajor && a.K <= 4096));
      const long long t = use7 ? t7 : t6;
      const double eff = use7 ? eff_of(t7) : eff_of(t6);
      const int big = use7 ? 7 : 6;
      if (a_kmajor && b_kmajor) {
        if (t >= 1024 || eff >= 0.95 || a.K >= 2048) return big;
      } else if (a_kmajor) {
        if (t >= 128) return big;
      } else {
        if (t >= 24) return big;
      }
    }
  }
  return 0;
}

extern "C" int rtdc_colsum(const void* X, int M, int N, int ld, float* ws, int nblk, float* out, int accumulate,
                           int is_bf16, hipStream_t st);
extern "C" int rtdc_colsum_rows(const float* ws, int W, int D, float* tmp, float* out, int accumulate,
                                hipStream_t st);
extern "C" int rtdc_gemm8_launch(const GemmArgs* args, int a_kmajor, int b_kmajor, int out_fp32, int bn,
                                 hipStream_t st);
extern "C" int rtdc_gemm8p_launch(const GemmArgs* args, int a_kmajor, int b_kmajor, int out_fp32, int bn,
                                  hipStream_t st);
extern "C" int rtdc_gemm4_launch(const GemmArgs* args, int a_kmajor, int b_kmajor, int out_fp32, hipStream_t st);
extern "C" int rtdc_gemm4b_launch(const GemmArgs* args, int a_kmajor, int b_kmajor, int out_fp32, hipStream_t st);
extern "C" int rtdc_gemm8b_launch(const GemmArgs* args, int a_kmajor, int b_kmajor, int out_fp32, hipStream_t st);

// cfg 12 / 13: the one-barrier-per-K-tile kernels (gemm4b.hip: 4 waves, any operand layout;
// gemm8b.hip: 8 waves, forward layout).  RTDC_GEMM4B_AUTO: 2 (default) cfg 12 for K-major x
// K-major products with K >= 2048 (Llama-3-8B step -0.7 %); 1 cfg 13 for every forward-layout
// product up to 8 rounds of 256x256 tiles (faster in isolation, but the GPT-2 step ran 4 %
// slower: profiles/gemm_8wave_one_barrier_r4.txt); 0 neither.  RTDC_GEMM4B=1 routes every
// 8-wave 256x256 choice (cfg 6 / 8) to cfg 12 (A/B).
static int g_gemm4b_auto = -1;
static int gemm4b_mode() {  // 0 off, 1 cfg 13 for the forward layout, 2 cfg 12 for K >= 2048 forwards
  if (g_gemm4b_auto < 0) {
    const char* e = getenv("RTDC_GEMM4B_AUTO");
    g_gemm4b_auto = e ? atoi(e) : 2;
  }
  return g_gemm4b_auto;
}
static bool gemm4b_auto() { return gemm4b_mode() == 1; }
extern "C" int rtdc_gemm4b_auto_set(int v) {
  const int old = gemm4b_mode();
  if (v >= 0) g_gemm4b_auto = v;
  return old;
}
static int g_gemm4b = -1;
static bool gemm4b_enabled() {
  if (g_gemm4b < 0) {
    const char* e = getenv("RTDC_GEMM4B");
    g_gemm4b = (e && e[0] == '1') ? 1 : 0;
  }
  return g_gemm4b == 1;
}
extern "C" int rtdc_gemm4b_set(int v) {
  const int old = gemm4b_enabled() ? 1 : 0;
  if (v >= 0) g_gemm4b = v ? 1 : 0;
  return old;
}

// cfg 10: the 4-wave 256x256 kernel (gemm_8ph.hip gemm4_kernel, 128x128 per wave).
// RTDC_GEMM4W=1 routes the 8-wave 256x256 choices (cfg 6 / 8) to it.
static bool gemm4w_enabled() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("RTDC_GEMM4W");
    v = (e && e[0] == '1') ? 1 : 0;
  }
  return v == 1;
}

// RTDC_GEMM_FEW_ROWS=0 keeps pick_cfg's choice for M <= 4096 products (A/B of pick_cfg_few_rows).
static bool few_rows_enabled() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("RTDC_GEMM_FEW_ROWS");
    v = (e && e[0] == '0') ? 0 : 1;
  }
  return v == 1;
}

// Persistent 8-wave kernel (gemm_8ph.hip gemm8p_kernel) for plain-K (no split-K) products with
// more tiles than CUs: the next tile's loads and this tile's epilogue overlap MFMA work instead
// of costing a prologue/epilogue bubble per tile (K = 768 GPT-2 products: 12 K-tiles per tile).
// K-major x K-major only: the MN-major variants exceed 256 VGPRs with the persistent state.
// RTDC_GEMM_PERSIST=0 disables it.
static bool persist_enabled() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("RTDC_GEMM_PERSIST");
    v = (e && e[0] == '0') ? 0 : 1;
  }
  return v == 1;
}

// Split-K for long-K / few-tile products (weight gradients): choose the slice count s that
// minimises a wave-quantised time model
//     T(s) = ceil(tiles*s / slots) * ceil(ktiles / s) * t_ktile  +  s * M*N * 8 B / HBM
// (slots = concurrent blocks on 256 CUs, t_ktile = one block's time per 64-deep k-tile, the
// second term the fp32 slab write + reduce read).  Grid sizes just past a multiple of the
// slots cost a whole extra wave (e.g. 27 tiles x 19 slices = 513 blocks = 3 waves of 1-block-
// per-CU work), so the quantisation term matters more than "about 2 blocks per CU".
static int pick_splitk(const GemmArgs& a, long long tiles, int slots = 512, double t_ktile_us = 1.8) {
  const int ktiles = a.K / gemm::BK;
  if (!a.ws || tiles >= 200 || ktiles < 32) return 1;
  const double slab_us = (double)a.M * a.N * 8.0 / 4.0e6;  // bytes / (4 TB/s) in us
  int best = 1;
  double best_t = 1e30;
  // (up to 1024 slices: a single-tile product - the 64-channel convolutions' weight gradients
  // over 0.8-3.2 M pixels - needs ~512 of them to fill the chip)
  for (int s = 1; s <= 1024; ++s) {
    if (ktiles / s < 8 || (long long)s * a.M * a.N > a.ws_elems) break;
    const long long waves = (tiles * s + slots - 1) / slots;
    const double t = (double)waves * (double)((ktiles + s - 1) / s) * t_ktile_us + (s > 1 ? s * slab_us : 0.0);
    if (t < best_t - 1e-9) {
      best_t = t;
      best = s;
    }
  }
  return best;
}

// RTDC_GEMM_FEW_ROWS_X=0 drops pick_cfg_few_rows' measured exceptions (A/B)
static bool few_rows_exceptions() {
  const char* e = getenv("RTDC_GEMM_FEW_ROWS_X");
  return !(e && e[0] == '0');
}

// Few-row-tile products (M <= 4096: Llama-3-8B at 2048 tokens per GPU) with a K-major A and a
// bf16 output: choose among the 8-wave tiles by a wave-quantised time model instead of the
// M = 16384 rules of pick_cfg.  At M = 2048 an N = 4096 output is only 128 tiles of 256x256 -
// half of the 256 CUs idle - and the right answer differs per product: 256x128 tiles (one full
// round), 256x256 tiles with two K slices, or 256x192.  Per-K-tile block times (us) from
// benchmarks/gemm_bench.py --set llama --sweep (profiles/gemm_llama_sweep_r4.jsonl):
//   256x256  1.74 (1.58 persistent, > 256 tiles)   256x192  1.42 fwd / 1.37 dgrad
//   256x128  1.10 fwd / 1.16 dgrad
// Returns the cfg (6 / 7 / 11 / 12 / 13, or 0 under the measured exceptions below).
static int pick_cfg_few_rows(const GemmArgs& a, bool b_kmajor, bool can_split) {
  const int kt = a.K / gemm::BK, tm = (a.M + 255) / 256;
  const double slab_us = (double)a.M * a.N * 8.0 / 4.0e6;
  auto est = [&](int bn, double t_k) {
    const long long tiles = (long long)tm * ((a.N + bn - 1) / bn);
    double best = 1e30;
    for (int s = 1; s <= (can_split ? 8 : 1); ++s) {
      if (s > 1 && (kt / s < 8 || tiles >= 200 || (long long)s * a.M * a.N > a.ws_elems)) break;
      const long long waves = (tiles * s + 255) / 256;
      const double t = (double)waves * ((kt + s - 1) / s) * t_k + (s > 1 ? s * slab_us : 0.0);
      best = t < best ? t : best;
    }
    return best;
  };
  const long long t6 = (long long)tm * ((a.N + 255) / 256);
  // Measured exceptions to the model (Llama-3-8B at 2048 tokens, gemm_bench --sweep,
  // profiles/r6/llama_few_rows_cfg_r6.txt):
  //  * one partial round of 256x256 tiles on the forward layout (qkv: 192 tiles, K = 4096): the
  //    one-barrier 8-wave kernel runs at ~1.25 us per K-tile there - 1287 TF vs 1145 at 256x192;
  //  * at most half a round (o-proj: 128 tiles, K = 4096, both layouts): 128x128 tiles with two
  //    blocks per CU - 1052 / 1015 TF vs 958 / 930 at 256x128 (not past K = 4096: the down
  //    projection's K = 14336 forward loses on them, 1164 vs 1280).
  if (few_rows_exceptions()) {
    if (b_kmajor && t6 > 128 && t6 <= 256 && gemm4b_mode() != 0) return 13;
    if (t6 <= 128 && a.K <= 4096) return 0;
  }
  const double e6 = est(256, b_kmajor && t6 > 256 ? 1.58 : 1.74);
  const double e7 = (b_kmajor || a.K <= 4096) ? est(192, b_kmajor ? 1.42 : 1.37) : 1e30;
  const double e11 = est(128, b_kmajor ? 1.10 : 1.16);
  // cfg 13 (gemm8b.hip, 8 waves, one barrier per K-tile): ~1.45 us per 256x256 K-tile on the
  // forward layout (profiles/gemm_8wave_one_barrier_r4.txt); forward layout only
  const double e13 = b_kmajor && gemm4b_mode() == 1 ? est(256, 1.45) : 1e30;
  if (e13 < e6 && e13 < e7 && e13 < e11) return 13;
  const double e12 = b_kmajor && gemm4b_mode() == 2 ? est(256, 1.52) : 1e30;
  if (e12 < e6 && e12 < e7 && e12 < e11) return 12;
  if (e11 < e6 && e11 < e7) return 11;
  return e7 < e6 ? 7 : 6;
}

// RTDC_GEMM_TAIL=0 disables the tail split of rtdc_gemm_bf16 (read per call: A/B in one process).
static bool tail_split_enabled() {
  const char* e = getenv("RTDC_GEMM_TAIL");
  return !(e && e[0] == '0');
}

// cs_rows_out (optional): with cs_ws set and cs_out null the column sums are DEFERRED - the
// 8-wave gelu-backward epilogue leaves its partial rows in cs_ws, *cs_rows_out = their count
// (0: this kernel choice wrote none; the caller reduces C itself).
extern "C" int rtdc_gemm_bf16(const GemmArgs* args, int a_kmajor, int b_kmajor, int out_fp32, int batch,
                              hipStream_t stream, int* cs_rows_out) {
  if (cs_rows_out) *cs_rows_out = 0;
  GemmArgs a = *args;
  if (a.K % gemm::BK != 0 || a.M % 8 != 0 || a.N % 8 != 0) return 1;
  int cfg = pick_cfg(a, batch, a_kmajor, b_kmajor);
  if (a.tile_cfg < 0 && few_rows_enabled() && batch == 1 && a.causal == 0 && a_kmajor && !out_fp32 &&
      a.M >= 256 && a.M <= 4096 && a.N >= 128 && a.K >= 8 * gemm::BK) {
    const bool plain = a.act == 0 && a.bias_type == 0 && !a.cs_out && !a.cs_ws;
    cfg = pick_cfg_few_rows(a, b_kmajor, plain && a.ws != nullptr);
  }
  if ((cfg == 6 || cfg == 8) && a.tile_cfg < 0 && gemm4w_enabled()) cfg = 10;
  if ((cfg == 6 || cfg == 8) && a.tile_cfg < 0 && gemm4b_enabled()) cfg = 12;
  // RTDC_GEMM4B_AUTO=1: the one-barrier 8-wave kernel for the forward layout up to 8 rounds of
  // 256x256 tiles (beyond that - the LM head's 12608 tiles - the persistent 8-wave kernel hides
  // the per-tile prologue better)
  if (cfg >= 6 && cfg <= 9 && a.tile_cfg < 0 && gemm4b_auto() && a_kmajor && b_kmajor && batch == 1 &&
      (long long)((a.M + 255) / 256) * ((a.N + 255) / 256) <= 2048)
    cfg = 13;
  if ((cfg == 6 || cfg == 8) && a.tile_cfg < 0 && gemm4b_mode() == 2 && a_kmajor && b_kmajor && a.K >= 2048) cfg = 12;
  if (cfg == 13 && !(a_kmajor && b_kmajor)) cfg = 6;  // the 8-wave one-barrier kernel: forward layout only
  // Tail split: a forward-layout product on 256x256 tiles whose last round of tiles fills at
  // most half the 256 CUs (Llama-3-8B gate|up at 2048 tokens: 8 x 112 = 896 tiles = 3.5 rounds)
  // runs its whole rounds as one launch and the remaining column tiles on 256x128 tiles - twice
  // the blocks, one full round at ~1.10 us per K-tile instead of half a round at ~1.52 - as a
  // second (model: 389 -> 362 us for gate|up).  Same per-element K order in both kernels.
  if (a.tile_cfg < 0 && (cfg == 6 || cfg == 8 || cfg == 12) && batch == 1 && a.causal == 0 && a_kmajor &&
      b_kmajor && !out_fp32 && !a.cs_out && !a.cs_ws && !a.Cin && !a.aux_in && !a.aux_out && a.act == 0 &&
      !a.stats_mean && !a.bnb_x &&
      a.N % 256 == 0 && a.K >= 16 * gemm::BK && tail_split_enabled()) {
    const int tm = (a.M + 255) / 256, tn = a.N / 256;
    if (tm <= 256 && 256 % tm == 0 && (long long)tm * tn > 256) {
      const int tail_cols = tn % (256 / tm);
      if (tail_cols > 0 && tail_cols * tm <= 128) {
        const int n1 = (tn - tail_cols) * 256;
        // both halves accumulate every element over the full K in one pass (no split-K slabs:
        // ws = null makes pick_splitk return 1), so the result is bitwise the unsplit kernel's
        GemmArgs h = a;
        h.N = n1;
        h.tile_cfg = cfg;
        h.ws = nullptr;
        int rc = rtdc_gemm_bf16(&h, 1, 1, 0, 1, stream, nullptr);
        if (rc) return rc;
        GemmArgs t = a;
        t.N = a.N - n1;
        t.tile_cfg = 11;
        t.ws = nullptr;
        t.B = a.B + (long long)n1 * a.ldb;
        t.C = (bf16_t*)a.C + n1;
        if (a.bias) t.bias = (const char*)a.bias + (long long)n1 * (a.bias_type == 2 ? 4 : 2);
        return rtdc_gemm_bf16(&t, 1, 1, 0, 1, stream, nullptr);
      }
    }
  }
  // the 8-wave kernels write bf16 outputs 16 B at a time through tile-relative 32-bit buffer
  // offsets (gemm_8ph.hip tile_epilogue)
  const uintptr_t al = (uintptr_t)a.C | (uintptr_t)a.Cin | (uintptr_t)a.aux_in | (uintptr_t)a.aux_out |
                       (uintptr_t)a.bias;
  if (cfg >= 6 && cfg <= 13 && !out_fp32 && ((al & 15) != 0 || (a.ldc & 7) != 0 || a.ldc >= (1 << 22))) cfg = 0;
  // ... and take no residual with an input-gradient activation (their epilogue then has no
  // conditional load; the models never ask for this combination)
  if (cfg >= 6 && cfg <= 13 && (a.act == 3 || a.act == 4 || a.act == 6) && a.Cin && a.beta != 0.f) cfg = 0;
  a.splitk = 1;
  // split-K when the output tiles cannot fill the chip and K is long (weight gradients)
  const bool plain = a.act == 0 && a.bias_type == 0 && a.causal == 0 && batch == 1;
  long long tiles = cfg == 3 ? ntiles<Cfg256x256>(a) : cfg == 1 ? ntiles<Cfg256x128>(a)
                  : cfg == 2 ? ntiles<Cfg128x256>(a) : cfg == 4 ? ntiles<Cfg256x64>(a)
                  : cfg == 5 ? ntiles<Cfg64x256>(a) : ntiles<Cfg128x128>(a);
  // cfg 11: the 8-wave kernel on 256x128 tiles (bf16 output, K-major A)
  if (cfg == 11 && (out_fp32 || !a_kmajor)) cfg = 6;
  const bool big = cfg >= 6 && cfg <= 13;  // counted-vmcnt pipelines (gemm_8ph.hip, gemm4b.hip, gemm8b.hip)
  const int bn = (cfg == 7 || cfg == 9) ? 192 : cfg == 11 ? 128 : 256;
  if (big) {
    if (batch != 1 || a.causal != 0) return 1;
    tiles = (long long)((a.M + 255) / 256) * ((a.N + bn - 1) / bn);
  }
  // 8-phase 256x256: one 512-thread block per CU; 128x128: two per CU; ~1.8 us per k-tile either way
  if (plain && (cfg <= 7 || (cfg >= 10 && cfg <= 13)))
    a.splitk = cfg >= 6 ? pick_splitk(a, tiles, 256, cfg == 7 ? 1.35 : cfg == 11 ? 1.0 : cfg == 12 ? 1.52 : cfg == 13 ? 1.45 : 1.8)
                        : pick_splitk(a, tiles);
  if (cfg == 10) {
    const int rc = rtdc_gemm4_launch(&a, a_kmajor, b_kmajor, out_fp32, stream);
    if (rc) return rc;
  } else if (cfg == 12) {
    const int rc = rtdc_gemm4b_launch(&a, a_kmajor, b_kmajor, out_fp32, stream);
    if (rc) return rc;
  } else if (cfg == 13) {
    const int rc = rtdc_gemm8b_launch(&a, a_kmajor, b_kmajor, out_fp32, stream);
    if (rc) return rc;
  } else if (big) {
    // cfg 8 / 9 force the persistent form; 6 / 7 take it automatically where it applies
    const bool persist = (cfg == 8 || cfg == 9) || (cfg != 11 && persist_enabled() && a.splitk == 1 && a_kmajor &&
                                                    b_kmajor && tiles > 256 && a.K >= 2 * gemm::BK);
    const int rc = persist ? rtdc_gemm8p_launch(&a, a_kmajor, b_kmajor, out_fp32, bn, stream)
                           : rtdc_gemm8_launch(&a, a_kmajor, b_kmajor, out_fp32, bn, stream);
    if (rc) return rc;
  } else if (out_fp32) {
    if (a_kmajor && b_kmajor) launch_layout<true, true, float>(a, cfg, batch, stream);
    else if (a_kmajor && !b_kmajor) launch_layout<true, false, float>(a, cfg, batch, stream);
    else if (!a_kmajor && !b_kmajor) launch_layout<false, false, float>(a, cfg, batch, stream);
    else launch_layout<false, true, float>(a, cfg, batch, stream);
  } else {
    if (a_kmajor && b_kmajor) launch_layout<true, true, bf16_t>(a, cfg, batch, stream);
    else if (a_kmajor && !b_kmajor) launch_layout<true, false, bf16_t>(a, cfg, batch, stream);
    else if (!a_kmajor && !b_kmajor) launch_layout<false, false, bf16_t>(a, cfg, batch, stream);
    else launch_layout<false, true, bf16_t>(a, cfg, batch, stream);
  }
  if (a.splitk > 1) {
    if (out_fp32) launch_splitk_reduce<float>(a, stream);
    else launch_splitk_reduce<bf16_t>(a, stream);
  }
  if (!a.cs_out && a.cs_ws && cs_rows_out && big && (a.act == 3 || a.act == 6) && !out_fp32 && a.splitk == 1) {
    const int W = ((a.M + 255) / 256) * (bn == 256 ? 2 : 4);
    if ((long long)W * a.N <= a.cs_ws_elems) *cs_rows_out = W;
  }
  if (a.cs_out) {
    // column sums of C: the 8-wave gelu-backward epilogue left one partial row per (row tile,
    // wave row) in cs_ws; anything else reduces C itself
    const int tiles_m = (a.M + 255) / 256;
    if (big && (a.act == 3 || a.act == 6) && !out_fp32) {
      const int W = tiles_m * (bn == 256 ? 2 : 4);
      if ((long long)(W + 64) * a.N > a.cs_ws_elems) return 1;
      const int rc = rtdc_colsum_rows(a.cs_ws, W, a.N, a.cs_ws + (long long)W * a.N, a.cs_out, 0, stream);
      if (rc) return rc;
    } else {
      const int nblk = a.M / 64 < 1 ? 1 : (a.M / 64 > 256 ? 256 : a.M / 64);
      if ((long long)(nblk + 64) * a.N > a.cs_ws_elems) return 1;
      const int rc = rtdc_colsum(a.C, a.M, a.N, a.ldc, a.cs_ws, nblk, a.cs_out, 0, out_fp32 ? 0 : 1, stream);
      if (rc) return rc;
    }
  }
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

// ---- 3x3 / stride-1 / pad-1 convolution weight gradient with input reuse ----------------
// dW[co][kh][kw][ci] = sum over pixels p of dy[p][co] * x[p + (kh-1, kw-1)][ci] (NHWC bf16,
// fp32 out).  The implicit GEMM (mode 2) gathers im2col(X) per 256-column tile: X is read once
// per tap (9x) plus dY once per column tile - 1.24 GB for a 56x56x64 layer at batch 256, which
// ran the Cout = 64 weight gradients at ~380 TF (156 us).  Here a block owns a 64(co) x 64(ci)
// output tile for ALL nine taps and walks chunks of RC = 64 / W whole image rows: per chunk it
// stages dY (64 pixels x 64 co) and the X halo the nine taps need ((RC+2) x (W+2) pixels x 64 ci,
// zero rows / columns outside the image) once, and the taps are row offsets into that halo
// (the transposing LDS read takes one row address per lane, so a shifted tap costs nothing).
// 12 waves: wave (kh, quadrant) accumulates taps (kh, 0..2) of a 32x32 quadrant.  Staging is
// global_load_lds into three LDS buffers (two chunks in flight under this chunk's MFMAs,
// counted vmcnt, one barrier per chunk; the padding slots load from a zero line); the
// transposing reads use the asm protocol of common.h (the builtin form drains vmcnt).  Blocks
// split the chunks; fp32 partial slabs are summed by splitk_reduce_kernel (fixed order).
namespace wg3 {
constexpr int kThreads = 768;
// KP pixels per chunk (64 or 128): NSL 16-B staging slots per thread, LDS bytes per buffer
template <int KP> struct Cfg {
  static constexpr int NSL = KP == 128 ? 4 : 3, kDyBytes = KP * 128, kBuf = NSL * kThreads * 16;
  static constexpr int kMaxHalo = (NSL * kThreads - KP * 8) / 8;
};
__device__ __forceinline__ int swz(int row) { return (row & 7) ^ (((row >> 3) & 1) << 2); }
__device__ __forceinline__ int off(int row, int ch) {  // 128-B rows of 8 16-B chunks, swizzled
  return row * 128 + ((ch ^ swz(row)) << 4);
}
struct Args {
  const bf16_t* x;
  const bf16_t* dy;
  float* out;
  int B, H, W, Cin, Cout, RC, cpi, nchunks, per, halo;
  long long slab;
};
// 16 columns c0.. of rows r_lo / r_hi of an image as a 16x16x32 MFMA operand (lane l: column
// c0 + (l&15), rows 8(l>>4) + j): two transposing reads, retired by the caller's lgkm wait
__device__ __forceinline__ TrPair frag(const char* img, int r_lo, int r_hi, int c0, int lane) {
  const int p = lane & 3, c = (c0 >> 3) + (p >> 1), b = (p & 1) << 3;
  TrPair f;
  f.lo = ds_tr16(img + off(r_lo, c) + b);
  f.hi = ds_tr16(img + off(r_hi, c) + b);
  return f;
}
}  // namespace wg3

template <int KP>
__global__ __launch_bounds__(768, 1) void conv3x3_wgrad_kernel(wg3::Args a) {
  using namespace wg3;
  constexpr int NSL = Cfg<KP>::NSL, kDyBytes = Cfg<KP>::kDyBytes, kBuf = Cfg<KP>::kBuf, KS = KP / 32, NDY = KP * 8;
  __shared__ __attribute__((aligned(16))) char smem[3 * kBuf];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int kh = wv >> 2, quad = wv & 3, co_s = (quad >> 1) * 32, ci_s = (quad & 1) * 32;
  const int ntc = a.Cin / 64;
  const int co0 = (blockIdx.x / ntc) * 64, ci0 = (blockIdx.x % ntc) * 64;
  const int c_begin = blockIdx.y * a.per, c_end = min(a.nchunks, c_begin + a.per);
  const int W2 = a.W + 2, npieces = NDY + a.halo * 8, npx = a.RC * a.W;
  // this lane's operand rows (chunk pixels k; chunk-invariant): dY row k, halo row of tap (kh, 0)
  const int q4 = (lane & 15) >> 2, g = lane >> 4;
  int kr[KS][2], hb[KS][2];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int k = ks * 32 + 8 * g + 4 * h + q4;
      kr[ks][h] = k;
      hb[ks][h] = k < npx ? (k / a.W + kh) * W2 + k % a.W : 0;  // (padding pixels: dY row is 0)
    }
  // this thread's three staging slots (slot i -> LDS byte 16 i of a buffer), chunk-invariant
  // but for the image / row origin: source row offset from the chunk's first row, column,
  // channel offset (logical chunk of the swizzled slot); dr = -2: padding (zero line)
  int s_dr[NSL], s_w[NSL], s_c[NSL];
#pragma unroll
  for (int j = 0; j < NSL; ++j) {
    const int i = tid + j * kThreads;
    s_dr[j] = -2;
    s_w[j] = 0;
    s_c[j] = 0;
    if (i < NDY) {
      const int r = i >> 3;
      if (r < npx) {
        s_dr[j] = r / a.W;
        s_w[j] = r % a.W;
        s_c[j] = ((i & 7) ^ swz(r)) * 8;
      }
    } else if (i < npieces) {
      const int r = (i - NDY) >> 3, hr = r / W2;
      s_dr[j] = hr - 1;
      s_w[j] = r - hr * W2 - 1;
      s_c[j] = ((i & 7) ^ swz(r)) * 8;
    }
  }
  auto issue = [&](int ch, char* buf) {
    const int b = ch / a.cpi, h0 = (ch - b * a.cpi) * a.RC;
#pragma unroll
    for (int j = 0; j < NSL; ++j) {
      const int i = tid + j * kThreads, hh = h0 + s_dr[j], ww = s_w[j];
      const bool ok = s_dr[j] != -2 && (unsigned)hh < (unsigned)a.H && (unsigned)ww < (unsigned)a.W;
      const long long pix = (long long)(b * a.H + hh) * a.W + ww;
      const bf16_t* src = !ok ? (const bf16_t*)g_conv_zero
                          : i < NDY ? a.dy + pix * a.Cout + co0 + s_c[j]
                                    : a.x + pix * a.Cin + ci0 + s_c[j];
      __builtin_amdgcn_global_load_lds((const void*)src, LDS_PTR(buf + (j * kThreads + wv * 64) * 16), 16, 0, 0);
    }
  };
  f32x4 acc[3][2][2];
#pragma unroll
  for (int t = 0; t < 3; ++t)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[t][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int n = c_end - c_begin;
  if (n > 0) issue(c_begin, smem);
  if (n > 1) issue(c_begin + 1, smem + kBuf);
  for (int t = 0; t < n; ++t) {
    // this chunk's three loads are in; the next chunk's may still be in flight
    if (t + 1 < n)
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NSL) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // every thread's slots landed; buffer (t+2)%3 was last read in step t-1
    if (t + 2 < n) issue(c_begin + t + 2, smem + ((t + 2) % 3) * kBuf);
    const char* buf = smem + (t % 3) * kBuf;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      TrPair af[2], bfr[3][2];
#pragma unroll
      for (int fm = 0; fm < 2; ++fm) af[fm] = frag(buf, kr[ks][0], kr[ks][1], co_s + 16 * fm, lane);
#pragma unroll
      for (int kw = 0; kw < 3; ++kw)
#pragma unroll
        for (int fn = 0; fn < 2; ++fn)
          bfr[kw][fn] = frag(buf + kDyBytes, hb[ks][0] + kw, hb[ks][1] + kw, ci_s + 16 * fn, lane);
      lgkm_wait0();
      bf16x8 A[2], Bv[3][2];
#pragma unroll
      for (int fm = 0; fm < 2; ++fm) A[fm] = tr_use(af[fm]);
#pragma unroll
      for (int kw = 0; kw < 3; ++kw)
#pragma unroll
        for (int fn = 0; fn < 2; ++fn) Bv[kw][fn] = tr_use(bfr[kw][fn]);
#pragma unroll
      for (int kw = 0; kw < 3; ++kw)
#pragma unroll
        for (int fm = 0; fm < 2; ++fm)
#pragma unroll
          for (int fn = 0; fn < 2; ++fn)
            acc[kw][fm][fn] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[fm], Bv[kw][fn], acc[kw][fm][fn], 0, 0, 0);
    }
  }
  // C[m = co][n = ci]: lane holds rows 4(l>>4) + r of column l & 15
  float* out = a.out + (long long)blockIdx.y * a.slab;
  const int K9 = 9 * a.Cin;
#pragma unroll
  for (int kw = 0; kw < 3; ++kw)
#pragma unroll
    for (int fm = 0; fm < 2; ++fm)
#pragma unroll
      for (int fn = 0; fn < 2; ++fn)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int co = co0 + co_s + 16 * fm + 4 * g + r, ci = ci0 + ci_s + 16 * fn + (lane & 15);
          out[(long long)co * K9 + (kh * 3 + kw) * a.Cin + ci] = acc[kw][fm][fn][r];
        }
}

static bool conv3_wgrad_enabled() {
  static int v = -1;  // RTDC_CONV3_WGRAD=0: the implicit-GEMM weight gradient (A/B)
  if (v < 0) {
    const char* e = getenv("RTDC_CONV3_WGRAD");
    v = (e && e[0] == '0') ? 0 : 1;
  }
  return v == 1;
}

// mode-2 arguments of a 3x3 / stride 1 / pad 1 weight gradient -> conv3x3_wgrad_kernel (+ the
// split reduce); 1 = shape not taken (the caller runs the implicit GEMM)
static int launch_conv3x3_wgrad(const GemmArgs& ga, hipStream_t st) {
  const int H = ga.cv_H, W = ga.cv_W, Cin = ga.cv_C, Cout = ga.M;
  if (Cin % 64 || Cout % 64 || W < 1 || W > 64 || H < 1 || ga.lda != Cout) return 1;
  const int B = ga.cv_npix / (H * W);
  // 128-pixel chunks (half the barriers and staging rounds per pixel) when whole rows fill at
  // least 3/4 of them and the halo fits; else 64
  static int kp_env = -1;  // RTDC_CONV3_KP=128: 128-pixel chunks where they fit (A/B; default 64)
  if (kp_env < 0) {
    const char* e = getenv("RTDC_CONV3_KP");
    kp_env = (e && e[0] == '1') ? 128 : 64;
  }
  int KP = 128, RC = 128 / W;
  RC = RC < H ? RC : H;
  if (kp_env == 64 || RC * W * 4 < 3 * 128 || (RC + 2) * (W + 2) > wg3::Cfg<128>::kMaxHalo) {
    KP = 64;
    RC = 64 / W;
    RC = RC < H ? RC : H;
  }
  const int halo = (RC + 2) * (W + 2);
  if (KP == 64 && halo > wg3::Cfg<64>::kMaxHalo) return 1;
  wg3::Args a{};
  a.x = (const bf16_t*)ga.B;
  a.dy = (const bf16_t*)ga.A;
  a.B = B; a.H = H; a.W = W; a.Cin = Cin; a.Cout = Cout; a.RC = RC; a.halo = halo;
  a.cpi = (H + RC - 1) / RC;
  a.nchunks = B * a.cpi;
  a.slab = (long long)Cout * 9 * Cin;
  const int tiles = (Cout / 64) * (Cin / 64);
  // measured per conv (ResNet-18, profiles/resnet18_r3_conv3_wgrad): 56x56x64 84 vs 146 us,
  // 28x28x128 82 vs 121 us, but 14x14x256 92 vs 83 us and 7x7x512 92 vs 91 us - the implicit
  // GEMM's 128x128 tiles already fill the chip there, so it keeps the products of > 4 tiles
  if (tiles > 4) return 1;
  int S = 256 / tiles;
  S = S < 1 ? 1 : S;
  S = S < a.nchunks ? S : a.nchunks;
  if (S > 1 && (!ga.ws || (long long)S * a.slab > ga.ws_elems))
    S = ga.ws ? (int)(ga.ws_elems / a.slab) : 1;
  S = S < 1 ? 1 : S;
  a.per = (a.nchunks + S - 1) / S;
  S = (a.nchunks + a.per - 1) / a.per;
  a.out = S > 1 ? ga.ws : (float*)ga.C;
  if (KP == 128)
    hipLaunchKernelGGL(conv3x3_wgrad_kernel<128>, dim3(tiles, S), dim3(wg3::kThreads), 0, st, a);
  else
    hipLaunchKernelGGL(conv3x3_wgrad_kernel<64>, dim3(tiles, S), dim3(wg3::kThreads), 0, st, a);
  if (S > 1) {
    GemmArgs r = ga;
    r.N = 9 * Cin;
    r.ldc = 9 * Cin;
    r.splitk = S;
    r.Cin = nullptr;
    r.beta = 0.f;
    launch_splitk_reduce<float>(r, st);
  }
  return 0;
}

// Implicit-GEMM convolution products on the same MFMA kernel (see ConvStagerK / ConvStagerMN):
//   mode 1: C[npix][N] (bf16) = im2col(X)[npix][K] . B[N][K]^T     conv forward / stride-1 dgrad
//   mode 2: C[M][N]   (fp32) = A[K=npix][M]^T . im2col(X)[npix][N] weight gradient (split-K)
extern "C" int rtdc_conv_gemm(const GemmArgs* args, int mode, hipStream_t stream) {
  GemmArgs a = *args;
  // C a multiple of 64 (one tap per k tile) or a divisor of 64 that is a multiple of 8 (16-B
  // chunks never straddle a tap: the space-to-depth stem, C = 16)
  const bool c_ok = a.cv_C % 64 == 0 || (a.cv_C % 8 == 0 && 64 % a.cv_C == 0);
  if (!c_ok || a.cv_npix >= (1 << 24) || a.K % gemm::BK != 0 || a.N % 8 != 0) return 1;
  if (mode == 2 && a.M % 8 != 0) return 1;  // mode 1: rows (pixels) are clamped + masked, any count
  if ((long long)a.cv_H * a.cv_W * a.cv_C * ((long long)a.cv_npix / ((long long)a.cv_Ho * a.cv_Wo)) >= (1LL << 31))
    return 1;
  a.splitk = 1;
  if (mode == 1) {
    if (a.M != a.cv_npix) return 1;
    // stats rows are per BM-row tile: 256 (256x64 tiles) or 128
    if (a.bnb_x) {
      // BatchNorm-backward statistics of the (stride-1 dgrad) output: 8-wave tiles only
      if (!a.stats_mean || !a.stats_m2 || !a.bnb_mean || !a.bnb_rstd || !a.bnb_gamma || !a.bnb_beta) return 1;
      if (a.N <= 64) launch_cfg<Cfg256x64w8, true, true, bf16_t, 4>(a, 1, stream);
      else launch_cfg<Cfg128x128w8, true, true, bf16_t, 4>(a, 1, stream);
    } else if (a.stats_mean) {
      if (a.N <= 64 && conv64_w8()) launch_cfg<Cfg256x64w8, true, true, bf16_t, 3>(a, 1, stream);
      else if (a.N <= 64) launch_conv<Cfg256x64, true, true, bf16_t, 3>(a, stream);
      else if (conv128_w8()) launch_cfg<Cfg128x128w8, true, true, bf16_t, 3>(a, 1, stream);
      else launch_conv<Cfg128x128, true, true, bf16_t, 3>(a, stream);
    } else {
      if (a.N <= 64 && conv64_w8()) launch_cfg<Cfg256x64w8, true, true, bf16_t, 1>(a, 1, stream);
      else if (a.N <= 64) launch_conv<Cfg256x64, true, true, bf16_t, 1>(a, stream);
      else if (conv128_w8()) launch_cfg<Cfg128x128w8, true, true, bf16_t, 1>(a, 1, stream);
      else launch_conv<Cfg128x128, true, true, bf16_t, 1>(a, stream);
    }
  } else if (mode == 2) {
    if (a.K < a.cv_npix || a.stats_mean) return 1;
    if (conv3_wgrad_enabled() && a.cv_KW == 3 && a.N == 9 * a.cv_C && a.cv_stride == 1 && a.cv_pad == 1 &&
        a.cv_Ho == a.cv_H && a.cv_Wo == a.cv_W && launch_conv3x3_wgrad(a, stream) == 0)
      return hipGetLastError() == hipSuccess ? 0 : 2;
    const bool narrow = a.M <= 64;
    a.splitk = pick_splitk(a, narrow ? ntiles<Cfg64x256>(a) : ntiles<Cfg128x128>(a), conv_stages() > 2 ? 256 : 512);
    if (narrow && conv64wg_w8()) launch_cfg<Cfg64x256w8, false, false, float, 2>(a, 1, stream);
    else if (narrow) launch_conv<Cfg64x256, false, false, float, 2>(a, stream);
    else if (conv128_w8()) launch_cfg<Cfg128x128w8, false, false, float, 2>(a, 1, stream);
    else launch_conv<Cfg128x128, false, false, float, 2>(a, stream);
    if (a.splitk > 1) launch_splitk_reduce<float>(a, stream);
  } else {
    return 1;
  }
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

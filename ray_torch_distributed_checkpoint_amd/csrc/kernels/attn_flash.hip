// Fused causal flash attention (forward + backward) for gfx950, bf16 in / fp32 accumulate.
//
// Reads Q, K, V in place from the packed QKV activations [B, T, (H + 2*Hkv) * Dh] written by
// the c_attn GEMM (GQA: q-head h uses kv-head h / (H/Hkv)) and never materialises the
// T x T score matrix.  v_mfma_f32_16x16x32_bf16 everywhere; every product is laid out so
// the accumulator of one MFMA is the B operand of the next with no data movement
// (cdna_hip_programming.md §3 "An accumulator tile as the next MFMA's operand"): the score
// tile is computed transposed (D[key][q]) so a lane owns one query row and its P values feed
// the P.V MFMA directly; the k-order permutation this implies (key = 32s + 16(j>>2) + 4g +
// (j&3) for element j of lane group g) is reproduced on the other operand by reading V / dO
// / Q / K tiles with the transposing LDS read ds_read_b64_tr_b16 (4 consecutive rows x 16
// columns per 16-lane group).
//
//   fwd     : block = 64 query rows (4 waves x 16) of one (b, h); K/V tiles of 64 keys
//             streamed through LDS by global_load_lds; online softmax in the log2 domain;
//             writes O and the row log-sum-exp.
//   bwd_dkdv: block = 64 keys (4 waves x 16) of one (b, kv-head); loops over the query
//             blocks at or after the diagonal and over the q-heads of the GQA group; keeps
//             dK/dV in registers - no atomics.
//   bwd_dq  : block = 64 query rows; loops over key blocks up to the diagonal.  Recomputing
//             P here instead of accumulating dQ with float atomics keeps the backward
//             bitwise reproducible (MI355X_MICROARCH.md §Global float atomics).
//   delta   : D[b,h,t] = sum_d dO * O (the softmax-backward row term), computed by bwd_dq
//             in its prologue (bwd_dq runs first); delta_kernel is the standalone form.
// Requires T % 64 == 0 and Dh in {64, 128}.
//
// Pipelining (all three loops): the streamed tiles (K/V for fwd and dQ; Q, dO and the 64
// LSE / delta values of a query block for dK/dV) go through an NS-slot LDS ring with NS-1
// tiles in flight.  Every streamed byte arrives by global_load_lds; the operands a wave keeps
// in registers are loaded - and waited for - before the loop, so no ordinary load sits
// between a DMA and its wait (hipcc waits vmcnt(0) at the first use of an ordinary load while
// a DMA is in flight: cdna_hip_programming.md §5 "Pipelining across barriers").  A step ends
// with a counted `s_waitcnt vmcnt(n)` that retires exactly the next tile (n = the DMA
// instructions of the tiles issued after it) and a raw s_barrier (a __syncthreads() would
// drain the DMA queue).  The tile of step j+NS-1 is issued at the top of step j into the slot
// that step j-1 read, which every wave has left: its reads completed (lgkmcnt(0)) before the
// barrier that closed step j-1.  All LDS is one __shared__ array.
// NS (ring slots) is chosen at launch (fa_ns below): LDS per block grows with NS and sets how
// many blocks share a CU, so deeper rings trade occupancy for DMA depth.
#include "common.h"

#include <cstdlib>

namespace rtdc {
namespace fa {

constexpr int BQ = 64, BKV = 64, NT = 256;
constexpr float LOG2E = 1.4426950408889634f;

struct Args {
  const bf16_t* qkv;  // [B, T, W]
  bf16_t* out;        // [B, T, H*Dh]
  float* lse;         // [B*H, T] row log-sum-exp of the scaled scores, base 2 (log2 domain)
  const bf16_t* dout; // [B, T, H*Dh]
  float* delta;       // [B*H, T] (written by bwd_dq, read by bwd_dkdv)
  bf16_t* dqkv;       // [B, T, W]
  int B, T, H, Hkv;
  float scale;
  int xcd_remap;  // 1: the blocks of one head share an XCD (and its L2); 2: + heavy blocks first
                  // across all the XCD's heads
  int diag;       // timing-only builds (wrong results): bit 1 skips the loop's DMA waits
  // optional [B*T/16][W] fp32: per 16-row group, the column sums of the bf16 dQ / dK / dV rows
  // the backward kernels store (the qkv projection's bias gradient, reduced later without
  // re-reading dqkv: ops/gemm.py offer_colsum_partials)
  float* cs_ws;
  // GQA head split of dK/dV (qs > 1): block (key block, kv-head, qsub) covers q-heads
  // qsub*grp/qs .. +grp/qs of the group and writes its fp32 partial dK|dV rows to
  // part [qs][B*T][Hkv][2*Dh]; dkdv_reduce_kernel sums them in qsub order (deterministic)
  float* part;
  int qs;
  // delta already in `delta` (delta_kernel ran first): the dQ kernels compute their own copy for
  // their rows but do not store it - dK/dV may be reading it concurrently (rtdc_flash_bwd `which`)
  int delta_ready;
};

// column sums over a wave's 16 rows of its stored fragment values v (lane = row (lane & 15) x
// 4 columns 4g..4g+3 of each 16-column block d): one partial row per 16-row group
template <int DT>
__device__ __forceinline__ void wave_colsum16(const f32x4 (&v)[DT], float mul, float* dst, int lane) {
  const int g = lane >> 4;
#pragma unroll
  for (int d = 0; d < DT; ++d) {
    float s[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) s[r] = row16_sum(bf2f(f2bf(v[d][r] * mul)));
    if ((lane & 15) == 0) *(f32x4*)(dst + 16 * d + 4 * g) = f32x4{s[0], s[1], s[2], s[3]};
  }
}

// (block-in-head, head) of this workgroup
__device__ __forceinline__ void grid_pos(const Args& a, int& x, int& y) {
  if (a.xcd_remap) {
    xcd_grid(x, y, a.xcd_remap == 2);
  } else {
    x = blockIdx.x;
    y = blockIdx.y;
  }
}

// [64 rows][DH] bf16 LDS image, 16-B chunks XOR-swizzled per row by (row & 7) at Dh 64,
// 2 (row & 7) at Dh 128: bank-conflict-free for both readers - the ds_read_b128 row reads
// (frag_rows) and the 32-lane ds_read_b64_tr_b16 halves (frag_cols).  Round 4's (row >> 1) & 7
// (Dh 64) and (row & 15) (Dh 128) left every transposing read 2-way (two rows of a 32-lane half
// on one bank; round-5 PMC: 1.0-1.3 conflict cycles per LDS instruction in the flash kernels).
template <int DH>
__device__ __forceinline__ int toff(int row, int chunk) {
  if constexpr (DH == 64) return row * 128 + ((chunk ^ (row & 7)) << 4);
  else return row * 256 + ((chunk ^ ((row & 7) << 1)) << 4);
}

// global -> LDS copy of rows [r0, r0+64) (row stride ld elements, column offset col0) by all
// 4 waves: 1 KiB global_load_lds pieces, swizzle applied on the source address.
// DH/32 DMA instructions per wave.
// HOIST = false keeps the per-piece 64-bit address math: the Dh = 64 backward kernels measured
// faster that way (GPT-2 bwd 122 vs 129 us), the forward and the Dh = 128 kernels slower
// (GPT-2 fwd 44.7 vs 43.3 us, Llama bwd 268 vs 264 us)
template <int DH, bool HOIST = true>
__device__ __forceinline__ void stage(const bf16_t* base, long long ld, int r0, int col0, char* tile, int wave,
                                      int lane) {
  constexpr int RB = DH * 2, CPR = RB / 16, RPP = 1024 / RB, PIECES = 64 * RB / 1024, PPW = PIECES / 4;
  // wave-uniform tile origin (scalar math) + a 32-bit per-lane offset that does not depend on
  // r0 (the swizzle uses the tile-local row), so it is computed once per kernel, not per tile
  const bf16_t* tb = base + (long long)r0 * ld + col0;
#pragma unroll
  for (int ii = 0; ii < PPW; ++ii) {
    const int piece = wave * PPW + ii;
    const int row = piece * RPP + lane / CPR;
    const int pch = lane % CPR;
    int lch;
    if constexpr (DH == 64) lch = pch ^ (row & 7);
    else lch = pch ^ ((row & 7) << 1);
    const bf16_t* src = HOIST ? tb + (row * (int)ld + lch * 8) : base + (long long)(r0 + row) * ld + col0 + lch * 8;
    __builtin_amdgcn_global_load_lds((const void*)src, LDS_PTR(tile + piece * 1024), 16, 0, 0);
  }
}

// MFMA operand with rows = tile rows [R0, R0+16), k = columns 32*ks + 8g + j  (ds_read_b128)
template <int DH>
__device__ __forceinline__ bf16x8 frag_rows(const char* tile, int R0, int ks, int lane) {
  return *(const bf16x8*)(tile + toff<DH>(R0 + (lane & 15), ks * 4 + (lane >> 4)));
}

// MFMA operand with rows = tile columns [d0, d0+16), k = tile rows in the accumulator order
// kbase + 16(j>>2) + 4g + (j&3): two transposing reads (ds_read_b64_tr_b16) issued as asm
// (common.h ds_tr16 protocol: lgkm_wait0() then tr_use() before the MFMA reads them).
// Addressing: with the tile-row base kbase + 16h a multiple of 16,
// the swizzle term depends on the lane only, so each lane keeps one LDS offset per 16-column
// group d (tr_lane_offsets, computed once per kernel) and every read is that offset + the slot
// base (one add per d per step) + an immediate (kbase + 16h) * row bytes - instead of ~6 VALU of
// address arithmetic per transposing read in the VALU-bound softmax loop.
template <int DH>
__device__ __forceinline__ void tr_lane_offsets(uint32_t (&off)[DH / 16], int lane) {
  constexpr int RB = DH * 2;
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int lr = 4 * g + q, pb = p >> 1;
  const int f = DH == 64 ? (lr & 7) : ((lr & 7) << 1);
#pragma unroll
  for (int d = 0; d < DH / 16; ++d) off[d] = lr * RB + ((((2 * d) + pb) ^ f) << 4) + ((p & 1) << 3);
}

template <int OFF>
__device__ __forceinline__ bf16x4 ds_tr16_at(uint32_t addr) {
  bf16x4 r;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "i"(OFF) : "memory");
  return r;
}

// frag_cols_tr(tile, KB, 16 d, lane) given lane_addr = LDS address of the tile + off[d]
template <int DH, int KB>
__device__ __forceinline__ TrPair frag_cols_at(uint32_t lane_addr) {
  TrPair f;
  f.lo = ds_tr16_at<KB * DH * 2>(lane_addr);
  f.hi = ds_tr16_at<(KB + 16) * DH * 2>(lane_addr);
  return f;
}

__device__ __forceinline__ uint32_t lds_addr(const char* p) {
  return (uint32_t)(uintptr_t)((const __attribute__((address_space(3))) char*)p);
}

// 16-B global load of row `row` columns [c, c+8) -> bf16x8
__device__ __forceinline__ bf16x8 gload8(const bf16_t* p) { return *(const bf16x8*)p; }

// make the compiler retire an ordinary load HERE (its own s_waitcnt before this use), not at
// the first use inside the DMA loop
__device__ __forceinline__ void settle(const bf16x8& x) { asm volatile("" ::"v"(__builtin_bit_cast(f32x4, x))); }
__device__ __forceinline__ void settle(float x) { asm volatile("" ::"v"(x)); }

// s_waitcnt vmcnt(n) for a wave-uniform runtime n: rounded DOWN to an encoded immediate
// (waiting for more of the in-flight DMA than needed is always safe).
#define RTDC_FA_VM(n) asm volatile("s_waitcnt vmcnt(" #n ")" ::: "memory")
__device__ __forceinline__ void wait_vm_upto(int n) {
  if (n >= 18) RTDC_FA_VM(18);
  else if (n >= 16) RTDC_FA_VM(16);
  else if (n >= 10) RTDC_FA_VM(10);
  else if (n >= 9) RTDC_FA_VM(9);
  else if (n >= 8) RTDC_FA_VM(8);
  else if (n >= 5) RTDC_FA_VM(5);
  else if (n >= 4) RTDC_FA_VM(4);
  else RTDC_FA_VM(0);
}
#undef RTDC_FA_VM

// close a pipeline step: this wave's LDS reads retired, then the block barrier (raw: the
// DMA in flight stays in flight)
__device__ __forceinline__ void step_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// two accumulator tiles (rows 16*(2s) and 16*(2s+1)) -> one bf16 B operand
__device__ __forceinline__ bf16x8 pack_pair(const f32x4& a, const f32x4& b) {
  bf16x8 r;
  r[0] = (short)f2bf(a[0]); r[1] = (short)f2bf(a[1]); r[2] = (short)f2bf(a[2]); r[3] = (short)f2bf(a[3]);
  r[4] = (short)f2bf(b[0]); r[5] = (short)f2bf(b[1]); r[6] = (short)f2bf(b[2]); r[7] = (short)f2bf(b[3]);
  return r;
}

// 2^x as the bare v_exp_f32.  exp2f() adds a denormal-range fix-up around it (compare, select,
// add, select, ldexp: 6 VALU instead of 1 - measured in the loop's .s), and the softmax
// loops are VALU-issue bound; probabilities below 2^-126 only need to underflow to 0.
__device__ __forceinline__ float fexp2(float x) { return __builtin_amdgcn_exp2f(x); }

__device__ __forceinline__ f32x4 mfma(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// ------------------------------------------------------------------------------ forward
// DBV: output column blocks of 16 whose V fragments are read per batch (registers vs LDS
// latency per batch)
template <int DH, int NS, int DBV = 4>
__global__ __launch_bounds__(256, 2) void fwd_kernel(Args a) {
  constexpr int KS = DH / 32, DT = DH / 16, DB = DT < DBV ? DT : DBV, TILE = 64 * DH * 2, PER = DH / 16;
  __shared__ __attribute__((aligned(16))) char smem[2 * NS * TILE];  // K[NS], V[NS]
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4;
  const int nqb = a.T / BQ;
  int bx, bh;
  grid_pos(a, bx, bh);
  const int qb = nqb - 1 - bx;  // heaviest (longest causal prefix) blocks first
  const int b = bh / a.H, h = bh % a.H;
  const int grp = a.H / a.Hkv, kvh = h / grp;
  const int C = a.H * DH, W = C + 2 * a.Hkv * DH;
  const bf16_t* base = a.qkv + (long long)b * a.T * W;
  const int qcol = h * DH, kcol = C + kvh * DH, vcol = C + a.Hkv * DH + kvh * DH;
  const int q0w = qb * BQ + wave * 16;
  const int myq = q0w + (lane & 15);
  const float c = a.scale * LOG2E;
  uint32_t troff[DH / 16];
  tr_lane_offsets<DH>(troff, lane);
  const int nkb = qb + 1;

#define KT(s) (smem + (s) * TILE)
#define VT(s) (smem + (NS + (s)) * TILE)
#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (s < nkb) {
      stage<DH>(base, W, s * BKV, kcol, KT(s), wave, lane);
      stage<DH>(base, W, s * BKV, vcol, VT(s), wave, lane);
    }
  bf16x8 qf[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) qf[ks] = gload8(base + (long long)myq * W + qcol + ks * 32 + g * 8);
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) settle(qf[ks]);
  step_barrier();

  f32x4 o[DT];
#pragma unroll
  for (int d = 0; d < DT; ++d) o[d] = f32x4{0.f, 0.f, 0.f, 0.f};
  // row sums of P on the matrix core: an all-ones A operand makes every row of the P.V-shaped
  // product the sum over the keys, so lacc[*] = l for the lane's query row (no VALU adds, no
  // cross-lane reduction at the end; the sum is over the same bf16 P the numerator uses)
  f32x4 lacc = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 ones;
#pragma unroll
  for (int e = 0; e < 8; ++e) ones[e] = (short)0x3F80;
  float m = -INFINITY;

  for (int kb = 0; kb < nkb; ++kb) {
    const int cur = kb % NS;
    if (kb + NS - 1 < nkb) {
      const int nx = (kb + NS - 1) % NS;
      stage<DH>(base, W, (kb + NS - 1) * BKV, kcol, KT(nx), wave, lane);
      stage<DH>(base, W, (kb + NS - 1) * BKV, vcol, VT(nx), wave, lane);
    }
    const char* kt = KT(cur);
    const uint32_t vbase = lds_addr(VT(cur));
    f32x4 s[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      s[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) s[t] = mfma(frag_rows<DH>(kt, 16 * t, ks, lane), qf[ks], s[t]);
    }
    // causal mask on the diagonal block, running max of the raw scores (c > 0: scaling into the
    // log2 domain commutes with max, so it folds into one FMA per probability)
    float mx = -INFINITY;
    const bool diag = (kb == qb);
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = s[t][r];
        if (diag) {
          const int key = kb * BKV + 16 * t + 4 * g + r;
          if (key > myq) v = -INFINITY;
        }
        s[t][r] = v;
        mx = fmaxf(mx, v);
      }
    mx = max_rows4(mx);
    // lazy rescale: the running max moves (and O, l are rescaled) only when some row of the
    // wave would otherwise see probabilities above 2^8 - after the first key blocks the max
    // rarely grows that much, so the 4*DT+4 multiplies and the exp are skipped (wave-uniform)
    if (__any(mx * c > m + 8.f)) {
      const float mn = fmaxf(m, mx * c);
      const float alpha = fexp2(m - mn);
      m = mn;
#pragma unroll
      for (int r = 0; r < 4; ++r) lacc[r] *= alpha;
#pragma unroll
      for (int d = 0; d < DT; ++d)
#pragma unroll
        for (int r = 0; r < 4; ++r) o[d][r] *= alpha;
    }
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) s[t][r] = fexp2(fmaf(s[t][r], c, -m));
    const bf16x8 p0 = pack_pair(s[0], s[1]), p1 = pack_pair(s[2], s[3]);
    lacc = mfma(ones, p0, lacc);
    lacc = mfma(ones, p1, lacc);
#pragma unroll
    for (int d0 = 0; d0 < DT; d0 += DB) {
      TrPair vq[DB][2];
#pragma unroll
      for (int d = 0; d < DB; ++d) {
        const uint32_t la = vbase + troff[d0 + d];
        vq[d][0] = frag_cols_at<DH, 0>(la);
        vq[d][1] = frag_cols_at<DH, 32>(la);
      }
      lgkm_wait0();
#pragma unroll
      for (int d = 0; d < DB; ++d) {
        o[d0 + d] = mfma(tr_use(vq[d][0]), p0, o[d0 + d]);
        o[d0 + d] = mfma(tr_use(vq[d][1]), p1, o[d0 + d]);
      }
    }
    if (kb + 1 < nkb && !(a.diag & 1)) wait_vm_upto(PER * (min(kb + NS - 1, nkb - 1) - kb - 1));
    step_barrier();
  }
#undef KT
#undef VT
  const float l = lacc[0];
  const float inv = 1.f / l;
  bf16_t* orow = a.out + ((long long)b * a.T + myq) * C + h * DH;
#pragma unroll
  for (int d = 0; d < DT; ++d) {
    const uint2 v = make_uint2(pack_bf2(o[d][0] * inv, o[d][1] * inv), pack_bf2(o[d][2] * inv, o[d][3] * inv));
    *(uint2*)(orow + 16 * d + 4 * g) = v;
  }
  if (g == 0) a.lse[(long long)bh * a.T + myq] = m + log2f(l);
}

// Forward, software-pipelined across key tiles inside each wave: the S = K.Q MFMAs of tile kb+1
// are issued before the softmax of tile kb, so one wave's matrix work runs under its own
// exp/max/pack VALU instead of waiting for a co-resident wave to fill the gap (the serial
// S -> max -> exp -> P.V chain of fwd_kernel).  K therefore streams one tile further ahead than
// V: a 3-slot K ring and a 2-slot V ring (40 KiB, the same 4 blocks per CU as fwd_kernel's
// 2+2 slots would allow at this register count).  Step kb issues K(kb+2) and V(kb+1) - into the
// slots of K(kb-1) (read in step kb-2) and V(kb-1) (read in step kb-1) - and retires both
// before its closing barrier, so each DMA has one step to land, as in fwd_kernel.  Same math in
// the same order as fwd_kernel: bitwise equal output.
template <int DH>
__global__ __launch_bounds__(256, 2) void fwd3_kernel(Args a) {
  constexpr int KS = DH / 32, DT = DH / 16, DB = DT < 4 ? DT : 4, TILE = 64 * DH * 2;
  __shared__ __attribute__((aligned(16))) char smem[5 * TILE];  // K[3], V[2]
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4;
  const int nqb = a.T / BQ;
  int bx, bh;
  grid_pos(a, bx, bh);
  const int qb = nqb - 1 - bx;
  const int b = bh / a.H, h = bh % a.H;
  const int grp = a.H / a.Hkv, kvh = h / grp;
  const int C = a.H * DH, W = C + 2 * a.Hkv * DH;
  const bf16_t* base = a.qkv + (long long)b * a.T * W;
  const int qcol = h * DH, kcol = C + kvh * DH, vcol = C + a.Hkv * DH + kvh * DH;
  const int q0w = qb * BQ + wave * 16;
  const int myq = q0w + (lane & 15);
  const float c = a.scale * LOG2E;
  uint32_t troff[DH / 16];
  tr_lane_offsets<DH>(troff, lane);
  const int nkb = qb + 1;

#define KT(s) (smem + (s) * TILE)
#define VT(s) (smem + (3 + (s)) * TILE)
  stage<DH>(base, W, 0, kcol, KT(0), wave, lane);
  stage<DH>(base, W, 0, vcol, VT(0), wave, lane);
  if (nkb > 1) stage<DH>(base, W, BKV, kcol, KT(1), wave, lane);
  bf16x8 qf[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) qf[ks] = gload8(base + (long long)myq * W + qcol + ks * 32 + g * 8);
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) settle(qf[ks]);  // (retires the DMA above with it)
  step_barrier();

  auto scores = [&](const char* kt, f32x4 (&s)[4]) {
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      s[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) s[t] = mfma(frag_rows<DH>(kt, 16 * t, ks, lane), qf[ks], s[t]);
    }
  };
  f32x4 o[DT];
#pragma unroll
  for (int d = 0; d < DT; ++d) o[d] = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 lacc = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 ones;
#pragma unroll
  for (int e = 0; e < 8; ++e) ones[e] = (short)0x3F80;
  float m = -INFINITY;
  f32x4 s[4];
  scores(KT(0), s);

  for (int kb = 0; kb < nkb; ++kb) {
    if (kb + 2 < nkb) stage<DH>(base, W, (kb + 2) * BKV, kcol, KT((kb + 2) % 3), wave, lane);
    if (kb + 1 < nkb) stage<DH>(base, W, (kb + 1) * BKV, vcol, VT((kb + 1) & 1), wave, lane);
    // next tile's scores first: independent of this tile's softmax
    f32x4 sn[4];
    if (kb + 1 < nkb) scores(KT((kb + 1) % 3), sn);
    const uint32_t vbase = lds_addr(VT(kb & 1));
    float mx = -INFINITY;
    const bool diag = (kb == qb);
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = s[t][r];
        if (diag) {
          const int key = kb * BKV + 16 * t + 4 * g + r;
          if (key > myq) v = -INFINITY;
        }
        s[t][r] = v;
        mx = fmaxf(mx, v);
      }
    mx = max_rows4(mx);
    if (__any(mx * c > m + 8.f)) {
      const float mn = fmaxf(m, mx * c);
      const float alpha = fexp2(m - mn);
      m = mn;
#pragma unroll
      for (int r = 0; r < 4; ++r) lacc[r] *= alpha;
#pragma unroll
      for (int d = 0; d < DT; ++d)
#pragma unroll
        for (int r = 0; r < 4; ++r) o[d][r] *= alpha;
    }
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) s[t][r] = fexp2(fmaf(s[t][r], c, -m));
    const bf16x8 p0 = pack_pair(s[0], s[1]), p1 = pack_pair(s[2], s[3]);
    lacc = mfma(ones, p0, lacc);
    lacc = mfma(ones, p1, lacc);
#pragma unroll
    for (int d0 = 0; d0 < DT; d0 += DB) {
      TrPair vq[DB][2];
#pragma unroll
      for (int d = 0; d < DB; ++d) {
        const uint32_t la = vbase + troff[d0 + d];
        vq[d][0] = frag_cols_at<DH, 0>(la);
        vq[d][1] = frag_cols_at<DH, 32>(la);
      }
      lgkm_wait0();
#pragma unroll
      for (int d = 0; d < DB; ++d) {
        o[d0 + d] = mfma(tr_use(vq[d][0]), p0, o[d0 + d]);
        o[d0 + d] = mfma(tr_use(vq[d][1]), p1, o[d0 + d]);
      }
    }
    // step kb+1 reads K(kb+2) and V(kb+1), both issued at the top of this step
    if (kb + 1 < nkb && !(a.diag & 1)) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    step_barrier();
#pragma unroll
    for (int t = 0; t < 4; ++t) s[t] = sn[t];
  }
#undef KT
#undef VT
  const float l = lacc[0];
  const float inv = 1.f / l;
  bf16_t* orow = a.out + ((long long)b * a.T + myq) * C + h * DH;
#pragma unroll
  for (int d = 0; d < DT; ++d) {
    const uint2 v = make_uint2(pack_bf2(o[d][0] * inv, o[d][1] * inv), pack_bf2(o[d][2] * inv, o[d][3] * inv));
    *(uint2*)(orow + 16 * d + 4 * g) = v;
  }
  if (g == 0) a.lse[(long long)bh * a.T + myq] = m + log2f(l);
}

// Forward, 32 query rows per wave (block = 128 rows): every K fragment read from LDS feeds
// two S MFMAs and every V fragment two P.V MFMAs, halving LDS bytes per FLOP.  Same
// accumulator-as-operand layout and the same DMA ring as fwd_kernel.
template <int DH, int NS>
__global__ __launch_bounds__(256, 2) void fwd2_kernel(Args a) {
  constexpr int KS = DH / 32, DT = DH / 16, DB = DT < 4 ? DT : 4, TILE = 64 * DH * 2, QG = 2, BQ2 = 128, PER = DH / 16;
  __shared__ __attribute__((aligned(16))) char smem[2 * NS * TILE];  // K[NS], V[NS]
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4;
  const int nqb = a.T / BQ2;
  int bx, bh;
  grid_pos(a, bx, bh);
  const int qb = nqb - 1 - bx;  // heaviest (longest causal prefix) blocks first
  const int b = bh / a.H, h = bh % a.H;
  const int grp = a.H / a.Hkv, kvh = h / grp;
  const int C = a.H * DH, W = C + 2 * a.Hkv * DH;
  const bf16_t* base = a.qkv + (long long)b * a.T * W;
  const int qcol = h * DH, kcol = C + kvh * DH, vcol = C + a.Hkv * DH + kvh * DH;
  const int q0w = qb * BQ2 + wave * 32;  // this wave: rows [q0w, q0w + 32)
  int myq[QG];
#pragma unroll
  for (int qg = 0; qg < QG; ++qg) myq[qg] = q0w + 16 * qg + (lane & 15);
  const float c = a.scale * LOG2E;
  uint32_t troff[DH / 16];
  tr_lane_offsets<DH>(troff, lane);
  const int nkb = (qb + 1) * (BQ2 / BKV);

#define KT(s) (smem + (s) * TILE)
#define VT(s) (smem + (NS + (s)) * TILE)
#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (s < nkb) {
      stage<DH>(base, W, s * BKV, kcol, KT(s), wave, lane);
      stage<DH>(base, W, s * BKV, vcol, VT(s), wave, lane);
    }
  bf16x8 qf[QG][KS];
#pragma unroll
  for (int qg = 0; qg < QG; ++qg)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) qf[qg][ks] = gload8(base + (long long)myq[qg] * W + qcol + ks * 32 + g * 8);
#pragma unroll
  for (int qg = 0; qg < QG; ++qg)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) settle(qf[qg][ks]);
  step_barrier();

  f32x4 o[QG][DT];
  float m[QG], l[QG];
#pragma unroll
  for (int qg = 0; qg < QG; ++qg) {
    m[qg] = -INFINITY;
    l[qg] = 0.f;
#pragma unroll
    for (int d = 0; d < DT; ++d) o[qg][d] = f32x4{0.f, 0.f, 0.f, 0.f};
  }

  for (int kb = 0; kb < nkb; ++kb) {
    const int cur = kb % NS;
    if (kb + NS - 1 < nkb) {
      const int nx = (kb + NS - 1) % NS;
      stage<DH>(base, W, (kb + NS - 1) * BKV, kcol, KT(nx), wave, lane);
      stage<DH>(base, W, (kb + NS - 1) * BKV, vcol, VT(nx), wave, lane);
    }
    // keys of this tile all after this wave's last row: nothing to add (barriers still run)
    if (kb * BKV <= q0w + 31) {
      const char* kt = KT(cur);
      const uint32_t vbase = lds_addr(VT(cur));
      f32x4 sc[QG][4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
#pragma unroll
        for (int qg = 0; qg < QG; ++qg) sc[qg][t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          const bf16x8 kf = frag_rows<DH>(kt, 16 * t, ks, lane);
#pragma unroll
          for (int qg = 0; qg < QG; ++qg) sc[qg][t] = mfma(kf, qf[qg][ks], sc[qg][t]);
        }
      }
      const bool diag = (kb * BKV + BKV - 1 > q0w);
      bf16x8 pp[QG][2];
#pragma unroll
      for (int qg = 0; qg < QG; ++qg) {
        float mx = -INFINITY;
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float v = sc[qg][t][r];
            if (diag) {
              const int key = kb * BKV + 16 * t + 4 * g + r;
              if (key > myq[qg]) v = -INFINITY;
            }
            sc[qg][t][r] = v;
            mx = fmaxf(mx, v);
          }
        mx = max_rows4(mx);
        // lazy rescale (as fwd_kernel): the running max moves - and O, l are rescaled - only when
        // some row of the wave would otherwise see probabilities above 2^8 (wave-uniform branch;
        // a fully masked row keeps mx = -inf and never triggers it)
        if (__any(mx * c > m[qg] + 8.f)) {
          const float mn = fmaxf(m[qg], mx * c);
          const float alpha = fexp2(m[qg] - mn);
          m[qg] = mn;
          l[qg] *= alpha;
#pragma unroll
          for (int d = 0; d < DT; ++d)
#pragma unroll
            for (int r = 0; r < 4; ++r) o[qg][d][r] *= alpha;
        }
        const float mq = m[qg];
        float ps = 0.f;
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float pv = fexp2(fmaf(sc[qg][t][r], c, -mq));
            sc[qg][t][r] = pv;
            ps += pv;
          }
        l[qg] += ps;
        pp[qg][0] = pack_pair(sc[qg][0], sc[qg][1]);
        pp[qg][1] = pack_pair(sc[qg][2], sc[qg][3]);
      }
#pragma unroll
      for (int d0 = 0; d0 < DT; d0 += DB) {
        TrPair vq[DB][2];
#pragma unroll
        for (int d = 0; d < DB; ++d) {
          const uint32_t la = vbase + troff[d0 + d];
          vq[d][0] = frag_cols_at<DH, 0>(la);
          vq[d][1] = frag_cols_at<DH, 32>(la);
        }
        lgkm_wait0();
#pragma unroll
        for (int d = 0; d < DB; ++d) {
          const bf16x8 v0 = tr_use(vq[d][0]), v1 = tr_use(vq[d][1]);
#pragma unroll
          for (int qg = 0; qg < QG; ++qg) {
            o[qg][d0 + d] = mfma(v0, pp[qg][0], o[qg][d0 + d]);
            o[qg][d0 + d] = mfma(v1, pp[qg][1], o[qg][d0 + d]);
          }
        }
      }
    }
    if (kb + 1 < nkb && !(a.diag & 1)) wait_vm_upto(PER * (min(kb + NS - 1, nkb - 1) - kb - 1));
    step_barrier();
  }
#undef KT
#undef VT
#pragma unroll
  for (int qg = 0; qg < QG; ++qg) {
    const float lt = sum_rows4(l[qg]);
    const float inv = 1.f / lt;
    bf16_t* orow = a.out + ((long long)b * a.T + myq[qg]) * C + h * DH;
#pragma unroll
    for (int d = 0; d < DT; ++d) {
      const uint2 v = make_uint2(pack_bf2(o[qg][d][0] * inv, o[qg][d][1] * inv),
                                 pack_bf2(o[qg][d][2] * inv, o[qg][d][3] * inv));
      *(uint2*)(orow + 16 * d + 4 * g) = v;
    }
    if (g == 0) a.lse[(long long)bh * a.T + myq[qg]] = m[qg] + log2f(lt);
  }
}

// ------------------------------------------------------------------------------ delta
// delta[b][h][t] = sum_d O * dO over one head row; G = DH/8 lanes per row (16-B loads,
// consecutive lanes read consecutive 16 B), reduced with xor shuffles inside the lane group.
template <int DH>
__global__ __launch_bounds__(256) void delta_kernel(const bf16_t* __restrict__ out, const bf16_t* __restrict__ dout,
                                                   float* __restrict__ delta, int B, int T, int H) {
  constexpr int G = DH / 8;
  const long long gid = blockIdx.x * 256LL + threadIdx.x;
  const long long idx = gid / G;  // (b, t, h) row
  const int part = (int)(gid % G);
  float s = 0.f;
  if (idx < (long long)B * T * H) {
    const bf16_t* o = out + idx * DH + part * 8;
    const bf16_t* d = dout + idx * DH + part * 8;
    const uint4 x = *(const uint4*)o, y = *(const uint4*)d;
    const uint32_t xa[4] = {x.x, x.y, x.z, x.w}, ya[4] = {y.x, y.y, y.z, y.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      s += __uint_as_float(xa[i] << 16) * __uint_as_float(ya[i] << 16);
      s += __uint_as_float(xa[i] & 0xffff0000u) * __uint_as_float(ya[i] & 0xffff0000u);
    }
  }
#pragma unroll
  for (int off = 1; off < G; off <<= 1) s += __shfl_xor(s, off, 64);
  if (part == 0 && idx < (long long)B * T * H) {
    const int h = (int)(idx % H);
    const long long bt = idx / H;
    const int t = (int)(bt % T), b = (int)(bt / T);
    delta[((long long)b * H + h) * T + t] = s;
  }
}

// ------------------------------------------------------------------------------ dK / dV
// Ring slot = Q tile | dO tile | LSE[64] | delta[64] of one (q-head, q-block) step.  The 512 B
// of row constants come by DMA as well (waves 0-1: LSE halves, waves 2-3: delta halves, 8
// lanes x 16 B each), so every wave issues the same DH/16 + 1 DMA instructions per step.
template <int DH, int NS>
__global__ __launch_bounds__(256, 2) void bwd_dkdv_kernel(Args a) {
  constexpr int KS = DH / 32, DT = DH / 16, DB = DT < 4 ? DT : 4, TILE = 64 * DH * 2;
  constexpr int STG = 2 * TILE + 512, PER = DH / 16 + 1;
  __shared__ __attribute__((aligned(16))) char smem[NS * STG];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4;
  const int nkb = a.T / BKV;
  int kb, bkq;
  grid_pos(a, kb, bkq);  // key block, (batch, kv-head, q-head subset)
  const int qs = a.qs, bk = bkq / qs, qsub = bkq - bk * qs;
  const int b = bk / a.Hkv, kvh = bk % a.Hkv;
  const int grp = a.H / a.Hkv, gper = grp / qs;  // q-heads of the group this block covers
  const int C = a.H * DH, W = C + 2 * a.Hkv * DH;
  const bf16_t* base = a.qkv + (long long)b * a.T * W;
  const bf16_t* dob = a.dout + (long long)b * a.T * C;
  const int kcol = C + kvh * DH, vcol = C + a.Hkv * DH + kvh * DH;
  const int k0w = kb * BKV + wave * 16;
  const int mykey = k0w + (lane & 15);
  const float c = a.scale * LOG2E;
  uint32_t troff[DH / 16];
  tr_lane_offsets<DH>(troff, lane);

  const int nq = nkb - kb;      // q blocks at/after the diagonal
  const int total = nq * gper;  // steps over (q-head of this subset, q block)
  const float* rowsrc = wave < 2 ? (const float*)a.lse : a.delta;
  const int rowoff = 32 * (wave & 1) + 4 * (lane & 7);
  const int rowdst = 2 * TILE + 256 * (wave >> 1) + 128 * (wave & 1);
  auto issue = [&](int it) {
    char* st = smem + (it % NS) * STG;
    const int gi = it / nq, qb = kb + it % nq;
    const int h = kvh * grp + qsub * gper + gi;
    stage<DH, DH != 64>(base, W, qb * BQ, h * DH, st, wave, lane);
    stage<DH, DH != 64>(dob, C, qb * BQ, h * DH, st + TILE, wave, lane);
    const float* src = rowsrc + ((long long)b * a.H + h) * a.T + qb * BQ + rowoff;
    if (lane < 8) __builtin_amdgcn_global_load_lds((const void*)src, LDS_PTR(st + rowdst), 16, 0, 0);
  };
#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (s < total) issue(s);

  bf16x8 kf[KS], vf[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    kf[ks] = gload8(base + (long long)mykey * W + kcol + ks * 32 + g * 8);
    vf[ks] = gload8(base + (long long)mykey * W + vcol + ks * 32 + g * 8);
  }
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    settle(kf[ks]);
    settle(vf[ks]);
  }
  step_barrier();

  f32x4 dk[DT], dv[DT];
#pragma unroll
  for (int d = 0; d < DT; ++d) dk[d] = dv[d] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int it = 0; it < total; ++it) {
    if (it + NS - 1 < total) issue(it + NS - 1);
    const char* st = smem + (it % NS) * STG;
    const char* qt = st;
    const char* ot = st + TILE;
    const uint32_t qbase = lds_addr(qt), obase = lds_addr(ot);
    const float* lse_s = (const float*)(st + 2 * TILE);
    const float* del_s = lse_s + 64;
    const int qb = kb + it % nq;
    const bool diag = (qb == kb);
    f32x4 p[4], ds[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      f32x4 sacc = f32x4{0.f, 0.f, 0.f, 0.f}, dpacc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        sacc = mfma(frag_rows<DH>(qt, 16 * t, ks, lane), kf[ks], sacc);   // D[q][key]
        dpacc = mfma(frag_rows<DH>(ot, 16 * t, ks, lane), vf[ks], dpacc); // D[q][key]
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int ql = 16 * t + 4 * g + r;
        p[t][r] = fexp2(fmaf(sacc[r], c, -lse_s[ql]));
        ds[t][r] = dpacc[r] - del_s[ql];
      }
    }
    // causal mask only on the diagonal block (wave-uniform branch: no per-element selects on
    // the other steps - the loop is VALU-issue bound)
    if (diag) {
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (qb * BQ + 16 * t + 4 * g + r < mykey) p[t][r] = 0.f;
    }
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) ds[t][r] *= p[t][r];
    const bf16x8 p0 = pack_pair(p[0], p[1]), p1 = pack_pair(p[2], p[3]);
    const bf16x8 d0 = pack_pair(ds[0], ds[1]), d1 = pack_pair(ds[2], ds[3]);
#pragma unroll
    for (int e0 = 0; e0 < DT; e0 += DB) {
      TrPair fo[DB][2], fq[DB][2];
#pragma unroll
      for (int d = 0; d < DB; ++d) {
        const uint32_t lo = obase + troff[e0 + d], lq = qbase + troff[e0 + d];
        fo[d][0] = frag_cols_at<DH, 0>(lo);
        fo[d][1] = frag_cols_at<DH, 32>(lo);
        fq[d][0] = frag_cols_at<DH, 0>(lq);
        fq[d][1] = frag_cols_at<DH, 32>(lq);
      }
      lgkm_wait0();
#pragma unroll
      for (int d = 0; d < DB; ++d) {
        dv[e0 + d] = mfma(tr_use(fo[d][0]), p0, dv[e0 + d]);
        dv[e0 + d] = mfma(tr_use(fo[d][1]), p1, dv[e0 + d]);
        dk[e0 + d] = mfma(tr_use(fq[d][0]), d0, dk[e0 + d]);
        dk[e0 + d] = mfma(tr_use(fq[d][1]), d1, dk[e0 + d]);
      }
    }
    if (it + 1 < total && !(a.diag & 1)) wait_vm_upto(PER * (min(it + NS - 1, total - 1) - it - 1));
    step_barrier();
  }
  if (qs > 1) {  // fp32 partial of this q-head subset; dkdv_reduce_kernel finishes the rows
    float* prow = a.part + (((long long)qsub * a.B * a.T + (long long)b * a.T + mykey) * a.Hkv + kvh) * (2 * DH);
#pragma unroll
    for (int d = 0; d < DT; ++d) {
      *(f32x4*)(prow + 16 * d + 4 * g) = f32x4{dk[d][0] * a.scale, dk[d][1] * a.scale, dk[d][2] * a.scale,
                                               dk[d][3] * a.scale};
      *(f32x4*)(prow + DH + 16 * d + 4 * g) = dv[d];
    }
    return;
  }
  bf16_t* krow = a.dqkv + ((long long)b * a.T + mykey) * W;
#pragma unroll
  for (int d = 0; d < DT; ++d) {
    *(uint2*)(krow + kcol + 16 * d + 4 * g) =
        make_uint2(pack_bf2(dk[d][0] * a.scale, dk[d][1] * a.scale), pack_bf2(dk[d][2] * a.scale, dk[d][3] * a.scale));
    *(uint2*)(krow + vcol + 16 * d + 4 * g) = make_uint2(pack_bf2(dv[d][0], dv[d][1]), pack_bf2(dv[d][2], dv[d][3]));
  }
  if (a.cs_ws) {
    float* crow = a.cs_ws + (((long long)b * a.T + k0w) >> 4) * W;
    wave_colsum16<DT>(dk, a.scale, crow + kcol, lane);
    wave_colsum16<DT>(dv, 1.f, crow + vcol, lane);
  }
}

// dK / dV with 32 keys per wave (block = 128 keys, two 16-key groups per wave): every Q / dO
// fragment and row constant read from LDS feeds both key groups' S / dP MFMAs, and every
// transposed dO / Q fragment both groups' dV / dK MFMAs - half the LDS traffic per MFMA of
// bwd_dkdv_kernel, whose Dh = 64 loop is LDS-bound (per step and wave 24 ds_read_b128 + 32
// ds_read_b64_tr_b16 = 160 LDS-array cycles for 32 MFMAs, 12 waves per CU; MI355X_MICROARCH.md
// §LDS).  Same ring, row-constant DMA and output contract (incl. the GQA head split).
// (Dh = 128: 2 x 2 x 8 accumulators + 2 x 2 x 4 K / V fragments need the AGPR half of the
// register file, so one wave per SIMD)
template <int DH, int NS>
__global__ __launch_bounds__(256, DH == 64 ? 2 : 1) void bwd_dkdv2_kernel(Args a) {
  constexpr int KS = DH / 32, DT = DH / 16, DB = 2, TILE = 64 * DH * 2, KG = 2, BK2 = 128;
  constexpr int STG = 2 * TILE + 512, PER = DH / 16 + 1;
  __shared__ __attribute__((aligned(16))) char smem[NS * STG];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4;
  const int nqb = a.T / BQ;
  int kb, bkq;
  grid_pos(a, kb, bkq);  // 128-key block, (batch, kv-head, q-head subset)
  const int qs = a.qs, bk = bkq / qs, qsub = bkq - bk * qs;
  const int b = bk / a.Hkv, kvh = bk % a.Hkv;
  const int grp = a.H / a.Hkv, gper = grp / qs;
  const int C = a.H * DH, W = C + 2 * a.Hkv * DH;
  const bf16_t* base = a.qkv + (long long)b * a.T * W;
  const bf16_t* dob = a.dout + (long long)b * a.T * C;
  const int kcol = C + kvh * DH, vcol = C + a.Hkv * DH + kvh * DH;
  const int k0w = kb * BK2 + wave * 32;  // this wave's keys [k0w, k0w + 32)
  int mykey[KG];
#pragma unroll
  for (int kg = 0; kg < KG; ++kg) mykey[kg] = k0w + 16 * kg + (lane & 15);
  const float c = a.scale * LOG2E;
  uint32_t troff[DH / 16];
  tr_lane_offsets<DH>(troff, lane);

  const int qb0 = kb * (BK2 / BQ);  // first q block that meets the block's keys
  const int nq = nqb - qb0;
  const int total = nq * gper;
  const float* rowsrc = wave < 2 ? (const float*)a.lse : a.delta;
  const int rowoff = 32 * (wave & 1) + 4 * (lane & 7);
  const int rowdst = 2 * TILE + 256 * (wave >> 1) + 128 * (wave & 1);
  auto issue = [&](int it) {
    char* st = smem + (it % NS) * STG;
    const int gi = it / nq, qb = qb0 + it % nq;
    const int h = kvh * grp + qsub * gper + gi;
    stage<DH, DH != 64>(base, W, qb * BQ, h * DH, st, wave, lane);
    stage<DH, DH != 64>(dob, C, qb * BQ, h * DH, st + TILE, wave, lane);
    const float* src = rowsrc + ((long long)b * a.H + h) * a.T + qb * BQ + rowoff;
    if (lane < 8) __builtin_amdgcn_global_load_lds((const void*)src, LDS_PTR(st + rowdst), 16, 0, 0);
  };
#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (s < total) issue(s);

  bf16x8 kf[KG][KS], vf[KG][KS];
#pragma unroll
  for (int kg = 0; kg < KG; ++kg)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      kf[kg][ks] = gload8(base + (long long)mykey[kg] * W + kcol + ks * 32 + g * 8);
      vf[kg][ks] = gload8(base + (long long)mykey[kg] * W + vcol + ks * 32 + g * 8);
    }
#pragma unroll
  for (int kg = 0; kg < KG; ++kg)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      settle(kf[kg][ks]);
      settle(vf[kg][ks]);
    }
  step_barrier();

  f32x4 dk[KG][DT], dv[KG][DT];
#pragma unroll
  for (int kg = 0; kg < KG; ++kg)
#pragma unroll
    for (int d = 0; d < DT; ++d) dk[kg][d] = dv[kg][d] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int it = 0; it < total; ++it) {
    if (it + NS - 1 < total) issue(it + NS - 1);
    const char* st = smem + (it % NS) * STG;
    const int qb = qb0 + it % nq;
    // (wave-uniform) the tile's last query row is before this wave's first key: nothing to add
    if (qb * BQ + BQ - 1 >= k0w) {
      const char* qt = st;
      const char* ot = st + TILE;
      const uint32_t qbase = lds_addr(qt), obase = lds_addr(ot);
      const float* lse_s = (const float*)(st + 2 * TILE);
      const float* del_s = lse_s + 64;
      const bool diag = qb * BQ < k0w + 32;
      f32x4 p[KG][4], ds[KG][4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        f32x4 sacc[KG], dpacc[KG];
#pragma unroll
        for (int kg = 0; kg < KG; ++kg) sacc[kg] = dpacc[kg] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          const bf16x8 qa = frag_rows<DH>(qt, 16 * t, ks, lane), oa = frag_rows<DH>(ot, 16 * t, ks, lane);
#pragma unroll
          for (int kg = 0; kg < KG; ++kg) {
            sacc[kg] = mfma(qa, kf[kg][ks], sacc[kg]);    // D[q][key]
            dpacc[kg] = mfma(oa, vf[kg][ks], dpacc[kg]);  // D[q][key]
          }
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int ql = 16 * t + 4 * g + r;
          const float lv = lse_s[ql], dl = del_s[ql];
#pragma unroll
          for (int kg = 0; kg < KG; ++kg) {
            p[kg][t][r] = fexp2(fmaf(sacc[kg][r], c, -lv));
            ds[kg][t][r] = dpacc[kg][r] - dl;
          }
        }
      }
      if (diag) {  // causal mask where the tile meets this wave's keys (wave-uniform branch)
#pragma unroll
        for (int kg = 0; kg < KG; ++kg)
#pragma unroll
          for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r)
              if (qb * BQ + 16 * t + 4 * g + r < mykey[kg]) p[kg][t][r] = 0.f;
      }
      bf16x8 p0[KG], p1[KG], d0[KG], d1[KG];
#pragma unroll
      for (int kg = 0; kg < KG; ++kg) {
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r) ds[kg][t][r] *= p[kg][t][r];
        p0[kg] = pack_pair(p[kg][0], p[kg][1]);
        p1[kg] = pack_pair(p[kg][2], p[kg][3]);
        d0[kg] = pack_pair(ds[kg][0], ds[kg][1]);
        d1[kg] = pack_pair(ds[kg][2], ds[kg][3]);
      }
#pragma unroll
      for (int e0 = 0; e0 < DT; e0 += DB) {
        TrPair fo[DB][2], fq[DB][2];
#pragma unroll
        for (int d = 0; d < DB; ++d) {
          const uint32_t lo = obase + troff[e0 + d], lq = qbase + troff[e0 + d];
          fo[d][0] = frag_cols_at<DH, 0>(lo);
          fo[d][1] = frag_cols_at<DH, 32>(lo);
          fq[d][0] = frag_cols_at<DH, 0>(lq);
          fq[d][1] = frag_cols_at<DH, 32>(lq);
        }
        lgkm_wait0();
#pragma unroll
        for (int d = 0; d < DB; ++d) {
          const bf16x8 o0 = tr_use(fo[d][0]), o1 = tr_use(fo[d][1]);
          const bf16x8 q0 = tr_use(fq[d][0]), q1 = tr_use(fq[d][1]);
#pragma unroll
          for (int kg = 0; kg < KG; ++kg) {
            dv[kg][e0 + d] = mfma(o0, p0[kg], dv[kg][e0 + d]);
            dv[kg][e0 + d] = mfma(o1, p1[kg], dv[kg][e0 + d]);
            dk[kg][e0 + d] = mfma(q0, d0[kg], dk[kg][e0 + d]);
            dk[kg][e0 + d] = mfma(q1, d1[kg], dk[kg][e0 + d]);
          }
        }
      }
    }
    if (it + 1 < total && !(a.diag & 1)) wait_vm_upto(PER * (min(it + NS - 1, total - 1) - it - 1));
    step_barrier();
  }
#pragma unroll
  for (int kg = 0; kg < KG; ++kg) {
    if (qs > 1) {
      float* prow = a.part + (((long long)qsub * a.B * a.T + (long long)b * a.T + mykey[kg]) * a.Hkv + kvh) * (2 * DH);
#pragma unroll
      for (int d = 0; d < DT; ++d) {
        *(f32x4*)(prow + 16 * d + 4 * g) = f32x4{dk[kg][d][0] * a.scale, dk[kg][d][1] * a.scale,
                                                 dk[kg][d][2] * a.scale, dk[kg][d][3] * a.scale};
        *(f32x4*)(prow + DH + 16 * d + 4 * g) = dv[kg][d];
      }
      continue;
    }
    bf16_t* krow = a.dqkv + ((long long)b * a.T + mykey[kg]) * W;
#pragma unroll
    for (int d = 0; d < DT; ++d) {
      *(uint2*)(krow + kcol + 16 * d + 4 * g) = make_uint2(pack_bf2(dk[kg][d][0] * a.scale, dk[kg][d][1] * a.scale),
                                                           pack_bf2(dk[kg][d][2] * a.scale, dk[kg][d][3] * a.scale));
      *(uint2*)(krow + vcol + 16 * d + 4 * g) =
          make_uint2(pack_bf2(dv[kg][d][0], dv[kg][d][1]), pack_bf2(dv[kg][d][2], dv[kg][d][3]));
    }
    if (a.cs_ws) {
      float* crow = a.cs_ws + (((long long)b * a.T + k0w + 16 * kg) >> 4) * W;
      wave_colsum16<DT>(dk[kg], a.scale, crow + kcol, lane);
      wave_colsum16<DT>(dv[kg], 1.f, crow + vcol, lane);
    }
  }
}

// dK | dV rows from the qs fp32 partials of a head-split dK/dV pass: dqkv[b, t, K|V cols] =
// bf16(sum over qsub in order).  Block = 16 rows x 1024 columns of the [Hkv][2*Dh] partial row
// (blockIdx.y picks the column half when Hkv*2*Dh = 2048); thread = 4 columns, 16-B loads.  With
// cs_ws it also writes the 16-row column sums of the stored bf16 values (the qkv bias gradient
// partials, as the unsplit kernel's wave_colsum16 does).
template <int DH>
__global__ __launch_bounds__(256) void dkdv_reduce_kernel(Args a) {
  const int KV = a.Hkv * 2 * DH;
  const int col = (blockIdx.y * 256 + threadIdx.x) * 4;  // column in the [Hkv][2][DH] row
  if (col >= KV) return;
  const long long rows = (long long)a.B * a.T, r0 = (long long)blockIdx.x * 16;
  const int C = a.H * DH, W = C + 2 * a.Hkv * DH;
  const int kvh = col / (2 * DH), rem = col % (2 * DH);
  const int dcol = rem < DH ? C + kvh * DH + rem : C + a.Hkv * DH + kvh * DH + (rem - DH);
  float cs[4] = {0.f, 0.f, 0.f, 0.f};
  for (int i = 0; i < 16; ++i) {
    const long long r = r0 + i;
    f32x4 acc = *(const f32x4*)(a.part + r * KV + col);
    for (int q = 1; q < a.qs; ++q) {
      const f32x4 v = *(const f32x4*)(a.part + ((long long)q * rows + r) * KV + col);
      acc[0] += v[0]; acc[1] += v[1]; acc[2] += v[2]; acc[3] += v[3];
    }
    const uint2 o = make_uint2(pack_bf2(acc[0], acc[1]), pack_bf2(acc[2], acc[3]));
    *(uint2*)(a.dqkv + r * W + dcol) = o;
    if (a.cs_ws) {
      cs[0] += __uint_as_float(o.x << 16); cs[1] += __uint_as_float(o.x & 0xffff0000u);
      cs[2] += __uint_as_float(o.y << 16); cs[3] += __uint_as_float(o.y & 0xffff0000u);
    }
  }
  if (a.cs_ws) *(f32x4*)(a.cs_ws + (r0 >> 4) * W + dcol) = f32x4{cs[0], cs[1], cs[2], cs[3]};
}

// ------------------------------------------------------------------------------ dQ
template <int DH, int NS>
__global__ __launch_bounds__(256, 2) void bwd_dq_kernel(Args a) {
  constexpr int KS = DH / 32, DT = DH / 16, DB = DT < 4 ? DT : 4, TILE = 64 * DH * 2, PER = DH / 16;
  __shared__ __attribute__((aligned(16))) char smem[2 * NS * TILE];  // K[NS], V[NS]
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4;
  const int nqb = a.T / BQ;
  int bx, bh;
  grid_pos(a, bx, bh);
  const int qb = nqb - 1 - bx;
  const int b = bh / a.H, h = bh % a.H;
  const int grp = a.H / a.Hkv, kvh = h / grp;
  const int C = a.H * DH, W = C + 2 * a.Hkv * DH;
  const bf16_t* base = a.qkv + (long long)b * a.T * W;
  const int qcol = h * DH, kcol = C + kvh * DH, vcol = C + a.Hkv * DH + kvh * DH;
  const int myq = qb * BQ + wave * 16 + (lane & 15);
  const float c = a.scale * LOG2E;
  uint32_t troff[DH / 16];
  tr_lane_offsets<DH>(troff, lane);
  const long long r = (long long)bh * a.T + myq;
  const int nkb = qb + 1;

#define KT(s) (smem + (s) * TILE)
#define VT(s) (smem + (NS + (s)) * TILE)
#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (s < nkb) {
      stage<DH, DH != 64>(base, W, s * BKV, kcol, KT(s), wave, lane);
      stage<DH, DH != 64>(base, W, s * BKV, vcol, VT(s), wave, lane);
    }
  bf16x8 qf[KS], of[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    qf[ks] = gload8(base + (long long)myq * W + qcol + ks * 32 + g * 8);
    of[ks] = gload8(a.dout + ((long long)b * a.T + myq) * C + h * DH + ks * 32 + g * 8);
  }
  // delta = sum_d dO * O of this row (the softmax-backward row term): the lane's 8*KS columns
  // of O against its dO fragment, summed over the 4 lane rows; stored for the dK/dV kernel,
  // which runs after this one
  bf16x8 ofw[KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) ofw[ks] = gload8(a.out + ((long long)b * a.T + myq) * C + h * DH + ks * 32 + g * 8);
  const float lse2 = a.lse[r];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    settle(qf[ks]);
    settle(of[ks]);
    settle(ofw[ks]);
  }
  settle(lse2);
  float dsum = 0.f;
#pragma unroll
  for (int ks = 0; ks < KS; ++ks)
#pragma unroll
    for (int e = 0; e < 8; ++e)
      dsum = fmaf(bf2f((bf16_t)of[ks][e]), bf2f((bf16_t)ofw[ks][e]), dsum);
  const float del = sum_rows4(dsum);
  if (g == 0 && !a.delta_ready) a.delta[r] = del;
  step_barrier();

  f32x4 dq[DT];
#pragma unroll
  for (int d = 0; d < DT; ++d) dq[d] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int kb = 0; kb < nkb; ++kb) {
    const int cur = kb % NS;
    if (kb + NS - 1 < nkb) {
      const int nx = (kb + NS - 1) % NS;
      stage<DH, DH != 64>(base, W, (kb + NS - 1) * BKV, kcol, KT(nx), wave, lane);
      stage<DH, DH != 64>(base, W, (kb + NS - 1) * BKV, vcol, VT(nx), wave, lane);
    }
    const char* kt = KT(cur);
    const char* vt = VT(cur);
    const uint32_t kbase_lds = lds_addr(kt);
    const bool diag = (kb == qb);
    f32x4 ds[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      f32x4 sacc = f32x4{0.f, 0.f, 0.f, 0.f}, dpacc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        sacc = mfma(frag_rows<DH>(kt, 16 * t, ks, lane), qf[ks], sacc);   // D[key][q]
        dpacc = mfma(frag_rows<DH>(vt, 16 * t, ks, lane), of[ks], dpacc); // D[key][q]
      }
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const float pv = fexp2(fmaf(sacc[rr], c, -lse2));
        ds[t][rr] = pv * (dpacc[rr] - del);
      }
    }
    if (diag) {  // causal mask on the diagonal block only (wave-uniform)
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int rr = 0; rr < 4; ++rr)
          if (kb * BKV + 16 * t + 4 * g + rr > myq) ds[t][rr] = 0.f;
    }
    const bf16x8 d0 = pack_pair(ds[0], ds[1]), d1 = pack_pair(ds[2], ds[3]);
#pragma unroll
    for (int e0 = 0; e0 < DT; e0 += DB) {
      TrPair fk[DB][2];
#pragma unroll
      for (int d = 0; d < DB; ++d) {
        const uint32_t lk = kbase_lds + troff[e0 + d];
        fk[d][0] = frag_cols_at<DH, 0>(lk);
        fk[d][1] = frag_cols_at<DH, 32>(lk);
      }
      lgkm_wait0();
#pragma unroll
      for (int d = 0; d < DB; ++d) {
        dq[e0 + d] = mfma(tr_use(fk[d][0]), d0, dq[e0 + d]);
        dq[e0 + d] = mfma(tr_use(fk[d][1]), d1, dq[e0 + d]);
      }
    }
    if (kb + 1 < nkb && !(a.diag & 1)) wait_vm_upto(PER * (min(kb + NS - 1, nkb - 1) - kb - 1));
    step_barrier();
  }
#undef KT
#undef VT
  bf16_t* qrow = a.dqkv + ((long long)b * a.T + myq) * W + qcol;
#pragma unroll
  for (int d = 0; d < DT; ++d)
    *(uint2*)(qrow + 16 * d + 4 * g) =
        make_uint2(pack_bf2(dq[d][0] * a.scale, dq[d][1] * a.scale), pack_bf2(dq[d][2] * a.scale, dq[d][3] * a.scale));
  if (a.cs_ws)
    wave_colsum16<DT>(dq, a.scale, a.cs_ws + (((long long)b * a.T + qb * BQ + wave * 16) >> 4) * W + qcol, lane);
}

// dQ with 32 query rows per wave (block = 128 rows): every K / V fragment read from LDS (row and
// transposed) feeds the MFMAs of two 16-row query groups, halving LDS bytes per MFMA of
// bwd_dq_kernel - the change that took dK/dV from 130 to 82 us at GPT-2 shapes (bwd_dkdv2_kernel).
// Same DMA ring, delta prologue, causal skip / mask and output contract.
template <int DH, int NS>
__global__ __launch_bounds__(256, 2) void bwd_dq2_kernel(Args a) {
  constexpr int KS = DH / 32, DT = DH / 16, DB = DT < 4 ? DT : 4, TILE = 64 * DH * 2, PER = DH / 16;
  constexpr int QG = 2, BQ2 = 128;
  __shared__ __attribute__((aligned(16))) char smem[2 * NS * TILE];  // K[NS], V[NS]
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4;
  const int nqb = a.T / BQ2;
  int bx, bh;
  grid_pos(a, bx, bh);
  const int qb = nqb - 1 - bx;  // heaviest (longest causal prefix) blocks first
  const int b = bh / a.H, h = bh % a.H;
  const int grp = a.H / a.Hkv, kvh = h / grp;
  const int C = a.H * DH, W = C + 2 * a.Hkv * DH;
  const bf16_t* base = a.qkv + (long long)b * a.T * W;
  const int qcol = h * DH, kcol = C + kvh * DH, vcol = C + a.Hkv * DH + kvh * DH;
  const int q0w = qb * BQ2 + wave * 32;  // this wave: rows [q0w, q0w + 32)
  int myq[QG];
#pragma unroll
  for (int qg = 0; qg < QG; ++qg) myq[qg] = q0w + 16 * qg + (lane & 15);
  const float c = a.scale * LOG2E;
  uint32_t troff[DH / 16];
  tr_lane_offsets<DH>(troff, lane);
  const int nkb = (qb + 1) * (BQ2 / BKV);

#define KT(s) (smem + (s) * TILE)
#define VT(s) (smem + (NS + (s)) * TILE)
#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (s < nkb) {
      stage<DH, DH != 64>(base, W, s * BKV, kcol, KT(s), wave, lane);
      stage<DH, DH != 64>(base, W, s * BKV, vcol, VT(s), wave, lane);
    }
  bf16x8 qf[QG][KS], of[QG][KS], ofw[QG][KS];
  float lse2[QG];
#pragma unroll
  for (int qg = 0; qg < QG; ++qg) {
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      qf[qg][ks] = gload8(base + (long long)myq[qg] * W + qcol + ks * 32 + g * 8);
      of[qg][ks] = gload8(a.dout + ((long long)b * a.T + myq[qg]) * C + h * DH + ks * 32 + g * 8);
      ofw[qg][ks] = gload8(a.out + ((long long)b * a.T + myq[qg]) * C + h * DH + ks * 32 + g * 8);
    }
    lse2[qg] = a.lse[(long long)bh * a.T + myq[qg]];
  }
#pragma unroll
  for (int qg = 0; qg < QG; ++qg) {
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      settle(qf[qg][ks]);
      settle(of[qg][ks]);
      settle(ofw[qg][ks]);
    }
    settle(lse2[qg]);
  }
  // delta = sum_d dO * O per row (the softmax-backward row term), stored for the dK/dV kernel
  float del[QG];
#pragma unroll
  for (int qg = 0; qg < QG; ++qg) {
    float dsum = 0.f;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int e = 0; e < 8; ++e) dsum = fmaf(bf2f((bf16_t)of[qg][ks][e]), bf2f((bf16_t)ofw[qg][ks][e]), dsum);
    del[qg] = sum_rows4(dsum);
    if (g == 0 && !a.delta_ready) a.delta[(long long)bh * a.T + myq[qg]] = del[qg];
  }
  step_barrier();

  f32x4 dq[QG][DT];
#pragma unroll
  for (int qg = 0; qg < QG; ++qg)
#pragma unroll
    for (int d = 0; d < DT; ++d) dq[qg][d] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int kb = 0; kb < nkb; ++kb) {
    const int cur = kb % NS;
    if (kb + NS - 1 < nkb) {
      const int nx = (kb + NS - 1) % NS;
      stage<DH, DH != 64>(base, W, (kb + NS - 1) * BKV, kcol, KT(nx), wave, lane);
      stage<DH, DH != 64>(base, W, (kb + NS - 1) * BKV, vcol, VT(nx), wave, lane);
    }
    // keys of this tile all after this wave's last row: nothing to add (barriers still run)
    if (kb * BKV <= q0w + 31) {
      const char* kt = KT(cur);
      const char* vt = VT(cur);
      const uint32_t kbase_lds = lds_addr(kt);
      const bool diag = kb * BKV + BKV - 1 > q0w;
      f32x4 ds[QG][4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        f32x4 sacc[QG], dpacc[QG];
#pragma unroll
        for (int qg = 0; qg < QG; ++qg) sacc[qg] = dpacc[qg] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          const bf16x8 kf = frag_rows<DH>(kt, 16 * t, ks, lane), vf = frag_rows<DH>(vt, 16 * t, ks, lane);
#pragma unroll
          for (int qg = 0; qg < QG; ++qg) {
            sacc[qg] = mfma(kf, qf[qg][ks], sacc[qg]);    // D[key][q]
            dpacc[qg] = mfma(vf, of[qg][ks], dpacc[qg]);  // D[key][q]
          }
        }
#pragma unroll
        for (int qg = 0; qg < QG; ++qg)
#pragma unroll
          for (int rr = 0; rr < 4; ++rr) {
            const float pv = fexp2(fmaf(sacc[qg][rr], c, -lse2[qg]));
            ds[qg][t][rr] = pv * (dpacc[qg][rr] - del[qg]);
          }
      }
      if (diag) {  // causal mask where the tile meets this wave's rows (wave-uniform)
#pragma unroll
        for (int qg = 0; qg < QG; ++qg)
#pragma unroll
          for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int rr = 0; rr < 4; ++rr)
              if (kb * BKV + 16 * t + 4 * g + rr > myq[qg]) ds[qg][t][rr] = 0.f;
      }
      bf16x8 d0[QG], d1[QG];
#pragma unroll
      for (int qg = 0; qg < QG; ++qg) {
        d0[qg] = pack_pair(ds[qg][0], ds[qg][1]);
        d1[qg] = pack_pair(ds[qg][2], ds[qg][3]);
      }
#pragma unroll
      for (int e0 = 0; e0 < DT; e0 += DB) {
        TrPair fk[DB][2];
#pragma unroll
        for (int d = 0; d < DB; ++d) {
          const uint32_t lk = kbase_lds + troff[e0 + d];
          fk[d][0] = frag_cols_at<DH, 0>(lk);
          fk[d][1] = frag_cols_at<DH, 32>(lk);
        }
        lgkm_wait0();
#pragma unroll
        for (int d = 0; d < DB; ++d) {
          const bf16x8 k0 = tr_use(fk[d][0]), k1 = tr_use(fk[d][1]);
#pragma unroll
          for (int qg = 0; qg < QG; ++qg) {
            dq[qg][e0 + d] = mfma(k0, d0[qg], dq[qg][e0 + d]);
            dq[qg][e0 + d] = mfma(k1, d1[qg], dq[qg][e0 + d]);
          }
        }
      }
    }
    if (kb + 1 < nkb && !(a.diag & 1)) wait_vm_upto(PER * (min(kb + NS - 1, nkb - 1) - kb - 1));
    step_barrier();
  }
#undef KT
#undef VT
#pragma unroll
  for (int qg = 0; qg < QG; ++qg) {
    bf16_t* qrow = a.dqkv + ((long long)b * a.T + myq[qg]) * W + qcol;
#pragma unroll
    for (int d = 0; d < DT; ++d)
      *(uint2*)(qrow + 16 * d + 4 * g) = make_uint2(pack_bf2(dq[qg][d][0] * a.scale, dq[qg][d][1] * a.scale),
                                                   pack_bf2(dq[qg][d][2] * a.scale, dq[qg][d][3] * a.scale));
    if (a.cs_ws)
      wave_colsum16<DT>(dq[qg], a.scale, a.cs_ws + (((long long)b * a.T + q0w + 16 * qg) >> 4) * W + qcol, lane);
  }
}

}  // namespace fa
}  // namespace rtdc

using namespace rtdc;

// ring depth: RTDC_FA_NS = 2 | 3 | 4 at Dh = 64.  Measured on GPT-2 shapes (B16 T1024 H12,
// benchmarks/attn_bench.py): NS 2 / 3 / 4 = fwd 108 / 113 / 135 us, bwd 285 / 335 / 357 us -
// every extra slot costs a co-resident block per CU (32 / 48 / 64 KiB of LDS per block), and
// at these 8-16-step loops occupancy hides more HBM latency than a deeper ring.  Dh = 128
// stays at 2 (a third slot leaves one block per CU).
static int fa_diag() {
  static const int v = getenv("RTDC_FA_DIAG") ? atoi(getenv("RTDC_FA_DIAG")) : 0;
  return v;
}

static int fa_xcd() {
  // 2 (default): one head's blocks share an XCD and each XCD runs the long blocks of all its
  // heads first (GPT-2 fwd 84 -> 48 us vs the plain grid order 0); 1: XCD grouping only
  static const int v = getenv("RTDC_FA_XCD") ? atoi(getenv("RTDC_FA_XCD")) : 2;
  return v;
}

static int fa_ns(int Dh) {
  static const int forced = getenv("RTDC_FA_NS") ? atoi(getenv("RTDC_FA_NS")) : 0;
  if (Dh == 128) return 2;
  return forced >= 2 && forced <= 4 ? forced : 2;
}

#define FA_DISPATCH(KERNEL, DH, NSV, GRID, ARGS)                                                        \
  do {                                                                                                   \
    if ((NSV) == 4) hipLaunchKernelGGL((KERNEL<DH, (DH == 64 ? 4 : 2)>), GRID, dim3(256), 0, st, ARGS); \
    else if ((NSV) == 3) hipLaunchKernelGGL((KERNEL<DH, (DH == 64 ? 3 : 2)>), GRID, dim3(256), 0, st, ARGS); \
    else hipLaunchKernelGGL((KERNEL<DH, 2>), GRID, dim3(256), 0, st, ARGS);                              \
  } while (0)

extern "C" int rtdc_flash_fwd(const void* qkv, void* out, float* lse, int B, int T, int H, int Hkv, int Dh,
                              float scale, hipStream_t st) {
  if (T % 64 != 0 || (Dh != 64 && Dh != 128) || H % Hkv != 0) return 1;
  fa::Args a{};
  a.qkv = (const bf16_t*)qkv; a.out = (bf16_t*)out; a.lse = lse;
  a.B = B; a.T = T; a.H = H; a.Hkv = Hkv; a.scale = scale; a.xcd_remap = fa_xcd(); a.diag = fa_diag();
  // measured (benchmarks/attn_bench.py, before the DMA ring): 32 rows/wave wins at Dh = 128
  // (Llama: 101 vs 108 us), 16 rows/wave at Dh = 64 (GPT-2: 100 vs 109 us); RTDC_FA_FWD=1|2
  // forces one
  const char* fwd_env = getenv("RTDC_FA_FWD");  // (read per call: tests A/B it in one process)
  const int forced = fwd_env ? atoi(fwd_env) : 0;
  const int variant = forced ? forced : (Dh == 128 ? 2 : 1);
  const int ns = fa_ns(Dh);
  if (variant == 3 && Dh == 64) {  // software-pipelined 16 rows per wave
    dim3 grid(T / 64, B * H);
    hipLaunchKernelGGL((fa::fwd3_kernel<64>), grid, dim3(256), 0, st, a);
  } else if (variant == 2 && T % 128 == 0) {  // 32 rows per wave
    dim3 grid(T / 128, B * H);
    if (Dh == 64) FA_DISPATCH(fa::fwd2_kernel, 64, ns, grid, a);
    else FA_DISPATCH(fa::fwd2_kernel, 128, ns, grid, a);
  } else {
    dim3 grid(T / 64, B * H);
    static const int db = getenv("RTDC_FA_DB") ? atoi(getenv("RTDC_FA_DB")) : 4;
    if (Dh == 64 && ns == 2 && db == 2) hipLaunchKernelGGL((fa::fwd_kernel<64, 2, 2>), grid, dim3(256), 0, st, a);
    else if (Dh == 64) FA_DISPATCH(fa::fwd_kernel, 64, ns, grid, a);
    else FA_DISPATCH(fa::fwd_kernel, 128, ns, grid, a);
  }
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

// delta[b][h][t] = rowsum(dO * O) alone (before dQ and dK/dV run concurrently on two streams)
extern "C" int rtdc_flash_delta(const void* out, const void* dout, float* delta, int B, int T, int H, int Dh,
                                hipStream_t st) {
  if (Dh != 64 && Dh != 128) return 1;
  const long long threads = (long long)B * T * H * (Dh / 8);
  dim3 grid((unsigned)((threads + 255) / 256));
  if (Dh == 64)
    hipLaunchKernelGGL(fa::delta_kernel<64>, grid, dim3(256), 0, st, (const bf16_t*)out, (const bf16_t*)dout, delta, B,
                       T, H);
  else
    hipLaunchKernelGGL(fa::delta_kernel<128>, grid, dim3(256), 0, st, (const bf16_t*)out, (const bf16_t*)dout, delta,
                       B, T, H);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

// which: bit 0 the dQ pass (it also stores delta unless delta_ready), bit 1 the dK/dV pass (+ the
// GQA head-split reduction).  Both bits: dQ then dK/dV on `st`.  One bit with delta_ready lets the
// caller run the two passes on two streams (ops/attention.py).
extern "C" int rtdc_flash_bwd(const void* qkv, const void* out, const void* dout, const float* lse, float* delta,
                              void* dqkv, int B, int T, int H, int Hkv, int Dh, float scale, float* cs_ws,
                              float* part, int qs, int which, int delta_ready, hipStream_t st) {
  if (T % 64 != 0 || (Dh != 64 && Dh != 128) || H % Hkv != 0) return 1;
  if (qs < 1 || (H / Hkv) % qs != 0 || (qs > 1 && part == nullptr) || ((Hkv * 2 * Dh) % 4) != 0) return 1;
  // dQ first: it also computes the row terms delta = rowsum(dO * O) that dK/dV read
  fa::Args a{};
  a.qkv = (const bf16_t*)qkv; a.out = (bf16_t*)out; a.dout = (const bf16_t*)dout; a.lse = (float*)lse;
  a.delta = delta;
  a.dqkv = (bf16_t*)dqkv;
  a.cs_ws = cs_ws;
  a.B = B; a.T = T; a.H = H; a.Hkv = Hkv; a.scale = scale; a.xcd_remap = fa_xcd(); a.diag = fa_diag();
  a.part = part; a.qs = qs; a.delta_ready = delta_ready;
  if (which < 1 || which > 3 || (which != 3 && !delta_ready)) return 1;
  const bool run_dq = which & 1, run_dkdv = which & 2;
  dim3 g1(T / 64, B * Hkv * qs), g2(T / 64, B * H);
  const int ns = fa_ns(Dh);
  // dK/dV at Dh = 64: 32 keys per wave (bwd_dkdv2_kernel) unless RTDC_FA_DKDV=1 (16 keys per wave)
  const char* dkdv_env = getenv("RTDC_FA_DKDV");  // (read per call: tests A/B it in one process)
  const int dkdv_v = dkdv_env ? atoi(dkdv_env) : 2;
  // dQ: 32 query rows per wave (bwd_dq2_kernel; GPT-2 63 -> 59 us, Llama-3-8B shapes 165 -> 140 us
  // per call, benchmarks/attn_bench.py under rocprofv3) unless RTDC_FA_DQ=1 (16 rows per wave)
  const char* dq_env = getenv("RTDC_FA_DQ");  // (read per call: tests A/B it in one process)
  const bool dq2 = (dq_env ? atoi(dq_env) : 2) == 2 && T % 128 == 0;
  const dim3 g2b(T / 128, B * H);
  if (Dh == 64) {
    if (run_dq) {
      if (dq2) FA_DISPATCH(fa::bwd_dq2_kernel, 64, ns, g2b, a);
      else FA_DISPATCH(fa::bwd_dq_kernel, 64, ns, g2, a);
    }
    if (run_dkdv) {
      if (dkdv_v == 2 && T % 128 == 0) {
        dim3 g3(T / 128, B * Hkv * qs);
        FA_DISPATCH(fa::bwd_dkdv2_kernel, 64, ns, g3, a);
      } else {
        FA_DISPATCH(fa::bwd_dkdv_kernel, 64, ns, g1, a);
      }
    }
  } else {
    if (run_dq) {
      if (dq2) FA_DISPATCH(fa::bwd_dq2_kernel, 128, ns, g2b, a);
      else FA_DISPATCH(fa::bwd_dq_kernel, 128, ns, g2, a);
    }
    if (run_dkdv) {
      if (dkdv_env && dkdv_v == 2 && T % 128 == 0) {  // opt-in at Dh = 128 (occupancy 1)
        dim3 g3(T / 128, B * Hkv * qs);
        FA_DISPATCH(fa::bwd_dkdv2_kernel, 128, ns, g3, a);
      } else {
        FA_DISPATCH(fa::bwd_dkdv_kernel, 128, ns, g1, a);
      }
    }
  }
  if (qs > 1 && run_dkdv) {
    const int KV = Hkv * 2 * Dh;
    dim3 gr((unsigned)((long long)B * T / 16), (unsigned)((KV / 4 + 255) / 256));
    if (Dh == 64) hipLaunchKernelGGL(fa::dkdv_reduce_kernel<64>, gr, dim3(256), 0, st, a);
    else hipLaunchKernelGGL(fa::dkdv_reduce_kernel<128>, gr, dim3(256), 0, st, a);
  }
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

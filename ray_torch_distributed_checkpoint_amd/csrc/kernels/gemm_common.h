// Shared pieces of the bf16 MFMA GEMM kernels (gemm_bf16.hip, gemm_8ph.hip): LDS image
// swizzles, per-lane glds stagers (plain and implicit-GEMM convolution gathers), MFMA
// fragment loads (K-major ds_read_b128 / MN-major ds_read_b64_tr_b16) and the fused epilogue.
#pragma once
#include "common.h"
#include "args.h"

#include <type_traits>

namespace rtdc {

namespace gemm {
constexpr int BK = 64;
}

template <int BM_, int BN_, int WM_, int WN_>
struct TileCfg {
  static constexpr int BM = BM_, BN = BN_, WM = WM_, WN = WN_;
  static constexpr int NW = WM * WN, NT = 64 * NW;
  static constexpr int TM = BM / WM / 16, TN = BN / WN / 16;  // MFMA tiles per wave
  static constexpr int A_BYTES = BM * gemm::BK * 2, B_BYTES = BN * gemm::BK * 2;
  static constexpr int STAGE = A_BYTES + B_BYTES;
  static_assert((BM / 8) % NW == 0 && (BN / 8) % NW == 0, "pieces must split evenly over waves");
};

// ---- LDS image helpers ----------------------------------------------------------------
// K-major image: ROWS rows x 128 B (64 bf16 of k).  16-B chunk c of row r lives at physical
// chunk c ^ ((r >> 1) & 7): a ds_read_b128 lane group (16 distinct rows, same logical chunk)
// then touches 16 distinct 16-B slots of the 256-B bank row.
__device__ __forceinline__ int kmaj_off(int row, int chunk) {
  return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4);
}
// MN-major image: 64 k-rows x (2*ROWS) B.  Chunk c of k-row kr lives at c ^ f(kr); a 32-lane
// half of ds_read_b64_tr_b16 reads 8 k-rows {q, 8+q : q < 4} x 2 chunks -> 16 distinct 16-B
// bank slots.  ROWS >= 128 (k-rows start on the same bank, stride 256/512 B): f < 16 keeps the
// chunk inside its row.  ROWS = 64 (128-B k-rows, two per bank row: kr&1 already separates
// halves): f in {0,2,4,6} from bits 1 and 3 of kr.
template <int ROWS>
__device__ __forceinline__ int mnmaj_swz(int kr) {
  if constexpr (ROWS >= 128)
    return ((kr & 3) | (((kr >> 3) & 1) << 2)) << 1;
  else
    return (((kr >> 1) & 1) | (((kr >> 3) & 1) << 1)) << 1;
}

// Per-lane global sources of one operand tile, computed once per block.
#ifndef RTDC_STAGER32
#define RTDC_STAGER32 0
#endif
template <bool KMAJOR, int ROWS, int NW>
struct Stager {
  static constexpr int PIECES = ROWS / 8;  // 1 KiB pieces per 64-deep k tile
  static constexpr int PPW = PIECES / NW;
#if RTDC_STAGER32
  // A/B build (-DRTDC_STAGER32=1): a wave-uniform base + 32-bit per-lane element offsets (half
  // the VGPRs of 64-bit per-lane pointers; the launcher keeps operands under 2^31 elements)
  const bf16_t* base;
  uint32_t off[PPW];
#else
  const bf16_t* src[PPW];
#endif
  long long kmul;  // element stride per unit of k

  __device__ __forceinline__ void init(const bf16_t* X, int ld, int rows, int r0, int wave, int lane) {
#pragma unroll
    for (int ii = 0; ii < PPW; ++ii) {
      const int piece = wave * PPW + ii;
      long long o;
      if constexpr (KMAJOR) {
        const int row = piece * 8 + (lane >> 3);
        const int lchunk = (lane & 7) ^ ((row >> 1) & 7);
        int gr = r0 + row;
        gr = gr < rows ? gr : rows - 1;
        o = (long long)gr * ld + lchunk * 8;
      } else {
        constexpr int CPR = ROWS / 8;     // 16-B chunks per k-row
        constexpr int KRP = 1024 / (ROWS * 2);  // k-rows per piece
        const int kr = piece * KRP + lane / CPR;
        const int lchunk = (lane % CPR) ^ mnmaj_swz<ROWS>(kr);
        int gc = r0 + lchunk * 8;
        gc = gc < rows ? gc : rows - 8;
        o = (long long)kr * ld + gc;
      }
#if RTDC_STAGER32
      off[ii] = (uint32_t)o;
#else
      src[ii] = X + o;
#endif
    }
#if RTDC_STAGER32
    base = X;
#endif
    kmul = KMAJOR ? 1 : ld;
  }

  __device__ __forceinline__ const bf16_t* addr(int ii, long long koff) const {
#if RTDC_STAGER32
    return base + (koff + off[ii]);
#else
    return src[ii] + koff;
#endif
  }

  __device__ __forceinline__ void issue(int k0, char* lds_tile, int wave) const {
    const long long koff = (long long)k0 * kmul;
#pragma unroll
    for (int ii = 0; ii < PPW; ++ii) {
      const int piece = wave * PPW + ii;
      __builtin_amdgcn_global_load_lds((const void*)addr(ii, koff), LDS_PTR(lds_tile + piece * 1024), 16, 0, 0);
    }
  }
  // one piece (1 KiB per wave) of issue(): lets a schedule interleave the DMA with MFMAs
  __device__ __forceinline__ void issue_one(int k0, char* lds_tile, int wave, int ii) const {
    const long long koff = (long long)k0 * kmul;
    const int piece = wave * PPW + ii;
    __builtin_amdgcn_global_load_lds((const void*)addr(ii, koff), LDS_PTR(lds_tile + piece * 1024), 16, 0, 0);
  }
};

// ---- implicit-GEMM convolution stagers ---------------------------------------------------
// Zero source for taps that fall into the padding (global_load_lds needs a real address).
__device__ __attribute__((aligned(16))) uint4 g_conv_zero[4];

// q = x / d for 0 <= x < 2^24 via the fp32 reciprocal (one correction step is exact there)
__device__ __forceinline__ int fdivq(int x, int d, float rd) {
  int q = (int)((float)x * rd);
  const int r = x - q * d;
  q += (r < 0) ? -1 : (r >= d ? 1 : 0);
  return q;
}

// Mode 1: A (K-major) = im2col(X) gathered on the fly.  With C % 64 == 0 a 64-deep k tile lies
// inside one tap, so row m of the tile is 128 contiguous bytes of X at pixel
// (b, ho*s - p + kh, wo*s - p + kw), channels c0..c0+63 - exactly the 8 x 16-B pieces the
// plain K-major stager moves; out-of-image taps read the zero page.  With C | 64 (C = 16, 32:
// the space-to-depth ResNet stem) a k tile spans 64/C taps and each 16-B chunk has its own
// tap offset to[] and channel offset co[] (k = tap*C + c throughout).
template <int ROWS, int NW>
struct ConvStagerK {
  static constexpr int PIECES = ROWS / 8, PPW = PIECES / NW;
  const bf16_t* X;
  int hb[PPW], wb[PPW], pb[PPW], co[PPW], to[PPW];
  int H, W, C, KW;
  float rKW;

  __device__ __forceinline__ void init(const GemmArgs& a, const bf16_t* Xp, int rows, int r0, int wave, int lane) {
    X = Xp;
    H = a.cv_H; W = a.cv_W; C = a.cv_C; KW = a.cv_KW;
    rKW = 1.f / (float)KW;
    const float rWo = 1.f / (float)a.cv_Wo, rHo = 1.f / (float)a.cv_Ho;
#pragma unroll
    for (int ii = 0; ii < PPW; ++ii) {
      const int piece = wave * PPW + ii;
      const int row = piece * 8 + (lane >> 3);
      const int lchunk = (lane & 7) ^ ((row >> 1) & 7);
      int gr = r0 + row;
      gr = gr < rows ? gr : rows - 1;
      const int q = fdivq(gr, a.cv_Wo, rWo), wo = gr - q * a.cv_Wo;
      const int b = fdivq(q, a.cv_Ho, rHo), ho = q - b * a.cv_Ho;
      hb[ii] = ho * a.cv_stride - a.cv_pad;
      wb[ii] = wo * a.cv_stride - a.cv_pad;
      pb[ii] = b * H;
      const int kc = lchunk * 8;  // k offset of this chunk inside the 64-deep tile
      to[ii] = C >= 64 ? 0 : kc / C;
      co[ii] = kc - to[ii] * C;
    }
  }

  __device__ __forceinline__ void issue(int k0, char* lds_tile, int wave) const {
    const int tap0 = k0 / C, c0 = k0 - tap0 * C;
    const int kh0 = tap0 / KW, kw0 = tap0 - kh0 * KW;
#pragma unroll
    for (int ii = 0; ii < PPW; ++ii) {
      const int piece = wave * PPW + ii;
      int kh = kh0, kw = kw0;
      if (C < 64) {  // wave-uniform: several taps per k tile
        const int tap = tap0 + to[ii];
        kh = fdivq(tap, KW, rKW);
        kw = tap - kh * KW;
      }
      const int h = hb[ii] + kh, w = wb[ii] + kw;
      const bool ok = (unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W;
      const bf16_t* src = ok ? X + (size_t)((pb[ii] + h) * W + w) * C + c0 + co[ii] : (const bf16_t*)g_conv_zero;
      __builtin_amdgcn_global_load_lds((const void*)src, LDS_PTR(lds_tile + piece * 1024), 16, 0, 0);
    }
  }
};

// Mode 2: B (MN-major) = im2col(X) with k = output pixel, n = tap*C + c (weight gradient
// dW = dY^T . im2col(X)).  A lane's 16-B chunk has a fixed (tap, c) for the whole loop; its
// k-row (pixel) advances by 64 per tile and is decomposed with fp32-reciprocal divisions.
template <int ROWS, int NW>
struct ConvStagerMN {
  static constexpr int PIECES = ROWS / 8, PPW = PIECES / NW;
  static constexpr int CPR = ROWS / 8, KRP = 1024 / (ROWS * 2);
  const bf16_t* X;
  int kr[PPW], dh[PPW], dw[PPW], cc[PPW];
  int H, W, C, Ho, Wo, stride, npix;
  float rWo, rHo;

  __device__ __forceinline__ void init(const GemmArgs& a, const bf16_t* Xp, int cols, int c0, int wave, int lane) {
    X = Xp;
    H = a.cv_H; W = a.cv_W; C = a.cv_C; Ho = a.cv_Ho; Wo = a.cv_Wo; stride = a.cv_stride; npix = a.cv_npix;
    rWo = 1.f / (float)Wo;
    rHo = 1.f / (float)Ho;
#pragma unroll
    for (int ii = 0; ii < PPW; ++ii) {
      const int piece = wave * PPW + ii;
      kr[ii] = piece * KRP + lane / CPR;
      const int lchunk = (lane % CPR) ^ mnmaj_swz<ROWS>(kr[ii]);
      int gc = c0 + lchunk * 8;
      gc = gc < cols ? gc : cols - 8;
      const int tap = gc / C, c = gc - tap * C, kh = tap / a.cv_KW, kw = tap - kh * a.cv_KW;
      dh[ii] = kh - a.cv_pad;
      dw[ii] = kw - a.cv_pad;
      cc[ii] = c;
    }
  }

  __device__ __forceinline__ void issue(int k0, char* lds_tile, int wave) const {
#pragma unroll
    for (int ii = 0; ii < PPW; ++ii) {
      const int piece = wave * PPW + ii;
      const int pix = k0 + kr[ii];
      const int q = fdivq(pix, Wo, rWo), wo = pix - q * Wo;
      const int b = fdivq(q, Ho, rHo), ho = q - b * Ho;
      const int h = ho * stride + dh[ii], w = wo * stride + dw[ii];
      const bool ok = pix < npix && (unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W;
      const bf16_t* src = ok ? X + (size_t)((b * H + h) * W + w) * C + cc[ii] : (const bf16_t*)g_conv_zero;
      __builtin_amdgcn_global_load_lds((const void*)src, LDS_PTR(lds_tile + piece * 1024), 16, 0, 0);
    }
  }
};

// Fragment for v_mfma_f32_16x16x32_bf16: lane l holds X(row = R0 + (l&15), k = ks*32 + 8(l>>4) + j).
template <bool KMAJOR, int ROWS>
__device__ __forceinline__ bf16x8 load_frag(const char* lds_tile, int R0, int ks, int lane) {
  if constexpr (KMAJOR) {
    const int row = R0 + (lane & 15);
    const int chunk = ks * 4 + (lane >> 4);
    return *(const bf16x8*)(lds_tile + kmaj_off(row, chunk));
  } else {
    const int idx = lane & 15, q = idx >> 2, p = idx & 3, g = lane >> 4;
    const int c = (R0 >> 3) + (p >> 1);
    bf16x4 v[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int kr = ks * 32 + 8 * g + 4 * h + q;
      const int off = kr * (ROWS * 2) + ((c ^ mnmaj_swz<ROWS>(kr)) << 4) + ((p & 1) << 3);
      v[h] = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
          (__attribute__((address_space(3))) bf16x4*)(lds_tile + off));
    }
    bf16x8 r;
    r[0] = v[0][0]; r[1] = v[0][1]; r[2] = v[0][2]; r[3] = v[0][3];
    r[4] = v[1][0]; r[5] = v[1][1]; r[6] = v[1][2]; r[7] = v[1][3];
    return r;
  }
}

// MN-major fragment through the asm transposing read (common.h ds_tr16 protocol): same lane
// contract as load_frag<false, ROWS>, returned as the two unassembled halves.  The builtin
// form costs an `s_waitcnt vmcnt(0)` (a drain of every staged tile in flight) in front of each
// group of reads.
template <int ROWS>
__device__ __forceinline__ TrPair load_frag_tr(const char* lds_tile, int R0, int ks, int lane) {
  const int idx = lane & 15, q = idx >> 2, p = idx & 3, g = lane >> 4;
  const int c = (R0 >> 3) + (p >> 1);
  const int kr0 = ks * 32 + 8 * g + q, kr1 = kr0 + 4;
  TrPair f;
  f.lo = ds_tr16(lds_tile + kr0 * (ROWS * 2) + ((c ^ mnmaj_swz<ROWS>(kr0)) << 4) + ((p & 1) << 3));
  f.hi = ds_tr16(lds_tile + kr1 * (ROWS * 2) + ((c ^ mnmaj_swz<ROWS>(kr1)) << 4) + ((p & 1) << 3));
  return f;
}

// fragment register type per operand layout: K-major = compiler-tracked ds_read_b128,
// MN-major = asm TrPair (retire with lgkm_wait0(), read through fval())
template <bool KMAJOR>
struct Frag {
  using T = bf16x8;
};
template <>
struct Frag<false> {
  using T = TrPair;
};

template <bool KMAJOR, int ROWS>
__device__ __forceinline__ typename Frag<KMAJOR>::T load_fragx(const char* lds_tile, int R0, int ks, int lane) {
  if constexpr (KMAJOR) return load_frag<true, ROWS>(lds_tile, R0, ks, lane);
  else return load_frag_tr<ROWS>(lds_tile, R0, ks, lane);
}

__device__ __forceinline__ bf16x8 fval(bf16x8& f) { return f; }
__device__ __forceinline__ bf16x8 fval(TrPair& f) { return tr_use(f); }

template <typename OutT>
__device__ __forceinline__ void load4(const OutT* p, float* v);
template <>
__device__ __forceinline__ void load4<float>(const float* p, float* v) {
  f32x4 x = *(const f32x4*)p;
  v[0] = x[0]; v[1] = x[1]; v[2] = x[2]; v[3] = x[3];
}
template <>
__device__ __forceinline__ void load4<bf16_t>(const bf16_t* p, float* v) {
  uint2 x = *(const uint2*)p;
  v[0] = __uint_as_float(x.x << 16); v[1] = __uint_as_float(x.x & 0xffff0000u);
  v[2] = __uint_as_float(x.y << 16); v[3] = __uint_as_float(x.y & 0xffff0000u);
}
template <typename OutT>
__device__ __forceinline__ void store4(OutT* p, const float* v);
template <>
__device__ __forceinline__ void store4<float>(float* p, const float* v) {
  f32x4 x = {v[0], v[1], v[2], v[3]};
  *(f32x4*)p = x;
}
template <>
__device__ __forceinline__ void store4<bf16_t>(bf16_t* p, const float* v) {
  uint2 x = make_uint2(pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3]));
  *(uint2*)p = x;
}

// Fused epilogue for one lane fragment C[m][n..n+3] (v = alpha-scaled accumulators):
// + bias (bf16/fp32), + beta*Cin, then activation: relu | gelu (pre-activation to aux_out) |
// * gelu'(aux_in) | * relu'(aux_in).
template <typename OutT>
__device__ __forceinline__ void epilogue4(const GemmArgs& a, OutT* C, const OutT* Cin, int m, int n, float* v) {
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

// 8-wide (16-B) form of epilogue4 for bf16 outputs: v = C[m][n..n+7], n % 8 == 0, every
// operand 16-B aligned and ldc % 8 == 0 (checked by the launcher).  Half the global instructions of two epilogue4 calls.
// Buffer descriptor over `bytes` bytes from base + byte_off (wave-uniform inputs; the
// readfirstlanes make that provable to hipcc, else it wraps every buffer op in a waterfall
// loop - cdna_hip_programming.md T20).  A voffset >= bytes (BUF_OOB) loads 0 / drops the store,
// which replaces per-lane bounds branches: records are capped below BUF_OOB.
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
constexpr uint32_t BUF_OOB = 0x80000000u;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, long long byte_off, long long bytes) {
  const uintptr_t u = (uintptr_t)base + byte_off;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)u);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(u >> 32));
  const long long cap = (long long)BUF_OOB - 16;
  const int n = __builtin_amdgcn_readfirstlane((int)(bytes < 0 ? 0 : (bytes > cap ? cap : bytes)));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), 0, n, 0x00020000);
}
__device__ __forceinline__ u32x4 buf_load16(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0);
}
__device__ __forceinline__ void buf_store16(__amdgpu_buffer_rsrc_t r, uint32_t off, u32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(v, r, (int)off, 0, 0);
}
__device__ __forceinline__ void unpack8bf(const u32x4& x, float* v) {
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    v[2 * r] = __uint_as_float(x[r] << 16);
    v[2 * r + 1] = __uint_as_float(x[r] & 0xffff0000u);
  }
}
__device__ __forceinline__ u32x4 pack8bf(const float* v) {
  return u32x4{pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3]), pack_bf2(v[4], v[5]), pack_bf2(v[6], v[7])};
}

// Two MFMA 16x16 fragments x0 / x1 of the same rows (lane: row m, columns 4g..4g+3 of the
// fragment, g = lane >> 4) -> one 8-column run per lane.  v_permlane16_swap exchanges the odd
// 16-lane rows of its first operand with the even rows of its second, so after four swaps
// lane rows g = 0, 1, 2, 3 hold columns 0-7 of x0, 0-7 of x1, 8-15 of x0, 8-15 of x1
// (v = alpha-scaled).  All 64 lanes must execute it (no divergent branch around it).
__device__ __forceinline__ void pair_frags(const f32x4& x0, const f32x4& x1, float alpha, float* v) {
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const auto s = __builtin_amdgcn_permlane16_swap(__float_as_uint(x0[r]), __float_as_uint(x1[r]), false, false);
    v[r] = __uint_as_float(s[0]) * alpha;
    v[4 + r] = __uint_as_float(s[1]) * alpha;
  }
}

// XCD-aware bijective remap of a flat tile id + GROUP_M super-rows (cdna_hip_programming.md
// T1): consecutive tiles on one XCD share A row-panels in its L2.
__device__ __forceinline__ void tile_coords(int bid, int tiles_m, int tiles_n, int& tm, int& tn) {
  const int nwg = tiles_m * tiles_n;
  int wgid = bid;
  if (nwg > 8) {
    const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  }
  constexpr int GROUP_M = 8;
  const int group = wgid / (GROUP_M * tiles_n);
  const int first_m = group * GROUP_M;
  const int gsize = min(tiles_m - first_m, GROUP_M);
  tm = first_m + (wgid % (GROUP_M * tiles_n)) % gsize;
  tn = (wgid % (GROUP_M * tiles_n)) / gsize;
}

}  // namespace rtdc

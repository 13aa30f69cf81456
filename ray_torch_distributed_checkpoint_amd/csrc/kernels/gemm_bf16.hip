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
// Geometry: 128x128 output tile, BK = 64, 256 threads = 4 waves (2x2), each wave 64x64 =
// 4x4 v_mfma_f32_16x16x32_bf16 tiles.  LDS: 2 buffers x (A 16 KiB + B 16 KiB) = 64 KiB.
// Staging: global_load_lds_dwordx4 (1 KiB per wave-instruction, LDS image lane-linear), the
// bank-conflict swizzle applied on the SOURCE address and on the read (cdna_hip_programming.md
// §5.4 rule 21).  The MFMA is issued with the operands swapped (B-data as MFMA "A") so each
// lane's accumulator holds 4 consecutive n of one output row: 8-16 B vector stores.
//
// Batching (attention) uses blockIdx.z with a two-level (outer, inner) stride per operand;
// causal modes skip/limit work for the triangular attention products.
#include "common.h"
#include "args.h"

namespace rtdc {

namespace gemm {
constexpr int BM = 128, BN = 128, BK = 64, NT = 256;
constexpr int TILE_BYTES = 128 * BK * 2;  // 16 KiB per operand tile
}

// ---- LDS image helpers ----------------------------------------------------------------
// K-major image: 128 rows x 128 B (64 bf16 of k).  16-B chunk c of row r lives at
// physical chunk c ^ ((r >> 1) & 7): a ds_read_b128 lane group (16 distinct rows, same
// logical chunk) then touches 16 distinct 16-B slots of the 256-B bank row.
__device__ __forceinline__ int kmaj_off(int row, int chunk) {
  return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4);
}
// MN-major image: 64 k-rows x 256 B (128 bf16 of m or n).  Chunk c of k-row kr lives at
// c ^ f(kr); a 32-lane half of ds_read_b64_tr_b16 reads 8 k-rows x 2 chunks -> 16 slots.
__device__ __forceinline__ int mnmaj_swz(int kr) {
  return ((kr & 3) | (((kr >> 3) & 1) << 2)) << 1;
}

// Issue the global->LDS copy of one operand tile (rows [r0, r0+128), k [k0, k0+64)).
template <bool KMAJOR>
__device__ __forceinline__ void stage_tile(const bf16_t* __restrict__ X, int ld, int rows,
                                           int r0, int k0, char* lds_tile, int wave, int lane) {
#pragma unroll
  for (int ii = 0; ii < 4; ++ii) {
    const int piece = wave * 4 + ii;  // 16 pieces of 1 KiB
    const bf16_t* src;
    if constexpr (KMAJOR) {
      const int row = piece * 8 + (lane >> 3);
      const int pchunk = lane & 7;
      const int lchunk = pchunk ^ ((row >> 1) & 7);
      int gr = r0 + row;
      gr = gr < rows ? gr : rows - 1;
      src = X + (long long)gr * ld + k0 + lchunk * 8;
    } else {
      const int kr = piece * 4 + (lane >> 4);
      const int pchunk = lane & 15;
      const int lchunk = pchunk ^ mnmaj_swz(kr);
      int gc = r0 + lchunk * 8;
      gc = gc < rows ? gc : rows - 8;
      src = X + (long long)(k0 + kr) * ld + gc;
    }
    __builtin_amdgcn_global_load_lds((const void*)src, LDS_PTR(lds_tile + piece * 1024), 16, 0, 0);
  }
}

// Fragment for v_mfma_f32_16x16x32_bf16: lane l holds X(row = R0 + (l&15), k = ks*32 + 8(l>>4) + j).
template <bool KMAJOR>
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
      const int off = kr * 256 + ((c ^ mnmaj_swz(kr)) << 4) + ((p & 1) << 3);
      v[h] = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
          (__attribute__((address_space(3))) bf16x4*)(lds_tile + off));
    }
    bf16x8 r;
    r[0] = v[0][0]; r[1] = v[0][1]; r[2] = v[0][2]; r[3] = v[0][3];
    r[4] = v[1][0]; r[5] = v[1][1]; r[6] = v[1][2]; r[7] = v[1][3];
    return r;
  }
}

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

template <bool AK, bool BKM, typename OutT>
__global__ __launch_bounds__(256, 2) void gemm_bf16_kernel(GemmArgs a) {
  using namespace gemm;
  __shared__ __attribute__((aligned(16))) char smem[4 * TILE_BYTES];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;  // 2x2 waves, 64x64 each

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
  const int nt = ke > kb ? (ke - kb) / BK : 0;

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // buffer b: A tile at smem + 2*b*TILE_BYTES, B tile right after it
#define BUF_A(b) (smem + (b) * 2 * TILE_BYTES)
#define BUF_B(b) (smem + (b) * 2 * TILE_BYTES + TILE_BYTES)

  if (nt > 0) {
    stage_tile<AK>(A, a.lda, a.M, m0, kb, BUF_A(0), wave, lane);
    stage_tile<BKM>(B, a.ldb, a.N, n0, kb, BUF_B(0), wave, lane);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  for (int t = 0; t < nt; ++t) {
    const int cur = t & 1;
    if (t + 1 < nt) {
      stage_tile<AK>(A, a.lda, a.M, m0, kb + (t + 1) * BK, BUF_A(cur ^ 1), wave, lane);
      stage_tile<BKM>(B, a.ldb, a.N, n0, kb + (t + 1) * BK, BUF_B(cur ^ 1), wave, lane);
    }
    const char* tA = BUF_A(cur);
    const char* tB = BUF_B(cur);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 fa[4], fb[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) fa[i] = load_frag<AK>(tA, wm * 64 + i * 16, ks, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[j] = load_frag<BKM>(tB, wn * 64 + j * 16, ks, lane);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[i][j], 0, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

#undef BUF_A
#undef BUF_B
  // ---- epilogue: lane holds C[m][n..n+3] ----
  OutT* C = (OutT*)a.C + coff;
  const OutT* Cin = a.Cin ? (const OutT*)a.Cin + coff : nullptr;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + wm * 64 + i * 16 + (lane & 15);
    if (m >= a.M) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = n0 + wn * 64 + j * 16 + 4 * (lane >> 4);
      if (n >= a.N) continue;
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = acc[i][j][r] * a.alpha;
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
      } else if (a.act == 3 || a.act == 4) {
        float h[4];
        load4<bf16_t>(a.aux_in + off, h);
#pragma unroll
        for (int r = 0; r < 4; ++r)
          v[r] *= (a.act == 3) ? gelu_tanh_grad(h[r]) : (h[r] > 0.f ? 1.f : 0.f);
      }
      store4<OutT>(C + off, v);
    }
  }
}

}  // namespace rtdc

using namespace rtdc;

extern "C" int rtdc_gemm_bf16(const GemmArgs* args, int a_kmajor, int b_kmajor, int out_fp32,
                              int batch, hipStream_t stream) {
  const GemmArgs& a = *args;
  if (a.K % gemm::BK != 0 || a.M % 8 != 0 || a.N % 8 != 0) return 1;
  const int tiles = ((a.M + gemm::BM - 1) / gemm::BM) * ((a.N + gemm::BN - 1) / gemm::BN);
  dim3 grid(tiles, 1, batch), block(gemm::NT);
#define LAUNCH(AK, BKM, T) hipLaunchKernelGGL((gemm_bf16_kernel<AK, BKM, T>), grid, block, 0, stream, a)
  if (out_fp32) {
    if (a_kmajor && b_kmajor) LAUNCH(true, true, float);
    else if (a_kmajor && !b_kmajor) LAUNCH(true, false, float);
    else if (!a_kmajor && !b_kmajor) LAUNCH(false, false, float);
    else LAUNCH(false, true, float);
  } else {
    if (a_kmajor && b_kmajor) LAUNCH(true, true, bf16_t);
    else if (a_kmajor && !b_kmajor) LAUNCH(true, false, bf16_t);
    else if (!a_kmajor && !b_kmajor) LAUNCH(false, false, bf16_t);
    else LAUNCH(false, true, bf16_t);
  }
#undef LAUNCH
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

// Shared device helpers for the gfx950 (CDNA4 / MI355X) kernels.
//
// Everything here is written for wave64: lane ids are `threadIdx.x & 63`, cross-lane
// reductions run over 64 lanes with __shfl_xor, and vector loads are 16 B per lane.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rtdc {

typedef uint16_t bf16_t;  // raw bf16 bits in memory
typedef __attribute__((ext_vector_type(8))) short bf16x8;
typedef __attribute__((ext_vector_type(4))) short bf16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;

#define LDS_PTR(p) ((__attribute__((address_space(3))) void*)(p))

// ---- transposing LDS read (ds_read_b64_tr_b16) as inline asm ---------------------------
// The __builtin_amdgcn_ds_read_tr16_b64 form makes hipcc (ROCm 7.2) emit `s_waitcnt
// vmcnt(0)` in front of every such read while any global_load_lds is in flight (checked in the
// .s: one full drain of the DMA pipeline per group of transposing reads), which serialises
// every DMA-fed loop that reads an MN-major / transposed operand.  The asm form is invisible
// to hipcc's wait bookkeeping, so the protocol is explicit (cdna_hip_programming.md §5.7):
// issue with ds_tr16(), retire with lgkm_wait0(), then pass each result through tr_use()
// (an asm that names the registers, so no consumer is scheduled above the wait) before any
// other use.  LDS ops return in order; an lgkmcnt(0) also covers hipcc's own LDS ops.
struct TrPair {
  bf16x4 lo, hi;
};

__device__ __forceinline__ bf16x4 ds_tr16(const char* p) {
  bf16x4 r;
  const uint32_t a = (uint32_t)(uintptr_t)((const __attribute__((address_space(3))) char*)p);
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r) : "v"(a) : "memory");
  return r;
}

// max without fmaxf's NaN-canonicalising v_max x,x,x on each operand
__device__ __forceinline__ float vmax_raw(float a, float b) {
  float r;
  asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

// all-reduce max over the lanes l, l^16, l^32, l^48 (the 4 rows of 16 lanes of a wave64) with the
// gfx950 VALU row swaps - no LDS round trip (a __shfl_xor is a ds_bpermute plus its lgkm wait).
// permlane16_swap(x, x) leaves rows (0,0,2,2) in one result and (1,1,3,3) in the other, and
// permlane32_swap(x, x) the halves (lo,lo) / (hi,hi): the max of each pair is the xor-16 /
// xor-32 reduction.
__device__ __forceinline__ float max_rows4(float v) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = vmax_raw(__uint_as_float(r[0]), __uint_as_float(r[1]));
  const auto q = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return vmax_raw(__uint_as_float(q[0]), __uint_as_float(q[1]));
}

__device__ __forceinline__ float sum_rows4(float v) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  const auto q = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(q[0]) + __uint_as_float(q[1]);
}

// XCD-aware bijective remap of a 2-D grid (cdna_hip_programming.md T1): the hardware deals
// consecutive workgroups round-robin to the 8 XCDs (flat id % 8), each with its own L2.  Returns
// the logical (x, y) such that each XCD receives a CONTIGUOUS run of the x-fastest logical order:
// the blocks of one y (e.g. all query blocks of one attention head) share one L2 instead of
// pulling the same K/V through all eight.
// x_major: when every XCD gets whole rows (gridDim.y % 8 == 0), walk the XCD's rows x-major
// instead (x = 0 of all its rows first, then x = 1, ...): with x ordered heaviest-first this
// starts every long block early instead of leaving the last row's long block as the tail.
__device__ __forceinline__ void xcd_grid(int& x, int& y, bool x_major = false) {
  const int nx = gridDim.x, n = nx * gridDim.y;
  const int bid = blockIdx.x + blockIdx.y * nx;
  const int xcd = bid & 7, q = n >> 3, r = n & 7;
  if (x_major && (gridDim.y & 7) == 0) {
    const int rows = gridDim.y >> 3, local = bid >> 3;  // this XCD: rows [xcd*rows, +rows)
    x = local / rows;
    y = xcd * rows + (local - x * rows);
    return;
  }
  const int l = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  y = l / nx;
  x = l - y * nx;
}

__device__ __forceinline__ void lgkm_wait0() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

__device__ __forceinline__ bf16x8 tr_use(TrPair& f) {
  asm volatile("" : "+v"(f.lo), "+v"(f.hi));
  bf16x8 r;
  r[0] = f.lo[0]; r[1] = f.lo[1]; r[2] = f.lo[2]; r[3] = f.lo[3];
  r[4] = f.hi[0]; r[5] = f.hi[1]; r[6] = f.hi[2]; r[7] = f.hi[3];
  return r;
}

__device__ __forceinline__ float bf2f(bf16_t v) {
  return __uint_as_float(((uint32_t)v) << 16);
}

// Round-to-nearest-even f32 -> bf16.  A plain cast lowers to v_cvt_pk_bf16_f32 on gfx950
// (keeps NaN a NaN, MI355X_MICROARCH.md "Correctness boundaries").
__device__ __forceinline__ bf16_t f2bf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(bf16_t, b);
}

__device__ __forceinline__ uint32_t pack_bf2(float lo, float hi) {
  return (uint32_t)f2bf(lo) | ((uint32_t)f2bf(hi) << 16);
}

// Wave64 all-reduces entirely in the VALU: DPP within each 16-lane row (quad_perm xor 1 and
// xor 2, row_half_mirror, row_mirror pair every lane with one from the other quad / half), then
// the gfx950 row swaps across rows (max_rows4 above).  __shfl_xor lowers to ds_bpermute: six
// dependent LDS round trips with an lgkm wait each.  Every lane ends with the bitwise-same value
// (each step adds a commutative pair).
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float row16_sum(float v) {
  v += dpp_f<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_f<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_f<0x141>(v);  // row_half_mirror
  v += dpp_f<0x140>(v);  // row_mirror
  return v;
}
__device__ __forceinline__ float row16_max(float v) {
  v = vmax_raw(v, dpp_f<0xB1>(v));
  v = vmax_raw(v, dpp_f<0x4E>(v));
  v = vmax_raw(v, dpp_f<0x141>(v));
  v = vmax_raw(v, dpp_f<0x140>(v));
  return v;
}
__device__ __forceinline__ float wave_sum(float v) { return sum_rows4(row16_sum(v)); }
__device__ __forceinline__ float wave_max(float v) { return max_rows4(row16_max(v)); }

// Block reduction for blockDim.x == NT (multiple of 64).  `red` must hold NT/64 floats.
template <int NT>
__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  if (l == 0) red[w] = v;
  __syncthreads();
  float r = 0.f;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) r += red[i];
  __syncthreads();
  return r;
}

template <int NT>
__device__ __forceinline__ float block_max(float v, float* red) {
  v = wave_max(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  if (l == 0) red[w] = v;
  __syncthreads();
  float r = -INFINITY;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) r = fmaxf(r, red[i]);
  __syncthreads();
  return r;
}

// tanh-approximation GELU (GPT-2) and its derivative, through the logistic form
//   0.5 (1 + tanh(u)) = s = 1 / (1 + e^{-2u}),   1 - tanh(u)^2 = 4 s (1 - s)
// so each costs one v_exp_f32 and one v_rcp_f32 instead of a libm tanhf (these run in the
// GEMM epilogues of c_fc forward and c_proj dgrad, over 50M elements per GPT-2 layer).
// |x| large: e -> inf gives s = 0 (x * 0 = -0 for x -> -inf, the exact limit) and e -> 0 gives
// s = 1; no NaN for finite x.
__device__ __forceinline__ float gelu_sigmoid_arg(float x) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f, m2log2e = -2.0f * 1.4426950408889634f;
  const float u = k0 * fmaf(k1 * x, x * x, x);
  return __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(m2log2e * u));
}
__device__ __forceinline__ float gelu_tanh(float x) { return x * gelu_sigmoid_arg(x); }
__device__ __forceinline__ float gelu_tanh_grad(float x) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  const float s = gelu_sigmoid_arg(x);
  return fmaf(2.f * x * s * (1.f - s) * k0, fmaf(3.f * k1, x * x, 1.f), s);
}
// gelu(x) and gelu'(x) from one sigmoid (the forward epilogue that stores the derivative for
// the backward: act 5)
__device__ __forceinline__ float gelu_tanh_and_grad(float x, float& g) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  const float s = gelu_sigmoid_arg(x);
  g = fmaf(2.f * x * s * (1.f - s) * k0, fmaf(3.f * k1, x * x, 1.f), s);
  return x * s;
}

// Philox4x32-10 counter-based RNG: deterministic function of (seed, counter), so dropout
// masks are regenerated in backward and on resume from (seed, offset) alone.
struct Philox {
  __device__ static inline uint4 round(uint4 c, uint2 k) {
    const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
    uint32_t hi0 = __umulhi(M0, c.x), lo0 = M0 * c.x;
    uint32_t hi1 = __umulhi(M1, c.z), lo1 = M1 * c.z;
    return make_uint4(hi1 ^ c.y ^ k.x, lo1, hi0 ^ c.w ^ k.y, lo0);
  }
  __device__ static inline uint4 gen(uint64_t seed, uint64_t ctr_hi, uint64_t ctr_lo) {
    uint4 c = make_uint4((uint32_t)ctr_lo, (uint32_t)(ctr_lo >> 32), (uint32_t)ctr_hi,
                         (uint32_t)(ctr_hi >> 32));
    uint2 k = make_uint2((uint32_t)seed, (uint32_t)(seed >> 32));
#pragma unroll
    for (int i = 0; i < 10; ++i) {
      c = round(c, k);
      k.x += 0x9E3779B9u;
      k.y += 0xBB67AE85u;
    }
    return c;
  }
};

__device__ __forceinline__ float u32_to_unit(uint32_t x) {  // [0,1)
  return (float)(x >> 8) * (1.0f / 16777216.0f);
}

}  // namespace rtdc

// Llama-3 elementwise ops for gfx950: rotary position embedding on the packed QKV buffer and
// the SwiGLU gate.  Trig comes from host-precomputed cos/sin tables [T][Dh/2] (theta=500000),
// never from on-device sin/cos (cdna_hip_programming.md Appendix B "Element-wise"); bf16 moves
// 16 B per lane.
#include "common.h"

namespace rtdc {

__device__ __forceinline__ void ld8r(const bf16_t* p, float* v) {
  uint4 x = *(const uint4*)p;
  uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[2 * i] = __uint_as_float(w[i] << 16);
    v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}
__device__ __forceinline__ void st8r(bf16_t* p, const float* v) {
  *(uint4*)p = make_uint4(pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3]), pack_bf2(v[4], v[5]), pack_bf2(v[6], v[7]));
}

// HF "rotate_half" convention: (x1, x2) = halves of each head;
//   fwd: y1 = x1 c - x2 s ; y2 = x2 c + x1 s        bwd (sign = -1): rotate by -theta.
// One thread handles 8 pairs (i .. i+7) of one (token, head).  Heads [0, Hq+Hk) are rotated
// (q and k), the V heads are copied, so `out` is the full packed tensor.
__global__ __launch_bounds__(256) void rope_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y,
                                                  const float* __restrict__ cosb, const float* __restrict__ sinb,
                                                  int ntok, int T, int nrot_heads, int ntot_heads, int Dh,
                                                  float sign) {
  const int half = Dh / 2, per_head = half / 8;
  const long long total = (long long)ntok * ntot_heads * per_head;
  for (long long w = blockIdx.x * 256LL + threadIdx.x; w < total; w += (long long)gridDim.x * 256) {
    const int c8 = (int)(w % per_head);
    const long long th = w / per_head;
    const int head = (int)(th % ntot_heads);
    const long long tok = th / ntot_heads;
    const int t = (int)(tok % T);
    const long long base = (tok * ntot_heads + head) * Dh;
    const int i0 = c8 * 8;
    float a[8], b[8];
    ld8r(x + base + i0, a);
    ld8r(x + base + half + i0, b);
    if (head < nrot_heads) {
      const float* cs = cosb + (long long)t * half + i0;
      const float* sn = sinb + (long long)t * half + i0;
      float o1[8], o2[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float c = cs[e], s = sn[e] * sign;
        o1[e] = a[e] * c - b[e] * s;
        o2[e] = b[e] * c + a[e] * s;
      }
      st8r(y + base + i0, o1);
      st8r(y + base + half + i0, o2);
    } else {
      st8r(y + base + i0, a);
      st8r(y + base + half + i0, b);
    }
  }
}

__device__ __forceinline__ float silu(float g) { return g / (1.f + __expf(-g)); }

// gu: [M][2F] = [gate | up] (one fused GEMM output); h = silu(gate) * up  -> [M][F]
__global__ __launch_bounds__(256) void swiglu_fwd_kernel(const bf16_t* __restrict__ gu, bf16_t* __restrict__ h,
                                                        long long M, int F) {
  const long long total = M * (F / 8);
  for (long long w = blockIdx.x * 256LL + threadIdx.x; w < total; w += (long long)gridDim.x * 256) {
    const long long m = w / (F / 8);
    const int f = (int)(w % (F / 8)) * 8;
    float g[8], u[8], o[8];
    ld8r(gu + m * 2 * F + f, g);
    ld8r(gu + m * 2 * F + F + f, u);
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = silu(g[e]) * u[e];
    st8r(h + m * F + f, o);
  }
}

// dgu = [dh * up * silu'(gate) | dh * silu(gate)]
__global__ __launch_bounds__(256) void swiglu_bwd_kernel(const bf16_t* __restrict__ gu, const bf16_t* __restrict__ dh,
                                                        bf16_t* __restrict__ dgu, long long M, int F) {
  const long long total = M * (F / 8);
  for (long long w = blockIdx.x * 256LL + threadIdx.x; w < total; w += (long long)gridDim.x * 256) {
    const long long m = w / (F / 8);
    const int f = (int)(w % (F / 8)) * 8;
    float g[8], u[8], d[8], og[8], ou[8];
    ld8r(gu + m * 2 * F + f, g);
    ld8r(gu + m * 2 * F + F + f, u);
    ld8r(dh + m * F + f, d);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float sg = 1.f / (1.f + __expf(-g[e]));
      const float si = g[e] * sg;
      og[e] = d[e] * u[e] * (sg * (1.f + g[e] * (1.f - sg)));
      ou[e] = d[e] * si;
    }
    st8r(dgu + m * 2 * F + f, og);
    st8r(dgu + m * 2 * F + F + f, ou);
  }
}

}  // namespace rtdc

using namespace rtdc;

static inline unsigned grid_of(long long work) {
  long long b = (work + 255) / 256;
  if (b > 16384) b = 16384;
  if (b < 1) b = 1;
  return (unsigned)b;
}

extern "C" int rtdc_rope(const void* x, void* y, const float* cosb, const float* sinb, int ntok, int T,
                         int nrot_heads, int ntot_heads, int Dh, int inverse, hipStream_t st) {
  if (Dh % 16 != 0) return 1;
  const long long work = (long long)ntok * ntot_heads * (Dh / 16);
  hipLaunchKernelGGL(rope_kernel, dim3(grid_of(work)), dim3(256), 0, st, (const bf16_t*)x, (bf16_t*)y, cosb, sinb,
                     ntok, T, nrot_heads, ntot_heads, Dh, inverse ? -1.f : 1.f);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

extern "C" int rtdc_swiglu_fwd(const void* gu, void* h, long long M, int F, hipStream_t st) {
  if (F % 8 != 0) return 1;
  hipLaunchKernelGGL(swiglu_fwd_kernel, dim3(grid_of(M * (F / 8))), dim3(256), 0, st, (const bf16_t*)gu, (bf16_t*)h,
                     M, F);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

extern "C" int rtdc_swiglu_bwd(const void* gu, const void* dh, void* dgu, long long M, int F, hipStream_t st) {
  if (F % 8 != 0) return 1;
  hipLaunchKernelGGL(swiglu_bwd_kernel, dim3(grid_of(M * (F / 8))), dim3(256), 0, st, (const bf16_t*)gu,
                     (const bf16_t*)dh, (bf16_t*)dgu, M, F);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

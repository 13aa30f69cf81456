// fp32 GEMM on the gfx950 f32-input MFMA (v_mfma_f32_16x16x4_f32: exact f32, k-ordered fmaf
// chain - cdna_hip_programming.md §3 "FP32-input MFMA") with fused bias / ReLU / residual /
// ReLU-backward epilogues.  Serves the fp32 reference workload (the toy MLP of
// R/my_ray_module.py:94-112 at batch 16: M = 16, K = 784/512, N = 512/10), which is latency-
// bound, so the kernel favours arbitrary strides and shapes (no divisibility requirements)
// over peak throughput: any operand layout is described by (row stride, k stride).
//
// Latency-first structure (the toy GEMMs are 0.1-13 MFLOP, far from any throughput limit):
// a block owns a 16(M) x 64(N) output tile and splits K over KW waves (KW = 1..16, chosen so
// every wave has >= 4 four-deep k-steps); lanes load their MFMA operands straight from global
// memory (L2-resident, no LDS staging, no barriers in the loop, 4-step unroll keeps ~20 loads
// in flight) and the KW partial tiles are summed in LDS in fixed wave order before the fused
// epilogue - deterministic, one launch.
#include "common.h"
#include "args.h"

namespace rtdc {

namespace gf32 {
constexpr int BM = 16, BN = 64;
}

__global__ __launch_bounds__(1024) void gemm_f32_kernel(GemmF32Args a) {
  using namespace gf32;
  __shared__ float part[16][BM * BN];  // per-wave partial tiles (64 KiB at KW = 16)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int kw = blockDim.x >> 6;
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
  const int gm = m0 + (lane & 15);
  const bool mok = gm < a.M;
  f32x4 acc[4] = {f32x4{0, 0, 0, 0}, f32x4{0, 0, 0, 0}, f32x4{0, 0, 0, 0}, f32x4{0, 0, 0, 0}};
  int gn[4];
  bool nok[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    gn[j] = n0 + 16 * j + (lane & 15);
    nok[j] = gn[j] < a.N;
  }
  const int ksteps = (a.K + 3) / 4;
#pragma unroll 4
  for (int ks = wave; ks < ksteps; ks += kw) {
    const int gk = ks * 4 + (lane >> 4);
    const bool kok = gk < a.K;
    const float av = (mok && kok) ? a.A[(long long)gm * a.sam + (long long)gk * a.sak] : 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float bv = (nok[j] && kok) ? a.B[(long long)gk * a.sbk + (long long)gn[j] * a.sbn] : 0.f;
      acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc[j], 0, 0, 0);
    }
  }
  // D layout of 16x16x4 f32: lane holds rows 4*(lane>>4)+r, column lane&15
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) part[wave][(4 * (lane >> 4) + r) * BN + 16 * j + (lane & 15)] = acc[j][r];
  __syncthreads();
  const float dscale = a.drop_p > 0.f ? 1.f / (1.f - a.drop_p) : 1.f;
  const unsigned long long doff = a.drop_offset + (a.drop_base ? (unsigned long long)*a.drop_base : 0ull);
  for (int e = tid; e < BM * BN; e += blockDim.x) {
    const int m = m0 + e / BN, n = n0 + e % BN;
    if (m >= a.M || n >= a.N) continue;
    float v = 0.f;
    for (int w = 0; w < kw; ++w) v += part[w][e];
    const long long off = (long long)m * a.ldc + n;
    v *= a.alpha;
    if (a.bias) v += a.bias[n];
    if (a.Cin && a.beta != 0.f) v += a.beta * a.Cin[off];
    if (a.act == 1) {
      if (a.aux_out) a.aux_out[off] = v;
      v = fmaxf(v, 0.f);
      if (a.drop_p > 0.f) {  // fused inverted dropout (ReLU -> Dropout of the toy MLP)
        const uint4 r = Philox::gen(a.drop_seed, 0, doff + (unsigned long long)(off >> 2));
        const int l = (int)(off & 3);
        const uint32_t u = l == 0 ? r.x : (l == 1 ? r.y : (l == 2 ? r.z : r.w));
        v = u32_to_unit(u) >= a.drop_p ? v * dscale : 0.f;
      }
    } else if (a.act == 4) {
      v = a.aux_in[off] > 0.f ? v : 0.f;
    }
    a.C[off] = v;
  }
}

}  // namespace rtdc

using namespace rtdc;

extern "C" int rtdc_gemm_f32(const GemmF32Args* args, hipStream_t st) {
  const GemmF32Args& a = *args;
  const int ksteps = (a.K + 3) / 4;
  int kw = ksteps / 16;  // >= 16 k-steps (four 4-deep unrolled rounds) per wave
  kw = kw < 1 ? 1 : (kw > 16 ? 16 : kw);
  dim3 grid((a.N + gf32::BN - 1) / gf32::BN, (a.M + gf32::BM - 1) / gf32::BM), block(64 * kw);
  hipLaunchKernelGGL(gemm_f32_kernel, grid, block, 0, st, a);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

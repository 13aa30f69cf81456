// fp32 GEMM on the gfx950 f32-input MFMA (v_mfma_f32_16x16x4_f32: exact f32, k-ordered fmaf
// chain - cdna_hip_programming.md §3 "FP32-input MFMA") with fused bias / ReLU / residual /
// ReLU-backward epilogues.  Serves the fp32 reference workload (the toy MLP of
// R/my_ray_module.py:94-112 at batch 16: M = 16, K = 784/512, N = 512/10), which is latency-
// bound, so the kernel favours arbitrary strides and shapes (no divisibility requirements)
// over peak throughput: any operand layout is described by (row stride, k stride).
//
// Tile 32(M) x 64(N) x 32(K), 4 waves as 2x2, each wave 16x32 = 2 MFMA tiles.
#include "common.h"
#include "args.h"

namespace rtdc {

namespace gf32 {
constexpr int BM = 32, BN = 64, BK = 32;
}

__global__ __launch_bounds__(256) void gemm_f32_kernel(GemmF32Args a) {
  using namespace gf32;
  __shared__ float As[BK][BM + 1];
  __shared__ float Bs[BK][BN + 1];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
  f32x4 acc[2] = {f32x4{0, 0, 0, 0}, f32x4{0, 0, 0, 0}};
  const bool a_kfast = a.sak == 1;
  const bool b_nfast = a.sbn == 1;
  for (int k0 = 0; k0 < a.K; k0 += BK) {
    for (int idx = tid; idx < BM * BK; idx += 256) {
      int m, k;
      if (a_kfast) { m = idx / BK; k = idx % BK; } else { k = idx / BM; m = idx % BM; }
      const int gm = m0 + m, gk = k0 + k;
      As[k][m] = (gm < a.M && gk < a.K) ? a.A[gm * a.sam + gk * a.sak] : 0.f;
    }
    for (int idx = tid; idx < BN * BK; idx += 256) {
      int n, k;
      if (b_nfast) { k = idx / BN; n = idx % BN; } else { n = idx / BK; k = idx % BK; }
      const int gn = n0 + n, gk = k0 + k;
      Bs[k][n] = (gn < a.N && gk < a.K) ? a.B[gk * a.sbk + gn * a.sbn] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < BK / 4; ++kk) {
      const float av = As[kk * 4 + (lane >> 4)][wm * 16 + (lane & 15)];
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const float bv = Bs[kk * 4 + (lane >> 4)][wn * 32 + j * 16 + (lane & 15)];
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc[j], 0, 0, 0);
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int n = n0 + wn * 32 + j * 16 + (lane & 15);
    if (n >= a.N) continue;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = m0 + wm * 16 + (lane >> 4) * 4 + r;
      if (m >= a.M) continue;
      const long long off = (long long)m * a.ldc + n;
      float v = acc[j][r] * a.alpha;
      if (a.bias) v += a.bias[n];
      if (a.Cin && a.beta != 0.f) v += a.beta * a.Cin[off];
      if (a.act == 1) {
        if (a.aux_out) a.aux_out[off] = v;
        v = fmaxf(v, 0.f);
      } else if (a.act == 4) {
        v = a.aux_in[off] > 0.f ? v : 0.f;
      }
      a.C[off] = v;
    }
  }
}

}  // namespace rtdc

using namespace rtdc;

extern "C" int rtdc_gemm_f32(const GemmF32Args* args, hipStream_t st) {
  const GemmF32Args& a = *args;
  dim3 grid((a.N + gf32::BN - 1) / gf32::BN, (a.M + gf32::BM - 1) / gf32::BM), block(256);
  hipLaunchKernelGGL(gemm_f32_kernel, grid, block, 0, st, a);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

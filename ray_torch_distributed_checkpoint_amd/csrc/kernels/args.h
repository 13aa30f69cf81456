// Launch-argument structs shared by the HIP kernels and the host bindings.
#pragma once
#include <stdint.h>

namespace rtdc {

// bf16 MFMA GEMM (gemm_bf16.hip)
struct GemmArgs {
  const uint16_t* A;
  const uint16_t* B;
  void* C;
  const void* Cin;        // added as beta*Cin (same dtype as C); may alias C
  const void* bias;       // [N], bf16 or fp32
  const uint16_t* aux_in; // act-backward input (pre-activation), ld = ldc
  uint16_t* aux_out;      // act-forward pre-activation output, ld = ldc
  int M, N, K;
  int lda, ldb, ldc;
  long long sA0, sA1, sB0, sB1, sC0, sC1;
  int batch_inner;
  float alpha, beta;
  const float* alpha_dev;  // optional device scalar multiplied into alpha (upstream loss grad)
  int act;        // 0 none, 1 relu, 2 gelu_tanh (aux_out = pre-activation), 3 *gelu'(aux_in),
                  // 4 *relu'(aux_in), 5 gelu_tanh (aux_out = gelu'(pre-activation)), 6 *aux_in
  int causal;     // 0 none, 1 skip tiles with n0 > m_last, 2 k < m0+BM, 3 k >= m0
  int bias_type;  // 0 none, 1 bf16, 2 fp32
  // split-K (plain epilogue only): fp32 partial slabs [splitk][M][N] reduced by a second kernel
  float* ws;
  long long ws_elems;
  int splitk;     // set by the launcher
  int tile_cfg;   // -1 = auto; else force a tile configuration (benchmarks)
  // implicit-GEMM convolution (rtdc_conv_gemm): operand gathered from an NHWC tensor
  // X [B][cv_H][cv_W][cv_C] through a KHxKW window (stride, pad) over a cv_Ho x cv_Wo grid of
  // cv_npix output pixels.  Mode 1: A(m = pixel, k = tap*C + c), mode 2: B(k = pixel, n = tap*C + c).
  int cv_H, cv_W, cv_C, cv_Ho, cv_Wo, cv_KW, cv_stride, cv_pad, cv_npix;
  // optional fused BatchNorm statistics of the (bf16-rounded) output, mode 1 only:
  // per row-tile t and column n: mean and M2 over the tile's rows -> [tiles_m][N] each
  float* stats_mean;
  float* stats_m2;
  // optional column sums of the bf16 output C (bias gradient of the next layer down):
  // cs_out [N] (overwritten), cs_ws >= (tiles_m * 4 + 64) * N floats of scratch.  Fused into
  // the 8-wave kernels' gelu-backward epilogue, a separate reduction otherwise.
  float* cs_out;
  float* cs_ws;
  long long cs_ws_elems;
  // optional fused BatchNorm-BACKWARD statistics (implicit-GEMM stride-1 dgrad, mode 1): the
  // output C is the gradient g at the output of relu(BN(x)) with x = bnb_x ([M][N], ld = ldc);
  // per row-tile t and column n: sum g*mask and sum g*mask*xhat -> stats_mean / stats_m2
  // (mask = BN(x) > 0 recomputed from x, xhat = (x - mean) * rstd)
  const uint16_t* bnb_x;
  const float* bnb_mean;
  const float* bnb_rstd;
  const float* bnb_gamma;
  const float* bnb_beta;
  const uint16_t* bnb_y;  // optional: mask = bnb_y > 0 (BN + residual + ReLU output) instead
};

// fp32 MFMA GEMM (gemm_f32.hip)
struct GemmF32Args {
  const float* A;
  const float* B;
  float* C;
  const float* Cin;
  const float* bias;
  const float* aux_in;
  float* aux_out;
  int M, N, K;
  long long sam, sak, sbk, sbn;  // A(m,k) = A[m*sam + k*sak]; B(k,n) = B[k*sbk + n*sbn]
  int ldc;
  float alpha, beta;
  int act;  // 0 none, 1 relu (aux_out gets pre-activation if set), 4 relu-backward via aux_in
  // fused dropout after the ReLU (act 1, drop_p > 0): element i = m * ldc + n keeps with
  // Philox4x32(seed, counter = drop_offset (+ *drop_base) + i / 4) lane i % 4 >= drop_p - the
  // dropout kernel's exact stream, so the fused and unfused forms draw the same mask
  float drop_p;
  unsigned long long drop_seed, drop_offset;
  const long long* drop_base;
};

}  // namespace rtdc

// Launchers of the 8-wave / 4-wave 256-row GEMM kernels (kernels and schedules: gemm_8ph.h).
#include "gemm_8ph.h"

#include <cstdlib>

using namespace rtdc;

static int g_num_cus = 0;

#ifndef RTDC_G4_ONLY  // (-DRTDC_G4_ONLY: a quick build of the 4-wave kernel alone for ISA inspection)
// Launch the 8-phase kernel (batch 1, no causal modes).  a->splitk is honoured as set.
// bn: 256, 192 or 128 (output tile columns; 128: bf16 output, K-major A only - else returns 1)
extern "C" int rtdc_gemm8_launch(const GemmArgs* args, int a_kmajor, int b_kmajor, int out_fp32, int bn,
                                 hipStream_t st) {
  const GemmArgs& a = *args;
  const unsigned tiles = (unsigned)(((a.M + 255) / 256) * ((a.N + bn - 1) / bn));
  dim3 grid(tiles, a.splitk > 1 ? a.splitk : 1, 1), block(512);
  if (bn == 128) {
    if (out_fp32 || !a_kmajor) return 1;
    if (b_kmajor) hipLaunchKernelGGL((g8::gemm8_kernel<true, true, bf16_t, 128>), grid, block, 0, st, a);
    else hipLaunchKernelGGL((g8::gemm8_kernel<true, false, bf16_t, 128>), grid, block, 0, st, a);
    return hipGetLastError() == hipSuccess ? 0 : 2;
  }
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

// Persistent launch (gemm8p_kernel): grid = min(tiles, #CUs rounded down to a multiple of 8);
// plain (non split-K) products with K >= 128 only.
extern "C" int rtdc_gemm8p_launch(const GemmArgs* args, int a_kmajor, int b_kmajor, int out_fp32, int bn,
                                  hipStream_t st) {
  const GemmArgs& a = *args;
  if (a.splitk > 1 || a.K < 2 * gemm::BK) return 1;
  if (g_num_cus == 0) {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
    g_num_cus = n;
  }
  const long long tiles = (long long)((a.M + 255) / 256) * ((a.N + bn - 1) / bn);
  long long gsz = (g_num_cus / 8) * 8;
  if (gsz < 8) gsz = 8;
  if (tiles < gsz) gsz = tiles;
  dim3 grid((unsigned)gsz, 1, 1), block(512);
#define G8P(AK, BKM, T)                                                                             \
  do {                                                                                              \
    if (bn == 192) hipLaunchKernelGGL((g8::gemm8p_kernel<AK, BKM, T, 192>), grid, block, 0, st, a); \
    else hipLaunchKernelGGL((g8::gemm8p_kernel<AK, BKM, T, 256>), grid, block, 0, st, a);           \
  } while (0)
  if (out_fp32) {
    if (a_kmajor && b_kmajor) G8P(true, true, float);
    else if (a_kmajor) G8P(true, false, float);
    else if (!b_kmajor) G8P(false, false, float);
    else G8P(false, true, float);
  } else {
    if (a_kmajor && b_kmajor) G8P(true, true, bf16_t);
    else if (a_kmajor) G8P(true, false, bf16_t);
    else if (!b_kmajor) G8P(false, false, bf16_t);
    else G8P(false, true, bf16_t);
  }
#undef G8P
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

#endif  // RTDC_G4_ONLY

// Grouped 8-wave launch (gemm8g_kernel): n <= 8 products, every one K % 64 == 0, splitk 1,
// 256x256 tiles; layouts and output dtype shared.  Returns 1 for an unsupported group.
extern "C" int rtdc_gemm8_grouped(const GemmArgs* args, int n, int a_kmajor, int b_kmajor, int out_fp32,
                                  hipStream_t st) {
  if (n < 1 || n > g8::G8_MAX_GROUP) return 1;
  g8::GemmGroup gg{};
  int tiles = 0;
  for (int i = 0; i < n; ++i) {
    const GemmArgs& a = args[i];
    if (a.K % gemm::BK != 0 || a.K < gemm::BK || a.splitk > 1 || a.M % 8 != 0 || a.N % 8 != 0) return 1;
    gg.g[i] = a;
    gg.g[i].splitk = 1;
    gg.start[i] = tiles;
    tiles += ((a.M + 255) / 256) * ((a.N + 255) / 256);
  }
  gg.start[n] = tiles;
  gg.n = n;
  if (!out_fp32 || a_kmajor || b_kmajor) return 1;
  // persistent form (gemm8gp_kernel) when every product has the same K >= 128: one block per CU
  // walks its tiles with the next tile's loads in flight under this tile's epilogue.
  // RTDC_G8G_PERSIST=0 keeps one block per tile (A/B switch; read once).
  static int persist = -1;
  if (persist < 0) {
    const char* e = std::getenv("RTDC_G8G_PERSIST");
    persist = (e && e[0] == '0') ? 0 : 1;
  }
  bool same_k = args[0].K >= 2 * gemm::BK;
  for (int i = 1; i < n; ++i) same_k = same_k && args[i].K == args[0].K;
  if (persist && same_k) {
    if (g_num_cus == 0) {
      int dev = 0, c = 0;
      if (hipGetDevice(&dev) != hipSuccess ||
          hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || c <= 0)
        c = 256;
      g_num_cus = c;
    }
    long long gsz = (g_num_cus / 8) * 8;
    if (gsz < 8) gsz = 8;
    if (tiles < gsz) gsz = tiles;
    hipLaunchKernelGGL((g8::gemm8gp_kernel<false, false>), dim3((unsigned)gsz), dim3(512), 0, st, gg);
    return hipGetLastError() == hipSuccess ? 0 : 2;
  }
  dim3 grid((unsigned)tiles, 1, 1), block(512);
  hipLaunchKernelGGL((g8::gemm8g_kernel<false, false, float>), grid, block, 0, st, gg);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

// 4-wave 256x256 kernel (gemm4_kernel): same contract as rtdc_gemm8_launch with bn = 256.
extern "C" int rtdc_gemm4_launch(const GemmArgs* args, int a_kmajor, int b_kmajor, int out_fp32, hipStream_t st) {
  const GemmArgs& a = *args;
  const unsigned tiles = (unsigned)(((a.M + 255) / 256) * ((a.N + 255) / 256));
  dim3 grid(tiles, a.splitk > 1 ? a.splitk : 1, 1), block(256);
#define G4(AK, BKM, T) hipLaunchKernelGGL((g8::gemm4_kernel<AK, BKM, T>), grid, block, 0, st, a)
  if (out_fp32) {
    if (a_kmajor && b_kmajor) G4(true, true, float);
    else if (a_kmajor) G4(true, false, float);
    else if (!b_kmajor) G4(false, false, float);
    else G4(false, true, float);
  } else {
    if (a_kmajor && b_kmajor) G4(true, true, bf16_t);
    else if (a_kmajor) G4(true, false, bf16_t);
    else if (!b_kmajor) G4(false, false, bf16_t);
    else G4(false, true, bf16_t);
  }
#undef G4
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

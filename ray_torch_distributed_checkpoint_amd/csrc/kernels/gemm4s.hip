// Persistent stream-K 4-wave GEMM launcher (kernel: gemm4s.h; per-epilogue instantiations:
// gemm4s_a0/a2/a3.hip, compiled in parallel).
#include "gemm4s.h"

using namespace rtdc;

// Workspace per (device, stream): arrival counters (zeroed once; every finisher resets its own)
// and 2 x G partial images.  Two launches on one stream are ordered; launches on different
// streams use different workspaces.  Allocated outside graph capture only (a launch that would
// need a first allocation while its stream is capturing returns 3: the caller picks another
// kernel).
#include <map>
#include <mutex>
#include <utility>

namespace {
struct SkWs {
  int* cnt = nullptr;
  float* part = nullptr;
  int cnt_n = 0;
  long long part_n = 0;
};
std::mutex g_sk_mu;
std::map<std::pair<int, hipStream_t>, SkWs> g_sk_ws;
int g_ncu[64] = {0};

int num_cus(int dev) {
  if (dev < 0 || dev >= 64) return 256;
  if (!g_ncu[dev]) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    g_ncu[dev] = n;
  }
  return g_ncu[dev];
}
}  // namespace

// plan of a product on G blocks (host side of the kernel's SkArgs); returns false when there is
// nothing to split (the caller may still launch: d * G == tiles)
static void sk_plan(int tiles, int nt, int G, g8::SkArgs& s) {
  s.G = G;
  s.tiles = tiles;
  s.nt = nt;
  const int full = tiles / G, rem = tiles % G;
  s.d = rem == 0 ? full : (full > 0 ? full - 1 : 0);
  const long long I = (long long)(tiles - s.d * G) * nt;
  s.I_sk = (int)I;
  s.P = I > 0 ? (int)((I + G - 1) / G) : 0;
}

extern "C" int rtdc_gemm4s_launch(const GemmArgs* args, int a_kmajor, int b_kmajor, hipStream_t st) {
  const GemmArgs& a = *args;
  if (a.K % gemm::BK || a.splitk > 1 || !a_kmajor || (a.act != 0 && a.act != 2 && a.act != 3)) return 1;
  // buffer-descriptor DMA: every operand byte offset must fit the 32-bit range
  const long long eA = (long long)a.M * a.lda, eB = b_kmajor ? (long long)a.N * a.ldb : (long long)a.K * a.ldb;
  if (eA * 2 >= (1LL << 31) || eB * 2 >= (1LL << 31)) return 1;
  int dev = 0;
  hipGetDevice(&dev);
  const int tiles_m = (a.M + 255) / 256, tiles_n = (a.N + 255) / 256;
  const int tiles = tiles_m * tiles_n, nt = a.K / gemm::BK;
  int G = num_cus(dev) & ~7;
  // at least ~4 K-tiles per block
  const long long work = (long long)tiles * nt;
  while (G > 8 && work < 4LL * G) G -= 8;
  g8::SkArgs s{};
  sk_plan(tiles, nt, G, s);
  s.tiles_m = tiles_m;
  s.tiles_n = tiles_n;
  if (s.I_sk > 0) {
    std::lock_guard<std::mutex> lk(g_sk_mu);
    SkWs& w = g_sk_ws[{dev, st}];
    const int need_cnt = tiles - s.d * G;
    const long long need_part = 2LL * G * 256 * 256;
    if (w.cnt_n < need_cnt || w.part_n < need_part) {
      hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
      if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return 3;
      // (the previous buffers may still be in use by launches in flight on this stream)
      if (hipStreamSynchronize(st) != hipSuccess) return 2;
      if (w.cnt) hipFree(w.cnt);
      if (w.part) hipFree(w.part);
      w.cnt = nullptr;
      w.part = nullptr;
      const int cn = need_cnt > 4096 ? need_cnt : 4096;
      const long long pn = need_part > 2LL * 256 * 65536 ? need_part : 2LL * 256 * 65536;
      if (hipMalloc((void**)&w.cnt, (size_t)cn * sizeof(int)) != hipSuccess) return 2;
      if (hipMalloc((void**)&w.part, (size_t)pn * sizeof(float)) != hipSuccess) return 2;
      if (hipMemset(w.cnt, 0, (size_t)cn * sizeof(int)) != hipSuccess) return 2;
      w.cnt_n = cn;
      w.part_n = pn;
    }
    s.cnt = w.cnt;
    s.part = w.part;
  }
  switch (a.act) {
    case 0: return g8::gemm4s_launch_a0(a, s, a_kmajor, b_kmajor, st);
    case 2: return g8::gemm4s_launch_a2(a, s, a_kmajor, b_kmajor, st);
    case 3: return g8::gemm4s_launch_a3(a, s, a_kmajor, b_kmajor, st);
    default: return 1;
  }
}

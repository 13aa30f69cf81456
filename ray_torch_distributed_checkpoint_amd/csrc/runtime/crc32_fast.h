// CRC-32 (IEEE 802.3, the zip / torch.save record checksum) at memory speed on the host.
//
// The checkpoint writers checksum every byte they write; the system zlib's table-driven crc32
// runs at ~0.7 GB/s per core here, so 8 writer threads capped a rank's save at ~4.5 GB/s
// (profiles/ckpt_engine_sweep.txt) while the disk takes more (8 concurrent ranks: 8.75 GB/s).
// This is carry-less-multiply folding: four 128-bit lanes of the message are folded forward
// 512 bits at a time with PCLMULQDQ (x^k mod P multipliers), then into one lane 128 bits at a
// time.  The folded lane is congruent to the whole message modulo P, so the raw (un-inverted)
// CRC register run over its 16 bytes from state 0 - plus the < 16-byte tail - gives the CRC.
// No Barrett step: the last 16+tail bytes go through a 256-entry table.  Bit-reflected domain
// throughout, as zlib's crc32 (init / final inversion included): crc32_fast(c, p, n) ==
// crc32(c, p, n) for every input (tests/test_units_cpu.py checks it against zlib).
#pragma once

#include <cstddef>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <zlib.h>

#if defined(__x86_64__)
#include <immintrin.h>
#endif

namespace rtdc {
namespace crc {

struct Table {
  uint32_t t[256];
  Table() {
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t c = i;
      for (int k = 0; k < 8; ++k) c = (c >> 1) ^ (0xEDB88320u & (0u - (c & 1u)));
      t[i] = c;
    }
  }
};

inline const Table& table() {
  static const Table tb;
  return tb;
}

// raw register update (no inversions)
inline uint32_t raw_bytes(uint32_t r, const uint8_t* p, size_t n) {
  const uint32_t* t = table().t;
  for (size_t i = 0; i < n; ++i) r = t[(r ^ p[i]) & 0xffu] ^ (r >> 8);
  return r;
}

#if defined(__x86_64__)
// x^k mod P multipliers (bit-reflected, 33-bit): fold distance 512 bits (low half, high half),
// then 128 bits
constexpr uint64_t K512_LO = 0x154442bd4ull, K512_HI = 0x1c6e41596ull;
constexpr uint64_t K128_LO = 0x1751997d0ull, K128_HI = 0x0ccaa009eull;

__attribute__((target("pclmul,sse4.1"))) inline __m128i fold(__m128i x, __m128i k, __m128i next) {
  const __m128i lo = _mm_clmulepi64_si128(x, k, 0x00);
  const __m128i hi = _mm_clmulepi64_si128(x, k, 0x11);
  return _mm_xor_si128(_mm_xor_si128(lo, hi), next);
}

__attribute__((target("pclmul,sse4.1"))) inline uint32_t pclmul(uint32_t crc, const uint8_t* p, size_t n) {
  // n >= 64
  const __m128i k512 = _mm_set_epi64x((long long)K512_HI, (long long)K512_LO);
  const __m128i k128 = _mm_set_epi64x((long long)K128_HI, (long long)K128_LO);
  __m128i x0 = _mm_loadu_si128((const __m128i*)(p + 0));
  __m128i x1 = _mm_loadu_si128((const __m128i*)(p + 16));
  __m128i x2 = _mm_loadu_si128((const __m128i*)(p + 32));
  __m128i x3 = _mm_loadu_si128((const __m128i*)(p + 48));
  x0 = _mm_xor_si128(x0, _mm_cvtsi32_si128((int)~crc));
  p += 64;
  n -= 64;
  while (n >= 64) {
    x0 = fold(x0, k512, _mm_loadu_si128((const __m128i*)(p + 0)));
    x1 = fold(x1, k512, _mm_loadu_si128((const __m128i*)(p + 16)));
    x2 = fold(x2, k512, _mm_loadu_si128((const __m128i*)(p + 32)));
    x3 = fold(x3, k512, _mm_loadu_si128((const __m128i*)(p + 48)));
    p += 64;
    n -= 64;
  }
  __m128i x = fold(x0, k128, x1);
  x = fold(x, k128, x2);
  x = fold(x, k128, x3);
  while (n >= 16) {
    x = fold(x, k128, _mm_loadu_si128((const __m128i*)p));
    p += 16;
    n -= 16;
  }
  alignas(16) uint8_t lane[16];
  _mm_store_si128((__m128i*)lane, x);
  uint32_t r = raw_bytes(0u, lane, 16);
  r = raw_bytes(r, p, n);
  return ~r;
}

inline bool have_pclmul() {
  // RTDC_CRC_ZLIB=1: the system zlib's table CRC instead (A/B of the writers' checksum cost)
  static const int v = (__builtin_cpu_supports("pclmul") && __builtin_cpu_supports("sse4.1") &&
                        !(std::getenv("RTDC_CRC_ZLIB") && std::getenv("RTDC_CRC_ZLIB")[0] == '1'))
                           ? 1
                           : 0;
  return v == 1;
}
#endif

// zlib-compatible crc32(crc, p, n)
inline uint32_t crc32_fast(uint32_t crc, const void* data, size_t n) {
  const uint8_t* p = (const uint8_t*)data;
#if defined(__x86_64__)
  if (n >= 64 && have_pclmul()) return pclmul(crc, p, n);
#endif
  // zlib's length argument is 32-bit: chunk
  while (n > 0) {
    const uInt c = (uInt)(n > (1u << 30) ? (1u << 30) : n);
    crc = (uint32_t)::crc32(crc, p, c);
    p += c;
    n -= c;
  }
  return crc;
}

}  // namespace crc
}  // namespace rtdc

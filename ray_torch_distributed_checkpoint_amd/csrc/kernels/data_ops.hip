// Token-id sort for the deterministic embedding backward, and the synthetic token source of
// the training loop (gfx950, wave64).
//
// sort_ids: stable LSD radix sort of n token ids (< 2^nbits) producing (sorted ids, original
// positions) - what embed_bwd_wte_kernel walks to sum each run of equal ids in token order
// without float atomics.  It replaces torch.sort (rocprim radix sort + merge +
// fill_reverse_indices: three ATen/rocprim launches per step).  The whole sort is ONE
// workgroup of 16 waves: the GPT-2 step sorts 16k ids, far too few to fill a chip, and the
// sort runs on a side stream under the forward pass, so one CU is the right footprint.
// Per 8-bit digit pass:
//   1. each wave counts the digits of its contiguous segment into its own LDS histogram row
//      (lanes with equal digits are found with 8 ballots; the lowest such lane adds the count -
//      no atomics, so no ordering question);
//   2. one exclusive scan over (digit, wave) turns the 16 x 256 counts into write offsets;
//   3. each wave re-walks its segment in order and writes every element to
//      offset[wave][digit] + (rank among the equal-digit lanes below it), then advances the
//      offset - stable by construction (segment order, then lane order).
// Keys / values ping-pong through two 32-bit global buffers (L2-resident); the last pass
// writes the int64 outputs.
#include "common.h"

#include <cstdlib>

namespace rtdc {

constexpr int SORT_WAVES = 16;
constexpr int SORT_RADIX = 256;

__device__ __forceinline__ uint64_t peers_of(uint32_t d, bool valid) {
  // mask of the valid lanes whose 8-bit digit equals this lane's
  uint64_t m = __ballot(valid);
#pragma unroll
  for (int b = 0; b < 8; ++b) {
    const bool bit = (d >> b) & 1u;
    const uint64_t bal = __ballot(valid && bit);
    m &= bit ? bal : ~bal;
  }
  return m;
}

// Segments of at most SORT_REG_CHUNKS 64-element chunks per wave (n <= 16 x 16 x 64 = 16384, the
// GPT-2 step's token count) are held in registers for a whole pass: every load of the pass is
// issued at once, where the chunk loop below waits for one global load per chunk and phase (the
// kernel ran 230-320 us per step that way, latency-bound, on the side stream under the LM head).
constexpr int SORT_REG_CHUNKS = 16;

__global__ __launch_bounds__(1024) void sort_ids_reg_kernel(const int64_t* __restrict__ ids, int n, int passes,
                                                            uint32_t* __restrict__ k0, uint32_t* __restrict__ v0,
                                                            uint32_t* __restrict__ k1, uint32_t* __restrict__ v1,
                                                            int64_t* __restrict__ sorted, int64_t* __restrict__ perm) {
  __shared__ uint32_t hist[SORT_WAVES][SORT_RADIX];
  __shared__ uint32_t dsum[SORT_RADIX];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int chunks = (n + 63) >> 6;
  const int cper = (chunks + SORT_WAVES - 1) / SORT_WAVES;  // <= SORT_REG_CHUNKS (host-checked)
  const int beg = min(n, w * cper * 64), end = min(n, (w + 1) * cper * 64);
  const int nch = (end - beg + 63) >> 6;
  const uint64_t below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));

  for (int p = 0; p < passes; ++p) {
    const int shift = 8 * p;
    const uint32_t* sk = (p & 1) ? k0 : k1;
    const uint32_t* sv = (p & 1) ? v0 : v1;
    uint32_t* dk = (p & 1) ? k1 : k0;
    uint32_t* dv = (p & 1) ? v1 : v0;
    const bool last = (p == passes - 1);
#pragma unroll
    for (int j = 0; j < SORT_RADIX / 64; ++j) hist[w][lane + 64 * j] = 0u;
    // the wave's whole segment, all loads in flight together
    uint32_t kr[SORT_REG_CHUNKS], vr[SORT_REG_CHUNKS];
#pragma unroll
    for (int j = 0; j < SORT_REG_CHUNKS; ++j) {
      const int i = beg + 64 * j + lane;
      kr[j] = 0u;
      vr[j] = 0u;
      if (j < nch && i < end) {
        if (p == 0) {
          kr[j] = (uint32_t)ids[i];
          vr[j] = (uint32_t)i;
        } else {
          kr[j] = sk[i];
          vr[j] = sv[i];
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
    // 1. per-wave digit counts
#pragma unroll
    for (int j = 0; j < SORT_REG_CHUNKS; ++j) {
      if (j < nch) {
        const bool valid = beg + 64 * j + lane < end;
        const uint32_t d = (kr[j] >> shift) & 0xffu;
        const uint64_t m = peers_of(d, valid);
        if (valid && (m & below) == 0) hist[w][d] += (uint32_t)__popcll(m);
        __builtin_amdgcn_wave_barrier();
      }
    }
    __syncthreads();
    // 2. exclusive scan in (digit-major, wave-minor) order
    if (threadIdx.x < SORT_RADIX) {
      const int d = threadIdx.x;
      uint32_t run = 0;
#pragma unroll
      for (int ww = 0; ww < SORT_WAVES; ++ww) {
        const uint32_t c = hist[ww][d];
        hist[ww][d] = run;
        run += c;
      }
      dsum[d] = run;
    }
    __syncthreads();
    if (w == 0) {
      uint32_t v[4], s = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        v[j] = dsum[lane * 4 + j];
        s += v[j];
      }
      uint32_t inc = s;
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {
        const uint32_t o = __shfl_up(inc, off, 64);
        if (lane >= off) inc += o;
      }
      uint32_t ex = inc - s;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        dsum[lane * 4 + j] = ex;
        ex += v[j];
      }
    }
    __syncthreads();
    if (threadIdx.x < SORT_RADIX) {
      const int d = threadIdx.x;
      const uint32_t b = dsum[d];
#pragma unroll
      for (int ww = 0; ww < SORT_WAVES; ++ww) hist[ww][d] += b;
    }
    __syncthreads();
    // 3. stable scatter (segment order, then lane order)
#pragma unroll
    for (int j = 0; j < SORT_REG_CHUNKS; ++j) {
      if (j < nch) {
        const bool valid = beg + 64 * j + lane < end;
        const uint32_t d = (kr[j] >> shift) & 0xffu;
        const uint64_t m = peers_of(d, valid);
        const uint32_t at = hist[w][d] + (uint32_t)__popcll(m & below);
        __builtin_amdgcn_wave_barrier();
        if (valid) {
          if (last) {
            sorted[at] = (int64_t)kr[j];
            perm[at] = (int64_t)vr[j];
          } else {
            dk[at] = kr[j];
            dv[at] = vr[j];
          }
          if ((m & below) == 0) hist[w][d] += (uint32_t)__popcll(m);
        }
        __builtin_amdgcn_wave_barrier();
      }
    }
    __syncthreads();
  }
}

__global__ __launch_bounds__(1024) void sort_ids_kernel(const int64_t* __restrict__ ids, int n, int passes,
                                                        uint32_t* __restrict__ k0, uint32_t* __restrict__ v0,
                                                        uint32_t* __restrict__ k1, uint32_t* __restrict__ v1,
                                                        int64_t* __restrict__ sorted, int64_t* __restrict__ perm) {
  __shared__ uint32_t hist[SORT_WAVES][SORT_RADIX];
  __shared__ uint32_t dsum[SORT_RADIX];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  // segments are whole 64-element chunks so only a wave's last chunk is partial
  const int chunks = (n + 63) >> 6;
  const int cper = (chunks + SORT_WAVES - 1) / SORT_WAVES;
  const int beg = min(n, w * cper * 64), end = min(n, (w + 1) * cper * 64);
  const uint64_t below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));

  for (int p = 0; p < passes; ++p) {
    const int shift = 8 * p;
    const uint32_t* sk = (p & 1) ? k0 : k1;  // pass 0 reads ids; odd passes read k0, even k1
    const uint32_t* sv = (p & 1) ? v0 : v1;
    uint32_t* dk = (p & 1) ? k1 : k0;
    uint32_t* dv = (p & 1) ? v1 : v0;
    const bool last = (p == passes - 1);
#pragma unroll
    for (int j = 0; j < SORT_RADIX / 64; ++j) hist[w][lane + 64 * j] = 0u;
    __builtin_amdgcn_wave_barrier();
    // 1. per-wave digit counts
    for (int base = beg; base < end; base += 64) {
      const int i = base + lane;
      const bool valid = i < end;
      uint32_t key = 0;
      if (valid) key = (p == 0) ? (uint32_t)ids[i] : sk[i];
      const uint32_t d = (key >> shift) & 0xffu;
      const uint64_t m = peers_of(d, valid);
      if (valid && (m & below) == 0) hist[w][d] += (uint32_t)__popcll(m);
      __builtin_amdgcn_wave_barrier();
    }
    __syncthreads();
    // 2. exclusive scan in (digit-major, wave-minor) order
    if (threadIdx.x < SORT_RADIX) {
      const int d = threadIdx.x;
      uint32_t run = 0;
#pragma unroll
      for (int ww = 0; ww < SORT_WAVES; ++ww) {
        const uint32_t c = hist[ww][d];
        hist[ww][d] = run;
        run += c;
      }
      dsum[d] = run;
    }
    __syncthreads();
    if (w == 0) {  // exclusive scan of the 256 digit totals: 4 per lane + a wave scan
      uint32_t v[4], s = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        v[j] = dsum[lane * 4 + j];
        s += v[j];
      }
      uint32_t inc = s;
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {
        const uint32_t o = __shfl_up(inc, off, 64);
        if (lane >= off) inc += o;
      }
      uint32_t ex = inc - s;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        dsum[lane * 4 + j] = ex;
        ex += v[j];
      }
    }
    __syncthreads();
    if (threadIdx.x < SORT_RADIX) {
      const int d = threadIdx.x;
      const uint32_t b = dsum[d];
#pragma unroll
      for (int ww = 0; ww < SORT_WAVES; ++ww) hist[ww][d] += b;
    }
    __syncthreads();
    // 3. stable scatter
    for (int base = beg; base < end; base += 64) {
      const int i = base + lane;
      const bool valid = i < end;
      uint32_t key = 0, val = 0;
      if (valid) {
        if (p == 0) {
          key = (uint32_t)ids[i];
          val = (uint32_t)i;
        } else {
          key = sk[i];
          val = sv[i];
        }
      }
      const uint32_t d = (key >> shift) & 0xffu;
      const uint64_t m = peers_of(d, valid);
      const uint32_t at = hist[w][d] + (uint32_t)__popcll(m & below);
      __builtin_amdgcn_wave_barrier();
      if (valid) {
        if (last) {
          sorted[at] = (int64_t)key;
          perm[at] = (int64_t)val;
        } else {
          dk[at] = key;
          dv[at] = val;
        }
        if ((m & below) == 0) hist[w][d] += (uint32_t)__popcll(m);
      }
      __builtin_amdgcn_wave_barrier();
    }
    __syncthreads();  // the next pass reads what other waves wrote (same CU: workgroup scope)
  }
}

// Synthetic token stream (workloads.SyntheticTokens): sequence `ids[b]` is the tokens
// tok(j) = mix(ids[b] * (T + 1) + j, seed) % vocab, j in [0, T]; inputs = tok[0:T], targets =
// tok[1:T+1], both written contiguously (what a data loader hands the model).  `mix` is the
// integer hash of workloads._mix (values < 2^31 before each multiply: exact in 64 bits).
__device__ __forceinline__ uint64_t mix31(uint64_t x, uint64_t seed_add) {
  x = (x + seed_add) & 0x7FFFFFFFull;
#pragma unroll
  for (int r = 0; r < 3; ++r) x = ((x ^ (x >> 13)) * 1103515245ull + 12345ull) & 0x7FFFFFFFull;
  return x;
}

__global__ __launch_bounds__(256) void synth_tokens_kernel(const int64_t* __restrict__ ids, int B, int T,
                                                           long long vocab, unsigned long long seed_add,
                                                           int64_t* __restrict__ inp, int64_t* __restrict__ tgt) {
  const long long e = (long long)blockIdx.x * 256 + threadIdx.x;
  const long long per = (long long)T + 1;
  if (e >= (long long)B * per) return;
  const long long b = e / per, j = e - b * per;
  const uint64_t x = (uint64_t)ids[b] * (uint64_t)per + (uint64_t)j;
  const int64_t tok = (int64_t)(mix31(x, seed_add) % (uint64_t)vocab);
  if (j < T) inp[b * T + j] = tok;
  if (j > 0) tgt[b * T + j - 1] = tok;
}

}  // namespace rtdc

using namespace rtdc;

// ws: 4 * n uint32 (two key/value ping-pong buffers).  nbits: bits of the largest id.
extern "C" int rtdc_sort_ids(const int64_t* ids, int n, int nbits, uint32_t* ws, int64_t* sorted, int64_t* perm,
                             hipStream_t st) {
  if (n <= 0) return 0;
  if (nbits < 1 || nbits > 32) return 1;
  const int passes = (nbits + 7) / 8;
  uint32_t* k0 = ws;
  uint32_t* v0 = ws + n;
  uint32_t* k1 = ws + 2LL * n;
  uint32_t* v1 = ws + 3LL * n;
  const int chunks = (n + 63) / 64, cper = (chunks + SORT_WAVES - 1) / SORT_WAVES;
  if (cper <= SORT_REG_CHUNKS && !(getenv("RTDC_SORT_REG") && getenv("RTDC_SORT_REG")[0] == '0'))
    hipLaunchKernelGGL(sort_ids_reg_kernel, dim3(1), dim3(SORT_WAVES * 64), 0, st, ids, n, passes, k0, v0, k1, v1,
                       sorted, perm);
  else
    hipLaunchKernelGGL(sort_ids_kernel, dim3(1), dim3(SORT_WAVES * 64), 0, st, ids, n, passes, k0, v0, k1, v1,
                       sorted, perm);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

extern "C" int rtdc_synth_tokens(const int64_t* ids, int B, int T, long long vocab, unsigned long long seed_add,
                                 int64_t* inp, int64_t* tgt, hipStream_t st) {
  if (B <= 0 || T <= 0 || vocab <= 0) return 1;
  const long long n = (long long)B * (T + 1);
  hipLaunchKernelGGL(synth_tokens_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, ids, B, T, vocab,
                     seed_add, inp, tgt);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

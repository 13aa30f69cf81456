// One-shot all-reduce over hipIpc-mapped peer buffers (intra-node, xGMI), for small gradient
// buckets where a ring collective is latency-bound (7 point-to-point links per
// MI355X; a one-shot read of all peers uses all 7 at once and has one hop of latency).
//
// Every rank owns ONE uncached (MTYPE UC) device allocation, exported with hipIpcGetMemHandle
// and mapped by every peer:
//     [ flag (64 B) | staging parity 0 (cap B) | staging parity 1 (cap B) ]
// A call with epoch e (a per-communicator counter, identical on every rank because collectives
// are issued in the same order everywhere) uses staging parity e & 1.  The counter lives in
// DEVICE memory (one word per rank, never shared): every kernel of a call reads e = counter + 1
// and a final one-thread kernel advances it, so a call captured into a hipGraph advances the
// epoch on every replay (a host counter would be frozen into the captured kernel arguments):
//   1. stage_kernel copies the local tensor into the own staging slot of parity e & 1;
//   2. oneshot_kernel: block 0 publishes flag = e (system-scope release); every block waits
//      until all ranks' flags reached e (system-scope acquire loads), then sums its share of
//      the elements over ranks 0..world-1 IN RANK ORDER (fp32 accumulation) - every rank
//      computes bitwise the same result - and writes it back in place.
// Reuse safety: a rank writes parity p again only in call e + 2, after it passed the wait of
// call e + 1, which every peer can only publish after finishing call e's reads.
// Uncached staging means no L2 on any XCD ever holds a stale or dirty copy of it.
// The wait is BOUNDED (wall_clock64, 100 MHz): on timeout the kernel records an error in a
// host-visible word, fills the bucket with NaN (never a silently un-reduced gradient) and
// exits, so a missing peer can never leave waves spinning on the GPU.
// The error is STICKY: once set, later calls on this rank neither stage nor publish - they
// NaN-fill their bucket at once.  Restaging would break the reuse argument above (a rank that
// timed out in call e+1 never passed its wait, so a late peer may still be reading call e's
// slot of the parity that call e+2 would overwrite), and publishing would let a late peer
// reduce against a rank that no longer participates.  A late peer therefore completes at most
// the calls this rank published before its timeout, then times out itself on the next one.
#include "common.h"

namespace rtdc {
namespace p2p {

constexpr int MAXW = 8;
constexpr int FLAG_BYTES = 64;
typedef __attribute__((ext_vector_type(4))) unsigned int v4u;

struct Peers {
  const char* base[MAXW];  // every rank's mapped allocation (own included)
};

__device__ __forceinline__ unsigned load_flag(const unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// T: float or bf16_t.  n elements (n * sizeof(T) a multiple of 16), 16-B vectors.
__device__ __forceinline__ int sticky_error(const int* err) {
  return __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ __launch_bounds__(256) void stage_kernel(const unsigned* __restrict__ epoch_dev, char* own, long long cap,
                                                   const uint4* __restrict__ src, long long nv, const int* err) {
  if (sticky_error(err)) return;  // a timed-out rank never restages (see the header)
  const unsigned epoch = *epoch_dev + 1u;
  uint4* dst = (uint4*)(own + FLAG_BYTES + (long long)(epoch & 1u) * cap);
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < nv; i += (long long)gridDim.x * 256) dst[i] = src[i];
}

__global__ void advance_kernel(unsigned* epoch_dev) {
  if (threadIdx.x == 0 && blockIdx.x == 0) *epoch_dev += 1u;
}

template <typename T>
__global__ __launch_bounds__(256) void oneshot_kernel(Peers peers, int world, int rank, const unsigned* epoch_dev,
                                                      long long cap, T* __restrict__ out, long long n,
                                                      float scale, int* err, long long timeout_ticks) {
  __shared__ int bad;
  const unsigned epoch = *epoch_dev + 1u;  // advanced by advance_kernel after this call
  if (threadIdx.x == 0) {
    // sticky: after a timeout this rank neither publishes nor waits (see the header)
    int timed_out = sticky_error(err);
    unsigned* mine = (unsigned*)peers.base[rank];
    if (blockIdx.x == 0 && !timed_out) __hip_atomic_store(mine, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    const long long t0 = wall_clock64();
    for (int r = 0; r < world && !timed_out; ++r) {
      const unsigned* f = (const unsigned*)peers.base[r];
      while ((int)(load_flag(f) - epoch) < 0) {
        if (wall_clock64() - t0 > timeout_ticks) {
          timed_out = 1;
          __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          break;
        }
        __builtin_amdgcn_s_sleep(2);
      }
    }
    bad = timed_out;
  }
  __syncthreads();
  constexpr int V = 16 / sizeof(T);  // elements per 16-B vector
  const long long nv = n / V;
  if (bad) {
    // a peer never arrived: poison this rank's bucket with NaN instead of leaving the local,
    // un-reduced gradient in place (which would let the optimizer silently apply a
    // rank-dependent update); the host raises on the error word at the next finalize
    const uint4 qnan = sizeof(T) == 4 ? make_uint4(0x7FC00000u, 0x7FC00000u, 0x7FC00000u, 0x7FC00000u)
                                      : make_uint4(0x7FC07FC0u, 0x7FC07FC0u, 0x7FC07FC0u, 0x7FC07FC0u);
    for (long long i = blockIdx.x * 256LL + threadIdx.x; i < nv; i += (long long)gridDim.x * 256) ((uint4*)out)[i] = qnan;
    return;
  }
  const long long off = FLAG_BYTES + (long long)(epoch & 1u) * cap;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < nv; i += (long long)gridDim.x * 256) {
    float acc[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = 0.f;
    for (int r = 0; r < world; ++r) {
      const v4u q = __builtin_nontemporal_load((const v4u*)(peers.base[r] + off) + i);
      const uint32_t w[4] = {q[0], q[1], q[2], q[3]};
      if constexpr (sizeof(T) == 4) {
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[e] += __uint_as_float(w[e]);
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          acc[2 * e] += __uint_as_float(w[e] << 16);
          acc[2 * e + 1] += __uint_as_float(w[e] & 0xffff0000u);
        }
      }
    }
    uint4 o;
    if constexpr (sizeof(T) == 4) {
      o = make_uint4(__float_as_uint(acc[0] * scale), __float_as_uint(acc[1] * scale),
                     __float_as_uint(acc[2] * scale), __float_as_uint(acc[3] * scale));
    } else {
      o = make_uint4(pack_bf2(acc[0] * scale, acc[1] * scale), pack_bf2(acc[2] * scale, acc[3] * scale),
                     pack_bf2(acc[4] * scale, acc[5] * scale), pack_bf2(acc[6] * scale, acc[7] * scale));
    }
    ((uint4*)out)[i] = o;
  }
}

}  // namespace p2p
}  // namespace rtdc

using namespace rtdc;

// One call on stream st: stage (local tensor -> own staging slot), one-shot sum, epoch advance.
// bases: world mapped allocations (own at [rank]); data: the local tensor, reduced in place.
// blocks: grid size (few: the kernel reads HBM of every peer; a small grid leaves the CUs to
// the backward pass).  Every argument is call-invariant, so the call is hipGraph-capturable.
extern "C" int rtdc_p2p_oneshot(const void* const* bases, int world, int rank, unsigned* epoch_dev, long long cap,
                                void* data, long long n, int is_bf16, float scale, int* err,
                                long long timeout_ticks, int blocks, hipStream_t st) {
  if (world < 1 || world > p2p::MAXW || rank < 0 || rank >= world) return 1;
  const long long bytes = n * (is_bf16 ? 2 : 4);
  if (bytes % 16 != 0 || bytes > cap || ((uintptr_t)data & 15) != 0) return 1;
  p2p::Peers peers{};
  for (int r = 0; r < world; ++r) peers.base[r] = (const char*)bases[r];
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(p2p::stage_kernel, dim3(blocks), dim3(256), 0, st, (const unsigned*)epoch_dev,
                     (char*)bases[rank], cap, (const uint4*)data, bytes / 16, (const int*)err);
  if (is_bf16)
    hipLaunchKernelGGL(p2p::oneshot_kernel<bf16_t>, dim3(blocks), dim3(256), 0, st, peers, world, rank,
                       (const unsigned*)epoch_dev, cap, (bf16_t*)data, n, scale, err, timeout_ticks);
  else
    hipLaunchKernelGGL(p2p::oneshot_kernel<float>, dim3(blocks), dim3(256), 0, st, peers, world, rank,
                       (const unsigned*)epoch_dev, cap, (float*)data, n, scale, err, timeout_ticks);
  hipLaunchKernelGGL(p2p::advance_kernel, dim3(1), dim3(64), 0, st, epoch_dev);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

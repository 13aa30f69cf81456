// Fused optimizers over FLAT parameter/state buffers (gfx950).
//
// The framework keeps every parameter, gradient and optimizer state of a model in one
// contiguous buffer per kind (FlatParamSpace), so an optimizer step is ONE launch over a
// chunk table instead of ATen's multi-tensor-apply foreach chain (reference: SGD(momentum=0.9)
// at R/my_ray_module.py:142,160 -> torch/optim/sgd.py _multi_tensor_sgd).  A chunk is a slice
// of one parameter (never crossing parameters) carrying that parameter's weight-decay flag;
// segments are 64-element aligned so every lane moves 16 B per load.
//
// AdamW: fp32 master + m + v, optional bf16 shadow written in the same pass (the copy the
// bf16 MFMA kernels read).  grad_scale folds the DDP 1/world pre-divide into the step.
// A chunk carries two offsets: `start` into the flat parameter / gradient / shadow buffers and
// `sstart` into the optimizer-state buffers.  Without ZeRO they are equal; under ZeRO-1 the
// state buffers hold only this rank's owned shards back to back (1/world of the bytes), so
// `sstart` is the chunk's position in that compact buffer.
// Semantics follow torch.optim.AdamW / SGD (decoupled weight decay; SGD first-step clone).
//
// `skip` (optional): a communicator health word (the one-shot P2P all-reduce's host-coherent
// error flag, csrc/runtime/p2p_comm.cpp).  When a gradient collective earlier on this stream
// timed out it poisoned its bucket with NaN and set the word; the update then becomes a no-op,
// so a NaN gradient can never reach the parameters or the optimizer state - also inside a
// replayed hipGraph, where no host code runs between the collective and the step.
#include "common.h"

namespace rtdc {

__device__ __forceinline__ bool comm_poisoned(const int* skip) {
  return skip != nullptr && __hip_atomic_load(skip, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0;
}

struct Chunk {
  long long start;   // offset into p / g / shadow
  int len;
  int decay;
  long long sstart;  // offset into the optimizer state (m, v / momentum buffer)
};
static_assert(sizeof(Chunk) == 24, "chunk table rows are 3 x int64");

__global__ __launch_bounds__(256) void adamw_kernel(const Chunk* __restrict__ chunks, int nchunks,
                                                   float* __restrict__ p, const float* __restrict__ g,
                                                   float* __restrict__ m, float* __restrict__ v,
                                                   bf16_t* __restrict__ shadow, float lr, float b1,
                                                   float b2, float eps, float wd, float bc1,
                                                   float bc2_sqrt, float grad_scale, const int* skip) {
  if (comm_poisoned(skip)) return;
  const float step_size = lr / bc1;
  for (int ci = blockIdx.x; ci < nchunks; ci += gridDim.x) {
    const Chunk c = chunks[ci];
    const float decay = c.decay ? (1.f - lr * wd) : 1.f;
    for (int i = threadIdx.x * 4; i < c.len; i += 256 * 4) {
      const long long o = c.start + i, so = c.sstart + i;
      if (i + 4 <= c.len) {
        f32x4 pp = *(f32x4*)(p + o), gg = *(const f32x4*)(g + o);
        f32x4 mm = *(f32x4*)(m + so), vv = *(f32x4*)(v + so);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float gr = gg[e] * grad_scale;
          float pe = pp[e] * decay;
          mm[e] = b1 * mm[e] + (1.f - b1) * gr;
          vv[e] = b2 * vv[e] + (1.f - b2) * gr * gr;
          const float denom = sqrtf(vv[e]) / bc2_sqrt + eps;
          pe -= step_size * mm[e] / denom;
          pp[e] = pe;
        }
        *(f32x4*)(p + o) = pp;
        *(f32x4*)(m + so) = mm;
        *(f32x4*)(v + so) = vv;
        if (shadow) *(uint2*)(shadow + o) = make_uint2(pack_bf2(pp[0], pp[1]), pack_bf2(pp[2], pp[3]));
      } else {
        for (int e = 0; e < 4 && i + e < c.len; ++e) {
          const long long oe = o + e, se = so + e;
          const float gr = g[oe] * grad_scale;
          float pe = p[oe] * decay;
          m[se] = b1 * m[se] + (1.f - b1) * gr;
          v[se] = b2 * v[se] + (1.f - b2) * gr * gr;
          const float denom = sqrtf(v[se]) / bc2_sqrt + eps;
          pe -= step_size * m[se] / denom;
          p[oe] = pe;
          if (shadow) shadow[oe] = f2bf(pe);
        }
      }
    }
  }
}

// torch SGD: d = g*s + wd*p ; buf = first ? d : mom*buf + (1-damp)*d ; d = nesterov ? d + mom*buf : buf
// p -= lr*d
__global__ __launch_bounds__(256) void sgd_kernel(const Chunk* __restrict__ chunks, int nchunks,
                                                 float* __restrict__ p, const float* __restrict__ g,
                                                 float* __restrict__ buf, bf16_t* __restrict__ shadow,
                                                 float lr, float momentum, float dampening, float wd,
                                                 int nesterov, int first, float grad_scale, const int* skip) {
  if (comm_poisoned(skip)) return;
  for (int ci = blockIdx.x; ci < nchunks; ci += gridDim.x) {
    const Chunk c = chunks[ci];
    const float w = c.decay ? wd : 0.f;
    auto upd = [&](float gv, float& pe, float& b) {
      float d = gv * grad_scale;
      d += w * pe;
      if (momentum != 0.f) {
        b = first ? d : momentum * b + (1.f - dampening) * d;
        d = nesterov ? d + momentum * b : b;
      }
      pe -= lr * d;
    };
    const bool vec = (c.start & 3) == 0 && (c.sstart & 3) == 0;
    // 4 elements per lane and iteration (16-B loads of p, g and the momentum buffer)
    for (int i = threadIdx.x * 4; i < c.len; i += 256 * 4) {
      const long long o = c.start + i, so = c.sstart + i;
      if (vec && i + 4 <= c.len) {
        f32x4 pp = *(f32x4*)(p + o);
        const f32x4 gg = *(const f32x4*)(g + o);
        f32x4 bb = (momentum != 0.f && !first) ? *(f32x4*)(buf + so) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float pe = pp[e], b = bb[e];
          upd(gg[e], pe, b);
          pp[e] = pe;
          bb[e] = b;
        }
        *(f32x4*)(p + o) = pp;
        if (momentum != 0.f) *(f32x4*)(buf + so) = bb;
        if (shadow) *(uint2*)(shadow + o) = make_uint2(pack_bf2(pp[0], pp[1]), pack_bf2(pp[2], pp[3]));
      } else {
        for (int e = 0; e < 4 && i + e < c.len; ++e) {
          const long long oe = o + e, se = so + e;
          float pe = p[oe], b = (momentum != 0.f && !first) ? buf[se] : 0.f;
          upd(g[oe], pe, b);
          if (momentum != 0.f) buf[se] = b;
          p[oe] = pe;
          if (shadow) shadow[oe] = f2bf(pe);
        }
      }
    }
  }
}

__global__ __launch_bounds__(256) void f32_to_bf16_kernel(const float* __restrict__ x, bf16_t* __restrict__ y,
                                                         long long n) {
  for (long long i = (blockIdx.x * 256LL + threadIdx.x) * 4; i < n; i += gridDim.x * 256LL * 4) {
    if (i + 4 <= n) {
      f32x4 v = *(const f32x4*)(x + i);
      *(uint2*)(y + i) = make_uint2(pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3]));
    } else {
      for (long long e = i; e < n; ++e) y[e] = f2bf(x[e]);
    }
  }
}

// y[c][r] = bf16(x[r][c]) for a row-major fp32 [R][C] matrix: the K-major image of a weight for
// the products that read it transposed (ops/shadow.py shadow_t_of).  64x64 tiles through LDS
// (padded rows: conflict-free column reads), 16-B loads, 8-B stores.
__global__ __launch_bounds__(256) void f32_to_bf16_t_kernel(const float* __restrict__ x, bf16_t* __restrict__ y,
                                                           int R, int C) {
  __shared__ float t[64][65];
  const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int rr = ty + 16 * i, r = r0 + rr, c = c0 + 4 * tx;
    float v[4] = {0.f, 0.f, 0.f, 0.f};
    if (r < R) {
      if (c + 4 <= C && (C & 3) == 0) {
        const f32x4 q = *(const f32x4*)(x + (long long)r * C + c);
        v[0] = q[0]; v[1] = q[1]; v[2] = q[2]; v[3] = q[3];
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = c + e < C ? x[(long long)r * C + c + e] : 0.f;
      }
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) t[rr][4 * tx + e] = v[e];
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int cc = ty + 16 * i, c = c0 + cc, r = r0 + 4 * tx;
    if (c >= C) continue;
    bf16_t* o = y + (long long)c * R + r;
    if (r + 4 <= R && (R & 3) == 0) {
      *(uint2*)o = make_uint2(pack_bf2(t[4 * tx][cc], t[4 * tx + 1][cc]), pack_bf2(t[4 * tx + 2][cc], t[4 * tx + 3][cc]));
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (r + e < R) o[e] = f2bf(t[4 * tx + e][cc]);
    }
  }
}

__global__ __launch_bounds__(256) void bf16_to_f32_kernel(const bf16_t* __restrict__ x, float* __restrict__ y,
                                                         long long n, float scale) {
  for (long long i = (blockIdx.x * 256LL + threadIdx.x) * 4; i < n; i += gridDim.x * 256LL * 4) {
    if (i + 4 <= n) {
      const uint2 u = *(const uint2*)(x + i);
      f32x4 v;
      v[0] = __uint_as_float(u.x << 16) * scale;
      v[1] = __uint_as_float(u.x & 0xffff0000u) * scale;
      v[2] = __uint_as_float(u.y << 16) * scale;
      v[3] = __uint_as_float(u.y & 0xffff0000u) * scale;
      *(f32x4*)(y + i) = v;
    } else {
      for (long long e = i; e < n; ++e) y[e] = bf2f(x[e]) * scale;
    }
  }
}

// sum of squares per chunk -> partial[ci] (for grad-norm clipping); deterministic
__global__ __launch_bounds__(256) void sumsq_kernel(const Chunk* __restrict__ chunks, int nchunks,
                                                   const float* __restrict__ g, float* __restrict__ partial) {
  __shared__ float red[4];
  for (int ci = blockIdx.x; ci < nchunks; ci += gridDim.x) {
    const Chunk c = chunks[ci];
    float s = 0.f;
    for (int i = threadIdx.x; i < c.len; i += 256) {
      const float x = g[c.start + i];
      s += x * x;
    }
    s = block_sum<256>(s, red);
    if (threadIdx.x == 0) partial[ci] = s;
  }
}

}  // namespace rtdc

using namespace rtdc;

static inline int grid_for(int nchunks) { return nchunks < 4096 ? nchunks : 4096; }

extern "C" int rtdc_adamw(const void* chunks, int nchunks, float* p, const float* g, float* m,
                          float* v, void* shadow, float lr, float b1, float b2, float eps, float wd,
                          float bc1, float bc2_sqrt, float grad_scale, const int* skip, hipStream_t st) {
  if (nchunks <= 0) return 0;
  hipLaunchKernelGGL(adamw_kernel, dim3(grid_for(nchunks)), dim3(256), 0, st, (const Chunk*)chunks,
                     nchunks, p, g, m, v, (bf16_t*)shadow, lr, b1, b2, eps, wd, bc1, bc2_sqrt, grad_scale, skip);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

extern "C" int rtdc_sgd(const void* chunks, int nchunks, float* p, const float* g, float* buf,
                        void* shadow, float lr, float momentum, float dampening, float wd,
                        int nesterov, int first, float grad_scale, const int* skip, hipStream_t st) {
  if (nchunks <= 0) return 0;
  hipLaunchKernelGGL(sgd_kernel, dim3(grid_for(nchunks)), dim3(256), 0, st, (const Chunk*)chunks,
                     nchunks, p, g, buf, (bf16_t*)shadow, lr, momentum, dampening, wd, nesterov, first,
                     grad_scale, skip);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

extern "C" int rtdc_f32_to_bf16(const float* x, void* y, long long n, hipStream_t st) {
  long long blocks = (n / 4 + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(f32_to_bf16_kernel, dim3((unsigned)blocks), dim3(256), 0, st, x, (bf16_t*)y, n);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

extern "C" int rtdc_f32_to_bf16_t(const float* x, void* y, int R, int C, hipStream_t st) {
  if (R <= 0 || C <= 0) return 0;
  hipLaunchKernelGGL(f32_to_bf16_t_kernel, dim3((unsigned)((C + 63) / 64), (unsigned)((R + 63) / 64)), dim3(256), 0,
                     st, x, (bf16_t*)y, R, C);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

// ---- batched bf16 transpose: dst[c][r] = src[r][c] for up to kTMaxJobs row-major [R][C]
// matrices in one launch (the K-major images of a model's weights, ops/shadow.py
// kmajor_refresh).  Block = one 64x64 tile of one job: 16-B loads of 8 rows x 8 columns per
// pass into an LDS tile padded by one 16-B chunk per row, 16-B stores of 8 consecutive output
// columns gathered from one LDS column.  Requires R % 8 == 0 and C % 8 == 0.
typedef __attribute__((ext_vector_type(4))) unsigned int tu32x4;
constexpr int kTMaxJobs = 96;
struct TJobs {
  const bf16_t* src[kTMaxJobs];
  bf16_t* dst[kTMaxJobs];
  int R[kTMaxJobs], C[kTMaxJobs];
  int start[kTMaxJobs + 1];  // first tile of each job (prefix sums)
  int n;
};

__global__ __launch_bounds__(256) void bf16_transpose_multi_kernel(const TJobs* __restrict__ jobs) {
  __shared__ __attribute__((aligned(16))) bf16_t t[64][72];
  const int b = blockIdx.x;
  int j = 0;
  {  // job of this tile: the last job whose start <= b (n <= 96: a short scalar scan)
    const int n = jobs->n;
    for (int i = 1; i < n; ++i) j = jobs->start[i] <= b ? i : j;
  }
  const int R = jobs->R[j], C = jobs->C[j];
  const int tiles_c = (C + 63) / 64;
  const int tile = b - jobs->start[j];
  const int r0 = (tile / tiles_c) * 64, c0 = (tile % tiles_c) * 64;
  const bf16_t* src = jobs->src[j];
  bf16_t* dst = jobs->dst[j];
  const int tid = threadIdx.x;
  // load: thread -> (row tid / 8 + 32 p, 8 columns at 8 * (tid % 8))
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int rr = tid / 8 + 32 * p, cc = 8 * (tid % 8);
    tu32x4 v = {0u, 0u, 0u, 0u};
    if (r0 + rr < R && c0 + cc < C) v = *(const tu32x4*)(src + (long long)(r0 + rr) * C + c0 + cc);
    *(tu32x4*)&t[rr][cc] = v;
  }
  __syncthreads();
  // store: thread -> (output row = input column tid / 8 + 32 p, 8 output columns = input rows)
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int oc = tid / 8 + 32 * p, orr = 8 * (tid % 8);
    if (c0 + oc >= C || r0 + orr >= R) continue;
    uint32_t w[4];
#pragma unroll
    for (int e = 0; e < 4; ++e)
      w[e] = (uint32_t)t[orr + 2 * e][oc] | ((uint32_t)t[orr + 2 * e + 1][oc] << 16);
    *(tu32x4*)(dst + (long long)(c0 + oc) * R + r0 + orr) = tu32x4{w[0], w[1], w[2], w[3]};
  }
}

extern "C" int rtdc_bf16_transpose_multi(const void* const* src, void* const* dst, const int* R, const int* C, int n,
                                         void* jobs_dev, hipStream_t st) {
  if (n <= 0) return 0;
  if (n > kTMaxJobs) return 1;
  TJobs h{};
  int tiles = 0;
  for (int i = 0; i < n; ++i) {
    if (R[i] % 8 || C[i] % 8) return 1;
    h.src[i] = (const bf16_t*)src[i];
    h.dst[i] = (bf16_t*)dst[i];
    h.R[i] = R[i];
    h.C[i] = C[i];
    h.start[i] = tiles;
    tiles += ((R[i] + 63) / 64) * ((C[i] + 63) / 64);
  }
  h.start[n] = tiles;
  h.n = n;
  // the table goes to device memory ahead of the kernel on the same stream (larger than the
  // kernel-argument segment)
  if (hipMemcpyAsync(jobs_dev, &h, sizeof(TJobs), hipMemcpyHostToDevice, st) != hipSuccess) return 2;
  hipLaunchKernelGGL(bf16_transpose_multi_kernel, dim3((unsigned)tiles), dim3(256), 0, st, (const TJobs*)jobs_dev);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

extern "C" int rtdc_bf16_transpose_jobs_bytes() { return (int)sizeof(TJobs); }

extern "C" int rtdc_sumsq(const void* chunks, int nchunks, const float* g, float* partial, hipStream_t st) {
  if (nchunks <= 0) return 0;
  hipLaunchKernelGGL(sumsq_kernel, dim3(grid_for(nchunks)), dim3(256), 0, st, (const Chunk*)chunks,
                     nchunks, g, partial);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

extern "C" int rtdc_bf16_to_f32(const void* x, float* y, long long n, float scale, hipStream_t st) {
  long long blocks = (n / 4 + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(bf16_to_f32_kernel, dim3((unsigned)blocks), dim3(256), 0, st, (const bf16_t*)x, y, n, scale);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

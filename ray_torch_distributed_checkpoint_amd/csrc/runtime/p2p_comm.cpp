// Intra-node one-shot all-reduce communicator over hipIpc-mapped peer buffers (kernel and
// protocol: kernels/p2p_allreduce.hip).  Used by the gradient-bucket engine for buckets at or
// below a size threshold, where RCCL's ring is latency-bound; larger buckets stay on RCCL.
//
// Lifecycle: construct (allocates this rank's uncached [flag | 2 x staging] buffer) ->
// handle() bytes are exchanged over the process group (parallel/p2p.py) -> open(handles) maps
// every peer -> allreduce_(t) per collective, on the caller's current stream.
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>

#include <cstring>
#include <string>
#include <vector>

extern "C" int rtdc_p2p_oneshot(const void* const* bases, int world, int rank, unsigned* epoch_dev, long long cap,
                                void* data, long long n, int is_bf16, float scale, int* err,
                                long long timeout_ticks, int blocks, hipStream_t st);

namespace rtdc_p2p {

class P2PComm {
 public:
  static constexpr long long kFlag = 64;

  P2PComm(int rank, int world, long long capacity_bytes, int device, double timeout_s, int blocks)
      : rank_(rank), world_(world), cap_((capacity_bytes + 255) / 256 * 256), device_(device), blocks_(blocks) {
    TORCH_CHECK(world >= 1 && world <= 8 && rank >= 0 && rank < world, "P2PComm: world in [1, 8]");
    TORCH_CHECK(cap_ > 0, "P2PComm: capacity must be positive");
    check(hipSetDevice(device_), "hipSetDevice");
    // uncached: no L2 of any XCD (ours or a peer's) ever caches the staging or the flag
    check(hipExtMallocWithFlags(&own_, (size_t)(kFlag + 2 * cap_), hipDeviceMallocUncached), "hipExtMallocWithFlags");
    check(hipMemset(own_, 0, (size_t)(kFlag + 2 * cap_)), "hipMemset");
    check(hipHostMalloc((void**)&err_, sizeof(int), hipHostMallocCoherent), "hipHostMalloc");
    // device-resident epoch counter (graph-capturable calls: kernels/p2p_allreduce.hip)
    check(hipMalloc((void**)&epoch_dev_, 64), "hipMalloc");
    check(hipMemset(epoch_dev_, 0, 64), "hipMemset");
    *err_ = 0;
    int rate_khz = 0;
    if (hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, device_) != hipSuccess || rate_khz <= 0)
      rate_khz = 100000;
    timeout_ticks_ = (long long)(timeout_s * 1e3 * rate_khz);
    bases_.assign(world_, nullptr);
    bases_[rank_] = own_;
  }

  ~P2PComm() {
    for (int r = 0; r < world_; ++r)
      if (r != rank_ && bases_[r]) hipIpcCloseMemHandle(bases_[r]);
    if (own_) hipFree(own_);
    if (epoch_dev_) hipFree(epoch_dev_);
    if (err_) hipHostFree(err_);
  }

  pybind11::bytes handle() const {
    hipIpcMemHandle_t h;
    check(hipIpcGetMemHandle(&h, own_), "hipIpcGetMemHandle");
    return pybind11::bytes(reinterpret_cast<const char*>(&h), sizeof(h));
  }

  void open(const std::vector<std::string>& handles) {
    TORCH_CHECK((int)handles.size() == world_, "P2PComm.open: one handle per rank");
    check(hipSetDevice(device_), "hipSetDevice");
    for (int r = 0; r < world_; ++r) {
      if (r == rank_) continue;
      TORCH_CHECK(handles[r].size() == sizeof(hipIpcMemHandle_t), "P2PComm.open: bad handle size");
      hipIpcMemHandle_t h;
      std::memcpy(&h, handles[r].data(), sizeof(h));
      void* p = nullptr;
      check(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle");
      bases_[r] = p;
    }
    opened_ = true;
  }

  // in-place all-reduce of a contiguous fp32 / bf16 CUDA tensor on the current stream
  // (average=True: the sum times 1/world)
  void allreduce_(at::Tensor t, bool average) {
    TORCH_CHECK(opened_, "P2PComm: open() first");
    TORCH_CHECK(t.is_cuda() && t.is_contiguous() && t.device().index() == device_, "P2PComm: contiguous tensor on the device");
    TORCH_CHECK(t.scalar_type() == at::kFloat || t.scalar_type() == at::kBFloat16, "P2PComm: fp32 or bf16");
    const long long bytes = t.numel() * (long long)t.element_size();
    TORCH_CHECK(bytes <= cap_, "P2PComm: tensor larger than the staging capacity");
    TORCH_CHECK(bytes % 16 == 0, "P2PComm: size must be a multiple of 16 bytes");
    if (*err_ != 0) TORCH_CHECK(false, "P2PComm: an earlier all-reduce timed out waiting for a peer");
    if (bytes == 0) return;
    ++epoch_;  // calls issued (host bookkeeping only: the kernels use the device counter)
    hipStream_t st = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA(device_).stream();
    const float scale = average ? 1.f / (float)world_ : 1.f;
    const int rc = rtdc_p2p_oneshot((const void* const*)bases_.data(), world_, rank_, epoch_dev_, cap_, t.data_ptr(),
                                    t.numel(), t.scalar_type() == at::kBFloat16 ? 1 : 0, scale, err_, timeout_ticks_,
                                    blocks_, st);
    TORCH_CHECK(rc == 0, "rtdc_p2p_oneshot failed (" + std::to_string(rc) + ")");
  }

  int error() const { return *err_; }
  // device-readable address of the error word (host-coherent): the fused optimizer kernels
  // skip their update when it is set (kernels/optim.hip comm_poisoned)
  int64_t error_ptr() const { return (int64_t)(uintptr_t)err_; }
  // stream-ordered copy of the error word into dst[idx] (pinned host int32) on the current
  // stream: a checkpoint snapshot records the outcome of exactly the collectives enqueued
  // before it, not the live sticky word (parallel/health.py capture_error_words)
  void snapshot_error(at::Tensor dst, int64_t idx) const {
    TORCH_CHECK(dst.scalar_type() == at::kInt && dst.is_contiguous() && idx >= 0 && idx < dst.numel(),
                "P2PComm.snapshot_error: contiguous int32 destination");
    hipStream_t st = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA(device_).stream();
    check(hipMemcpyAsync(dst.data_ptr<int>() + idx, err_, sizeof(int), hipMemcpyDefault, st), "hipMemcpyAsync");
  }
  long long capacity() const { return cap_; }
  int world() const { return world_; }
  int rank() const { return rank_; }
  long long epoch() const { return epoch_; }

 private:
  static void check(hipError_t e, const char* what) {
    TORCH_CHECK(e == hipSuccess, std::string(what) + ": " + hipGetErrorString(e));
  }

  int rank_, world_;
  long long cap_;
  int device_, blocks_;
  void* own_ = nullptr;
  int* err_ = nullptr;
  unsigned* epoch_dev_ = nullptr;
  long long timeout_ticks_ = 0;
  std::vector<void*> bases_;
  bool opened_ = false;
  unsigned epoch_ = 0;
};

}  // namespace rtdc_p2p

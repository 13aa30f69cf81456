// Native gradient-bucket engine for data-parallel training (the MI355X-native counterpart of
// c10d's C++ Reducer, T/include/torch/csrc/distributed/c10d/reducer.hpp:30-31,135,279,329,499,523).
//
// The gradients of all parameters live in ONE flat fp32 buffer (optim/flat.py).  A bucket is
// a contiguous [lo, hi) slice of it, fixed at construction (static plan in backward order:
// a small first bucket, then `bucket_cap` buckets - see parallel/ddp.py for the sizing
// rationale for 7 xGMI links).  Per step:
//   * mark_ready(p) is called from each parameter's post-accumulate-grad hook; it counts the
//     bucket down and launches every bucket whose turn has come, strictly in bucket order
//     (identical collective order on every rank - no rendezvous needed),
//   * the all-reduce runs IN PLACE on the slice on the process group's own stream (RCCL over
//     xGMI; averaging folded into the collective with ReduceOp::AVG), overlapped with the
//     rest of the backward pass - no copy-in/copy-out, no pre-divide kernel,
//   * finalize() (queued at the end of backward) launches what is left (parameters that got
//     no gradient), waits for every Work - which on RCCL makes the current stream wait, not
//     the host - applies the 1/world post-scale for backends without AVG (gloo), and resets.
// Reduced-precision communication (grad_comm_dtype="bf16"): when a bucket is ready its fp32
// slice is rounded into a parallel bf16 buffer on the compute stream (one streaming kernel),
// the bf16 slice is all-reduced (half the xGMI bytes of fp32), and as soon as that collective
// completes a side stream widens it back into the fp32 master-gradient slice - so `p.grad`
// still holds the averaged gradient and the optimizer is unchanged; the compute stream only
// waits for the side stream's event at the end of backward.
// Bucket bookkeeping is lock-free single-threaded state: autograd invokes the hooks from
// one engine thread per device.
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <torch/csrc/distributed/c10d/ProcessGroup.hpp>
#include <torch/csrc/distributed/c10d/Work.hpp>

#include <memory>
#include <mutex>

#include "p2p_comm.cpp"

extern "C" {
int rtdc_f32_to_bf16(const float* x, void* y, long long n, hipStream_t st);
int rtdc_bf16_to_f32(const void* x, float* y, long long n, float scale, hipStream_t st);
}

namespace rtdc_ddp {

// One widen stream and one P2P stream per device for the whole process, shared by every
// engine.  A pool stream per engine made each re-wrap (bench.py's bucket sweep) create a new
// HIP stream; past GPU_MAX_HW_QUEUES (4) streams share hardware queues round-robin, and a
// widen stream that lands on the compute stream's queue parks the compute kernels behind its
// wait on the all-reduce: +2..8 ms/step on the 2nd..4th bf16 wrap of GPT-2 (r4 sweep).
enum SharedStream { kWiden = 0, kP2P = 1 };
inline c10::hip::HIPStreamMasqueradingAsCUDA shared_stream(SharedStream kind, int dev) {
  static std::mutex mu;
  static std::vector<c10::optional<c10::hip::HIPStreamMasqueradingAsCUDA>> streams[2];
  std::lock_guard<std::mutex> lock(mu);
  auto& v = streams[kind];
  if ((int)v.size() <= dev) v.resize(dev + 1);
  if (!v[dev]) v[dev].emplace(c10::hip::getStreamFromPoolMasqueradingAsCUDA(/*isHighPriority=*/true, dev));
  return *v[dev];
}

class GradBucketEngine {
 public:
  // seg: per parameter (offset, numel) inside flat_grad, same order as param_bucket
  GradBucketEngine(at::Tensor flat_grad, std::vector<int64_t> bounds, std::vector<int64_t> param_bucket,
                   std::vector<std::pair<int64_t, int64_t>> seg, c10::intrusive_ptr<c10d::ProcessGroup> pg,
                   bool use_avg, double post_scale, c10::optional<at::Tensor> comm_buf, int64_t zero_world = 0,
                   int64_t zero_rank = 0)
      : flat_(std::move(flat_grad)), bounds_(std::move(bounds)), param_bucket_(std::move(param_bucket)),
        seg_(std::move(seg)), pg_(std::move(pg)), use_avg_(use_avg), post_scale_(post_scale),
        zero_world_(zero_world > 1 ? zero_world : 0), zero_rank_(zero_rank) {
    TORCH_CHECK(seg_.size() == param_bucket_.size(), "one segment per parameter");
    TORCH_CHECK(bounds_.size() >= 2, "need at least one bucket");
    const size_t nb = bounds_.size() - 1;
    if (comm_buf.has_value()) {
      lp_ = *comm_buf;
      TORCH_CHECK(lp_.scalar_type() == at::kBFloat16 && lp_.numel() == flat_.numel() &&
                      lp_.device() == flat_.device() && lp_.is_contiguous(),
                  "comm buffer: contiguous bf16 twin of the flat gradient buffer");
      if (flat_.is_cuda()) {
        side_.emplace(shared_stream(kWiden, flat_.device().index()));
        events_.resize(nb, nullptr);
        for (auto& e : events_) TORCH_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming) == hipSuccess,
                                            "hipEventCreate");
      }
    }
    if (zero_world_) {
      TORCH_CHECK(zero_rank_ >= 0 && zero_rank_ < zero_world_, "ZeRO rank out of range");
      for (size_t b = 0; b < nb; ++b)
        TORCH_CHECK((bounds_[b + 1] - bounds_[b]) % (64 * zero_world_) == 0,
                    "ZeRO: every bucket must be a multiple of 64 x world elements");
    }
    expected_.assign(nb, 0);
    for (int64_t b : param_bucket_) {
      TORCH_CHECK(b >= 0 && (size_t)b < nb, "bad bucket index");
      expected_[b] += 1;
    }
    pending_ = expected_;
    works_.resize(nb);
    launched_.assign(nb, false);
    marked_.assign(param_bucket_.size(), false);
  }

  void mark_ready(int64_t param_idx) {
    TORCH_CHECK(param_idx >= 0 && (size_t)param_idx < param_bucket_.size(), "bad parameter index");
    if (marked_[param_idx]) return;  // a second gradient of the same parameter this step
    marked_[param_idx] = true;
    pending_[param_bucket_[param_idx]] -= 1;
    launch_ready();
  }

  // defer_last: make the current stream wait for every bucket but the last one; the last
  // bucket's collective stays in flight until wait_tail() (the fused optimizer updates the
  // other parameters meanwhile - the last bucket holds the parameters whose gradients finish
  // last, e.g. GPT-2's tied 154 MB token table, so its all-reduce is the step's exposed tail).
  // Backends without an averaging collective (gloo) get the 1/world scale per part: the
  // final slices now, the deferred one in wait_tail().
  ~GradBucketEngine() {
    for (auto e : events_)
      if (e) hipEventDestroy(e);
    for (auto e : p2p_ready_)
      if (e) hipEventDestroy(e);
    for (auto e : p2p_done_)
      if (e) hipEventDestroy(e);
    for (auto e : piece_events_)
      if (e) hipEventDestroy(e);
  }

  void finalize(bool defer_last = false) {
    wait_tail();
    // parameters that produced no gradient this step contribute zeros (their slots may hold
    // a previous step's values when gradients are written in place): only unlaunched
    // buckets can contain them
    for (size_t i = 0; i < marked_.size(); ++i)
      if (!marked_[i]) flat_.slice(0, seg_[i].first, seg_[i].first + seg_[i].second).zero_();
    while (next_ < works_.size()) launch(next_++);
    const size_t last_b = works_.size() - 1;
    const bool defer = defer_last && works_.size() > 1 && !is_p2p(last_b);
    const size_t nwait = works_.size() - (defer ? 1 : 0);
    // the last bucket as pieces (set_tail_split), not deferred: its pieces complete here
    const bool pieces_now = !defer && !pieces_.empty();
    if (p2p_) {
      hipStream_t cur = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA(flat_.device().index()).stream();
      for (size_t b = 0; b < nwait; ++b)
        if (is_p2p(b)) TORCH_CHECK(hipStreamWaitEvent(cur, p2p_done_[b], 0) == hipSuccess, "hipStreamWaitEvent");
    }
    if (side_) {
      // the widened fp32 slices are final once the side stream passed each bucket's event
      // (a piece-split last bucket: its last piece's event - the side stream is in order)
      hipStream_t cur = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA(flat_.device().index()).stream();
      size_t last = nwait;
      while (last > 0 && is_p2p(last - 1)) --last;  // the side stream handled buckets < last
      if (last > 0) {
        hipEvent_t ev = (pieces_now && last - 1 == last_b) ? piece_events_[pieces_.size() - 1] : events_[last - 1];
        TORCH_CHECK(hipStreamWaitEvent(cur, ev, 0) == hipSuccess, "hipStreamWaitEvent");
      }
    } else {
      {
        pybind11::gil_scoped_release nogil;
        for (size_t b = 0; b < nwait; ++b)
          if (works_[b]) works_[b]->wait();
        if (pieces_now)
          for (auto& w : piece_works_) w->wait();
      }
      if (lp_.defined()) {  // CPU (gloo): widen in place after the blocking wait
        for (size_t b = 0; b < nwait; ++b)
          if (!(pieces_now && b == last_b)) widen(b);
        if (pieces_now)
          for (size_t i = 0; i < pieces_.size(); ++i) widen_range(pieces_[i].first, pieces_[i].second);
      } else if (!use_avg_ && post_scale_ != 1.0) {
        flat_.slice(0, 0, bounds_[nwait]).mul_(post_scale_);
      }
    }
    if (pieces_now) {
      pieces_.clear();
      piece_works_.clear();
    }
    if (defer) {
      if (!pieces_.empty()) {
        tail_piece_next_ = 0;  // pieces stay in flight: wait_tail_piece(i) / wait_tail()
        tail_pieces_pending_ = true;
      } else {
        tail_ = works_.back();
      }
    }
    for (size_t b = 0; b < nwait; ++b) works_[b].reset();
    pending_ = expected_;
    std::fill(launched_.begin(), launched_.end(), false);
    std::fill(marked_.begin(), marked_.end(), false);
    next_ = 0;
    ++steps_;
  }

  // stream-order the last bucket's all-reduce before later work (no-op when none is pending)
  void wait_tail() {
    if (tail_pieces_pending_) {
      while (tail_piece_next_ < pieces_.size()) wait_tail_piece((int64_t)tail_piece_next_);
      return;
    }
    if (!tail_) return;
    const size_t last = works_.size() - 1;
    if (side_) {
      hipStream_t cur = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA(flat_.device().index()).stream();
      TORCH_CHECK(hipStreamWaitEvent(cur, events_[last], 0) == hipSuccess, "hipStreamWaitEvent");
    } else {
      {
        pybind11::gil_scoped_release nogil;
        tail_->wait();
      }
      if (lp_.defined()) widen(last);
      else if (!use_avg_ && post_scale_ != 1.0) flat_.slice(0, tail_start(), bounds_.back()).mul_(post_scale_);
    }
    tail_.reset();
    works_[last].reset();
  }
  // ---- the last bucket as several collectives (set_tail_split) -------------------------
  // GPT-2's tied token table is one 154 MB gradient that completes at the very end of
  // backward: as ONE deferred collective the fused optimizer can only update it after all of
  // it landed.  Split into pieces of at most `max_elems`, the optimizer waits for piece i and
  // updates its slice while pieces i+1.. are still on the wire (optim/fused.py _launch_split).
  // All pieces launch together in order on every rank (same collective sequence everywhere).
  void set_tail_split(int64_t max_elems) {
    TORCH_CHECK(max_elems >= 0, "set_tail_split: max_elems >= 0");
    tail_max_ = max_elems;
  }
  // flat offsets where the pieces of a deferred tail start (empty: no piece-split tail pending)
  std::vector<int64_t> tail_piece_starts() const {
    std::vector<int64_t> out;
    if (tail_pieces_pending_)
      for (auto& pr : pieces_) out.push_back(pr.first);
    return out;
  }
  // make the current stream (CPU: the host) wait until piece i of the deferred tail is final
  void wait_tail_piece(int64_t i) {
    if (!tail_pieces_pending_) return;
    TORCH_CHECK(i >= 0 && (size_t)i < pieces_.size(), "wait_tail_piece: bad piece");
    while (tail_piece_next_ <= (size_t)i) {
      const size_t k = tail_piece_next_++;
      if (side_) {
        hipStream_t cur = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA(flat_.device().index()).stream();
        TORCH_CHECK(hipStreamWaitEvent(cur, piece_events_[k], 0) == hipSuccess, "hipStreamWaitEvent");
      } else {
        {
          pybind11::gil_scoped_release nogil;
          piece_works_[k]->wait();
        }
        if (lp_.defined()) widen_range(pieces_[k].first, pieces_[k].second);
        else if (!use_avg_ && post_scale_ != 1.0)
          flat_.slice(0, pieces_[k].first, pieces_[k].second).mul_(post_scale_);
      }
    }
    if (tail_piece_next_ >= pieces_.size()) {
      tail_pieces_pending_ = false;
      pieces_.clear();
      piece_works_.clear();
      works_.back().reset();
    }
  }

  // Route buckets of at most max_bytes (communicated bytes) through the one-shot hipIpc
  // all-reduce (runtime/p2p_comm.cpp) on a dedicated stream instead of RCCL; the rest stay on
  // the process group.  Collective order is unchanged (bucket order), so every rank routes the
  // same buckets.
  void set_p2p(std::shared_ptr<rtdc_p2p::P2PComm> comm, int64_t max_bytes) {
    TORCH_CHECK(flat_.is_cuda(), "p2p all-reduce needs a device gradient buffer");
    p2p_ = std::move(comm);
    p2p_max_bytes_ = max_bytes;
    const size_t nb = works_.size();
    if (!p2p_stream_)
      p2p_stream_.emplace(shared_stream(kP2P, flat_.device().index()));
    if (p2p_ready_.empty()) {
      p2p_ready_.resize(nb, nullptr);
      p2p_done_.resize(nb, nullptr);
      for (size_t b = 0; b < nb; ++b) {
        TORCH_CHECK(hipEventCreateWithFlags(&p2p_ready_[b], hipEventDisableTiming) == hipSuccess, "hipEventCreate");
        TORCH_CHECK(hipEventCreateWithFlags(&p2p_done_[b], hipEventDisableTiming) == hipSuccess, "hipEventCreate");
      }
    }
    via_p2p_.assign(nb, false);
    for (size_t b = 0; b < nb; ++b) {
      const int64_t bytes = (bounds_[b + 1] - bounds_[b]) * (lp_.defined() ? 2 : 4);
      via_p2p_[b] = p2p_ && bytes <= p2p_max_bytes_ && bytes <= p2p_->capacity() && bytes % 16 == 0;
    }
  }
  std::vector<bool> p2p_buckets() const { return via_p2p_; }

  int64_t comm_bytes_per_step() const {
    return (bounds_.back() - bounds_.front()) * (lp_.defined() ? 2 : 4);
  }
  // Make the CURRENT stream wait until bucket b's reduced gradient is final in the fp32 buffer
  // (an optimizer update of that slice may then run on it while backward continues): the
  // widen event (bf16 communication), the P2P done event, or - averaging backends - the
  // collective itself (Work::wait on a CUDA-like backend orders the current stream after it).
  // Backends that need the finalize() post-scale (SUM without a widen pass) cannot do this.
  bool can_stream_wait() const {
    return flat_.is_cuda() && !zero_world_ && (use_avg_ || side_.has_value() || post_scale_ == 1.0);
  }
  void stream_wait_bucket(int64_t b) {
    TORCH_CHECK(can_stream_wait(), "stream_wait_bucket: needs a device buffer, no ZeRO, and AVG or bf16 comm");
    TORCH_CHECK(b >= 0 && (size_t)b < works_.size() && launched_[b], "stream_wait_bucket: bucket not launched");
    hipStream_t cur = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA(flat_.device().index()).stream();
    if ((size_t)b + 1 == works_.size() && !pieces_.empty()) {  // a piece-split last bucket: all pieces
      if (side_) {
        TORCH_CHECK(hipStreamWaitEvent(cur, piece_events_[pieces_.size() - 1], 0) == hipSuccess, "hipStreamWaitEvent");
      } else {
        for (auto& w : piece_works_) w->wait();
      }
      return;
    }
    if (is_p2p(b)) {
      TORCH_CHECK(hipStreamWaitEvent(cur, p2p_done_[b], 0) == hipSuccess, "hipStreamWaitEvent");
    } else if (side_) {
      TORCH_CHECK(hipStreamWaitEvent(cur, events_[b], 0) == hipSuccess, "hipStreamWaitEvent");
    } else {
      TORCH_CHECK(works_[b], "stream_wait_bucket: no work");
      works_[b]->wait();
    }
  }
  bool tail_pending() const { return (bool)tail_ || tail_pieces_pending_; }
  int64_t tail_start() const { return bounds_[bounds_.size() - 2]; }

  int64_t num_buckets() const { return (int64_t)works_.size(); }
  int64_t steps() const { return steps_; }
  int64_t launched() const { return (int64_t)next_; }
  std::vector<int64_t> bucket_bytes() const {
    std::vector<int64_t> out;
    for (size_t b = 0; b + 1 < bounds_.size(); ++b)
      out.push_back((bounds_[b + 1] - bounds_[b]) * (lp_.defined() ? 2 : 4));
    return out;
  }

 private:
  void launch_ready() {
    while (next_ < works_.size() && pending_[next_] <= 0) launch(next_++);
  }

  bool is_p2p(size_t b) const { return !zero_world_ && p2p_ && b < via_p2p_.size() && via_p2p_[b]; }

  // ZeRO-1: the [lo, hi) range of bucket b this rank owns after the reduce-scatter
  std::pair<int64_t, int64_t> owned(size_t b) const {
    const int64_t lo = bounds_[b], hi = bounds_[b + 1];
    if (!zero_world_) return {lo, hi};
    const int64_t sh = (hi - lo) / zero_world_;
    return {lo + zero_rank_ * sh, lo + (zero_rank_ + 1) * sh};
  }

  void launch(size_t b) {
    const int64_t lo = bounds_[b], hi = bounds_[b + 1];
    at::Tensor src = flat_.slice(0, lo, hi);
    std::vector<at::Tensor> t{src};
    if (is_p2p(b)) {
      hipStream_t cur = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA(flat_.device().index()).stream();
      at::Tensor buf = src;
      if (lp_.defined()) {
        buf = lp_.slice(0, lo, hi);
        TORCH_CHECK(rtdc_f32_to_bf16(src.data_ptr<float>(), buf.data_ptr(), hi - lo, cur) == 0, "f32->bf16");
      }
      TORCH_CHECK(hipEventRecord(p2p_ready_[b], cur) == hipSuccess, "hipEventRecord");
      TORCH_CHECK(hipStreamWaitEvent(p2p_stream_->stream(), p2p_ready_[b], 0) == hipSuccess, "hipStreamWaitEvent");
      {
        c10::hip::HIPStreamGuardMasqueradingAsCUDA g(*p2p_stream_);
        // SUM when the process group has no AVG (gloo): the engine's post-scale then covers it
        p2p_->allreduce_(buf, use_avg_);
        if (lp_.defined()) widen(b);
        TORCH_CHECK(hipEventRecord(p2p_done_[b], p2p_stream_->stream()) == hipSuccess, "hipEventRecord");
      }
      launched_[b] = true;
      return;
    }
    if (b + 1 == works_.size() && tail_max_ > 0 && hi - lo > tail_max_ && !zero_world_) {
      launch_pieces(lo, hi);
      launched_[b] = true;
      return;
    }
    if (lp_.defined()) {
      at::Tensor dst = lp_.slice(0, lo, hi);
      if (flat_.is_cuda()) {
        hipStream_t cur = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA(flat_.device().index()).stream();
        TORCH_CHECK(rtdc_f32_to_bf16(src.data_ptr<float>(), dst.data_ptr(), hi - lo, cur) == 0, "f32->bf16");
      } else {
        dst.copy_(src);
      }
      t[0] = dst;
    }
    if (zero_world_) {
      // ZeRO-1: reduce-scatter in place - this rank's shard of the bucket receives the
      // average, the rest of the slice keeps the local gradient (never read)
      const auto [olo, ohi] = owned(b);
      at::Tensor out = t[0].slice(0, olo - lo, ohi - lo);
      c10d::ReduceScatterOptions ro;
      ro.reduceOp = use_avg_ ? c10d::ReduceOp(c10d::ReduceOp::AVG) : c10d::ReduceOp(c10d::ReduceOp::SUM);
      works_[b] = pg_->_reduce_scatter_base(out, t[0], ro);
    } else {
      c10d::AllreduceOptions opts;
      opts.reduceOp = use_avg_ ? c10d::ReduceOp(c10d::ReduceOp::AVG) : c10d::ReduceOp(c10d::ReduceOp::SUM);
      works_[b] = pg_->allreduce(t, opts);
    }
    launched_[b] = true;
    if (side_) {
      // widen back on the side stream right after the collective (Work::wait on a CUDA-like
      // backend only makes the current stream wait for the communication stream)
      c10::hip::HIPStreamGuardMasqueradingAsCUDA g(*side_);
      works_[b]->wait();
      widen(b);
      TORCH_CHECK(hipEventRecord(events_[b], side_->stream()) == hipSuccess, "hipEventRecord");
    }
  }

  // the last bucket [lo, hi) as pieces of <= tail_max_ elements (64-aligned), each its own
  // all-reduce (+ bf16 narrow / side-stream widen and a per-piece event)
  void launch_pieces(int64_t lo, int64_t hi) {
    pieces_.clear();
    piece_works_.clear();
    const int64_t n = (hi - lo + tail_max_ - 1) / tail_max_;
    const int64_t step = ((hi - lo + n - 1) / n + 63) / 64 * 64;
    for (int64_t a = lo; a < hi; a += step) pieces_.emplace_back(a, std::min(hi, a + step));
    if (side_)
      while (piece_events_.size() < pieces_.size()) {
        hipEvent_t e;
        TORCH_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming) == hipSuccess, "hipEventCreate");
        piece_events_.push_back(e);
      }
    c10d::AllreduceOptions opts;
    opts.reduceOp = use_avg_ ? c10d::ReduceOp(c10d::ReduceOp::AVG) : c10d::ReduceOp(c10d::ReduceOp::SUM);
    for (size_t i = 0; i < pieces_.size(); ++i) {
      const auto [a, e] = pieces_[i];
      at::Tensor t = flat_.slice(0, a, e);
      if (lp_.defined()) {
        at::Tensor dst = lp_.slice(0, a, e);
        if (flat_.is_cuda()) {
          hipStream_t cur = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA(flat_.device().index()).stream();
          TORCH_CHECK(rtdc_f32_to_bf16(t.data_ptr<float>(), dst.data_ptr(), e - a, cur) == 0, "f32->bf16");
        } else {
          dst.copy_(t);
        }
        t = dst;
      }
      std::vector<at::Tensor> tv{t};
      piece_works_.push_back(pg_->allreduce(tv, opts));
    }
    if (side_) {
      c10::hip::HIPStreamGuardMasqueradingAsCUDA g(*side_);
      for (size_t i = 0; i < pieces_.size(); ++i) {
        piece_works_[i]->wait();
        widen_range(pieces_[i].first, pieces_[i].second);
        TORCH_CHECK(hipEventRecord(piece_events_[i], side_->stream()) == hipSuccess, "hipEventRecord");
      }
    }
  }

  void widen_range(int64_t lo, int64_t hi) {
    const float scale = use_avg_ ? 1.f : (float)post_scale_;
    if (flat_.is_cuda()) {
      hipStream_t st = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA(flat_.device().index()).stream();
      TORCH_CHECK(rtdc_bf16_to_f32(lp_.slice(0, lo, hi).data_ptr(), flat_.slice(0, lo, hi).data_ptr<float>(), hi - lo,
                                   scale, st) == 0,
                  "bf16->f32");
    } else {
      at::Tensor f = flat_.slice(0, lo, hi);
      f.copy_(lp_.slice(0, lo, hi));
      if (scale != 1.f) f.mul_(scale);
    }
  }

  // bf16 reduced slice -> fp32 master gradient slice (x post-scale for SUM backends)
  void widen(size_t b) {
    const auto [lo, hi] = owned(b);  // (the whole bucket without ZeRO)
    const float scale = use_avg_ ? 1.f : (float)post_scale_;
    if (flat_.is_cuda()) {
      hipStream_t st = c10::hip::getCurrentHIPStreamMasqueradingAsCUDA(flat_.device().index()).stream();
      TORCH_CHECK(rtdc_bf16_to_f32(lp_.slice(0, lo, hi).data_ptr(), flat_.slice(0, lo, hi).data_ptr<float>(),
                                   hi - lo, scale, st) == 0,
                  "bf16->f32");
    } else {
      at::Tensor f = flat_.slice(0, lo, hi);
      f.copy_(lp_.slice(0, lo, hi));
      if (scale != 1.f) f.mul_(scale);
    }
  }

  at::Tensor flat_, lp_;
  c10::optional<c10::hip::HIPStreamMasqueradingAsCUDA> side_;
  std::vector<hipEvent_t> events_;
  std::vector<int64_t> bounds_, param_bucket_, expected_, pending_;
  std::vector<std::pair<int64_t, int64_t>> seg_;
  c10::intrusive_ptr<c10d::ProcessGroup> pg_;
  bool use_avg_;
  double post_scale_;
  int64_t zero_world_, zero_rank_;
  std::vector<c10::intrusive_ptr<c10d::Work>> works_;
  c10::intrusive_ptr<c10d::Work> tail_;
  std::vector<bool> launched_, marked_;
  std::shared_ptr<rtdc_p2p::P2PComm> p2p_;
  int64_t p2p_max_bytes_ = 0;
  std::vector<bool> via_p2p_;
  c10::optional<c10::hip::HIPStreamMasqueradingAsCUDA> p2p_stream_;
  std::vector<hipEvent_t> p2p_ready_, p2p_done_;
  size_t next_ = 0;
  int64_t steps_ = 0;
  int64_t tail_max_ = 0;                                  // set_tail_split (0: one collective)
  std::vector<std::pair<int64_t, int64_t>> pieces_;       // the last bucket's pieces this step
  std::vector<c10::intrusive_ptr<c10d::Work>> piece_works_;
  std::vector<hipEvent_t> piece_events_;
  bool tail_pieces_pending_ = false;
  size_t tail_piece_next_ = 0;
};

}  // namespace rtdc_ddp

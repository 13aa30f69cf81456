// Native checkpoint I/O engine (host side of the MI355X checkpoint path).
//
// Replaces the reference's blocking `torch.save` (one synchronous D2H per storage,
// R/my_ray_module.py:179-201 -> torch/serialization.py:1264-1286) and torch DCP's pageable
// `_OverlappingCpuLoader` + Python writer threads (torch/distributed/checkpoint/filesystem.py
// :141-208, :596-600) with:
//
//   device snapshot (HBM, taken by the caller on its compute stream)
//     -> bounded ring of pinned host slots (hipHostMalloc)            [PinnedRing]
//     -> D2H by the SDMA engines (hsa_amd_memory_async_copy, no AQL queue)  [enqueue thread]
//        (or hipMemcpyAsync on a dedicated copy stream: RTDC_CKPT_D2H=hip)
//     -> writer thread pool: event wait, CRC32 of the piece, pwrite     [writer threads]
//     -> per-file finalize: CRCs patched into the zip headers, central directory, fsync.
//
// Files are zip archives byte-compatible with `torch.load(weights_only=True)` (STORED records,
// data records 64-B aligned via an 'FB' extra field like PyTorchStreamWriter) so a `.pt` file
// or a DCP `__r_i.distcp` shard written here is readable by stock torch.  Nothing blocks the
// Python thread that submits a save: `submit` returns a job id, `wait`/`poll` report completion.
//
// Reads (restore) go the other way: `read_to_host` preads file ranges with a thread pool into
// caller memory (pinned or pageable); H2D and the cross-rank broadcast are issued from Python.
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <zlib.h>

#include "runtime/crc32_fast.h"
#include <fcntl.h>
#include <sys/resource.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

namespace rtdc_ckpt {

static bool g_have_gpu() {
  static int cached = -1;
  if (cached < 0) {
    int n = 0;
    cached = (hipGetDeviceCount(&n) == hipSuccess && n > 0) ? 1 : 0;
  }
  return cached == 1;
}

// ------------------------------------------------------------------------------------------
// zip layout.  ZIP64 is used exactly where the 32-bit fields overflow (the scheme
// PyTorchStreamWriter/miniz writes and torch.load reads): a record >= 4 GiB carries a zip64
// extra field (0x0001) with its 64-bit sizes in the local header and the central directory;
// a local header past 4 GiB carries its 64-bit offset in the central-directory extra; an
// archive whose central directory lies past 4 GiB or holds >= 65535 entries gets a zip64
// end-of-central-directory record + locator in front of the classic EOCD.
// ------------------------------------------------------------------------------------------
static constexpr uint64_t kZ32 = 0xFFFFFFFFull;

struct Record {
  std::string name;
  std::string inline_data;    // small records (pickle, version files)
  const char* src = nullptr;  // big record source (device or host pointer)
  uint64_t nbytes = 0;
  bool on_device = false;
  // layout
  uint64_t header_off = 0, data_off = 0;
  uint16_t extra_len = 0;     // local-header extra: zip64 sizes (if z64_size) + 'FB' padding
  bool z64_size = false;
  uint32_t crc = 0;
};

static void put16(std::string& s, uint16_t v) { s.push_back(v & 0xff); s.push_back(v >> 8); }
static void put32(std::string& s, uint32_t v) {
  for (int i = 0; i < 4; ++i) s.push_back((v >> (8 * i)) & 0xff);
}
static void put64(std::string& s, uint64_t v) {
  for (int i = 0; i < 8; ++i) s.push_back((char)((v >> (8 * i)) & 0xff));
}

static uint64_t rec_size(const Record& r) { return r.src ? r.nbytes : r.inline_data.size(); }

static std::string local_header(const Record& r, uint64_t size) {
  std::string h;
  put32(h, 0x04034b50);
  put16(h, r.z64_size ? 45 : 20);  // version needed (4.5 = zip64)
  put16(h, 0);   // flags
  put16(h, 0);   // STORED
  put16(h, 0);   // mod time
  put16(h, 0x21);  // mod date (1980-01-01)
  put32(h, r.crc);
  put32(h, r.z64_size ? (uint32_t)kZ32 : (uint32_t)size);
  put32(h, r.z64_size ? (uint32_t)kZ32 : (uint32_t)size);
  put16(h, (uint16_t)r.name.size());
  put16(h, r.extra_len);
  h += r.name;
  uint16_t pad = r.extra_len;
  if (r.z64_size) {
    put16(h, 0x0001);
    put16(h, 16);
    put64(h, size);
    put64(h, size);
    pad -= 20;
  }
  if (pad) {
    put16(h, 0x4246);  // 'FB' padding field (PyTorchStreamWriter uses the same tag)
    put16(h, (uint16_t)(pad - 4));
    h.append(pad - 4, 'Z');
  }
  return h;
}

// Records at least this large get their data at a 4 KiB-aligned FILE offset, so their
// slot-sized pieces can be written and read with O_DIRECT (DMA between the pinned ring and
// the device, no page-cache copy); smaller records are 64-B aligned like PyTorchStreamWriter.
static constexpr uint64_t kDirectMin = 1ull << 16, kPage = 4096;

// Assign archive-relative offsets; `abs_base` is the archive's file offset (for the 4 KiB
// alignment of big records).
static uint64_t layout_records(std::vector<Record>& recs, uint64_t base, uint64_t abs_base = 0) {
  uint64_t off = base;
  for (auto& r : recs) {
    r.header_off = off;
    r.z64_size = rec_size(r) >= kZ32;
    const uint64_t z = r.z64_size ? 20 : 0;
    uint64_t hdr = 30 + r.name.size() + z;
    uint64_t data = off + hdr;
    const uint64_t align = (r.src && r.nbytes >= kDirectMin) ? kPage : 64;
    uint64_t pad = (align - ((abs_base + data) % align)) % align;
    if (pad > 0 && pad < 4) pad += align;  // extra field needs >= 4 bytes
    r.extra_len = (uint16_t)(z + pad);
    r.data_off = data + pad;
    off = r.data_off + rec_size(r);
  }
  return off;
}

static uint64_t cd_entry_extra(const Record& r) {
  return (r.z64_size ? 16 : 0) + (r.header_off >= kZ32 ? 8 : 0);
}

static bool eocd64_needed(const std::vector<Record>& recs, uint64_t cd_off, uint64_t cd_bytes) {
  return recs.size() >= 0xFFFF || cd_off >= kZ32 || cd_bytes >= kZ32;
}

// central-directory bytes (entries only) of an archive whose data ends at cd_off
static uint64_t cd_entries_size(const std::vector<Record>& recs) {
  uint64_t n = 0;
  for (auto& r : recs) {
    const uint64_t e = cd_entry_extra(r);
    n += 46 + r.name.size() + (e ? 4 + e : 0);
  }
  return n;
}

static uint64_t cd_size(const std::vector<Record>& recs, uint64_t cd_off) {
  const uint64_t entries = cd_entries_size(recs);
  return entries + 22 + (eocd64_needed(recs, cd_off, entries) ? 56 + 20 : 0);
}

static std::string central_dir(const std::vector<Record>& recs, uint64_t cd_off) {
  std::string cd;
  for (auto& r : recs) {
    const uint64_t size = rec_size(r);
    const bool z64_off = r.header_off >= kZ32;
    const uint64_t extra = cd_entry_extra(r);
    put32(cd, 0x02014b50);
    put16(cd, 0x031e);  // made by: unix, 3.0
    put16(cd, extra ? 45 : 20);
    put16(cd, 0);
    put16(cd, 0);
    put16(cd, 0);
    put16(cd, 0x21);
    put32(cd, r.crc);
    put32(cd, r.z64_size ? (uint32_t)kZ32 : (uint32_t)size);
    put32(cd, r.z64_size ? (uint32_t)kZ32 : (uint32_t)size);
    put16(cd, (uint16_t)r.name.size());
    put16(cd, (uint16_t)(extra ? 4 + extra : 0));  // extra
    put16(cd, 0);  // comment
    put16(cd, 0);  // disk
    put16(cd, 0);  // internal attr
    put32(cd, 0);  // external attr
    put32(cd, z64_off ? (uint32_t)kZ32 : (uint32_t)r.header_off);
    cd += r.name;
    if (extra) {
      put16(cd, 0x0001);
      put16(cd, (uint16_t)extra);
      if (r.z64_size) {
        put64(cd, size);
        put64(cd, size);
      }
      if (z64_off) put64(cd, r.header_off);
    }
  }
  const uint64_t entries = cd.size();
  const bool z64 = eocd64_needed(recs, cd_off, entries);
  if (z64) {
    const uint64_t eocd64_off = cd_off + entries;
    put32(cd, 0x06064b50);
    put64(cd, 44);
    put16(cd, 45);
    put16(cd, 45);
    put32(cd, 0);
    put32(cd, 0);
    put64(cd, recs.size());
    put64(cd, recs.size());
    put64(cd, entries);
    put64(cd, cd_off);
    put32(cd, 0x07064b50);  // locator
    put32(cd, 0);
    put64(cd, eocd64_off);
    put32(cd, 1);
  }
  put32(cd, 0x06054b50);
  put16(cd, 0);
  put16(cd, 0);
  put16(cd, z64 ? 0xFFFF : (uint16_t)recs.size());
  put16(cd, z64 ? 0xFFFF : (uint16_t)recs.size());
  put32(cd, z64 ? (uint32_t)kZ32 : (uint32_t)entries);
  put32(cd, z64 ? (uint32_t)kZ32 : (uint32_t)cd_off);
  put16(cd, 0);
  return cd;
}

static void pwrite_all(int fd, const void* buf, size_t len, uint64_t off) {
  const char* p = (const char*)buf;
  while (len > 0) {
    ssize_t w = ::pwrite(fd, p, len, (off_t)off);
    if (w < 0) {
      if (errno == EINTR) continue;
      throw std::runtime_error(std::string("pwrite failed: ") + strerror(errno));
    }
    p += w;
    len -= (size_t)w;
    off += (uint64_t)w;
  }
}

static void pread_all(int fd, void* buf, size_t len, uint64_t off) {
  char* p = (char*)buf;
  while (len > 0) {
    ssize_t r = ::pread(fd, p, len, (off_t)off);
    if (r < 0) {
      if (errno == EINTR) continue;
      throw std::runtime_error(std::string("pread failed: ") + strerror(errno));
    }
    if (r == 0) throw std::runtime_error("pread: unexpected EOF");
    p += r;
    len -= (size_t)r;
    off += (uint64_t)r;
  }
}

// ------------------------------------------------------------------------------------------
// Pinned ring
// ------------------------------------------------------------------------------------------
class PinnedRing {
 public:
  PinnedRing(size_t nslots, size_t slot_bytes) : slot_bytes_(slot_bytes) {
    for (size_t i = 0; i < nslots; ++i) {
      void* p = nullptr;
      bool pinned = false;
      if (g_have_gpu() && hipHostMalloc(&p, slot_bytes, hipHostMallocDefault) == hipSuccess) pinned = true;
      if (!pinned) {
        if (posix_memalign(&p, 4096, slot_bytes) != 0) throw std::runtime_error("ring alloc failed");
      }
      slots_.push_back(p);
      pinned_.push_back(pinned);
      hipEvent_t ev = nullptr;
      // blocking sync: a writer waiting on its slot sleeps instead of spinning a core (the
      // default event spins, and 8 spinning writers exhaust a cgroup CPU quota that the
      // rank's launch thread shares - the whole process is then throttled mid-step)
      if (g_have_gpu()) hipEventCreateWithFlags(&ev, hipEventDisableTiming | hipEventBlockingSync);
      events_.push_back(ev);
      free_.push_back((int)i);
    }
  }
  ~PinnedRing() {
    for (size_t i = 0; i < slots_.size(); ++i) {
      if (pinned_[i]) hipHostFree(slots_[i]);
      else free(slots_[i]);
      if (events_[i]) hipEventDestroy(events_[i]);
    }
  }
  int acquire() {
    std::unique_lock<std::mutex> lk(mu_);
    cv_.wait(lk, [&] { return !free_.empty(); });
    int s = free_.front();
    free_.pop_front();
    return s;
  }
  void release(int s) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      free_.push_back(s);
    }
    cv_.notify_one();
  }
  void* ptr(int s) { return slots_[s]; }
  hipEvent_t event(int s) { return events_[s]; }
  size_t slot_bytes() const { return slot_bytes_; }
  size_t nslots() const { return slots_.size(); }
  bool pinned() const { return !pinned_.empty() && pinned_[0]; }

 private:
  size_t slot_bytes_;
  std::vector<void*> slots_;
  std::vector<bool> pinned_;
  std::vector<hipEvent_t> events_;
  std::deque<int> free_;
  std::mutex mu_;
  std::condition_variable cv_;
};

// ------------------------------------------------------------------------------------------
// SDMA drain.  A HIP copy stream is one of the process's GPU_MAX_HW_QUEUES (4) AQL queues,
// shared round-robin with every other stream: when it lands on the compute stream's queue, the
// barrier packet that orders each D2H copy blocks the kernels queued behind it, and a 1.5 GB
// drain costs the training step the whole copy time.  hsa_amd_memory_async_copy hands the
// piece straight to an SDMA engine (device -> pinned host, src agent != dst agent, so never a
// blit kernel on the CUs) with an HSA completion signal: no AQL packet, no CU, no queue shared
// with compute.  The snapshot's readiness is waited on the host first (the event recorded after
// the snapshot copies carries a system-scope release, so the bytes are visible to the DMA).
// ------------------------------------------------------------------------------------------
static bool agent_of(const void* p, hsa_agent_t* a) {
  hsa_amd_pointer_info_t info;
  std::memset(&info, 0, sizeof(info));
  info.size = sizeof(info);
  if (hsa_amd_pointer_info(p, &info, nullptr, nullptr, nullptr) != HSA_STATUS_SUCCESS) return false;
  if (info.type == HSA_EXT_POINTER_TYPE_UNKNOWN || info.agentOwner.handle == 0) return false;
  *a = info.agentOwner;
  return true;
}

// The pinned slot must be directly accessible by the GPU whose SDMA engine copies into it
// (hipHostMalloc normally grants every GPU; a process that sees several GPUs - one rank per
// GPU under torchrun - must not depend on it): add `gpu` to the slot's access list if missing,
// keeping every agent that already has access.
static bool ensure_access(void* slot, hsa_agent_t gpu) {
  hsa_amd_pointer_info_t info;
  std::memset(&info, 0, sizeof(info));
  info.size = sizeof(info);
  uint32_t n = 0;
  hsa_agent_t* agents = nullptr;
  if (hsa_amd_pointer_info(slot, &info, std::malloc, &n, &agents) != HSA_STATUS_SUCCESS) return false;
  bool has = false;
  std::vector<hsa_agent_t> all;
  for (uint32_t i = 0; i < n; ++i) {
    if (agents[i].handle == gpu.handle) has = true;
    all.push_back(agents[i]);
  }
  std::free(agents);
  if (has) return true;
  all.push_back(gpu);
  return hsa_amd_agents_allow_access((uint32_t)all.size(), all.data(), nullptr, slot) == HSA_STATUS_SUCCESS;
}

// host wait without spinning a core (the caller's event may use active synchronization)
static hipError_t wait_event_sleepy(hipEvent_t ev) {
  while (true) {
    hipError_t e = hipEventQuery(ev);
    if (e != hipErrorNotReady) return e;
    std::this_thread::sleep_for(std::chrono::microseconds(20));
  }
}

// ------------------------------------------------------------------------------------------
// Engine
// ------------------------------------------------------------------------------------------
// One file =a sequence of archives written back to back: a torch.save zip archive per tensor
// item (the DCP `__r_i.distcp` layout: each item at a recorded (offset, length), readable by
// `torch.load` on the slice), or a raw byte item (DCP BYTE_IO).  A `.pt` file is one archive.
struct Archive {
  std::vector<Record> recs;
  bool raw = false;
  uint64_t base = 0;      // file offset of the archive
  uint64_t data_end = 0;  // archive-relative end of the last record (central dir starts here)
  uint64_t size = 0;      // full archive size (incl. central directory)
};

// Assign archive bases and record offsets; returns the file size.
static uint64_t layout_archives(std::vector<Archive>& arcs) {
  uint64_t off = 0;
  for (auto& a : arcs) {
    a.base = off;
    if (a.raw) {
      uint64_t n = 0;
      for (auto& r : a.recs) {
        r.header_off = 0;
        r.data_off = n;
        r.extra_len = 0;
        n += rec_size(r);
      }
      a.data_end = n;
      a.size = n;
    } else {
      a.data_end = layout_records(a.recs, 0, off);
      a.size = a.data_end + cd_size(a.recs, a.data_end);
    }
    off += a.size;
  }
  return off;
}

struct FileJob {
  std::string path;
  std::vector<Archive> archives;
  int fd = -1;
  int dfd = -1;  // O_DIRECT descriptor of the same file (-1: filesystem refuses O_DIRECT)
  uint64_t total = 0;
  std::atomic<int> pending{0};
  // per big-record ordered piece CRCs, key = (archive << 24) | record
  std::map<long long, std::vector<std::pair<uint32_t, uint64_t>>> piece_crc;
  std::mutex mu;
  bool fsync_on = true;
  bool crc_on = true;
  std::string error;
};

static inline long long rkey(size_t a, size_t r) { return ((long long)a << 24) | (long long)r; }

struct SaveJob {
  int id;
  std::vector<std::shared_ptr<FileJob>> files;
  std::atomic<int> files_left{0};
  hipEvent_t ready = nullptr;  // device snapshot complete
  bool done = false;
  std::string error;
  double t_submit = 0, t_done = 0;
  std::atomic<double> t_d2h{0.0};  // last device piece landed in the pinned ring
  std::atomic<int> dev_left{0};
  uint64_t bytes = 0;
};

struct JobResult {
  std::string error;
  double durable_s = 0, d2h_s = 0;
};

static double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

class Engine {
 public:
  // `stream`: the copy stream (restore H2D, the hipMemcpy D2H fallback) - a stream the caller
  // already owns (PyTorch's pool).  0 creates a private one.  Every stream a process creates can
  // cost a hardware queue: with two ranks time-sharing one GPU, ONE extra idle stream per process
  // made the training step 10-15x slower (hardware-queue oversubscription; measured with a bare
  // hipStreamCreate, scripts/ab_r5/diag_postckpt.py, profiles/ckpt_engine_stream_r5.txt).
  Engine(size_t nslots, size_t slot_bytes, int nwriters, int device, bool direct_io = true, uintptr_t stream = 0)
      : ring_(nslots, slot_bytes), device_(device), direct_io_(direct_io) {
    if (g_have_gpu()) {
      hipSetDevice(device_);
      if (stream) {
        stream_ = reinterpret_cast<hipStream_t>(stream);
      } else {
        hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking);
        own_stream_ = true;
      }
      const char* m = std::getenv("RTDC_CKPT_D2H");
      const bool want_sdma = !(m && std::string(m) == "hip");
      // HIP has initialised the runtime already; hsa_init only takes a reference on it
      if (want_sdma && ring_.pinned() && hsa_init() == HSA_STATUS_SUCCESS && agent_of(ring_.ptr(0), &host_agent_)) {
        for (size_t i = 0; i < ring_.nslots(); ++i) {
          hsa_signal_t sg{0};
          if (hsa_signal_create(0, 0, nullptr, &sg) != HSA_STATUS_SUCCESS) break;
          sig_.push_back(sg);
        }
        sdma_ = sig_.size() == ring_.nslots();
      }
    }
    for (int i = 0; i < nwriters; ++i) writers_.emplace_back([this] { writer_loop(); });
    enqueuer_ = std::thread([this] { enqueue_loop(); });
  }
  ~Engine() {
    {
      std::lock_guard<std::mutex> lk(qmu_);
      stop_ = true;
    }
    qcv_.notify_all();
    if (enqueuer_.joinable()) enqueuer_.join();
    {
      std::lock_guard<std::mutex> lk(wmu_);
      wstop_ = true;
    }
    wcv_.notify_all();
    jcv_.notify_all();
    for (auto& t : writers_) t.join();
    if (stream_ && own_stream_) hipStreamDestroy(stream_);
    for (auto& sg : sig_) hsa_signal_destroy(sg);
  }

  // The copy stream is a PyTorch pool stream the Python side reserves for the engine
  // (ops/streams.py side_stream(dev, "ckpt")); should another user ever capture a hipGraph on the
  // same handle, enqueueing here would join (or invalidate) that capture: fail the job loudly.
  void check_stream_free() const {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (stream_ && hipStreamIsCapturing(stream_, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone)
      throw std::runtime_error("checkpoint engine: its copy stream is being captured into a hipGraph");
  }
  // "sdma" (hsa_amd_memory_async_copy) or "hip" (hipMemcpyAsync on the copy stream)
  std::string d2h_mode() const { return sdma_ ? "sdma" : (stream_ ? "hip" : "host"); }

  int submit(std::vector<std::shared_ptr<FileJob>> files, hipEvent_t ready) {
    auto job = std::make_shared<SaveJob>();
    job->t_submit = now_s();
    job->files = std::move(files);
    job->files_left = (int)job->files.size();
    job->ready = ready;
    for (auto& f : job->files) {
      f->total = layout_archives(f->archives);
      for (auto& a : f->archives)
        for (auto& r : a.recs) job->bytes += rec_size(r);
    }
    {
      std::lock_guard<std::mutex> lk(jmu_);
      job->id = next_id_++;
      jobs_[job->id] = job;
    }
    if (job->files.empty()) {
      finish_job(job);
      return job->id;
    }
    {
      std::lock_guard<std::mutex> lk(qmu_);
      save_q_.push_back(job);
    }
    qcv_.notify_all();
    return job->id;
  }

  bool poll(int id) {
    std::lock_guard<std::mutex> lk(jmu_);
    auto it = jobs_.find(id);
    if (it == jobs_.end()) {
      if (results_.count(id)) return true;
      throw std::runtime_error("poll: unknown checkpoint job id " + std::to_string(id));
    }
    return it->second->done;
  }

  // returns (error, seconds from submit to durable).  A finished job's outcome is kept (the
  // job itself - its staged buffers - is released), so a second waiter on the same id gets the
  // same answer - in particular the same error - instead of "unknown id == success".
  std::pair<std::string, double> wait(int id) {
    JobResult r = wait_result(id);
    return {r.error, r.durable_s};
  }

  // seconds from submit until the last device piece had landed in the pinned ring (the end of
  // the D2H traffic that overlaps training) and until durable; valid after wait()
  std::pair<double, double> timings(int id) {
    JobResult r = wait_result(id);
    return {r.d2h_s, r.durable_s};
  }

  JobResult wait_result(int id) {
    std::unique_lock<std::mutex> lk(jmu_);
    auto it = jobs_.find(id);
    if (it == jobs_.end()) {
      auto r = results_.find(id);
      if (r != results_.end()) return r->second;
      throw std::runtime_error("wait: unknown checkpoint job id " + std::to_string(id));
    }
    std::shared_ptr<SaveJob> job = it->second;
    jcv_.wait(lk, [&] { return job->done; });
    const double d2h = job->t_d2h.load();
    JobResult res{job->error, job->t_done - job->t_submit, d2h > 0 ? d2h - job->t_submit : 0.0};
    if (jobs_.erase(id)) {
      results_[id] = res;
      result_order_.push_back(id);
      while (result_order_.size() > 4096) {  // bounded history of finished jobs
        results_.erase(result_order_.front());
        result_order_.pop_front();
      }
    }
    return res;
  }

  size_t slot_bytes() const { return ring_.slot_bytes(); }
  bool pinned() const { return ring_.pinned(); }

  // Restore path: stream file ranges to device memory through the same pinned ring.
  // Ranges are split into slot-sized pieces; `nthreads` readers each take a piece, pread it
  // into a free pinned slot, enqueue the H2D copy on the engine's copy stream and release
  // the slot once that copy has landed - so the pread of one piece overlaps the DMA of the
  // others and host memory stays bounded by the ring.  Blocks until every byte is on the
  // device (the caller must not be using the destinations on another stream).
  void read_to_device(const std::string& path, const std::vector<uint64_t>& offs,
                      const std::vector<uint64_t>& lens, const std::vector<uintptr_t>& dsts, int nthreads) {
    if (!stream_) throw std::runtime_error("read_to_device: no GPU");
    if (offs.size() != lens.size() || offs.size() != dsts.size())
      throw std::runtime_error("read_to_device: offs/lens/dsts length mismatch");
    int fd = ::open(path.c_str(), O_RDONLY);
    if (fd < 0) throw std::runtime_error("open failed: " + path + ": " + strerror(errno));
    // page-aligned pieces are read with O_DIRECT straight into the (page-aligned) pinned slot
    int dfd = direct_io_ ? ::open(path.c_str(), O_RDONLY | O_DIRECT) : -1;
    struct stat stt;
    const uint64_t fsize = ::fstat(fd, &stt) == 0 ? (uint64_t)stt.st_size : 0;
    struct P { uint64_t off, len; char* dst; };
    std::vector<P> pieces;
    const uint64_t S = ring_.slot_bytes();
    for (size_t i = 0; i < offs.size(); ++i)
      for (uint64_t o = 0; o < lens[i]; o += S)
        pieces.push_back({offs[i] + o, std::min(S, lens[i] - o), (char*)dsts[i] + o});
    std::atomic<size_t> next{0};
    std::string err;
    std::mutex emu, cmu;
    auto work = [&] {
      hipSetDevice(device_);
      while (true) {
        const size_t k = next++;
        if (k >= pieces.size()) return;
        {
          std::lock_guard<std::mutex> lk(emu);
          if (!err.empty()) return;
        }
        const int s = ring_.acquire();
        try {
          const P& pc = pieces[k];
          const uint64_t rl = (pc.len + kPage - 1) / kPage * kPage;  // round up: O_DIRECT length
          bool done = false;
          if (dfd >= 0 && pc.off % kPage == 0 && rl <= S && pc.off + pc.len <= fsize) {
            ssize_t r = ::pread(dfd, ring_.ptr(s), rl, (off_t)pc.off);
            if (r >= (ssize_t)pc.len) done = true;  // may stop short of rl at end of file
          }
          if (!done) pread_all(fd, ring_.ptr(s), pieces[k].len, pieces[k].off);
          hipError_t e;
          {
            std::lock_guard<std::mutex> lk(cmu);
            e = hipMemcpyAsync(pieces[k].dst, ring_.ptr(s), pieces[k].len, hipMemcpyHostToDevice, stream_);
            if (e == hipSuccess) e = hipEventRecord(ring_.event(s), stream_);
          }
          if (e == hipSuccess) e = hipEventSynchronize(ring_.event(s));
          if (e != hipSuccess) throw std::runtime_error(std::string("restore H2D: ") + hipGetErrorString(e));
        } catch (std::exception& ex) {
          std::lock_guard<std::mutex> lk(emu);
          err = ex.what();
        }
        ring_.release(s);
      }
    };
    std::vector<std::thread> ts;
    const int nt = std::max(1, std::min<int>(std::min<int>(nthreads, (int)ring_.nslots()), (int)pieces.size()));
    for (int i = 0; i < nt; ++i) ts.emplace_back(work);
    for (auto& t : ts) t.join();
    ::close(fd);
    if (dfd >= 0) ::close(dfd);
    if (err.empty() && hipStreamSynchronize(stream_) != hipSuccess) err = "restore: copy stream failed";
    if (!err.empty()) throw std::runtime_error(err);
  }

 private:
  struct WJob {
    std::shared_ptr<SaveJob> job;
    std::shared_ptr<FileJob> file;
    long long key = -1;
    int piece = -1;
    int slot = -1;
    const void* host = nullptr;  // direct host source (no slot)
    uint64_t len = 0, off = 0;
    bool wait_event = false;   // copy-stream D2H: ring slot event
    bool wait_signal = false;  // SDMA D2H: ring slot HSA signal
    bool final_marker = false;
  };

  void enqueue_loop() {
    while (true) {
      std::shared_ptr<SaveJob> job;
      {
        std::unique_lock<std::mutex> lk(qmu_);
        qcv_.wait(lk, [&] { return stop_ || !save_q_.empty(); });
        if (stop_ && save_q_.empty()) return;
        job = save_q_.front();
        save_q_.pop_front();
      }
      try {
        run_job(job);
      } catch (std::exception& e) {
        job->error = e.what();
        finish_job(job);
      }
    }
  }

  void run_job(std::shared_ptr<SaveJob> job) {
    if (g_have_gpu()) hipSetDevice(device_);
    const size_t S = ring_.slot_bytes();
    int dev_pieces = 0;
    const char* first_dev = nullptr;
    for (auto& f : job->files)
      for (auto& a : f->archives)
        for (auto& r : a.recs)
          if (r.src && r.on_device) {
            dev_pieces += (int)((r.nbytes + S - 1) / S);
            if (!first_dev) first_dev = r.src;
          }
    job->dev_left = dev_pieces;
    if (dev_pieces == 0) job->t_d2h = now_s();
    // SDMA needs the source's GPU agent (a caching-allocator block is an ordinary HSA
    // allocation); anything else falls back to the copy stream for this job
    hsa_agent_t gpu_agent{0};
    bool sdma = sdma_ && first_dev && agent_of(first_dev, &gpu_agent);
    if (sdma && gpu_agent.handle != access_agent_) {
      // once per GPU agent: every ring slot reachable by its SDMA engines, else this engine
      // falls back to the copy stream for good
      for (size_t i = 0; i < ring_.nslots() && sdma; ++i) sdma = ensure_access(ring_.ptr((int)i), gpu_agent);
      if (sdma) access_agent_ = gpu_agent.handle;
      else sdma_ = false;
    }
    if (job->ready) {
      if (sdma) {
        hipError_t e = wait_event_sleepy(job->ready);
        if (e != hipSuccess) throw std::runtime_error(std::string("snapshot event: ") + hipGetErrorString(e));
      } else if (stream_) {
        check_stream_free();
        hipStreamWaitEvent(stream_, job->ready, 0);
      }
    }
    for (auto& f : job->files) {
      f->fd = ::open(f->path.c_str(), O_CREAT | O_TRUNC | O_WRONLY, 0644);
      if (f->fd < 0) throw std::runtime_error("open failed: " + f->path + ": " + strerror(errno));
      if (direct_io_) f->dfd = ::open(f->path.c_str(), O_WRONLY | O_DIRECT);
      int pieces = 1;  // the headers / small records / central directories (finalize)
      for (auto& a : f->archives)
        for (auto& r : a.recs)
          if (r.src) pieces += (int)((r.nbytes + S - 1) / S);
      f->pending = pieces;
      for (size_t ai = 0; ai < f->archives.size(); ++ai) {
        auto& a = f->archives[ai];
        for (size_t ri = 0; ri < a.recs.size(); ++ri) {
          auto& r = a.recs[ri];
          if (!r.src) continue;
          const int np = (int)((r.nbytes + S - 1) / S);
          {
            std::lock_guard<std::mutex> lk(f->mu);
            f->piece_crc[rkey(ai, ri)].assign(np, {0u, 0ull});
          }
          for (int p = 0; p < np; ++p) {
            const uint64_t o = (uint64_t)p * S;
            const uint64_t len = std::min<uint64_t>(S, r.nbytes - o);
            WJob w;
            w.job = job;
            w.file = f;
            w.key = rkey(ai, ri);
            w.piece = p;
            w.len = len;
            w.off = a.base + r.data_off + o;
            if (r.on_device) {
              const int s = ring_.acquire();
              if (sdma) {
                hsa_signal_store_screlease(sig_[s], 1);
                hsa_status_t st = hsa_amd_memory_async_copy(ring_.ptr(s), host_agent_, r.src + o, gpu_agent, len, 0,
                                                            nullptr, sig_[s]);
                if (st == HSA_STATUS_SUCCESS) {
                  w.wait_signal = true;
                } else {
                  // the runtime refused the DMA: this piece and the rest of the job (and every
                  // later one) go through the copy stream, ordered after the snapshot event
                  sdma = false;
                  sdma_ = false;
                  hsa_signal_store_screlease(sig_[s], 0);
                  if (stream_ && job->ready) hipStreamWaitEvent(stream_, job->ready, 0);
                }
              }
              if (!w.wait_signal) {
                check_stream_free();
                hipError_t e = hipMemcpyAsync(ring_.ptr(s), r.src + o, len, hipMemcpyDeviceToHost, stream_);
                if (e != hipSuccess) {
                  ring_.release(s);
                  throw std::runtime_error(std::string("hipMemcpyAsync: ") + hipGetErrorString(e));
                }
                hipEventRecord(ring_.event(s), stream_);
                w.wait_event = true;
              }
              w.slot = s;
            } else {
              w.host = r.src + o;
            }
            push_write(std::move(w));
          }
        }
      }
      WJob fin;
      fin.job = job;
      fin.file = f;
      fin.final_marker = true;
      push_write(std::move(fin));
    }
  }

  void push_write(WJob&& w) {
    {
      std::lock_guard<std::mutex> lk(wmu_);
      wq_.push_back(std::move(w));
    }
    wcv_.notify_one();
  }

  void writer_loop() {
    if (g_have_gpu()) hipSetDevice(device_);
    // background priority: CRC32 + pwrite must not take CPU time from the rank's training
    // thread (or a gloo all-reduce) while an async checkpoint drains (Linux: per-thread nice)
    setpriority(PRIO_PROCESS, (id_t)syscall(SYS_gettid), 10);
    while (true) {
      WJob w;
      {
        std::unique_lock<std::mutex> lk(wmu_);
        wcv_.wait(lk, [&] { return wstop_ || !wq_.empty(); });
        if (wq_.empty()) {
          if (wstop_) return;
          continue;
        }
        // a file's finalizer runs only after all its data pieces are written
        auto it = wq_.begin();
        for (; it != wq_.end(); ++it) {
          if (!it->final_marker || it->file->pending.load() == 1) break;
        }
        if (it == wq_.end()) {
          lk.unlock();
          std::this_thread::sleep_for(std::chrono::microseconds(200));
          continue;
        }
        w = std::move(*it);
        wq_.erase(it);
      }
      auto& f = *w.file;
      try {
        if (w.final_marker) {
          finalize_file(f);
        } else {
          const void* src = w.host;
          if (w.slot >= 0) {
            if (w.wait_event) {
              hipError_t e = hipEventSynchronize(ring_.event(w.slot));
              if (e != hipSuccess) throw std::runtime_error(std::string("D2H: ") + hipGetErrorString(e));
            }
            if (w.wait_signal) {
              // blocked wait: the writer sleeps on the signal's interrupt, no spinning core
              const hsa_signal_value_t v = hsa_signal_wait_scacquire(sig_[w.slot], HSA_SIGNAL_CONDITION_LT, 1,
                                                                     UINT64_MAX, HSA_WAIT_STATE_BLOCKED);
              if (v < 0) throw std::runtime_error("SDMA D2H copy failed");
            }
            if ((w.wait_event || w.wait_signal) && w.job->dev_left.fetch_sub(1) == 1) w.job->t_d2h = now_s();
            src = ring_.ptr(w.slot);
          }
          uint32_t c = 0;
          if (f.crc_on) c = rtdc::crc::crc32_fast(0u, src, w.len);  // PCLMUL folding: ~5 GB/s per writer from DRAM
          write_piece(f, src, w.len, w.off);
          if (w.slot >= 0) ring_.release(w.slot);
          w.slot = -1;
          std::lock_guard<std::mutex> lk(f.mu);
          f.piece_crc[w.key][w.piece] = {c, w.len};
        }
      } catch (std::exception& e) {
        if (w.slot >= 0) ring_.release(w.slot);
        std::lock_guard<std::mutex> lk(f.mu);
        f.error = e.what();
      }
      const int left = --f.pending;
      if (left == 0) {
        if (w.job->files_left.fetch_sub(1) == 1) finish_job(w.job);
      }
    }
  }

  // Page-aligned runs of a piece go through the O_DIRECT descriptor (pinned slot -> device,
  // no page-cache copy); an unaligned remainder (a record's last bytes) through the buffered
  // one.  The two never touch the same 4 KiB page, and fsync on the file covers both.
  static void write_piece(FileJob& f, const void* src, uint64_t len, uint64_t off) {
    const char* p = (const char*)src;
    if (f.dfd >= 0 && off % kPage == 0 && ((uintptr_t)p % kPage) == 0) {
      const uint64_t a = len / kPage * kPage;
      if (a > 0) {
        ssize_t w = ::pwrite(f.dfd, p, a, (off_t)off);
        if (w == (ssize_t)a) {
          p += a;
          off += a;
          len -= a;
        } else if (w < 0 && errno == EINVAL) {  // filesystem refuses: stay buffered from here
          ::close(f.dfd);
          f.dfd = -1;
        } else if (w < 0) {
          throw std::runtime_error(std::string("pwrite(O_DIRECT) failed: ") + strerror(errno));
        } else {  // short direct write: finish buffered
          p += w;
          off += (uint64_t)w;
          len -= (uint64_t)w;
        }
      }
    }
    if (len) pwrite_all(f.fd, p, len, off);
  }

  void finalize_file(FileJob& f) {
    if (!f.error.empty()) throw std::runtime_error(f.error);
    for (size_t ai = 0; ai < f.archives.size(); ++ai) {
      auto& a = f.archives[ai];
      for (size_t ri = 0; ri < a.recs.size(); ++ri) {
        auto& r = a.recs[ri];
        if (r.src) {
          uint32_t c = 0;
          if (f.crc_on) {
            auto& pcs = f.piece_crc[rkey(ai, ri)];
            bool first = true;
            for (auto& pc : pcs) {
              c = first ? pc.first : (uint32_t)crc32_combine(c, pc.first, (z_off_t)pc.second);
              first = false;
            }
          }
          r.crc = c;
        } else {
          r.crc = f.crc_on ? rtdc::crc::crc32_fast(0u, r.inline_data.data(), r.inline_data.size()) : 0;
        }
      }
      for (auto& r : a.recs) {
        if (!a.raw) {
          std::string h = local_header(r, rec_size(r));
          pwrite_all(f.fd, h.data(), h.size(), a.base + r.header_off);
        }
        if (!r.src && !r.inline_data.empty())
          pwrite_all(f.fd, r.inline_data.data(), r.inline_data.size(), a.base + r.data_off);
      }
      if (!a.raw) {
        std::string cd = central_dir(a.recs, a.data_end);
        pwrite_all(f.fd, cd.data(), cd.size(), a.base + a.data_end);
      }
    }
    if (f.fsync_on) ::fsync(f.fd);
    if (f.dfd >= 0) {
      ::close(f.dfd);
      f.dfd = -1;
    }
    ::close(f.fd);
    f.fd = -1;
  }

  void finish_job(std::shared_ptr<SaveJob> job) {
    for (auto& f : job->files) {
      if (!f->error.empty() && job->error.empty()) job->error = f->error;
      if (f->fd >= 0) {
        ::close(f->fd);
        f->fd = -1;
      }
      if (f->dfd >= 0) {
        ::close(f->dfd);
        f->dfd = -1;
      }
    }
    {
      std::lock_guard<std::mutex> lk(jmu_);
      job->t_done = now_s();
      job->done = true;
    }
    jcv_.notify_all();
  }

  PinnedRing ring_;
  int device_;
  bool direct_io_;
  hipStream_t stream_ = nullptr;
  bool own_stream_ = false;
  std::vector<std::thread> writers_;
  std::thread enqueuer_;
  std::mutex qmu_, wmu_, jmu_;
  std::condition_variable qcv_, wcv_, jcv_;
  std::deque<std::shared_ptr<SaveJob>> save_q_;
  std::deque<WJob> wq_;
  std::map<int, std::shared_ptr<SaveJob>> jobs_;
  std::map<int, JobResult> results_;  // outcomes of waited (finished) jobs
  bool sdma_ = false;
  uint64_t access_agent_ = 0;  // GPU agent the ring slots were made accessible to
  hsa_agent_t host_agent_{0};
  std::vector<hsa_signal_t> sig_;  // per ring slot: SDMA completion
  std::deque<int> result_order_;
  int next_id_ = 1;
  std::atomic<bool> stop_{false};
  bool wstop_ = false;
};

// Parallel pread of many (offset, len, dst) ranges of one file.
static void read_ranges(const std::string& path, const std::vector<uint64_t>& offs,
                        const std::vector<uint64_t>& lens, const std::vector<uintptr_t>& dsts, int nthreads) {
  int fd = ::open(path.c_str(), O_RDONLY);
  if (fd < 0) throw std::runtime_error("open failed: " + path);
  // split big ranges into 64 MiB pieces so threads share them
  struct P { uint64_t off, len; char* dst; };
  std::vector<P> pieces;
  const uint64_t PS = 64ull << 20;
  for (size_t i = 0; i < offs.size(); ++i)
    for (uint64_t o = 0; o < lens[i]; o += PS)
      pieces.push_back({offs[i] + o, std::min(PS, lens[i] - o), (char*)dsts[i] + o});
  std::atomic<size_t> next{0};
  std::string err;
  std::mutex emu;
  auto work = [&] {
    while (true) {
      size_t k = next++;
      if (k >= pieces.size()) return;
      try {
        pread_all(fd, pieces[k].dst, pieces[k].len, pieces[k].off);
      } catch (std::exception& e) {
        std::lock_guard<std::mutex> lk(emu);
        err = e.what();
      }
    }
  };
  std::vector<std::thread> ts;
  int nt = std::max(1, std::min<int>(nthreads, (int)pieces.size()));
  for (int i = 0; i < nt; ++i) ts.emplace_back(work);
  for (auto& t : ts) t.join();
  ::close(fd);
  if (!err.empty()) throw std::runtime_error(err);
}

// (absolute data offset, size) of the tensor record '<prefix>/data/0' of the zip archive that
// occupies [base, base + length) of an open file: EOCD (ZIP64 locator / record when present) ->
// central directory -> the record's local header.  The native form of dcp._zip_data_record, for
// all of a file's items at once (a GPT-2 train state restores ~600 records; per-item Python
// seeks + reads were a visible slice of a 0.1 s restore, and cold each is a disk round trip).
static uint16_t rd16(const char* p) { return (uint16_t)((uint8_t)p[0] | ((uint8_t)p[1] << 8)); }
static uint32_t rd32(const char* p) { return (uint32_t)rd16(p) | ((uint32_t)rd16(p + 2) << 16); }
static uint64_t rd64(const char* p) { return (uint64_t)rd32(p) | ((uint64_t)rd32(p + 4) << 32); }

static std::pair<uint64_t, uint64_t> zip_data_record(int fd, uint64_t base, uint64_t length) {
  const std::string sig_eocd("PK\x05\x06", 4);
  std::string tail;
  size_t eocd = std::string::npos;
  for (uint64_t tl : {std::min<uint64_t>(length, 2048), std::min<uint64_t>(length, 1u << 16)}) {
    tail.resize(tl);
    pread_all(fd, &tail[0], tl, base + length - tl);
    eocd = tail.rfind(sig_eocd);
    if (eocd != std::string::npos && eocd + 22 <= tail.size()) {
      const uint64_t n = rd16(&tail[eocd + 10]), cs = rd32(&tail[eocd + 12]), co = rd32(&tail[eocd + 16]);
      const bool z64 = n == 0xFFFF || cs == kZ32 || co == kZ32;
      if (z64 || co >= length - tl) break;
    }
  }
  if (eocd == std::string::npos || eocd + 22 > tail.size()) throw std::runtime_error("no zip end record");
  uint64_t n = rd16(&tail[eocd + 10]), cd_size = rd32(&tail[eocd + 12]), cd_off = rd32(&tail[eocd + 16]);
  if (n == 0xFFFF || cd_size == kZ32 || cd_off == kZ32) {
    if (eocd < 20 || tail.compare(eocd - 20, 4, std::string("PK\x06\x07", 4)) != 0)
      throw std::runtime_error("zip64 locator missing");
    const uint64_t z64_off = rd64(&tail[eocd - 20 + 8]);
    char rec[56];
    pread_all(fd, rec, 56, base + z64_off);
    if (std::string(rec, 4) != std::string("PK\x06\x06", 4)) throw std::runtime_error("bad zip64 end record");
    n = rd64(rec + 24);
    cd_size = rd64(rec + 40);
    cd_off = rd64(rec + 48);
  }
  std::string cd;
  const uint64_t tail_at = length - tail.size();
  if (cd_off >= tail_at && cd_off - tail_at + cd_size <= tail.size()) {
    cd = tail.substr(cd_off - tail_at, cd_size);
  } else {
    cd.resize(cd_size);
    pread_all(fd, &cd[0], cd_size, base + cd_off);
  }
  size_t pos = 0;
  for (uint64_t i = 0; i < n; ++i) {
    if (pos + 46 > cd.size() || rd32(&cd[pos]) != 0x02014B50u) throw std::runtime_error("corrupt central directory");
    uint64_t csize = rd32(&cd[pos + 20]), usize = rd32(&cd[pos + 24]);
    const size_t nlen = rd16(&cd[pos + 28]), elen = rd16(&cd[pos + 30]), clen = rd16(&cd[pos + 32]);
    uint64_t lho = rd32(&cd[pos + 42]);
    if (pos + 46 + nlen + elen > cd.size()) throw std::runtime_error("corrupt central directory");
    const std::string name = cd.substr(pos + 46, nlen);
    static const std::string suffix = "/data/0";
    if (name.size() >= suffix.size() && name.compare(name.size() - suffix.size(), suffix.size(), suffix) == 0) {
      if (csize == kZ32 || usize == kZ32 || lho == kZ32) {
        size_t e = 0;
        const char* ex = &cd[pos + 46 + nlen];
        while (e + 4 <= elen) {
          const uint16_t tag = rd16(ex + e), sz = rd16(ex + e + 2);
          if (e + 4 + sz > elen) throw std::runtime_error("corrupt zip64 extra field");
          if (tag == 1) {
            size_t v = e + 4;
            const size_t end = e + 4 + sz;
            auto next64 = [&](uint64_t& x) {
              if (v + 8 > end) throw std::runtime_error("short zip64 extra field");
              x = rd64(ex + v);
              v += 8;
            };
            if (usize == kZ32) next64(usize);
            if (csize == kZ32) next64(csize);
            if (lho == kZ32) next64(lho);
            break;
          }
          e += 4 + sz;
        }
      }
      char lh[30];
      pread_all(fd, lh, 30, base + lho);
      return {base + lho + 30 + rd16(lh + 26) + rd16(lh + 28), csize};
    }
    pos += 46 + nlen + elen + clen;
  }
  throw std::runtime_error("no tensor data record");
}

static std::vector<std::pair<uint64_t, uint64_t>> zip_data_records(const std::string& path,
                                                                   const std::vector<uint64_t>& bases,
                                                                   const std::vector<uint64_t>& lens, int nthreads) {
  int fd = ::open(path.c_str(), O_RDONLY);
  if (fd < 0) throw std::runtime_error("open failed: " + path);
  std::vector<std::pair<uint64_t, uint64_t>> out(bases.size());
  std::atomic<size_t> next{0};
  std::string err;
  std::mutex emu;
  auto work = [&] {
    while (true) {
      const size_t k = next++;
      if (k >= bases.size()) return;
      try {
        out[k] = zip_data_record(fd, bases[k], lens[k]);
      } catch (std::exception& e) {
        std::lock_guard<std::mutex> lk(emu);
        err = path + "@" + std::to_string(bases[k]) + ": " + e.what();
      }
    }
  };
  // a cold page cache makes every header a device round trip: overlap them
  const int nt = std::max(1, std::min<int>(nthreads, (int)(bases.size() / 32)));
  std::vector<std::thread> ts;
  for (int i = 1; i < nt; ++i) ts.emplace_back(work);
  work();
  for (auto& t : ts) t.join();
  ::close(fd);
  if (!err.empty()) throw std::runtime_error(err);
  return out;
}

}  // namespace rtdc_ckpt

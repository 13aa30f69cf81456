"""`torch.save`-compatible writer on the native checkpoint engine.

The reference persists `latest_model.pt` / `best_model.pt` with blocking `torch.save`
(R/my_ray_module.py:179-201), which copies every GPU storage to the host synchronously
(torch/serialization.py:1264-1286) and builds the zip in one thread.  Here the pickle of the
object graph (tensors replaced by persistent storage ids exactly like torch's, so
`torch.load(weights_only=True)` accepts it) is produced in Python, and the tensor bytes go
device -> pinned ring -> file through the C++ engine (csrc/runtime/ckpt_engine.cpp) with
optional HBM snapshot so the call can return before the write is durable.

Format produced (identical record set and order to PyTorchStreamWriter):
  archive/data.pkl, archive/.format_version, archive/.storage_alignment, archive/byteorder,
  archive/data/<k>..., archive/version, archive/.data/serialization_id
"""
from __future__ import annotations

import collections
import io
import os
import pickle
import threading
import time

import torch

from ..ops import _ext

_STORAGE_NAME = {
    torch.float64: "DoubleStorage", torch.float32: "FloatStorage", torch.float16: "HalfStorage",
    torch.int64: "LongStorage", torch.int32: "IntStorage", torch.int16: "ShortStorage", torch.int8: "CharStorage",
    torch.uint8: "ByteStorage", torch.bool: "BoolStorage", torch.bfloat16: "BFloat16Storage",
    torch.complex64: "ComplexFloatStorage", torch.complex128: "ComplexDoubleStorage",
}


class _StorageRef:
    __slots__ = ("dtype", "key", "numel")

    def __init__(self, dtype, key, numel):
        self.dtype, self.key, self.numel = dtype, key, numel


def _contig_stride(shape):
    st, acc = [], 1
    for s in reversed(shape):
        st.append(acc)
        acc *= max(int(s), 1)
    return tuple(reversed(st))


class _Pickler(pickle.Pickler):
    def __init__(self, f, tensors: list):
        super().__init__(f, protocol=2)
        self.tensors = tensors

    def persistent_id(self, obj):
        if isinstance(obj, _StorageRef):
            return ("storage", getattr(torch, _STORAGE_NAME[obj.dtype]), obj.key, "cpu", obj.numel)
        return None

    def reducer_override(self, obj):
        if isinstance(obj, torch.Tensor):
            if obj.dtype not in _STORAGE_NAME:
                raise TypeError(f"unsupported dtype for checkpoint: {obj.dtype}")
            key = str(len(self.tensors))
            self.tensors.append(obj)
            ref = _StorageRef(obj.dtype, key, obj.numel())
            return (torch._utils._rebuild_tensor_v2,
                    (ref, 0, tuple(obj.shape), _contig_stride(obj.shape), False, collections.OrderedDict()))
        return NotImplemented


def pickle_state(obj) -> tuple[bytes, list]:
    """(data.pkl bytes, tensors in storage-key order)."""
    buf = io.BytesIO()
    tensors: list = []
    _Pickler(buf, tensors).dump(obj)
    return buf.getvalue(), tensors


def build_records(pkl: bytes, storages: list, prefix: str = "archive"):
    """Engine record tuples for one torch.save archive.

    storages: list of (ptr, nbytes, on_device) in storage-key order.
    """
    sid = str(int.from_bytes(os.urandom(16), "little")).zfill(40)[:40]
    recs = [(f"{prefix}/data.pkl", pkl, 0, 0, False),
            (f"{prefix}/.format_version", b"1", 0, 0, False),
            (f"{prefix}/.storage_alignment", b"64", 0, 0, False),
            (f"{prefix}/byteorder", b"little", 0, 0, False)]
    for k, (ptr, nbytes, on_dev) in enumerate(storages):
        if nbytes == 0:
            recs.append((f"{prefix}/data/{k}", b"", 0, 0, False))
        else:
            recs.append((f"{prefix}/data/{k}", None, int(ptr), int(nbytes), bool(on_dev)))
    recs.append((f"{prefix}/version", b"3\n", 0, 0, False))
    recs.append((f"{prefix}/.data/serialization_id", sid.encode(), 0, 0, False))
    return recs


# ------------------------------------------------------------------------------ engine
_engine = None
_engine_lock = threading.Lock()


_engine_cfg: tuple | None = None


def default_writer_threads() -> int:
    """Writer threads of this rank from a per-NODE budget: half the CPUs this job may use
    (cgroup quota / affinity, utils/hostinfo.py; CRC32 + pwrite are CPU work) split over the
    node's ranks (LOCAL_WORLD_SIZE), 2..8 per rank; the threads run at background priority.  A per-rank
    default of min(8, ncpu/2) gave 8 ranks x 8 writers on one host, which starved the ranks'
    training threads during an async save."""
    from ..utils.hostinfo import available_cpus

    local = max(1, int(os.environ.get("LOCAL_WORLD_SIZE", "1") or 1))
    return max(2, min(8, available_cpus() // (2 * local)))


def configure_engine(nslots: int, slot_mb: int, writers: int = 0) -> None:
    """Size the process-wide engine (CheckpointConfig.pinned_ring_mb / ring_slot_mb /
    writer_threads); must run before the first checkpoint I/O of the process.  The
    RTDC_CKPT_SLOTS / RTDC_CKPT_SLOT_MB / RTDC_CKPT_WRITERS environment variables still
    override the individual fields (engine_config)."""
    global _engine_cfg
    if _engine is not None:
        return
    _engine_cfg = (int(nslots), int(slot_mb) << 20, int(writers or default_writer_threads()))


def engine_config():
    """(slots, slot bytes, writer threads): typed config (configure_engine) or defaults, each
    field overridable by its environment variable."""
    nslots, slot_bytes, writers = _engine_cfg or (8, 64 << 20, default_writer_threads())
    if os.environ.get("RTDC_CKPT_SLOTS"):
        nslots = int(os.environ["RTDC_CKPT_SLOTS"])
    if os.environ.get("RTDC_CKPT_SLOT_MB"):
        slot_bytes = int(os.environ["RTDC_CKPT_SLOT_MB"]) << 20
    if os.environ.get("RTDC_CKPT_WRITERS"):
        writers = int(os.environ["RTDC_CKPT_WRITERS"])
    return nslots, slot_bytes, writers


def get_engine():
    """Process-wide native checkpoint engine (bounded pinned ring: RTDC_CKPT_SLOTS x RTDC_CKPT_SLOT_MB)."""
    global _engine
    if _engine is None:
        with _engine_lock:
            if _engine is None:
                nslots, slot_bytes, writers = engine_config()
                dev = torch.cuda.current_device() if torch.cuda.is_available() else 0
                # the copy stream comes from PyTorch's pool (a private stream would add a
                # hardware queue to the process, see the Engine constructor), reserved for the
                # engine: the Stream object lives in ops/streams.py for the process lifetime and
                # every framework stream user draws its own pool entry there
                stream = 0
                if torch.cuda.is_available():
                    from ..ops.streams import side_stream

                    stream = side_stream(dev, "ckpt").cuda_stream
                _engine = _ext.ext().CkptEngine(nslots, slot_bytes, writers, dev, stream=stream)
    return _engine


class SaveHandle:
    """A submitted (possibly still running) native save.  `wait()` -> seconds to durable."""

    def __init__(self, job_id: int, keepalive, t0: float, nbytes: int, error_words=None):
        self.job_id, self._keep, self.t0, self.nbytes = job_id, keepalive, t0, nbytes
        # communicator error words captured right after the snapshot (parallel/health.py):
        # commit-or-refuse is decided from them, not from the live sticky word
        self._words = error_words
        self._result = None
        self._error: str | None = None
        self._lock = threading.Lock()  # waited on by the training thread AND the committer thread

    def d2h_seconds(self) -> float | None:
        """After wait(): seconds from submit until the last device piece was in the pinned
        ring (the end of the D2H traffic that overlaps training)."""
        try:
            return get_engine().timings(self.job_id)[0]
        except Exception:  # noqa: BLE001
            return None

    def done(self) -> bool:
        return self._result is not None or self._error is not None or get_engine().poll(self.job_id)

    def wait(self) -> float:
        """Seconds from submit to durable.  The outcome is cached: every waiter (any thread, any
        number of times) sees the same result, and a failed write raises for all of them."""
        with self._lock:
            if self._result is None and self._error is None:
                err, _secs = get_engine().wait(self.job_id)
                self._keep = None  # the snapshot (arena lease / clones) is drained: release it
                from ..parallel import health

                if not err and health.poisoned(self._words):
                    # a collective the snapshot depends on timed out (its NaN-poisoned state
                    # was staged): the write is never committed.  A timeout of a later step
                    # (after the snapshot) does not void this clean checkpoint
                    self._poisoned = True
                    err = "a P2P gradient all-reduce timed out before the snapshot (state poisoned)"
                if err:
                    self._error = str(err)
                else:
                    self._result = time.perf_counter() - self.t0
            if self._error is not None:
                if getattr(self, "_poisoned", False):
                    from ..parallel.health import CommPoisonedError

                    raise CommPoisonedError(f"refusing checkpoint commit: {self._error}")
                raise IOError(f"checkpoint write failed: {self._error}")
            return self._result


def snapshot_tensors(tensors: list, stream=None) -> list:
    """Detached, contiguous copies (device tensors stay on device: an HBM snapshot)."""
    out = []
    for t in tensors:
        t = t.detach()
        out.append(t.clone(memory_format=torch.contiguous_format))
    return out


def submit_files(files: list, keepalive, nbytes: int, ready_event=None, error_words=None) -> SaveHandle:
    """files: [(path, fsync, crc, [(raw, records), ...])] -> SaveHandle (non-blocking).
    error_words: parallel/health.py capture_error_words() taken at the snapshot."""
    t0 = time.perf_counter()
    ev = 0
    if ready_event is not None:
        ev = ready_event.cuda_event
    jid = get_engine().submit(files, ev)
    return SaveHandle(jid, (keepalive, ready_event), t0, nbytes, error_words)


def _storages_of(tensors):
    out = []
    for t in tensors:
        out.append((t.data_ptr(), t.numel() * t.element_size(), t.is_cuda))
    return out


def save(obj, path: str, *, async_: bool = False, fsync: bool = True, crc: bool = True,
         snapshot: bool | None = None) -> SaveHandle | None:
    """torch.save-compatible save through the native engine.

    async_=False: returns after the file is durable.  async_=True: takes an HBM/host snapshot
    (so the caller may keep mutating the tensors) and returns a SaveHandle immediately.
    Refuses (parallel/health.py CommPoisonedError) after a timed-out P2P gradient collective.
    """
    from ..parallel import health

    health.assert_healthy("checkpoint save", sync=False)  # decided again from the words captured at the snapshot
    pkl, tensors = pickle_state(obj)
    if snapshot is None:
        snapshot = async_
    lease = None
    if snapshot:
        from . import snapshot as _snap

        lease, contig = _snap.take(tensors)
    else:
        contig = [t.detach() if t.is_contiguous() else t.detach().clone(memory_format=torch.contiguous_format)
                  for t in tensors]
    words = health.capture_error_words()  # stream-ordered after the snapshot copies
    ready = None
    if any(t.is_cuda for t in contig):
        ready = torch.cuda.Event()
        ready.record()
    stor = _storages_of(contig)
    nbytes = sum(s[1] for s in stor)
    recs = build_records(pkl, stor, prefix=os.path.splitext(os.path.basename(path))[0] or "archive")
    h = submit_files([(path, fsync, crc, [(False, recs)])], [lease] + contig, nbytes, ready, words)
    if async_:
        return h
    h.wait()
    return None

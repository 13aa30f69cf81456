"""HBM snapshot of a checkpoint's tensors into persistent, reused arenas.

An async save copies the owned tensors on the compute stream, so the next optimizer step can
overwrite them while the engine drains the copy to disk (SURVEY §5.4 "snapshot").  Cloning
each tensor through the caching allocator (the round-1..4 path) carves ~1.5 GB (GPT-2-small
train state; ~12 GB for a Llama-3-8B rank shard) out of the blocks the training step itself
reuses, so the first steps after a save allocate fresh segments mid-step; and it costs one
copy launch per tensor (~450 for GPT-2 with AdamW state).

Here the snapshot goes into one device buffer per in-flight save, kept for the life of the
process and reused by the next save (288 GB of HBM holds it easily), and tensors that tile a
common storage - the flat parameter space and the fused optimizers' flat state buffers - are
copied as ONE span per storage: GPT-2's full train state is three D2D copies.  The snapshot
tensors are views into the arena at the same relative offsets, so the engine's records point
straight into it.

    lease, snaps = take([t0, t1, ...])      # snaps[i] is a contiguous copy of ts[i]
    ... keep `lease` alive until the engine has drained the snapshot, then drop it

RTDC_CKPT_ARENA=0 falls back to per-tensor clones (A/B switch).
"""
from __future__ import annotations

import os
import threading

import torch

_pool: dict = {}  # device -> list of free uint8 buffers
_lock = threading.Lock()
_ALIGN = 256


def enabled() -> bool:
    return os.environ.get("RTDC_CKPT_ARENA", "1") != "0"


class Lease:
    """Holds one arena buffer; returns it to the pool when dropped (after the drain)."""

    def __init__(self, buf: torch.Tensor | None):
        self.buf = buf

    def release(self) -> None:
        buf, self.buf = self.buf, None
        if buf is not None:
            with _lock:
                _pool.setdefault(buf.device, []).append(buf)

    def __del__(self):
        try:
            self.release()
        except Exception:  # interpreter shutdown
            pass


def _acquire(nbytes: int, device) -> torch.Tensor:
    with _lock:
        free = _pool.get(device, [])
        fit = [b for b in free if b.numel() >= nbytes]
        if fit:
            b = min(fit, key=lambda x: x.numel())
            free.remove(b)
            return b
        # a buffer too small for this save is dropped (the state grew): keep one per save size
        for b in list(free):
            free.remove(b)
    try:
        return torch.empty(nbytes, dtype=torch.uint8, device=device)
    except torch.cuda.OutOfMemoryError:
        # pooled arenas of other sizes (e.g. a larger plan of an earlier save) are what the
        # caching allocator cannot reclaim: drop every free one and retry once
        with _lock:
            _pool.clear()
        torch.cuda.empty_cache()
        return torch.empty(nbytes, dtype=torch.uint8, device=device)


def _bytes_view(t: torch.Tensor, lo: int, n: int) -> torch.Tensor:
    """uint8 view of bytes [lo, lo + n) of t's storage."""
    v = torch.empty(0, dtype=torch.uint8, device=t.device)
    return v.set_(t.untyped_storage(), lo, (n,))


def _plan(tensors: list):
    """Group contiguous device tensors by storage; a storage whose owned tensors cover most of
    the span between the first and last of them is copied as one span."""
    groups: dict = {}
    singles = []
    for i, t in enumerate(tensors):
        if t.is_cuda and t.is_contiguous() and t.numel() > 0:
            st = t.untyped_storage()
            groups.setdefault((st.data_ptr(), t.device), []).append(i)
        else:
            singles.append(i)
    spans = []
    for (_base, _dev), idx in groups.items():
        lo = min(tensors[i].storage_offset() * tensors[i].element_size() for i in idx)
        lo -= lo % 16  # arena offsets keep each view's alignment (a is 256-B aligned)
        hi = max((tensors[i].storage_offset() + tensors[i].numel()) * tensors[i].element_size() for i in idx)
        owned = sum(tensors[i].numel() * tensors[i].element_size() for i in idx)
        if len(idx) > 1 and hi - lo <= owned * 1.10 + (1 << 20):
            spans.append((idx, lo, hi))
        else:
            singles += idx
    return spans, sorted(singles)


def _layout(tensors: list):
    """(spans, singles, span arena offsets, single arena offsets, arena bytes): spans first,
    then single device tensors, each 256-B aligned."""
    spans, singles = _plan(tensors)
    off, place = 0, []
    for idx, lo, hi in spans:
        place.append(off)
        off += (hi - lo + _ALIGN - 1) // _ALIGN * _ALIGN
    single_off = {}
    for i in singles:
        t = tensors[i]
        if t.is_cuda:
            single_off[i] = off
            off += (t.numel() * t.element_size() + _ALIGN - 1) // _ALIGN * _ALIGN
    return spans, singles, place, single_off, max(off, _ALIGN)


def reserve(tensors: list) -> int:
    """Allocate (once) the arena a later `take(tensors)` needs, so the first checkpoint of a
    run does not allocate device memory between two training steps.  Returns its bytes."""
    tensors = [t.detach() for t in tensors]
    if not enabled() or not any(t.is_cuda for t in tensors):
        return 0
    *_, total = _layout(tensors)
    dev = next(t.device for t in tensors if t.is_cuda)
    Lease(_acquire(total, dev)).release()
    return total


def take(tensors: list) -> tuple[Lease | None, list]:
    """Snapshot `tensors` on the current stream.  Returns (lease, copies): device copies are
    views into one arena buffer (one copy per storage span), host tensors are cloned."""
    tensors = [t.detach() for t in tensors]
    if not enabled() or not any(t.is_cuda for t in tensors):
        return None, [t.clone(memory_format=torch.contiguous_format) for t in tensors]
    spans, singles, place, single_off, total = _layout(tensors)
    dev = next(t.device for t in tensors if t.is_cuda)
    buf = _acquire(total, dev)
    out: list = [None] * len(tensors)
    with torch.no_grad():
        for (idx, lo, hi), a in zip(spans, place):
            buf[a:a + hi - lo].copy_(_bytes_view(tensors[idx[0]], lo, hi - lo))
            for i in idx:
                t = tensors[i]
                b = a + t.storage_offset() * t.element_size() - lo
                out[i] = buf[b:b + t.numel() * t.element_size()].view(t.dtype).view(t.shape)
        for i in singles:
            t = tensors[i]
            if t.is_cuda:
                a = single_off[i]
                dst = buf[a:a + t.numel() * t.element_size()].view(t.dtype).view(t.shape)
                dst.copy_(t)
                out[i] = dst
            else:
                out[i] = t.clone(memory_format=torch.contiguous_format)
    return Lease(buf), out


def clear() -> None:
    """Free the pooled arenas (tests / memory pressure)."""
    with _lock:
        _pool.clear()

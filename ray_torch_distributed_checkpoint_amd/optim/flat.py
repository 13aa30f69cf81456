"""FlatParamSpace: one contiguous buffer per kind (params, grads, bf16 shadows, optimizer state).

The MI355X-first memory layout for data-parallel training: every parameter of a model is a
view into one flat fp32 buffer, every gradient a view into one flat fp32 buffer (the DDP
buckets are contiguous slices of it, so gradients are all-reduced in place - torch's
`gradient_as_bucket_view` without the copy-in/copy-out of reducer.hpp:329,499), and the
fused optimizers update the whole model in one launch over a chunk table.  Checkpoint
snapshots are a handful of large device-to-device copies instead of one copy per tensor.

Segments are 64-element aligned (16-B vector access for fp32/bf16) and laid out in the
order given (the DDP wrapper passes reverse registration order = approximate backward order).
"""
from __future__ import annotations

from dataclasses import dataclass

import torch

from ..ops.shadow import bind_shadow

ALIGN = 64
CHUNK = 16384  # elements per optimizer work item


@dataclass
class Segment:
    index: int
    offset: int
    numel: int
    shape: tuple
    channels_last: bool = False  # 4-D parameter stored [O][KH][KW][I] (conv weight = GEMM operand)


def _is_channels_last(p: torch.Tensor) -> bool:
    return p.dim() == 4 and not p.is_contiguous() and p.is_contiguous(memory_format=torch.channels_last)


class ZeroLayout:
    """ZeRO-1 ownership of a flat space (parallel/ddp.py `zero_stage=1`): every gradient bucket
    [start, end) - a multiple of 64 x world elements long - is split into `world` equal shards,
    rank r owns shard r of each.  The data-parallel engine reduce-scatters each bucket onto its
    owner, the fused optimizer updates owned elements only and keeps its state for them alone
    in COMPACT buffers (owned shards back to back: 1/world of the bytes), and `gather`
    all-gathers a flat buffer (parameters after every step) back to every rank.

    The layout is a pure function of (bucket plan, world), so every rank knows every other
    rank's shards: sharded checkpoints are planned without collectives (checkpoint/sharded.py).
    """

    def __init__(self, buckets, rank: int, world: int, group=None):
        self.buckets = [(int(a), int(b)) for a, b in buckets]
        self.rank, self.world, self.group = rank, world, group
        self.owned = self.owned_by(rank)
        # compact position of each owned range (the optimizer-state offset of its first element)
        self.compact_starts = []
        c = 0
        for oa, ob in self.owned:
            self.compact_starts.append(c)
            c += ob - oa
        self.compact_numel = c

    def owned_by(self, rank: int) -> list:
        out = []
        for a, b in self.buckets:
            n = b - a
            assert n % (64 * self.world) == 0, "ZeRO buckets must be multiples of 64 x world elements"
            sh = n // self.world
            out.append((a + rank * sh, a + (rank + 1) * sh))
        return out

    def compact_of(self, flat: int) -> int:
        """Compact (optimizer-state) offset of an owned flat offset."""
        import bisect

        i = bisect.bisect_right([oa for oa, _ in self.owned], flat) - 1
        oa, ob = self.owned[i]
        if not (oa <= flat < ob):
            raise ValueError(f"flat offset {flat} is not owned by rank {self.rank}")
        return self.compact_starts[i] + flat - oa

    def gather(self, buf: torch.Tensor) -> None:
        """Every bucket of `buf`: each rank's owned shard -> all ranks (in place)."""
        import torch.distributed as dist

        for (a, b), (oa, ob) in zip(self.buckets, self.owned):
            dist.all_gather_into_tensor(buf[a:b], buf[oa:ob], group=self.group)

    def gather_compact(self, compact: torch.Tensor, full: torch.Tensor) -> None:
        """All-gather a compact owned-shard buffer into a full flat buffer on every rank."""
        import torch.distributed as dist

        for (a, b), (oa, ob), c in zip(self.buckets, self.owned, self.compact_starts):
            dist.all_gather_into_tensor(full[a:b], compact[c:c + (ob - oa)], group=self.group)

    def owned_elements(self) -> int:
        return self.compact_numel


class FlatParamSpace:
    def __init__(self, params, device=None, shadow_dtype=torch.bfloat16, grads=True, align_after=None):
        params = list(params)
        assert params, "no parameters"
        seen = set()
        uniq = []
        for p in params:
            if id(p) not in seen:
                seen.add(id(p))
                uniq.append(p)
        self.params = uniq
        had_grad = any(p.grad is not None for p in uniq)
        self.device = torch.device(device) if device is not None else uniq[0].device
        self.segments: list[Segment] = []
        # "fresh" gradient mode (zero_grad(set_to_none=True)): p.grad is None until the first
        # contribution of the step, which the native backward writes straight into the flat
        # view (ops.gradbuf.grad_target); AccumulateGrad then adopts that view without a copy
        # or an add, and no memset of the buffer is needed.
        self.fresh = False
        self.step_id = 0
        off = 0
        align_after = align_after or {}
        for i, p in enumerate(uniq):
            assert p.dtype == torch.float32, "FlatParamSpace holds fp32 master parameters"
            # channels-last 4-D parameters (ResNet conv weights) keep that memory order in the
            # flat buffers: their bf16 shadow slice IS the [O, KH*KW*I] implicit-GEMM operand and
            # the weight-gradient GEMM writes its [O, KH*KW*I] output straight into the slice
            self.segments.append(Segment(i, off, p.numel(), tuple(p.shape), _is_channels_last(p)))
            off += (p.numel() + ALIGN - 1) // ALIGN * ALIGN
            a = align_after.get(i)
            if a:  # zero padding after this parameter (ZeRO bucket ends: multiples of 64 x world)
                off = (off + a - 1) // a * a
        self.numel = off
        self._seg_of = {id(p): s for p, s in zip(uniq, self.segments)}
        self.data = torch.zeros(off, dtype=torch.float32, device=self.device)
        with torch.no_grad():
            for p, s in zip(uniq, self.segments):
                self.view(self.data, s).copy_(p.detach())
                p.data = self.view(self.data, s)
                p._rtdc_space = self
        self.grad = None
        if grads:
            self.grad = torch.zeros(off, dtype=torch.float32, device=self.device)
            self.grad._rtdc_flat_grad = True  # (ops/gemm.py _deferrable: a gradient slot autograd adopts)
            if had_grad:
                for p, s in zip(uniq, self.segments):
                    p.grad = self.view(self.grad, s)
            else:
                # no gradient yet (a space built before the first backward: a restore's
                # init_state, a DDP wrap): start in the per-step mode zero_grad(set_to_none=True)
                # leaves, so the first backward takes the same kernels (grouped weight gradients
                # written into the slices) as every later one - a run restarted from a
                # checkpoint then reproduces the uninterrupted run's gradients bit for bit
                for p in uniq:
                    p.grad = None
                self.fresh = True
        self.shadow = None
        if shadow_dtype is not None and self.device.type == "cuda":
            self.shadow = torch.empty(off, dtype=shadow_dtype, device=self.device)
            self.refresh_shadows()
        self.grad_scale = 1.0
        # device address of a communicator error word (0: none); the fused optimizer kernels
        # skip their update when it is set (parallel/health.py)
        self.skip_ptr = 0
        self.zero: ZeroLayout | None = None
        self._offsets = None
        self._chunk_cache: dict = {}
        # [(flat offset, wait fn)] of gradient pieces whose all-reduce is still in flight
        # (DistributedDataParallel(defer_tail_to_optimizer=True)), ascending: everything below
        # the first offset is final, piece i spans [offset_i, offset_i+1) and is final after
        # its wait fn (which also waits for the pieces before it)
        self.pending_tail = None

    def wait_pending_tail(self) -> None:
        t = self.pending_tail
        if t is not None:
            self.pending_tail = None
            for _, wait in t:
                wait()

    @staticmethod
    def view(buf: torch.Tensor, s: Segment) -> torch.Tensor:
        flat = buf[s.offset:s.offset + s.numel]
        if s.channels_last:
            o, i, kh, kw = s.shape
            return flat.view(o, kh, kw, i).permute(0, 3, 1, 2)
        return flat.view(s.shape)

    def segment_of(self, p) -> Segment:
        s = self._seg_of.get(id(p))
        if s is None or self.params[s.index] is not p:
            raise KeyError("parameter not in this space")
        return s

    def grad_view(self, p) -> torch.Tensor:
        return self.view(self.grad, self.segment_of(p))

    def refresh_shadows(self):
        if self.shadow is None:
            return
        from ..ops._ext import gpu_ext

        gpu_ext().f32_to_bf16(self.data, self.shadow)
        for p, s in zip(self.params, self.segments):
            bind_shadow(p, self.view(self.shadow, s))

    def zero_grad(self, set_to_none: bool = False):
        if self.grad is None:
            return
        self.wait_pending_tail()
        if set_to_none:
            for p in self.params:
                p.grad = None
            self.fresh = True
            self.step_id += 1
            return
        self.fresh = False
        self.grad.zero_()
        for p, s in zip(self.params, self.segments):
            v = self.view(self.grad, s)
            if p.grad is None or p.grad.data_ptr() != v.data_ptr():
                p.grad = v

    def ensure_grad_views(self) -> list:
        """Fold gradients that autograd allocated outside the flat buffer back into it and
        return the parameters that have a gradient this step (the optimizers skip the rest,
        like torch).  One native pass over the parameters when the extension is loaded."""
        if self.grad is None:
            return [p for p in self.params if p.grad is not None]
        base = self.grad.data_ptr()
        st = self._grad_status(base)
        have = []
        for p, s, k in zip(self.params, self.segments, st):
            if k == 0:
                continue
            have.append(p)
            if k == 1:
                continue
            self.wait_pending_tail()  # never write into a slice a collective still owns
            v = self.view(self.grad, s)
            v.copy_(p.grad)
            p.grad = v
        return have

    def _grad_status(self, base: int):
        from ..ops import _ext

        if _ext.available():
            if self._offsets is None:
                self._offsets = [s.offset for s in self.segments]
            return _ext.ext().grad_status(self.params, base, self._offsets)
        out = []
        for p, s in zip(self.params, self.segments):
            g = p.grad
            out.append(0 if g is None else (1 if g.data_ptr() == base + 4 * s.offset else 2))
        return out

    def attach_grad_views(self):
        """Point every parameter's `.grad` at its flat slice (after a data-parallel reduce
        every slice holds the averaged gradient, whether or not this rank produced one)."""
        if self.grad is None:
            return
        for p, s in zip(self.params, self.segments):
            if p.grad is None:
                p.grad = self.view(self.grad, s)

    def set_zero(self, layout: ZeroLayout | None) -> None:
        self.zero = layout
        self._chunk_cache.clear()

    def _ranges(self, s: Segment):
        """[start, end) flat ranges of segment s this rank updates (all of it without ZeRO)."""
        a, b = s.offset, s.offset + s.numel
        if self.zero is None:
            return [(a, b)]
        out = []
        for oa, ob in self.zero.owned:
            lo, hi = max(a, oa), min(b, ob)
            if lo < hi:
                out.append((lo, hi))
        return out

    def state_offset(self, flat: int) -> int:
        """Optimizer-state offset of flat offset `flat` (compact under ZeRO-1)."""
        return flat if self.zero is None else self.zero.compact_of(flat)

    @property
    def state_numel(self) -> int:
        """Elements of one optimizer-state buffer: the whole space, or the owned shards."""
        return self.numel if self.zero is None else self.zero.compact_numel

    def _chunks(self, s: Segment, d):
        for a, b in self._ranges(s):
            so = self.state_offset(a)
            for st in range(a, b, CHUNK):
                yield st, min(CHUNK, b - st) | (int(bool(d)) << 32), so + (st - a)

    def owned_ranges(self, s: Segment) -> list:
        """[(flat start, flat end, state start)] of segment s this rank owns (all of it without
        ZeRO).  The fused optimizers' per-parameter state is these slices of the state buffers."""
        return [(a, b, self.state_offset(a)) for a, b in self._ranges(s)]

    def chunk_table_split(self, params_subset, decay_flags, split: int):
        """Two chunk tables: segments below flat offset `split`, and the rest."""
        key = ("split", tuple(id(p) for p in params_subset), tuple(decay_flags), split)
        hit = self._chunk_cache.get(key)
        if hit is not None:
            return hit
        lo, hi = [], []
        for p, d in zip(params_subset, decay_flags):
            s = self.segment_of(p)
            (lo if s.offset < split else hi).extend(self._chunks(s, d))
        out = tuple((torch.tensor(r if r else [(0, 0, 0)], dtype=torch.int64).to(self.device), len(r))
                    for r in (lo, hi))
        self._chunk_cache[key] = out
        return out

    def chunk_table_splits(self, params_subset, decay_flags, splits):
        """len(splits)+1 chunk tables: elements below flat offset splits[0], in
        [splits[i], splits[i+1]), ..., and from splits[-1] on.  A chunk that straddles a
        split is cut there (pieces of a deferred collective need not align to chunks)."""
        splits = tuple(int(x) for x in splits)
        key = ("splits", tuple(id(p) for p in params_subset), tuple(decay_flags), splits)
        hit = self._chunk_cache.get(key)
        if hit is not None:
            return hit
        import bisect

        parts = [[] for _ in range(len(splits) + 1)]
        for p, d in zip(params_subset, decay_flags):
            for start, lend, so in self._chunks(self.segment_of(p), d):
                n, flag = lend & 0xFFFFFFFF, lend & ~0xFFFFFFFF
                a, e = start, start + n
                while a < e:
                    k = bisect.bisect_right(splits, a)
                    cut = min(e, splits[k]) if k < len(splits) else e
                    parts[k].append((a, (cut - a) | flag, so + (a - start)))
                    a = cut
        out = tuple((torch.tensor(r if r else [(0, 0, 0)], dtype=torch.int64).to(self.device), len(r)) for r in parts)
        self._chunk_cache[key] = out
        return out

    def chunk_table(self, params_subset, decay_flags) -> tuple[torch.Tensor, int]:
        """int64 [nchunks, 3] rows of (start, len | decay<<32, state start) for the native
        optimizer kernels (only this rank's owned elements under ZeRO-1, whose state lives in
        compact buffers)."""
        key = (tuple(id(p) for p in params_subset), tuple(decay_flags))
        hit = self._chunk_cache.get(key)
        if hit is not None:
            return hit
        rows = []
        for p, d in zip(params_subset, decay_flags):
            rows.extend(self._chunks(self.segment_of(p), d))
        t = torch.tensor(rows if rows else [(0, 0, 0)], dtype=torch.int64).to(self.device)
        out = (t, len(rows))
        self._chunk_cache[key] = out
        return out

    def after_step(self) -> None:
        """End of an optimizer step: under ZeRO-1 every rank updated only its shards; gather
        the fp32 parameters back and rebuild the bf16 compute shadows."""
        if self.zero is None:
            return
        self.zero.gather(self.data)
        if self.shadow is not None:
            from ..ops._ext import gpu_ext

            gpu_ext().f32_to_bf16(self.data, self.shadow)
            # the in-place collective moved the parameters' version counters: the shadows are
            # current (converted just now), so re-stamp them instead of re-converting per tensor
            for p in self.params:
                p._rtdc_shadow_ver = p._version


def space_of(params) -> FlatParamSpace | None:
    sp = None
    for p in params:
        s = getattr(p, "_rtdc_space", None)
        if s is None:
            return None
        if sp is None:
            sp = s
        elif sp is not s:
            return None
    return sp

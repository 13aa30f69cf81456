"""Fused AdamW / SGD: one native launch per param group over the model's flat buffers.

API and `state_dict()` format match `torch.optim.AdamW` / `torch.optim.SGD` (state keys
`step`, `exp_avg`, `exp_avg_sq` / `momentum_buffer`), so checkpoints interoperate with stock
torch.  On the GPU the state tensors are views into flat fp32 buffers and the step is the
chunk-table kernel in csrc/kernels/optim.hip, which also refreshes the bf16 compute shadows.
On the CPU the same math runs per tensor with torch ops (reference path).

Host cost per step is O(#params) Python dict work and nothing else: AdamW step counts are
plain host integers (torch keeps one CPU tensor per parameter and does `step += 1` plus a
`float()` on each - ~150 tensor ops per GPT-2 step that left the GPU idle before the
optimizer launch); the per-parameter `step` tensors are materialised only by
`state_dict()` and parsed back by `load_state_dict()`, so checkpoints stay torch-compatible.
Like torch.optim, parameters without a gradient this step are skipped entirely (no weight
decay, no momentum), and the chunk table is built only from parameters that have one.
"""
from __future__ import annotations

import math

import torch

from ..ops._ext import gpu_ext
from ..ops.shadow import bump_generation
from .flat import FlatParamSpace, space_of


class _FlatOptimizer(torch.optim.Optimizer):
    _state_keys: tuple = ()

    def __init__(self, params, defaults):
        super().__init__(params, defaults)
        self._space: FlatParamSpace | None = None
        self._bufs: dict[str, torch.Tensor] = {}
        self._steps: dict = {}  # param -> number of optimizer steps taken (host int)
        self._bound: set = set()
        self._have = None  # parameters with a gradient this step (set by the native step)
        self._overlap = None  # optim.overlap.BackwardOverlap (updates run during backward)
        # DistributedDataParallel(zero_stage=1) leaves p.grad reduced only on this rank's shards:
        # only these optimizers (which update exactly the owned shards) may step such a model
        for p in self._all_params():
            p._rtdc_zero_capable = True

    # -- flat setup ------------------------------------------------------------------------
    def _all_params(self):
        return [p for g in self.param_groups for p in g["params"]]

    def _ensure_space(self):
        if self._space is not None:
            return self._space
        params = self._all_params()
        sp = space_of(params)
        if sp is None or any(p not in set(sp.params) for p in params):
            saved = [p.grad.detach().clone() if p.grad is not None else None for p in params]
            sp = FlatParamSpace(params)
            for p, g in zip(params, saved):
                if g is not None:
                    p.grad.copy_(g)
                else:
                    p.grad = None
        self._space = sp
        # optimizer state: the whole flat space, or (ZeRO-1) only this rank's owned shards,
        # back to back - 1/world of the bytes (FlatParamSpace.state_numel)
        for k in self._state_keys:
            self._bufs[k] = torch.zeros(sp.state_numel, dtype=torch.float32, device=sp.device)
        # adopt any state that already exists (e.g. loaded before the first step)
        for p in params:
            st = self.state.get(p)
            if st is None:
                continue
            for k in self._state_keys:
                if k in st and st[k] is not None:
                    self._adopt(p, k, st[k])
                    st[k] = self._state_value(p, k)
        return sp

    # -- per-parameter state views -------------------------------------------------------------
    def _zero(self):
        sp = self._space
        return None if sp is None else sp.zero

    def _state_value(self, p, k):
        """What `self.state[p][k]` holds: a view of the flat state buffer, or under ZeRO-1 a
        `FlatShardedTensor` over this rank's compact slices (checkpoint/sharded.py) - the value
        a sharded checkpoint writes and reads without any all-gather."""
        sp = self._space
        seg = sp.segment_of(p)
        z = sp.zero
        if z is None:
            return FlatParamSpace.view(self._bufs[k], seg)
        from ..checkpoint.sharded import FlatShardedTensor

        buf = self._bufs[k]
        local = [(a - seg.offset, buf[so:so + (b - a)]) for a, b, so in sp.owned_ranges(seg)]
        lo, hi = seg.offset, seg.offset + seg.numel
        ranges = []
        for r in range(z.world):
            rr = []
            for oa, ob in z.owned_by(r):
                a, b = max(lo, oa), min(hi, ob)
                if a < b:
                    rr.append((a - lo, b - lo))
            ranges.append(rr)
        return FlatShardedTensor(seg.shape, torch.float32, local, ranges, z.rank)

    def _adopt(self, p, k, v) -> None:
        """Copy a loaded/pre-existing state value into this optimizer's buffers (no-op when it
        already views them).  `v`: a full tensor of the parameter's shape, or a
        FlatShardedTensor whose local pieces cover this rank's owned ranges."""
        from ..checkpoint.sharded import FlatShardedTensor

        sp = self._space
        seg = sp.segment_of(p)
        buf = self._bufs[k]
        if isinstance(v, FlatShardedTensor):
            have = {s: t for s, t in v.local}
            for a, b, so in sp.owned_ranges(seg):
                t = have.get(a - seg.offset)
                if t is None or t.numel() != b - a:
                    raise ValueError(f"optimizer state {k!r}: sharded value does not cover owned range {a}-{b}")
                dst = buf[so:so + (b - a)]
                if t.data_ptr() != dst.data_ptr():
                    with torch.no_grad():
                        dst.copy_(t.reshape(-1).to(dst.device, dst.dtype))
            return
        if not torch.is_tensor(v):
            return
        if sp.zero is None:
            dst = FlatParamSpace.view(buf, seg)
            if v.data_ptr() != dst.data_ptr():
                with torch.no_grad():
                    dst.copy_(v.to(dst.device, dst.dtype))
            return
        # a full (replicated-layout) tensor: keep the owned ranges of its storage-order elements
        full = v.detach().to(buf.device, buf.dtype)
        if seg.channels_last:
            o, i, kh, kw = seg.shape
            full = full.permute(0, 2, 3, 1).contiguous()
        flat = full.reshape(-1)
        with torch.no_grad():
            for a, b, so in sp.owned_ranges(seg):
                buf[so:so + (b - a)].copy_(flat[a - seg.offset:b - seg.offset])

    def _bind_state(self, p):
        if p in self._bound:
            return self.state[p]
        st = self.state[p]
        for k in self._state_keys:
            if k not in st:
                st[k] = self._state_value(p, k)
        self._bound.add(p)
        return st

    def _flat_mode(self) -> bool:
        """Updates run over the flat buffers' chunk tables: always on the GPU (native kernels),
        and on the CPU under ZeRO-1 (owned shards only, compact state - reference path)."""
        if self._use_native():
            return True
        sp = space_of(self._all_params())
        return sp is not None and sp.zero is not None

    @torch.no_grad()
    def init_state(self) -> None:
        """Materialise every per-parameter state entry (zeros, step 0) without stepping, so
        `state_dict()` has its full structure before the first step - what a sharded
        checkpoint load fills in place (torch.distributed.checkpoint.state_dict does the same
        with a zero-grad step, T/distributed/checkpoint/state_dict.py `_init_optim_state`).
        Numerically a no-op for AdamW; for SGD a zero momentum buffer equals torch's
        first-step `buf = g` whenever dampening == 0."""
        flat = self._flat_mode()
        for p in self._all_params():
            st = self.state[p]
            if flat:
                self._ensure_space()
                self._bind_state(p)
            else:
                for k in self._state_keys:
                    if k not in st:
                        st[k] = torch.zeros_like(p, memory_format=torch.preserve_format)
            self._init_extra(p, st)
        self._materialize_steps()

    def _init_extra(self, p, st) -> None:
        pass

    # -- torch-compatible state dict -------------------------------------------------------
    def _materialize_steps(self) -> None:
        """Write the host step counters into the per-parameter `step` tensors torch keeps."""
        for p, n in self._steps.items():
            st = self.state.get(p)
            if st is not None:
                st["step"] = torch.tensor(float(n))

    def checkpoint_value(self, p, k, v):
        """The value a sharded checkpoint stores for state `k` of `p`: `v` itself, except a
        ZeRO-1 shard of a channels-last (ResNet conv) weight - its flat order is the storage
        order [O, KH, KW, I], not the torch shape's row-major order - which is consolidated
        into a full tensor (a sum of zero-filled shards: exact; collective over the group)."""
        from ..checkpoint.sharded import FlatShardedTensor

        if not isinstance(v, FlatShardedTensor):
            return v
        seg = self._space.segment_of(p)
        if not seg.channels_last:
            return v
        import torch.distributed as dist

        full = torch.zeros(seg.numel, dtype=v.dtype, device=self._space.device)
        for s0, t in v.local:
            full[s0:s0 + t.numel()].copy_(t)
        dist.all_reduce(full, group=self._space.zero.group)
        o, i, kh, kw = seg.shape
        return full.view(o, kh, kw, i).permute(0, 3, 1, 2)

    def consolidate_state(self) -> dict | None:
        """ZeRO-1: {state key: full flat buffer} all-gathered from every rank's compact shards
        (collective: call on every rank); None without ZeRO.  Only the torch-format
        `state_dict()` needs this - sharded checkpoints write the shards as they are."""
        sp = self._space
        if sp is None or sp.zero is None:
            return None
        full = {}
        for k, buf in self._bufs.items():
            f = torch.zeros(sp.numel, dtype=buf.dtype, device=buf.device)
            sp.zero.gather_compact(buf, f)
            full[k] = f
        return full

    def state_dict(self):
        """torch.optim format.  Under ZeRO-1 this is a collective that returns FULL state
        tensors (gathered copies); `checkpoint.state_dict.get_optimizer_state_dict` returns
        the sharded form instead."""
        full = self.consolidate_state()
        self._materialize_steps()
        sd = super().state_dict()
        if full is None:
            return sd
        # torch packs the live per-parameter dicts: replace the sharded values in copies
        ids = [i for g in sd["param_groups"] for i in g["params"]]
        state = {}
        for i, p in zip(ids, self._all_params()):
            st = sd["state"].get(i)
            if st is None:
                continue
            st = dict(st)
            seg = self._space.segment_of(p)
            for k in self._state_keys:
                if k in st:
                    st[k] = FlatParamSpace.view(full[k], seg)
            state[i] = st
        sd["state"] = state
        return sd

    def zero_grad(self, set_to_none: bool = True):
        from ..ops.gemm import flush_wgrads

        flush_wgrads()  # (a deferred weight gradient must not land after the reset)
        if self._space is not None and self._space.grad is not None:
            self._space.zero_grad(set_to_none=set_to_none)
        else:
            super().zero_grad(set_to_none=set_to_none)

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        self._steps = {}
        self._bound = set()
        for p in self._all_params():
            st = self.state.get(p)
            if st and "step" in st:
                self._steps[p] = int(float(st["step"]))
        if self._space is not None:
            for p in self._all_params():
                st = self.state.get(p)
                if not st:
                    continue
                for k in self._state_keys:
                    if k in st and st[k] is not None:
                        self._adopt(p, k, st[k])
                        st[k] = self._state_value(p, k)

    def _flat_step(self) -> None:
        """One step over the flat buffers: native chunk-table kernels on the GPU, the same
        chunk walk with torch ops on the CPU (ZeRO-1 reference path); then, under ZeRO-1, the
        parameter all-gather."""
        sp = self._ensure_space()
        have = sp.ensure_grad_views()
        self._have = None if len(have) == len(sp.params) else set(have)
        ov = self._overlap
        done = ov.updated if ov is not None else ()
        native = self._use_native()
        launches = []
        for group in self.param_groups:
            ps = [p for p in self._with_grad(group) if p not in done]
            if ps:
                launches += self._native_launches(group, ps) if native else self._cpu_launches(group, ps)
        self._launch_split(sp, launches)
        if ov is not None:
            ov.end_step()  # the compute stream waits for the updates that ran during backward
        sp.after_step()  # ZeRO-1: gather the updated shards
        bump_generation()  # masters / shadows changed in place: K-major weight images are stale

    @staticmethod
    def _rows(chunks, n):
        for start, lend, so in chunks[:n].tolist():
            yield start, lend & 0xFFFFFFFF, bool(lend >> 32), so

    def _cpu_launches(self, group, ps) -> list:
        raise NotImplementedError

    def _launch_split(self, sp, launches) -> None:
        """launches: [(params, decay_flags, fn(chunks, n))].  With a pending last-bucket
        all-reduce (DDP defer_tail_to_optimizer), update everything below its slice first,
        stream-wait for the collective, then the slice itself."""
        tail = sp.pending_tail
        if tail is None:
            for ps, flags, fn in launches:
                fn(*sp.chunk_table(ps, flags))
            return
        sp.pending_tail = None
        starts = [off for off, _ in tail]
        parts = [(sp.chunk_table_splits(ps, flags, starts), fn) for ps, flags, fn in launches]
        for tables, fn in parts:  # everything below the first in-flight piece
            if tables[0][1]:
                fn(*tables[0])
        for i, (_, wait) in enumerate(tail):  # piece i: wait for its collective, then update it
            wait()
            for tables, fn in parts:
                if tables[i + 1][1]:
                    fn(*tables[i + 1])

    def _use_native(self):
        ps = self._all_params()
        return bool(ps) and ps[0].is_cuda

    def _with_grad(self, group) -> list:
        have = self._have
        if have is None:
            return [p for p in group["params"] if p.grad is not None]
        return [p for p in group["params"] if p in have]

    @property
    def flat_space(self):
        return self._space


class FusedAdamW(_FlatOptimizer):
    _state_keys = ("exp_avg", "exp_avg_sq")

    def _init_extra(self, p, st) -> None:
        self._steps.setdefault(p, 0)

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2, amsgrad=False,
                 maximize=False):
        if amsgrad or maximize:
            raise NotImplementedError("amsgrad/maximize are not supported by the fused kernel")
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, amsgrad=False,
                                      maximize=False, foreach=None, capturable=False, differentiable=False,
                                      fused=None))

    def _native_launches(self, group, ps) -> list:
        """[(params, decay_flags, fn(chunks, n))] of one param group's native update of `ps`
        (advances their step counters)."""
        sp, ext = self._space, gpu_ext()
        for p in ps:
            self._bind_state(p)
        b1, b2 = group["betas"]
        wd = group["weight_decay"]
        out = []
        for step, sub in self._count(ps).items():
            def fn(chunks, n, group=group, b1=b1, b2=b2, wd=wd, step=step):
                ext.adamw(chunks, n, sp.data, sp.grad, self._bufs["exp_avg"], self._bufs["exp_avg_sq"],
                          sp.shadow, group["lr"], b1, b2, group["eps"], wd, 1 - b1 ** step,
                          math.sqrt(1 - b2 ** step), sp.grad_scale, sp.skip_ptr)

            out.append((sub, [wd != 0.0] * len(sub), fn))
        return out

    def _cpu_launches(self, group, ps) -> list:
        """CPU twin of `_native_launches` (ZeRO-1 on gloo): the per-tensor reference math of
        `step`, applied chunk by chunk to the owned flat slices and the compact state."""
        sp = self._space
        for p in ps:
            self._bind_state(p)
        b1, b2 = group["betas"]
        wd, lr, eps = group["weight_decay"], group["lr"], group["eps"]
        m_all, v_all = self._bufs["exp_avg"], self._bufs["exp_avg_sq"]
        out = []
        for step, sub in self._count(ps).items():
            def fn(chunks, n, step=step):
                for start, ln, decay, so in self._rows(chunks, n):
                    p = sp.data[start:start + ln]
                    g = sp.grad[start:start + ln]
                    if sp.grad_scale != 1.0:
                        g = g * sp.grad_scale
                    m, v = m_all[so:so + ln], v_all[so:so + ln]
                    if decay:
                        p.mul_(1 - lr * wd)
                    m.lerp_(g, 1 - b1)
                    v.mul_(b2).addcmul_(g, g, value=1 - b2)
                    denom = (v.sqrt() / math.sqrt(1 - b2 ** step)).add_(eps)
                    p.addcdiv_(m, denom, value=-lr / (1 - b1 ** step))

            out.append((sub, [wd != 0.0] * len(sub), fn))
        return out

    def _count(self, ps) -> dict:
        """Advance the step counter of every parameter in `ps`; {step: [params]}."""
        steps = self._steps
        by = {}
        for p in ps:
            n = steps.get(p, 0) + 1
            steps[p] = n
            by.setdefault(n, []).append(p)
        return by

    @torch.no_grad()
    def step(self, closure=None):
        from ..ops.gemm import flush_wgrads

        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        flush_wgrads()  # weight gradients deferred into a grouped launch (normally flushed by backward's end)
        if self._flat_mode():
            if self._use_native() and torch.cuda.is_current_stream_capturing():
                raise RuntimeError("FusedAdamW computes bias corrections on the host per step: not graph-capturable "
                                   "(use eager steps, or FusedSGD inside utils.graphs.CapturedStep)")
            self._flat_step()
            return loss
        sp = space_of(self._all_params())
        if sp is not None:
            sp.wait_pending_tail()
        for group in self.param_groups:
            b1, b2 = group["betas"]
            ps = self._with_grad(group)
            for step, sub in self._count(ps).items():
                for p in sub:
                    st = self.state[p]
                    if "exp_avg" not in st:
                        st["exp_avg"] = torch.zeros_like(p)
                        st["exp_avg_sq"] = torch.zeros_like(p)
                    g = p.grad
                    p.mul_(1 - group["lr"] * group["weight_decay"])
                    st["exp_avg"].lerp_(g, 1 - b1)
                    st["exp_avg_sq"].mul_(b2).addcmul_(g, g, value=1 - b2)
                    denom = (st["exp_avg_sq"].sqrt() / math.sqrt(1 - b2 ** step)).add_(group["eps"])
                    p.addcdiv_(st["exp_avg"], denom, value=-group["lr"] / (1 - b1 ** step))
        return loss


class FusedSGD(_FlatOptimizer):
    _state_keys = ("momentum_buffer",)

    def init_state(self) -> None:
        if all(g["momentum"] != 0.0 for g in self.param_groups):
            super().init_state()

    def __init__(self, params, lr=1e-3, momentum=0.0, dampening=0.0, weight_decay=0.0, nesterov=False,
                 maximize=False):
        if maximize:
            raise NotImplementedError("maximize is not supported by the fused kernel")
        super().__init__(params, dict(lr=lr, momentum=momentum, dampening=dampening, weight_decay=weight_decay,
                                      nesterov=nesterov, maximize=False, foreach=None, differentiable=False,
                                      fused=None))

    def _native_launches(self, group, ps) -> list:
        sp, ext = self._space, gpu_ext()
        mom = group["momentum"]
        wd = group["weight_decay"]
        # torch's first momentum step is `buf = d` (a clone): parameters without a buffer yet
        # form their own launch with first=True
        parts = [(ps, False)]
        if mom != 0.0:
            fresh = [p for p in ps if "momentum_buffer" not in self.state[p]]
            if fresh:
                old = [p for p in ps if "momentum_buffer" in self.state[p]]
                parts = [(fresh, True)] + ([(old, False)] if old else [])
            for p in fresh:
                self._bind_state(p)
        out = []
        for sub, first in parts:
            def fn(chunks, n, group=group, mom=mom, wd=wd, first=first):
                ext.sgd(chunks, n, sp.data, sp.grad, self._bufs["momentum_buffer"] if mom != 0.0 else None,
                        sp.shadow, group["lr"], mom, group["dampening"], wd, group["nesterov"], first,
                        sp.grad_scale, sp.skip_ptr)

            out.append((sub, [wd != 0.0] * len(sub), fn))
        return out

    def _cpu_launches(self, group, ps) -> list:
        """CPU twin of `_native_launches` (ZeRO-1 on gloo), torch.optim.SGD's math per chunk."""
        sp = self._space
        mom, wd, lr, damp, nest = (group["momentum"], group["weight_decay"], group["lr"], group["dampening"],
                                   group["nesterov"])
        parts = [(ps, False)]
        if mom != 0.0:
            fresh = [p for p in ps if "momentum_buffer" not in self.state[p]]
            if fresh:
                old = [p for p in ps if "momentum_buffer" in self.state[p]]
                parts = [(fresh, True)] + ([(old, False)] if old else [])
            for p in fresh:
                self._bind_state(p)
        buf_all = self._bufs.get("momentum_buffer")
        out = []
        for sub, first in parts:
            def fn(chunks, n, first=first):
                for start, ln, decay, so in self._rows(chunks, n):
                    p = sp.data[start:start + ln]
                    d = sp.grad[start:start + ln]
                    if sp.grad_scale != 1.0:
                        d = d * sp.grad_scale
                    if wd != 0 and decay:
                        d = d.add(p, alpha=wd)
                    if mom != 0:
                        b = buf_all[so:so + ln]
                        if first:
                            b.copy_(d)
                        else:
                            b.mul_(mom).add_(d, alpha=1 - damp)
                        d = d.add(b, alpha=mom) if nest else b
                    p.add_(d, alpha=-lr)

            out.append((sub, [wd != 0.0] * len(sub), fn))
        return out

    @torch.no_grad()
    def step(self, closure=None):
        from ..ops.gemm import flush_wgrads

        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        flush_wgrads()  # weight gradients deferred into a grouped launch (normally flushed by backward's end)
        if self._flat_mode():
            self._flat_step()
            return loss
        sp = space_of(self._all_params())
        if sp is not None:
            sp.wait_pending_tail()
        for group in self.param_groups:
            mom = group["momentum"]
            for p in self._with_grad(group):
                d = p.grad
                if group["weight_decay"] != 0:
                    d = d.add(p, alpha=group["weight_decay"])
                if mom != 0:
                    st = self.state[p]
                    buf = st.get("momentum_buffer")
                    if buf is None:
                        buf = torch.clone(d).detach()
                        st["momentum_buffer"] = buf
                    else:
                        buf.mul_(mom).add_(d, alpha=1 - group["dampening"])
                    d = d.add(buf, alpha=mom) if group["nesterov"] else buf
                p.add_(d, alpha=-group["lr"])
        return loss

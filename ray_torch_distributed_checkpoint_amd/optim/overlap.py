"""Fused optimizer updates overlapped with the backward pass.

A training step is `loss.backward(); opt.step()`: the update of every parameter waits for the
whole backward, although the last layers' gradients are final long before the first layers'
are.  The update is memory-bound (AdamW moves ~30 B per parameter: 3.7 GB for GPT-2-small,
0.64 ms of HBM time) while the backward's GEMMs are compute-bound, so on MI355X the two
overlap well.  `BackwardOverlap(opt, ddp=None)` registers post-accumulate-grad hooks (after
DDP's own) and, as soon as a group of parameters has its final gradient, launches the same
chunk-table kernel `opt.step()` would run for them on a low-priority side stream:

* single process: groups are ~`bucket_mb` slices of the flat parameter space; a group is
  final once every member's AccumulateGrad ran (autograd accumulates all uses of a leaf,
  e.g. GPT-2's tied token table, before its single AccumulateGrad);
* data parallel (native bucket engine): the groups are the DDP buckets; bucket b is updated
  once the engine launched its collective, the side stream first waiting for the reduced
  slice (`GradBucketEngine.stream_wait_bucket`: the collective itself with an averaging
  backend such as RCCL, or the bf16->fp32 widen / P2P event).

`opt.step()` then updates only what is left (parameters of groups that never completed,
e.g. unused ones) and makes the compute stream wait for the side stream, so the next forward
sees every update.  Per element the math is exactly `opt.step()`'s - results are bitwise
identical to the non-overlapped step (tests/test_optim_overlap_gpu.py).

Contract (why it is opt-in): one backward per optimizer step and no gradient edits between
backward and `step()` (clipping, unscaling) - the update has already run by then.  A second
gradient for an already-updated parameter in the same step raises.  Not with ZeRO-1 (the
shards are reduce-scattered and gathered around the step).
"""
from __future__ import annotations

from collections import defaultdict

import torch


class BackwardOverlap:
    def __init__(self, opt, ddp=None, bucket_mb: float = 32.0):
        if not opt._use_native():
            raise ValueError("BackwardOverlap needs the native (GPU) fused optimizer")
        sp = opt._ensure_space()
        self.opt, self.sp = opt, sp
        self.engine = None
        if ddp is not None and getattr(ddp, "world_size", 1) > 1:
            eng = getattr(ddp, "_engine", None)
            if eng is None or getattr(ddp, "zero", False) or not eng.can_stream_wait():
                raise ValueError("BackwardOverlap with DDP needs the native bucket engine, no ZeRO, and an averaging "
                                 "backend (RCCL) or bf16 gradient communication")
            self.engine = eng
            self.groups = [list(b.params) for b in ddp.buckets]
        else:
            from ..parallel.ddp import DistributedDataParallel

            # ~bucket_mb slices, but at most ~24 of them: each group costs one host-side hook
            # dispatch in the autograd thread (an 8B-parameter model at 32 MB would be ~1000)
            cap = max(1, int(bucket_mb * (1 << 20) / 4), sp.numel // 24)
            plan = DistributedDataParallel._plan([s.numel for s in sp.segments], cap, cap)
            self.groups = [[sp.params[i] for i in g] for g in plan]
        mine = {id(p) for p in opt._all_params()}
        self.groups = [[p for p in g if id(p) in mine] for g in self.groups]
        self.group_of = {id(p): gi for gi, g in enumerate(self.groups) for p in g}
        self.pgroup_of = {id(p): k for k, grp in enumerate(opt.param_groups) for p in grp["params"]}
        from ..ops.streams import side_stream

        self.stream = side_stream(sp.device, "overlap")
        self._reset()
        self._hooks = [p.register_post_accumulate_grad_hook(self._hook)
                       for g in self.groups for p in g]
        opt._overlap = self

    def _reset(self) -> None:
        self.pending = [len(g) for g in self.groups]
        self.next_bucket = 0
        self.updated: set = set()

    def remove(self) -> None:
        for h in self._hooks:
            h.remove()
        self._hooks = []
        if self.opt._overlap is self:
            self.opt._overlap = None

    # -- hooks (autograd thread) -------------------------------------------------------------
    def _fold(self, p) -> None:
        """A gradient autograd allocated outside the flat buffer is copied into its slice (the
        optimizer kernels read the flat buffer)."""
        g, sp = p.grad, self.sp
        if g is None:
            return
        base, end = sp.grad.data_ptr(), sp.grad.data_ptr() + sp.grad.numel() * 4
        if base <= g.data_ptr() < end:
            return
        v = sp.grad_view(p)
        with torch.no_grad():
            v.copy_(g)
        p.grad = v

    def _hook(self, p) -> None:
        from ..ops.gemm import when_grad_ready

        # (a weight gradient deferred into a grouped GEMM launch is final only after its flush)
        when_grad_ready(p, lambda: self._hook_final(p))

    def _hook_final(self, p) -> None:
        if p in self.updated:
            raise RuntimeError("BackwardOverlap: a second gradient for a parameter already updated this step "
                               "(gradient accumulation over several backward passes needs the plain optimizer "
                               "step)")
        if self.engine is not None:
            n = self.engine.launched()
            while self.next_bucket < n:
                b = self.next_bucket
                self.next_bucket += 1
                self._update(self.groups[b], bucket=b)
            return
        self._fold(p)
        gi = self.group_of.get(id(p))
        if gi is None:
            return
        self.pending[gi] -= 1
        if self.pending[gi] == 0:
            self._update(self.groups[gi])

    @torch.no_grad()
    def _update(self, ps, bucket: int | None = None) -> None:
        ps = [p for p in ps if p.grad is not None and p not in self.updated]
        if not ps:
            return
        dev = self.sp.device
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(dev))  # behind the kernels that wrote these gradients
        self.stream.wait_event(ev)
        by_group = defaultdict(list)
        for p in ps:
            by_group[self.pgroup_of[id(p)]].append(p)
        with torch.cuda.stream(self.stream):
            if bucket is not None:
                self.engine.stream_wait_bucket(bucket)
            for k, sub in by_group.items():
                for sub2, flags, fn in self.opt._native_launches(self.opt.param_groups[k], sub):
                    fn(*self.sp.chunk_table(sub2, flags))
        self.updated.update(ps)

    # -- opt.step() (main thread, after backward) --------------------------------------------
    def end_step(self) -> None:
        torch.cuda.current_stream(self.sp.device).wait_stream(self.stream)
        self._reset()

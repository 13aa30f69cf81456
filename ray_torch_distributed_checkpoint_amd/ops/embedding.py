"""Token + position embedding (gather) and its backward on native kernels.

The token-table gradient is a scatter-add where rows repeat; instead of float atomics (whose
summation order changes run to run) the token ids are stably sorted once and the native
kernel sums each run of equal ids in original token order: bitwise-reproducible gradients,
required for bit-exact resume (BASELINE config 5).  The sort is the native
one-workgroup radix sort (`data_ops.hip` sort_ids) on a side stream under the LM head's
cross-entropy kernel - no rocprim / ATen sort kernels in the step."""
from __future__ import annotations

import torch
import torch.nn.functional as F

from ._ext import gpu_ext
from .gradbuf import claimed_target, grad_target
from .shadow import shadow_of


def sort_ids(ids: torch.Tensor, num_rows: int):
    """(sorted ids, original positions) of a 1-D int64 GPU tensor of ids in [0, num_rows):
    stable, deterministic, one native kernel launch."""
    n = ids.numel()
    sidx = torch.empty(n, dtype=torch.int64, device=ids.device)
    perm = torch.empty(n, dtype=torch.int64, device=ids.device)
    ws = torch.empty(4 * max(n, 1), dtype=torch.int32, device=ids.device)
    gpu_ext().sort_ids(ids, sidx, perm, ws, max(1, int(num_rows - 1).bit_length()))
    return sidx, perm


def _side_stream(device) -> torch.cuda.Stream:
    from .streams import side_stream

    return side_stream(device, "sort")


class _PendingSort:
    """The backward's token sort, launched on the side stream when a kernel that tolerates one
    busy CU runs (`launch_pending_sorts`, called before the LM head's cross-entropy kernel).
    Launched right after the embedding, the one-workgroup sort held a CU during the first
    layer's persistent GEMM (one block per CU, every CU needed): qkv 123 vs 72 us."""

    def __init__(self, idx_c, rows):
        self.idx_c, self.rows, self.out = idx_c, rows, None

    def launch(self, side: bool = True):
        if self.out is None:
            dev = self.idx_c.device
            cur = torch.cuda.current_stream(dev)
            if side:
                st = _side_stream(dev)
                st.wait_stream(cur)
                with torch.cuda.stream(st):
                    sidx, perm = sort_ids(self.idx_c.reshape(-1), self.rows)
                    done = torch.cuda.Event()
                    done.record(st)
                sidx.record_stream(cur)
                perm.record_stream(cur)
            else:
                sidx, perm = sort_ids(self.idx_c.reshape(-1), self.rows)
                done = None
            self.out = (sidx, perm, done)
        return self.out


_pending: list = []
# RTDC_SORT_AT_XENT=0: launch the sort right after the embedding (A/B)
_SORT_AT_XENT = __import__("os").environ.get("RTDC_SORT_AT_XENT", "1") != "0"


def launch_pending_sorts() -> None:
    """Start the pending token sorts of this forward pass on the side stream (now)."""
    while _pending:
        _pending.pop().launch()


def _zero(ext, t: torch.Tensor) -> None:
    """Native zero fill (kernels/elementwise.hip fill_f32_kernel) of a contiguous fp32 slice."""
    if t.is_contiguous() and t.data_ptr() % 16 == 0:
        ext.fill_f32(t, 0.0)
    else:
        t.zero_()


class _Embedding(torch.autograd.Function):
    @staticmethod
    def forward(ctx, idx, wte, wpe, presort=True):
        B, T = idx.shape
        D = wte.shape[1]
        idx_c = idx.contiguous()
        out = torch.empty((B, T, D), dtype=torch.bfloat16, device=idx.device)
        gpu_ext().embed_fwd(idx_c, shadow_of(wte), shadow_of(wpe) if wpe is not None else None, out, T)
        # the backward's stable sort of the token ids depends only on idx: run it now on a side
        # stream, concurrently with the forward pass, instead of on the backward's critical path
        ctx.sorted = None
        if presort:
            ctx.sorted = _PendingSort(idx_c, wte.shape[0])
            if _SORT_AT_XENT:
                del _pending[:-3]  # (forwards whose sorts never launched: no backward followed)
                _pending.append(ctx.sorted)
            else:
                ctx.sorted.launch()
        ctx.save_for_backward(idx_c)
        ctx.shapes = (wte.shape, None if wpe is None else wpe.shape)
        ctx.params = (wte, wpe)
        return out

    @staticmethod
    def backward(ctx, dout):
        (idx,) = ctx.saved_tensors
        B, T = idx.shape
        wte_shape, wpe_shape = ctx.shapes
        wte, wpe = ctx.params
        dwte = grad_target(wte)
        accumulate = False
        if dwte is None:
            # tied table (GPT-2 LM head): add into the gradient the LM head already wrote
            dwte = claimed_target(wte)
            accumulate = dwte is not None
        ext = gpu_ext()
        if dwte is None:
            dwte = torch.empty(wte_shape, dtype=torch.float32, device=idx.device)
        if not accumulate:
            _zero(ext, dwte)  # rows no token uses (the kernel writes only the used ones)
        dwpe = None
        if wpe_shape is not None:
            dwpe = grad_target(wpe)
            if dwpe is None:
                dwpe = torch.empty(wpe_shape, dtype=torch.float32, device=idx.device)
            if T < wpe_shape[0]:
                _zero(ext, dwpe[T:])  # the kernel writes (not adds) positions [0, T)
        if ctx.sorted is not None:
            if ctx.sorted in _pending:
                _pending.remove(ctx.sorted)
            sidx, perm, done = ctx.sorted.launch(side=False) if ctx.sorted.out is None else ctx.sorted.out
            if done is not None:
                torch.cuda.current_stream(idx.device).wait_event(done)
        else:
            sidx, perm = sort_ids(idx.reshape(-1), wte_shape[0])
        ext.embed_bwd(sidx, perm, dout.contiguous(), dwte, dwpe, B, T, False, accumulate)
        return None, (None if accumulate else dwte), dwpe, None


def embedding(idx: torch.Tensor, wte: torch.Tensor, wpe: torch.Tensor | None = None,
              dtype=torch.bfloat16) -> torch.Tensor:
    if not idx.is_cuda:
        x = F.embedding(idx, wte)
        if wpe is not None:
            x = x + wpe[: idx.shape[1]].unsqueeze(0)
        return x
    # the backward's token sort is prepared during the forward only when a backward can follow
    return _Embedding.apply(idx, wte, wpe, torch.is_grad_enabled() and wte.requires_grad)

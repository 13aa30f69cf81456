"""GEMM entry points over the hand-written gfx950 MFMA kernels.

`gemm_bf16` is the raw launcher (layouts, batch strides, causal modes, fused epilogues);
`linear_fwd / linear_dgrad / linear_wgrad` are the three nn.Linear products expressed on it
(see csrc/kernels/gemm_bf16.hip for the operand-layout table).  `gemm_f32` is the exact-f32
MFMA path used by fp32 models (the reference toy MLP, R/my_ray_module.py:94-112).
"""
from __future__ import annotations

import os
import weakref

import torch

from ._ext import gpu_ext

ACT_NONE, ACT_RELU, ACT_GELU, ACT_GELU_BWD, ACT_RELU_BWD = 0, 1, 2, 3, 4
# GELU forward storing gelu'(pre-activation) (bf16) as the side output, and the dgrad epilogue
# that multiplies by it: the backward needs no transcendental
ACT_GELU_SAVE_GRAD, ACT_MUL = 5, 6
CAUSAL_NONE, CAUSAL_SKIP_UPPER, CAUSAL_K_UPTO_M, CAUSAL_K_FROM_M = 0, 1, 2, 3

_COLSUM_BLOCKS = 256
SPLITK_MAX_OUT = 200 * 256 * 256  # outputs that fill < 200 tiles of 256x256 (e.g. Llama-8B at 2k tokens/GPU)
SPLITK_WS_ELEMS = 64 << 20        # 256 MiB fp32 slab workspace cap
_ws_cache: dict = {}
# long-K weight gradients whose last round of output tiles is mostly empty run as two GEMMs
# (full rounds + a split-K tail); RTDC_WGRAD_ROUND_SPLIT=0 keeps one launch
_ROUND_SPLIT = os.environ.get("RTDC_WGRAD_ROUND_SPLIT", "1") != "0"


def workspace(device, numel: int, tag: str = "ws") -> torch.Tensor:
    """Per-device reusable fp32 scratch buffer (grown on demand, never shrunk)."""
    key = (str(device), tag)
    t = _ws_cache.get(key)
    if t is None or t.numel() < numel:
        t = torch.empty(max(numel, 1 << 16), dtype=torch.float32, device=device)
        _ws_cache[key] = t
    return t


def gemm_bf16(A, B, C, M, N, K, lda, ldb, ldc, a_kmajor=True, b_kmajor=True, *, Cin=None, bias=None,
              aux_in=None, aux_out=None, alpha=1.0, beta=0.0, act=ACT_NONE, causal=CAUSAL_NONE,
              batch=1, batch_inner=1, strides=(0, 0, 0, 0, 0, 0), tile_cfg=-1, alpha_dev=None, colsum_out=None):
    """colsum_out (fp32 [N]): also the column sums of C (fused into the gelu-backward epilogue
    of the 8-wave kernels, a separate reduction otherwise)."""
    sA0, sA1, sB0, sB1, sC0, sC1 = strides
    ws = None
    if act == ACT_NONE and bias is None and causal == CAUSAL_NONE and batch == 1 and M * N <= SPLITK_MAX_OUT:
        # split-K slabs for long-K / small-output GEMMs (weight gradients); the launcher decides
        ws = workspace(C.device, min(16 * M * N, SPLITK_WS_ELEMS), "splitk")
    cs_ws = None
    defer = colsum_out is not None and batch == 1 and _deferrable(colsum_out)
    if defer:
        # partial rows into a buffer of their own; the reduction joins the deferred window
        cs_ws = torch.empty(4 * ((M + 255) // 256) * N, dtype=torch.float32, device=C.device)
    elif colsum_out is not None:
        cs_ws = workspace(C.device, (max(4 * ((M + 255) // 256), _COLSUM_BLOCKS) + 64) * N, "colsum_gemm")
    rows = gpu_ext().gemm_bf16(A, B, C, Cin, bias, aux_in, aux_out, M, N, K, lda, ldb, ldc, a_kmajor, b_kmajor,
                               batch, batch_inner, sA0, sA1, sB0, sB1, sC0, sC1, float(alpha), float(beta), act,
                               causal, ws, tile_cfg, alpha_dev, None if defer else colsum_out, cs_ws)
    if defer and not (rows and _WG.add_job(cs_ws, rows, N, colsum_out, False)):
        colsum(C, out=colsum_out)  # this kernel left no partial rows (or nothing would flush them)
    return C


# Every product of the models runs on the hand-written gfx950 kernels (csrc/kernels/gemm_*):
# round 5 routed Llama-3-8B's few-row plain forwards / input gradients and GPT-2's LM-head
# logits to hipBLASLt where it measured faster; that vendor route was removed in round 6
# (benchmarks/gemm_bench.py keeps torch.matmul as the comparison oracle only).


def linear_fwd(x2d: torch.Tensor, w: torch.Tensor, bias=None, act=ACT_NONE, residual=None, aux_out=None,
               out_dtype=torch.bfloat16):
    """y[M,N] = act(x[M,K] @ w[N,K]^T + bias) (+ residual)."""
    M, K = x2d.shape
    N = w.shape[0]
    y = torch.empty((M, N), dtype=out_dtype, device=x2d.device)
    gemm_bf16(x2d, w, y, M, N, K, K, K, N, True, True, Cin=residual, bias=bias, aux_out=aux_out,
              beta=1.0 if residual is not None else 0.0, act=act)
    return y


def linear_dgrad(dy: torch.Tensor, w: torch.Tensor, act_bwd=ACT_NONE, aux_in=None, alpha=1.0, alpha_dev=None,
                 colsum_out=None, w_kmajor=None):
    """dx[M,K] = alpha (* alpha_dev[0]) * dy[M,N] @ w[N,K]  (optionally * act'(aux_in)).
    colsum_out (fp32 [K]): also sum_m dx[m, :] (the bias gradient of the layer that produced
    the activation), reduced by the GEMM epilogue instead of a second pass over dx.
    w_kmajor: the same weight as a K-major [K, N] bf16 image (ops/shadow.py kmajor_image): both
    operands then stream K-major (ds_read_b128 fragments instead of the transposing reads)."""
    M, N = dy.shape
    K = w.shape[1]
    dx = torch.empty((M, K), dtype=torch.bfloat16, device=dy.device)
    if w_kmajor is not None:
        gemm_bf16(dy, w_kmajor, dx, M, K, N, N, N, K, True, True, aux_in=aux_in, act=act_bwd, alpha=alpha,
                  alpha_dev=alpha_dev, colsum_out=colsum_out)
    else:
        gemm_bf16(dy, w, dx, M, K, N, N, K, K, True, False, aux_in=aux_in, act=act_bwd, alpha=alpha,
                  alpha_dev=alpha_dev, colsum_out=colsum_out)
    return dx


_ncu: dict = {}


def _num_cus(device) -> int:
    n = _ncu.get(device)
    if n is None:
        n = torch.cuda.get_device_properties(device).multi_processor_count
        _ncu[device] = n
    return n


def _round_split_rows(rows: int, cols: int, k: int, device) -> int:
    """Output rows for the full-rounds part of a long-K weight gradient, or 0 (no split).

    The 8-wave kernel runs one 256x256 tile per CU; an output of `tiles` tiles takes
    ceil(tiles / CUs) rounds, and a last round that is mostly empty idles the chip for a whole
    tile time (the GPT-2 LM head: 197 x 3 = 591 tiles = 2 full rounds + 79 tiles on 256 CUs).
    The rows that fill whole rounds run as one GEMM; the rest - too few tiles for a round -
    runs as a second one that the launcher splits along K (fp32 slabs + a fixed-order reduce),
    which spreads it over the chip: 2 + 1/3 rounds instead of 3 there."""
    if rows < 4096 or k < 64 * 64:
        return 0
    ncu = _num_cus(device)
    tn, tm = (cols + 255) // 256, (rows + 255) // 256
    tiles = tm * tn
    rem = tiles % ncu
    if tiles <= ncu or rem == 0 or rem * 2 > ncu:
        return 0
    tm_main = (tiles // ncu) * ncu // tn
    if (tm - tm_main) * tn >= 200:  # the tail must be a split-K candidate (gemm_bf16.hip pick_splitk)
        return 0
    return tm_main * 256


# ---- grouped weight gradients ---------------------------------------------------------------
# GPT-2's linear weight gradients are small outputs over a long K (tokens): 9..36 tiles of
# 256x256 each with K = 16384.  Launched one by one each needs split-K fp32 slabs plus a reduce
# kernel to fill 256 CUs (and the 768x768 one still runs at ~420 TF).  Deferred and launched
# together (gemm_8ph.hip gemm8g_kernel), two layers' eight products are 216 full-K tiles - one
# round of the chip, no slabs, no reduce.  A deferred product writes its output (a parameter's
# slice of the flat gradient buffer, handed to autograd before the kernel ran) at the flush, so
# every consumer of a parameter's "gradient ready" event goes through `when_grad_ready` (DDP
# bucket marks, the backward-overlapped optimizer), and the flush runs at the latest when the
# backward pass ends (an autograd final callback; DDP's finalize and the fused optimizers flush
# first too).  RTDC_WGRAD_GROUP=0 launches every weight gradient immediately.
_GROUP_ON = os.environ.get("RTDC_WGRAD_GROUP", "1") != "0"
_GROUP_MAX = 10       # products per launch (gemm8g_kernel G8_MAX_GROUP)
_GROUP_TILES = 200    # products with fewer output tiles than this are deferred
_BIG_TILES = 4096     # ... and, over a short K (< 4096 tokens), products of up to this many
# tiles per round (one 8-wave block per CU); groups are packed up to it (RTDC_WGRAD_ROUND: A/B of
# smaller groups that leave CUs to the compute stream's kernels while a group runs)
_ROUND = int(os.environ.get("RTDC_WGRAD_ROUND", "256"))
# RTDC_WGRAD_SIDE=1 launches the grouped products inside backward on a side stream, so the next
# layer's backward kernels can take the CUs a group leaves idle; the compute stream joins it at
# the end of backward.  It was -0.17 ms/step on GPT-2-small in round 3
# (profiles/wgrad_group_ab_r3.txt); with round 4's whole-round groups a group holds every CU and
# the compute stream's small kernels (norm backward, split-K reduces, column sums) run starved
# beside it: the compute stream is now faster on both models (GPT-2 -0.05 ms, Llama-3-8B
# -1.1 ms per step, profiles/wgrad_side_stream_ab_r4.txt), so it is the default.
_GROUP_SIDE = os.environ.get("RTDC_WGRAD_SIDE", "0") == "1"
# Short-K multi-round weight gradients packed into whole rounds (see _groupable);
# RTDC_WGRAD_GROUP_BIG=0 launches them one by one.
_GROUP_BIG = os.environ.get("RTDC_WGRAD_GROUP_BIG", "1") != "0"
# Deferred column sums: the bias / LayerNorm-parameter gradients are reductions of per-block
# partial rows; inside backward each leaves its partial rows in a buffer of its own and the
# reductions of a whole window run as ONE launch with the grouped weight gradients' flush
# (norm.hip colsum_multi_kernel; same per-reduction order, so bitwise the immediate result).
# ~4 reduction launches per GPT-2 layer otherwise.  RTDC_COLSUM_DEFER=0 reduces immediately.
_DEFER_ON = (os.environ.get("RTDC_COLSUM_DEFER", "1") != "0"
             and os.environ.get("RTDC_COLSUM_WIDE", "1") != "0")  # (same summation order only then)
_JOBS_MAX = 32  # reductions per launch (norm.hip kMultiJobs)


def _deferrable(out) -> bool:
    """A reduction into `out` may be deferred: a parameter's slice of a flat gradient buffer
    (FlatParamSpace), which AccumulateGrad adopts as p.grad without reading it.  Any other
    tensor handed to autograd may be cloned (read) right away - before the deferred kernel."""
    return (_DEFER_ON and _GROUP_ON and out is not None and out.is_cuda and out.dtype == torch.float32
            and out.is_contiguous() and out.dim() == 1 and out._base is not None
            and getattr(out._base, "_rtdc_flat_grad", False))


class _WgradGroup:
    def __init__(self):
        self.items = []      # (dy, x2d, out, tiles)
        self.jobs = []       # deferred column sums [ws, W, D, out alias, accumulate]
        self.tiles = 0
        self.ptrs = set()    # data_ptr of every pending output
        self.waiters = []    # (callback) in registration order, run after the flush
        self.cb_queued = False
        self.side = None     # RTDC_WGRAD_SIDE stream
        self.side_busy = False

    def _arm(self) -> bool:
        if not self.cb_queued:
            try:
                torch.autograd.Variable._execution_engine.queue_callback(self._end_of_backward)
            except RuntimeError:  # not inside a backward pass: nothing would flush - run now
                return False
            self.cb_queued = True
        return True

    def add_job(self, ws, W, D, out, accumulate) -> bool:
        """Defer `out (+)= column sums of the W partial rows ws[W][D]` to the next flush (False:
        not inside backward - the caller reduces now)."""
        if W < 1 or W > 4096 or not self._arm():
            return False
        if len(self.jobs) >= _JOBS_MAX:
            self.flush()
        # an alias, not `out` itself (see add())
        self.jobs.append([ws, int(W), int(D), out.view(out.shape), bool(accumulate)])
        self.ptrs.add(out.data_ptr())
        return True

    def pending_job(self, t):
        for j in self.jobs:
            if j[3].data_ptr() == t.data_ptr() and j[2] == t.numel():
                return j
        return None

    def add(self, dy, x2d, out, tiles, whole_rounds=False) -> bool:
        if not self._arm():
            return False
        # keep an alias, not `out` itself: AccumulateGrad adopts the returned tensor as p.grad
        # without a copy only while nothing else references it (otherwise it clones the still
        # unwritten buffer)
        if whole_rounds:
            # multi-round products (see _groupable): pack until the group is a whole number
            # of rounds - Llama-3-8B's four products of a layer at 2048 tokens are 896 + 1792
            # + 256 + 384 = 3328 tiles = 13 rounds, 14 when launched one by one
            if self.items and (len(self.items) >= _GROUP_MAX or not self.items[-1][4]):
                self.flush()
            self.items.append((dy, x2d, out.view(out.shape), tiles, True))
            self.tiles += tiles
            self.ptrs.add(out.data_ptr())
            if self.tiles % _ROUND == 0 or self.tiles > _BIG_TILES:
                self.flush()
            return True
        # greedy packing into rounds of the chip: launch the pending group first when this
        # product would not fit the round any more (GPT-2: 252-tile groups of 9 products)
        if self.items and (self.tiles + tiles > _ROUND or len(self.items) >= _GROUP_MAX or self.items[-1][4]):
            self.flush()
        self.items.append((dy, x2d, out.view(out.shape), tiles, False))
        self.tiles += tiles
        self.ptrs.add(out.data_ptr())
        if self.tiles >= _ROUND:
            self.flush()
        return True

    def _end_of_backward(self):
        self.cb_queued = False
        self.flush(join=True)

    def _launch_split(self, items):
        """A remainder far below a round (the last layer's products): each product on its own
        with split-K slabs, which spreads it over the chip."""
        for dy, x2d, out, _, _ in items:
            M, N = dy.shape
            K = x2d.shape[1]
            gemm_bf16(dy, x2d, out, N, K, M, N, K, K, False, False)

    def pending(self, t) -> bool:
        return t is not None and bool(self.ptrs) and t.data_ptr() in self.ptrs

    def pending_product(self, t) -> bool:
        """t is the output of a deferred weight-gradient PRODUCT (not a column-sum job: a
        second claim of a bias slot is the LayerNorm-offer protocol, see colsum())."""
        return t is not None and any(it[2].data_ptr() == t.data_ptr() for it in self.items)

    def _launch(self, items):
        for i in range(0, len(items), _GROUP_MAX):
            chunk = items[i:i + _GROUP_MAX]
            dims = []
            for dy, x2d, out, _, _ in chunk:
                M, N = dy.shape
                K = x2d.shape[1]
                dims += [N, K, M, N, K, K]
            gpu_ext().gemm_bf16_grouped([c[0] for c in chunk], [c[1] for c in chunk], [c[2] for c in chunk],
                                        dims, False, False)

    @staticmethod
    def _launch_jobs(jobs):
        for i in range(0, len(jobs), _JOBS_MAX):
            chunk = jobs[i:i + _JOBS_MAX]
            gpu_ext().colsum_multi([j[0] for j in chunk], [j[3] for j in chunk], [j[1] for j in chunk],
                                   [j[2] for j in chunk], [int(j[4]) for j in chunk])

    def flush(self, join: bool = False):
        """Launch the pending products and column sums, then run the callbacks waiting for
        them.  join=False (a flush inside backward) may leave them running on the side stream;
        join=True makes the current stream wait for everything launched there."""
        items, self.items, self.tiles = self.items, [], 0
        jobs, self.jobs = self.jobs, []
        waiters, self.waiters = self.waiters, []
        if join:
            # a backward that raised never ran its queued _end_of_backward: re-arm on the next
            # deferral instead of trusting a stale flag (a spare callback only flushes nothing)
            self.cb_queued = False
        dev_t = items[0][0] if items else (jobs[0][0] if jobs else None)
        if (dev_t is not None and _GROUP_SIDE and not join and dev_t.is_cuda
                and not torch.cuda.is_current_stream_capturing()):
            cur = torch.cuda.current_stream(dev_t.device)
            if self.side is None:
                from .streams import side_stream

                self.side = side_stream(dev_t.device, "wgrad")
            self.side.wait_stream(cur)  # operands written
            with torch.cuda.stream(self.side):
                if items:
                    self._launch(items)
                if jobs:
                    self._launch_jobs(jobs)
                for dy, x2d, _, _, _ in items:  # the compute stream may recycle them before the kernel ran
                    dy.record_stream(self.side)
                    x2d.record_stream(self.side)
                for j in jobs:
                    j[0].record_stream(self.side)
                self.ptrs = set()
                self.side_busy = True
                # (a DDP bucket / overlapped update triggered by these gradients is ordered
                # behind the grouped kernel: its events are recorded on this stream)
                for fn in waiters:
                    fn()
            return
        if items:
            if join and sum(it[3] for it in items) * 2 < _ROUND and not any(it[4] for it in items):
                self._launch_split(items)
            else:
                self._launch(items)
        if jobs:
            self._launch_jobs(jobs)
        self.ptrs = set()
        if self.side_busy and join:
            torch.cuda.current_stream(self.side.device).wait_stream(self.side)
            self.side_busy = False
        for fn in waiters:
            fn()


_WG = _WgradGroup()


def flush_wgrads() -> None:
    """Launch every deferred weight gradient now (and run the gradient-ready callbacks that
    waited for them); the current stream is ordered after all of them."""
    _WG.flush(join=True)


def when_grad_ready(p: torch.Tensor, fn) -> None:
    """Run fn() once p's gradient is final: now, or right after the flush that writes it.
    While grouped launches run on the side stream (RTDC_WGRAD_SIDE), fn runs with the side
    stream current, joined to the compute stream first: whatever fn enqueues (a DDP bucket's
    collective may cover gradients of both streams) is ordered after both."""
    if _WG.pending(p.grad):
        _WG.waiters.append(fn)
    elif _WG.side_busy:
        side = _WG.side
        side.wait_stream(torch.cuda.current_stream(side.device))
        with torch.cuda.stream(side):
            fn()
    else:
        fn()


def _groupable(dy, x2d, out, accumulate, alpha, alpha_dev) -> int:
    """Tiles of a weight gradient that may be deferred into a grouped launch, else 0: plain
    products that would otherwise split K (fewer than 200 output tiles, long K), or - over a
    short K (M < 4096 tokens: Llama-3-8B at 2048 per GPU) - multi-round products that are
    packed into whole rounds of the chip (returned negative)."""
    if not (_GROUP_ON and dy.is_cuda and out is not None and not accumulate and alpha == 1.0 and alpha_dev is None
            and out.dtype == torch.float32 and out.is_contiguous() and dy.is_contiguous() and x2d.is_contiguous()
            and dy.dtype == torch.bfloat16 and x2d.dtype == torch.bfloat16):
        return 0
    M, N = dy.shape
    K = x2d.shape[1]
    tiles = ((N + 255) // 256) * ((K + 255) // 256)
    if M % 64 or N % 8 or K % 8 or N < 256 or K < 256:
        return 0
    for t in (dy, x2d, out):
        if t.data_ptr() % 16:
            return 0
    if M < 64 * 64:
        return -tiles if _GROUP_BIG and M >= 1024 and 256 <= tiles <= _BIG_TILES else 0
    return tiles if tiles < _GROUP_TILES else 0


def linear_wgrad(dy: torch.Tensor, x2d: torch.Tensor, out=None, accumulate=False, alpha=1.0, alpha_dev=None):
    """dw[N,K] (fp32) = alpha (* alpha_dev[0]) * dy[M,N]^T @ x[M,K].  A product written into a
    flat-buffer gradient slice during backward may be deferred into a grouped launch (see
    `_WgradGroup`): its `out` is final after `flush_wgrads()` / at the end of backward."""
    M, N = dy.shape
    K = x2d.shape[1]
    tiles = _groupable(dy, x2d, out, accumulate, alpha, alpha_dev)
    if tiles and _WG.add(dy, x2d, out, abs(tiles), whole_rounds=tiles < 0):
        return out
    if out is None:
        out = torch.empty((N, K), dtype=torch.float32, device=dy.device)
    split = _round_split_rows(N, K, M, dy.device) if (_ROUND_SPLIT and dy.is_cuda and dy.is_contiguous()
                                                     and out.is_contiguous()) else 0
    if split:
        # rows [0, split) fill whole rounds of the chip; rows [split, N) go split-K (see above)
        for r0, r1 in ((0, split), (split, N)):
            o = out[r0:r1]
            gemm_bf16(dy[:, r0:r1], x2d, o, r1 - r0, K, M, N, K, K, False, False, Cin=o if accumulate else None,
                      beta=1.0 if accumulate else 0.0, alpha=alpha, alpha_dev=alpha_dev)
        return out
    gemm_bf16(dy, x2d, out, N, K, M, N, K, K, False, False, Cin=out if accumulate else None,
              beta=1.0 if accumulate else 0.0, alpha=alpha, alpha_dev=alpha_dev)
    return out


# Column sums that a gradient's producer computed on the way out (LayerNorm backward: the
# residual-stream gradient), keyed by the gradient tensor itself: (weakref, data_ptr, numel,
# last dim, version counter, sums).  colsum() of the same tensor takes them instead of
# re-reading it.  Entries whose tensor is gone are dropped on every offer.
_offered: list = []


def offer_colsum(t: torch.Tensor, sums: torch.Tensor) -> None:
    _offered[:] = [e for e in _offered if e[0]() is not None][-7:]
    _offered.append((weakref.ref(t), t.data_ptr(), t.numel(), t.shape[-1], t._version, sums))


# Per-row-group partial column sums a producer wrote on the way out ([W][N] fp32 rows, e.g. the
# flash-attention backward's dqkv): colsum() of the same matrix reduces them (deferred when it
# can) instead of reading the matrix.
_offered_partials: list = []


def partials_wanted() -> bool:
    return _DEFER_ON


def offer_colsum_partials(t: torch.Tensor, rows: torch.Tensor) -> None:
    _offered_partials[:] = [e for e in _offered_partials if e[0]() is not None][-3:]
    _offered_partials.append((weakref.ref(t), t.data_ptr(), t.numel(), t.shape[-1], t._version, rows))


def _take_partials(x2d: torch.Tensor):
    for k, (ref, ptr, numel, last, ver, rows) in enumerate(_offered_partials):
        t = ref()
        if (t is not None and ptr == x2d.data_ptr() and numel == x2d.numel() and last == x2d.shape[-1]
                and x2d.is_contiguous() and t._version == ver):
            del _offered_partials[k]
            return rows
    return None


def _take_colsum(x2d: torch.Tensor):
    for k, (ref, ptr, numel, last, ver, sums) in enumerate(_offered):
        t = ref()
        if (t is not None and ptr == x2d.data_ptr() and numel == x2d.numel() and last == x2d.shape[-1]
                and x2d.is_contiguous() and t._version == ver):
            del _offered[k]
            return sums
    return None


def colsum(x2d: torch.Tensor, out=None, accumulate=False):
    """fp32 column sums of a [M,N] matrix (bias gradient), deterministic two-stage reduce (or
    the sums the matrix's producer already offered, see offer_colsum)."""
    M, N = x2d.shape
    sums = _take_colsum(x2d)
    if sums is not None:
        if out is None or out.data_ptr() == sums.data_ptr():
            return sums if out is None else out
        job = _WG.pending_job(sums)
        if job is not None and not accumulate and _deferrable(out):
            # the sums are a deferred reduction: aim it at `out` instead of copying later
            _WG.ptrs.discard(sums.data_ptr())
            job[3] = out.view(out.shape)
            _WG.ptrs.add(out.data_ptr())
            return out
        if job is not None:
            flush_wgrads()
        if accumulate:
            out.add_(sums)
        else:
            out.copy_(sums)
        return out
    rows = _take_partials(x2d) if x2d.is_cuda else None
    if rows is not None and rows.shape[0] <= 4096 and rows.shape[1] == N:
        if _deferrable(out) and _WG.add_job(rows.view(-1), rows.shape[0], N, out, accumulate):
            return out
        if out is None:
            out = torch.empty((N,), dtype=torch.float32, device=x2d.device)
            accumulate = False
        gpu_ext().colsum_multi([rows.view(-1)], [out], [rows.shape[0]], [N], [int(accumulate)])
        return out
    nblk = min(_COLSUM_BLOCKS, max(1, M // 64))
    if (x2d.is_cuda and _deferrable(out) and x2d.dtype in (torch.bfloat16, torch.float32)
            and nblk >= 64 and x2d.stride(1) == 1):
        ws = torch.empty(nblk * N, dtype=torch.float32, device=x2d.device)
        gpu_ext().colsum_partial(x2d, M, N, x2d.stride(0), ws, nblk)
        if _WG.add_job(ws, nblk, N, out, accumulate):
            return out
        gpu_ext().colsum_multi([ws], [out], [nblk], [N], [int(accumulate)])
        return out
    if out is None:
        out = torch.empty((N,), dtype=torch.float32, device=x2d.device)
    ws = workspace(x2d.device, (nblk + 64) * N, "colsum")
    gpu_ext().colsum(x2d, M, N, x2d.stride(0), ws, nblk, out, accumulate)
    return out


def gemm_f32(A, B, C, M, N, K, sam, sak, sbk, sbn, ldc, *, Cin=None, bias=None, aux_in=None, aux_out=None,
             alpha=1.0, beta=0.0, act=ACT_NONE, dropout=None):
    """dropout: (p, seed, offset, device_base or None) - inverted dropout fused after the ReLU
    epilogue, drawing the Philox stream exactly like the standalone dropout kernel."""
    p, seed, offset, base = dropout if dropout is not None else (0.0, 0, 0, None)
    gpu_ext().gemm_f32(A, B, C, Cin, bias, aux_in, aux_out, M, N, K, sam, sak, sbk, sbn, ldc, float(alpha),
                       float(beta), act, float(p), int(seed), int(offset), base)
    return C

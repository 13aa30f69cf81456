"""Headline benchmark: samples/sec (+ sharded checkpoint save/restore wall-clock) on 1-8 MI355X.

Metric and configs come from BASELINE.json: "samples/sec/GPU + checkpoint save+restore
wall-clock at 1/2/4/8 MI355X".  Flagship = GPT-2-small DDP (BASELINE config 3): per GPU a
fixed micro-batch of 16 x 1024 tokens (weak scaling), bf16 compute on the hand-written
gfx950 kernels, fp32 master weights + fused AdamW, bucketed gradient all-reduce on RCCL
overlapped with backward.  Synthetic token data, random-init weights.

Timed region: exactly K full training steps (forward, backward + all-reduce, optimizer
step), bracketed by barrier + device synchronize, max over ranks.  After it, the checkpoint
phase measures a DCP-format sharded save of the full train state (model + AdamW state +
step): time until training can resume (HBM snapshot enqueued), time until every shard is
durable and `.metadata` committed, training throughput while the write is in flight, and
the restore wall-clock (sharded read + RCCL broadcast into the live model/optimizer).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--model gpt2-small] [--batch 16]
    python bench.py --model resnet18 [--batch 256] [--image-size 224]      (BASELINE config 2)
    python bench.py --model llama3-8b [--batch 1] [--seq-len 2048]         (BASELINE config 4)
    torchrun --nproc-per-node N bench.py --gpus N ...
"""
from __future__ import annotations

import argparse
import gc
import json
import os
import shutil
import sys
import tempfile
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

BASELINE = os.path.join(ROOT, "BASELINE.json")


def _baseline_metric():
    try:
        with open(BASELINE) as f:
            b = json.load(f)
        return b["metric"], b.get("published") or {}
    except Exception:
        return "samples/sec/GPU + checkpoint save+restore wall-clock at 1/2/4/8 MI355X", {}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--model", default="gpt2-small")
    ap.add_argument("--batch", type=int, default=None, help="samples per GPU per step (model default if unset)")
    ap.add_argument("--seq-len", type=int, default=None)
    ap.add_argument("--image-size", type=int, default=224)
    ap.add_argument("--bucket-mb", type=float, default=32.0)
    ap.add_argument("--grad-comm-dtype", default="fp32", choices=["fp32", "bf16"],
                    help="gradient all-reduce dtype (fp32 = torch DDP semantics)")
    ap.add_argument("--p2p-kb", type=float, default=0.0,
                    help="buckets <= this many KiB use the one-shot hipIpc all-reduce (0 = all on RCCL)")
    ap.add_argument("--zero", type=int, default=-1, choices=[-1, 0, 1],
                    help="1: ZeRO-1 (reduce-scatter gradients, sharded optimizer step, all-gather parameters); "
                         "-1 (default): ZeRO-1 for llama* at world > 1 (workloads.default_zero_stage), else 0")
    ap.add_argument("--overlap-opt", type=int, default=0, choices=[0, 1],
                    help="1: each bucket's fused optimizer update runs on a side stream as soon as its gradients "
                         "are final (optim/overlap.py; bitwise the plain step's result).  Off by default: measured "
                         "+0.1 ms on GPT-2 and ResNet-18 on one GPU (profiles/optim_overlap_ab.txt)")
    ap.add_argument("--no-ckpt", action="store_true")
    ap.add_argument("--ckpt-dir", default=None)
    ap.add_argument("--ckpt-scope", default="full", choices=["full", "model"],
                    help="full = model + optimizer train state (default); model = weights only")
    ap.add_argument("--ckpt-scope-fallback", action="store_true",
                    help="if the full train state does not fit on disk, measure model scope (flagged)")
    ap.add_argument("--overlap-steps", type=int, default=5)
    ap.add_argument("--backend", default="nccl", help="nccl (= RCCL on ROCm) | gloo (multi-rank rehearsal on 1 GPU)")
    ap.add_argument("--cpu", action="store_true",
                    help="run on the CPU (gloo; a plumbing rehearsal of the N-rank path, e.g. in CI - not a benchmark)")
    ap.add_argument("--force-dist", action="store_true",
                    help="run the distributed path (DDP + collectives) even with one rank (RCCL rehearsal)")
    ap.add_argument("--simulate-world", type=int, default=0,
                    help="checkpoint phase only (1 process): plan the sharded save/restore as rank "
                         "--simulate-rank of a W-rank data-parallel job and write/read just that rank's "
                         "shard (e.g. Llama-3-8B's full train-state 1/8 shard on one GPU)")
    ap.add_argument("--simulate-rank", type=int, default=0)
    ap.add_argument("--graph", default="0", choices=["auto", "0", "1"],
                    help="replay every step as a captured hipGraph (utils.graphs.CapturedStep, one graph per "
                         "synthetic batch: the same kernels, no per-launch host work); auto = on for ResNet-18 in "
                         "one process.  Off by default: ResNet-18 measured 8.14 vs 8.08 ms/step eager "
                         "(profiles/resnet_hipgraph_ab_r5.txt)")
    ap.add_argument("--sweep", type=int, default=1, choices=[0, 1],
                    help="N > 1: after the timed run, a short bucket_cap_mb x grad-comm-dtype sweep (comm.sweep)")
    ap.add_argument("--ckpt-budget-s", type=float, default=float(os.environ.get("RTDC_BENCH_CKPT_BUDGET_S", 300)),
                    help="wall-clock budget of the checkpoint phase; on overrun the measured headline is printed "
                         "with phase_timed_out and the run exits")
    ap.add_argument("--sweep-budget-s", type=float, default=float(os.environ.get("RTDC_BENCH_SWEEP_BUDGET_S", 240)))
    ap.add_argument("--pg-timeout-s", type=float, default=300.0, help="process-group (collective) timeout")
    args = ap.parse_args()
    args.batch_set, args.seq_len_set = args.batch is not None, args.seq_len is not None
    if args.batch is None:
        args.batch = 16
    if args.seq_len is None:
        args.seq_len = 1024

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # self-launch one process per GPU (before anything touches the GPU)
        import subprocess

        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
               "--master-addr=127.0.0.1", "--master-port=29517", os.path.abspath(__file__)] + sys.argv[1:]
        sys.exit(subprocess.call(cmd))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # --force-dist: the multi-GPU code path (process group, DDP with the native bucket engine and
    # an all-reduce of every bucket, preflight, in-sync check, bucket sweep, rank-sharded
    # checkpoint) in a 1-rank group - a one-GPU rehearsal of RCCL for the driver's 8-GPU run
    dist_on = world > 1 or args.force_dist
    if dist_on:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29561")
        os.environ.setdefault("RANK", str(rank))
        os.environ.setdefault("WORLD_SIZE", str(world))
    if args.cpu:
        dev = torch.device("cpu")
        args.backend = "gloo"
    else:
        ndev = max(1, torch.cuda.device_count())
        torch.cuda.set_device(local % ndev)
        dev = torch.device("cuda", local % ndev)
    if args.zero < 0:
        from ray_torch_distributed_checkpoint_amd.workloads import default_zero_stage

        args.zero = default_zero_stage(args.model, world)
    if dist_on:
        import datetime

        # a hung collective raises after the timeout instead of blocking forever (RCCL's
        # watchdog aborts the communicator; async error handling tears the rank down)
        os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
        to = datetime.timedelta(seconds=args.pg_timeout_s)
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev, timeout=to)
        else:
            dist.init_process_group(args.backend, timeout=to)

    from ray_torch_distributed_checkpoint_amd.checkpoint import dcp
    from ray_torch_distributed_checkpoint_amd.parallel.ddp import DistributedDataParallel
    from ray_torch_distributed_checkpoint_amd.ops import _ext

    if not args.cpu:
        _ext.gpu_ext()  # native kernels are mandatory on the GPU path
    sync = (lambda: None) if args.cpu else torch.cuda.synchronize
    _progress(rank, "process group up" if dist_on else "start")
    pre = preflight(world, rank, dev, args) if dist_on else None
    torch.manual_seed(1234)
    wl = build_workload(args, dev, rank)
    model, opt = wl["model"], wl["opt"]
    # the last bucket's all-reduce (GPT-2: the tied token table, whose gradient completes at the
    # end of backward) overlaps the fused optimizer's update of every other parameter
    net = DistributedDataParallel(model, bucket_cap_mb=args.bucket_mb, defer_tail_to_optimizer=True,
                                  grad_comm_dtype=args.grad_comm_dtype, p2p_max_kb=args.p2p_kb,
                                  zero_stage=args.zero, force_collectives=args.force_dist) if dist_on else model
    B, T = wl["batch"], wl["seq_len"]
    fwd_loss = wl["loss"]
    overlap = None
    if args.overlap_opt:
        from ray_torch_distributed_checkpoint_amd.optim import BackwardOverlap

        try:
            overlap = BackwardOverlap(opt, net if dist_on else None)
        except ValueError as e:  # e.g. fp32 gradients over gloo (no averaging collective)
            print(f"[bench] optimizer/backward overlap off: {e}", file=sys.stderr)

    seed = torch.ones((), dtype=torch.float32, device=dev)  # d(loss)/d(loss): no fill kernel per step

    from ray_torch_distributed_checkpoint_amd.utils.profiling import phase  # roctx ranges (--marker-trace)

    cur = {"net": net}

    def step(i):
        with phase("fwd"):
            loss = fwd_loss(cur["net"], i)
        with phase("bwd"):
            loss.backward(seed)
        with phase("opt"):
            opt.step()
            opt.zero_grad()
        # detached: a live loss keeps the step's autograd graph (its AccumulateGrad nodes) alive,
        # which a later hipGraph capture of the step must not inherit
        return loss.detach()

    _progress(rank, "workload built; warmup")
    for i in range(args.warmup):
        loss = step(i)
    graphs = None
    if args.graph == "1" or (args.graph == "auto" and args.model.startswith("resnet") and not dist_on and not args.cpu):
        # one captured step per synthetic batch (static inputs), replayed in capture order; the
        # captures share one memory pool and the optimizer is FusedSGD (graph-safe)
        from ray_torch_distributed_checkpoint_amd.utils.graphs import CapturedStep

        loss = None
        torch.cuda.synchronize()
        pool_id = torch.cuda.graph_pool_handle()
        graphs = [CapturedStep(lambda k=k: step(k), warmup=1, pool=pool_id) for k in range(wl["pool_len"])]
        _progress(rank, f"captured {len(graphs)} hipGraph steps")

    def run(i):
        return graphs[i % len(graphs)].replay() if graphs else step(i)

    sync()
    if dist_on:
        dist.barrier()
    sync()
    _progress(rank, f"timing {args.steps} steps")
    t0 = time.perf_counter()
    for i in range(args.steps):
        loss = run(i)
    sync()
    if dist_on:
        dist.barrier()
    sync()
    dt = time.perf_counter() - t0
    if dist_on:
        tt = torch.tensor([dt], device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = tt.item()
    ms_per_step = dt / args.steps * 1e3
    samples_per_s = world * B * args.steps / dt
    final_loss = loss.item()
    comm_plan = net.comm_plan() if dist_on else None
    # every rank must hold bitwise the same parameters (and, without ZeRO, optimizer state)
    in_sync = ranks_in_sync(model, opt, world, dev) if dist_on else None

    out = headline(args, wl, model, world, B, T, ms_per_step, samples_per_s, final_loss, overlap, dist_on,
                   comm_plan, pre, in_sync, dev)
    out["step_launch"] = f"hipgraph replay ({len(graphs)} captured steps)" if graphs else "eager"
    # from here on the headline is measured: a later phase that hangs (a stuck collective on a
    # first contact with a new node, a filesystem that stops answering) must not hide it
    wd = PhaseWatchdog(out, rank)
    _progress(rank, f"headline measured: {ms_per_step:.3f} ms/step")

    if not args.no_ckpt:
        # the throughput above is measured and must be reported even if the checkpoint phase
        # fails (e.g. a filesystem that refuses the shard writes): the failure is reported too
        with wd.phase("checkpoint", args.ckpt_budget_s):
            try:
                ck = checkpoint_phase(args, model, opt, net, run, world, rank, dev, dcp, sync)
            except Exception as e:  # noqa: BLE001
                ck = {"ckpt_unmeasured": f"checkpoint phase failed: {type(e).__name__}: {e}"[:300]}
                print(f"[bench] rank {rank}: {ck['ckpt_unmeasured']}", file=sys.stderr, flush=True)
        out.update(ck)

    if dist_on and args.sweep and args.zero == 0 and not args.overlap_opt:
        with wd.phase("sweep", args.sweep_budget_s):
            try:
                sweep = comm_sweep(args, model, opt, net, cur, step, world, sync)
            except Exception as e:  # noqa: BLE001
                sweep = {"error": f"{type(e).__name__}: {e}"[:300]}
        out["comm"]["sweep"] = sweep
    wd.stop()
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist_on:
        with wd.phase("teardown", 120.0, exit_code=0):
            dist.barrier()
            dist.destroy_process_group()
        wd.stop()


def _progress(rank: int, msg: str) -> None:
    """One stderr line per bench phase (stdout carries only the JSON line): a run that stops
    progressing shows where.  Rank 0 always; every rank with RTDC_BENCH_VERBOSE=1."""
    if rank == 0 or os.environ.get("RTDC_BENCH_VERBOSE", "0") == "1":
        print(f"[bench] rank {rank} {time.strftime('%H:%M:%S')} {msg}", file=sys.stderr, flush=True)


class PhaseWatchdog:
    """Wall-clock budget per post-headline phase.  If a phase overruns, rank 0 prints the JSON
    line with everything measured so far plus `"phase_timed_out": <name>` and the process ends
    with os._exit (no re-exec, no cleanup that could block on the hung collective)."""

    def __init__(self, out: dict, rank: int):
        import threading

        self.out, self.rank = out, rank
        self._lock = threading.Lock()
        self._cur = None  # (name, deadline, exit_code)
        self._beat = time.monotonic()
        self._t = threading.Thread(target=self._run, daemon=True, name="bench-watchdog")
        self._t.start()

    def _run(self):
        while True:
            time.sleep(0.5)
            with self._lock:
                cur = self._cur
            now = time.monotonic()
            if cur is not None and now - self._beat > 60.0:
                # heartbeat: a long phase is visibly alive (and a hung one names itself)
                self._beat = now
                _progress(self.rank, f"still in phase {cur[0]!r} ({cur[1] - now:.0f} s of budget left)")
            if cur is not None and now > cur[1]:
                name, _d, code = cur
                if self.rank == 0 and code != 0:
                    o = dict(self.out)
                    o["phase_timed_out"] = name
                    print(json.dumps(o), flush=True)
                print(f"[bench] rank {self.rank}: phase {name!r} exceeded its budget; exiting", file=sys.stderr,
                      flush=True)
                os._exit(code)

    def phase(self, name: str, budget_s: float, exit_code: int = 3):
        import contextlib

        @contextlib.contextmanager
        def cm():
            with self._lock:
                self._cur = (name, time.monotonic() + budget_s, exit_code)
                self._beat = time.monotonic()
            _progress(self.rank, f"phase {name!r} (budget {budget_s:.0f} s)")
            try:
                yield
            finally:
                with self._lock:
                    self._cur = None

        return cm()

    def stop(self):
        with self._lock:
            self._cur = None


def headline(args, wl, model, world, B, T, ms_per_step, samples_per_s, final_loss, overlap, dist_on, comm_plan,
             pre, in_sync, dev) -> dict:
    """The JSON line's fields known right after the timed run."""
    metric, published = _baseline_metric()
    base = published.get("samples_per_sec") if isinstance(published, dict) else None
    out = {
        "metric": metric,
        "value": round(samples_per_s, 3),
        "unit": wl["unit"],
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": (round(samples_per_s / base, 4) if base else None),
        "dtype": "bf16",
        "data": wl["data"],
        "config": {"model": args.model, "global_batch": B * world, "seq_len": T,
                   "parallelism": f"dp{world}", "micro_batch_per_gpu": B, "optimizer": wl["optim_name"],
                   "params": model.num_params()},
        "samples_per_sec_per_gpu": round(samples_per_s / world, 3),
        "model_tflops_per_gpu": round(wl["flops_per_sample"] * samples_per_s / world / 1e12, 2),
        "model_tflops_note": wl.get("flops_note", ""),
        # the attention FLOP convention is explicit, and the full-square figure of
        # rounds 1-4 is reported beside it so records stay comparable across rounds
        "flops_convention": "causal" if wl.get("flops_per_sample_full") else "dense",
        "final_loss": round(final_loss, 4),
    }
    if wl.get("flops_per_sample_full"):
        out["model_tflops_per_gpu_full_attn"] = round(wl["flops_per_sample_full"] * samples_per_s / world / 1e12, 2)
    if wl.get("tokens_per_sample"):
        out["tokens_per_sec"] = round(samples_per_s * wl["tokens_per_sample"], 1)
    # self-description of the communication setup (what ran, on how many ranks)
    comm = {"world_size": world, "backend": (dist.get_backend() if dist_on else None),
            "optimizer_overlapped_with_backward": overlap is not None,
            "rccl_version": _rccl_version(),
            "device": torch.cuda.get_device_name(dev) if dev.type == "cuda" else "cpu"}
    if dist_on:
        comm.update(comm_plan)
        comm["allreduce_GB_per_s_needed_at_this_step_time"] = round(
            comm["allreduce_bytes_per_step"] * 2 * (world - 1) / world / (ms_per_step / 1e3) / 1e9, 2)
        comm["preflight"] = pre
        out["ranks_in_sync"] = in_sync
    out["comm"] = comm
    return out


def preflight(world, rank, dev, args) -> dict:
    """Before anything is timed: one all-reduce of a known tensor checked on EVERY rank (the
    first time RCCL runs on a new node, a wrong result must stop the run, not skew it), the
    peer-access matrix of the visible GPUs, and all-reduce bus bandwidth at three sizes
    (xGMI evidence for the bucket sizing)."""
    t = torch.full((1 << 20,), float(rank + 1), device=dev)
    dist.all_reduce(t)
    want = world * (world + 1) / 2
    ok = bool((t == want).all().item())
    flags = torch.tensor([1 if ok else 0], device=dev)
    dist.all_reduce(flags, op=dist.ReduceOp.MIN)
    res = {"allreduce_check_ok_all_ranks": bool(flags.item())}
    if not res["allreduce_check_ok_all_ranks"]:
        raise RuntimeError(f"preflight: all-reduce returned wrong values on some rank (rank {rank} ok={ok})")
    if dev.type == "cuda":
        n = torch.cuda.device_count()
        res["peer_access"] = [[1 if i == j else int(torch.cuda.can_device_access_peer(i, j)) for j in range(n)]
                              for i in range(n)]
    bw = {}
    sizes = (1 << 20, 32 << 20, 256 << 20) if dev.type == "cuda" else (1 << 20,)
    for nbytes in sizes:
        x = torch.ones(nbytes // 4, device=dev)
        dist.all_reduce(x)
        if dev.type == "cuda":
            torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        iters = 5
        for _ in range(iters):
            dist.all_reduce(x)
        if dev.type == "cuda":
            torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / iters
        tt = torch.tensor([dt], device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = tt.item()
        bw[f"{nbytes >> 20}MB"] = {"ms": round(dt * 1e3, 3), "busbw_GBps": round(nbytes * 2 * (world - 1) / world / dt / 1e9, 2)}
        del x
    res["allreduce_fp32"] = bw
    return res


def _checksum(buf: torch.Tensor) -> list:
    """Order-sensitive integer checksum of a float buffer's bits (chunked: bounded memory)."""
    v = buf.detach().reshape(-1)
    bits = v.view(torch.int32) if v.element_size() == 4 else v.view(torch.int16)
    s1 = torch.zeros((), dtype=torch.int64, device=v.device)
    s2 = torch.zeros((), dtype=torch.int64, device=v.device)
    step = 1 << 26
    for a in range(0, bits.numel(), step):
        x = bits[a:a + step].to(torch.int64)
        w = (torch.arange(a, a + x.numel(), device=v.device, dtype=torch.int64) % 1000003) + 1
        s1 += x.sum()
        s2 += (x * w).sum()
    return [int(s1.item()), int(s2.item())]


def ranks_in_sync(model, opt, world, dev) -> bool:
    """Post-run cross-rank check: every rank holds bitwise the same parameters and (without
    ZeRO-1, where each rank keeps only its own shards) the same optimizer state."""
    sp = getattr(opt, "flat_space", None)
    bufs = [sp.data] if sp is not None else [p.detach() for p in model.parameters()]
    if sp is not None and sp.zero is None:
        bufs += list(getattr(opt, "_bufs", {}).values())
    mine = []
    for b in bufs:
        mine += _checksum(b)
    t = torch.tensor(mine, dtype=torch.int64, device=dev)
    lo, hi = t.clone(), t.clone()
    dist.all_reduce(lo, op=dist.ReduceOp.MIN)
    dist.all_reduce(hi, op=dist.ReduceOp.MAX)
    return bool(torch.equal(lo, hi))


def comm_sweep(args, model, opt, net, cur, step, world, sync) -> list:
    """bucket_cap_mb x gradient dtype, a few steps each on this node's fabric: the xGMI
    sizing evidence for the default plan (32 MiB fp32).  Re-wraps the same model (same flat
    space and optimizer); the timed headline above is untouched."""
    from ray_torch_distributed_checkpoint_amd.parallel.ddp import DistributedDataParallel

    _maybe_hang("sweep")
    out = []
    net.detach()
    cells = [(d, c) for d in ("fp32", "bf16") for c in (16.0, 32.0, 64.0, 128.0)]
    if os.environ.get("RTDC_SWEEP_CELLS"):  # e.g. "bf16:32,fp32:64" (A/B of single cells)
        cells = [(d, float(c)) for d, c in (x.split(":") for x in os.environ["RTDC_SWEEP_CELLS"].split(","))]
    for dtype, cap in cells:
        w = DistributedDataParallel(model, bucket_cap_mb=cap, defer_tail_to_optimizer=True, grad_comm_dtype=dtype,
                                    force_collectives=args.force_dist)
        cur["net"] = w
        for i in range(2):  # warm: lazy workspaces, the engine's first bucket plan
            step(i)
        # three windows of 5 steps, the fastest one reported (plus the mean): one host hiccup
        # inside a single short window would otherwise move a whole cell
        gc.collect()
        times = []
        for rep in range(3):
            sync()
            dist.barrier()
            t0 = time.perf_counter()
            n = 5
            for i in range(n):
                step(i)
            sync()
            dist.barrier()
            times.append((time.perf_counter() - t0) / n)
        tt = torch.tensor([min(times), sum(times) / len(times)], device=sp_device(model))
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        out.append({"bucket_cap_mb": cap, "grad_comm_dtype": dtype, "buckets": len(w.buckets),
                    "ms_per_step": round(tt[0].item() * 1e3, 3), "ms_per_step_mean": round(tt[1].item() * 1e3, 3)})
        _progress(dist.get_rank(), f"sweep cell {dtype}/{cap:g} MB: {out[-1]['ms_per_step']} ms/step")
        w.detach()
    cur["net"] = net
    return out


def sp_device(model):
    return next(model.parameters()).device


def _rccl_version():
    try:
        v = torch.cuda.nccl.version()
        return ".".join(str(x) for x in v) if isinstance(v, tuple) else str(v)
    except Exception:
        return None


def build_workload(args, dev, rank):
    """Model + optimizer + synthetic batch pool for one BASELINE.json config."""
    from ray_torch_distributed_checkpoint_amd import ops
    from ray_torch_distributed_checkpoint_amd.optim import FusedAdamW, FusedSGD

    g = torch.Generator(device=dev)
    g.manual_seed(1000 + rank)
    name = args.model
    if name.startswith("resnet"):
        from ray_torch_distributed_checkpoint_amd.models import ResNet18

        hw = args.image_size
        B = args.batch if args.batch_set else 256
        model = ResNet18(num_classes=10).to(dev)
        opt = FusedSGD(model.parameters(), lr=0.01, momentum=0.9, weight_decay=5e-5)
        pool = [(torch.randn(B, 3, hw, hw, device=dev, generator=g),
                 torch.randint(0, 10, (B,), device=dev, generator=g)) for _ in range(2)]

        def loss(net, i):
            x, y = pool[i % len(pool)]
            return ops.cross_entropy(net(x), y)

        return dict(model=model, opt=opt, batch=B, seq_len=hw, loss=loss, pool_len=len(pool),
                    unit=f"samples/s ({hw}x{hw} images, all GPUs)", optim_name="fused SGD momentum (fp32 master)",
                    data="synthetic (random images/labels), random-init weights",
                    flops_per_sample=model.flops_per_sample(hw))
    if name.startswith("llama"):
        from ray_torch_distributed_checkpoint_amd.models import Llama, LlamaConfig

        cfg = LlamaConfig.named(name)
        T = min(args.seq_len if args.seq_len_set else 2048, cfg.max_seq_len)
        B = args.batch if args.batch_set else 1
        model = Llama(cfg, device=dev)
        vocab = cfg.vocab_size
    else:
        from ray_torch_distributed_checkpoint_amd.models import GPT2, GPT2Config

        cfg = GPT2Config.named(name)
        T = min(args.seq_len, cfg.n_positions)
        B = args.batch
        model = GPT2(cfg).to(dev)
        vocab = cfg.vocab_size
    opt = FusedAdamW(model.parameters(), lr=6e-4, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.1)
    pool = [torch.randint(0, vocab, (B, T + 1), device=dev, generator=g) for _ in range(4)]
    # (inputs, shifted targets) as contiguous tensors, as a data loader delivers them
    pool = [(d[:, :-1].contiguous(), d[:, 1:].contiguous()) for d in pool]

    def loss(net, i):
        inp, tgt = pool[i % len(pool)]
        return net(inp, tgt)

    return dict(model=model, opt=opt, batch=B, seq_len=T, loss=loss, tokens_per_sample=T, pool_len=len(pool),
                unit=f"samples/s (sequences of {T} tokens, all GPUs)", optim_name="fused AdamW (fp32 master)",
                data="synthetic (random tokens), random-init weights",
                flops_per_sample=model.flops_per_token(T, causal=True) * T,
                flops_per_sample_full=model.flops_per_token(T, causal=False) * T,
                flops_note="6N + 6·L·d·T per token (N without the position/input embedding; causal attention: "
                           "the lower triangle only - rounds 1-4 counted the full square, ~7 % more on GPT-2)")


def _maybe_hang(phase: str) -> None:
    """RTDC_BENCH_HANG_PHASE=<phase>: fault injection for the watchdog test (a hung phase)."""
    if os.environ.get("RTDC_BENCH_HANG_PHASE") == phase:
        print(f"[bench] injected hang in phase {phase!r}", file=sys.stderr, flush=True)
        while True:
            time.sleep(60)


def checkpoint_phase(args, model, opt, net, step, world, rank, dev, dcp, sync):
    _maybe_hang("checkpoint")
    base = args.ckpt_dir or os.environ.get("RTDC_BENCH_CKPT_DIR") or tempfile.gettempdir()
    path = os.path.join(base, "rtdc_bench_ckpt")
    if rank == 0:
        shutil.rmtree(path, ignore_errors=True)
        os.makedirs(path, exist_ok=True)
    if dist.is_initialized():
        dist.barrier()

    from ray_torch_distributed_checkpoint_amd.checkpoint.state_dict import get_state_dict, set_state_dict

    scope = args.ckpt_scope
    sim = None
    if args.simulate_world and args.simulate_world > 1:
        if world != 1:
            raise ValueError("--simulate-world runs in a single process")
        sim = (args.simulate_world, args.simulate_rank)
    share = sim[0] if sim else max(world, 1)  # this rank writes ~1/share of the state
    # --simulate-world W --zero 1: the optimizer state of rank r's ZeRO-1 shard (owner chunks of
    # the W-rank layout, no all-gather) instead of the replicated dedup plan
    zsim = bool(sim) and args.zero == 1

    def state():
        if zsim:
            from ray_torch_distributed_checkpoint_amd.checkpoint.sharded import simulated_zero_optimizer_state

            msd = get_state_dict(model, None)[0]
            osd = simulated_zero_optimizer_state(model, opt, sim[0], sim[1], args.bucket_mb, args.grad_comm_dtype)
        else:
            msd, osd = get_state_dict(model, opt)
        return {"model": msd, "optim": osd, "step": 1} if scope == "full" else {"model": msd, "step": 1}

    def nbytes_of(sd):
        if torch.is_tensor(sd):
            return sd.numel() * sd.element_size()
        if isinstance(sd, dict):
            return sum(nbytes_of(v) for v in sd.values())
        return 0

    # the box's scratch disk bounds what one rank can write (Llama-3-8B full train state is
    # 96 GB on one GPU, 12 GB per rank at 8).  The scope is never reduced silently: a state
    # that does not fit is reported as unmeasured (or, with --ckpt-scope-fallback, measured at
    # model scope and flagged as downgraded).
    free = shutil.disk_usage(base).free
    downgraded = False
    if scope == "full" and nbytes_of(state()) / share * 1.15 > free:
        if not args.ckpt_scope_fallback:
            return {"ckpt_unmeasured": f"full train state ({nbytes_of(state()) / 1e9:.1f} GB) larger than free "
                                       f"disk ({free / 1e9:.0f} GB) at {base}; pass --ckpt-scope-fallback for a "
                                       f"model-only measurement"}
        scope, downgraded = "model", True
    if nbytes_of(state()) / share * 1.15 > free:
        return {"ckpt_unmeasured": f"state larger than free disk ({free / 1e9:.0f} GB)"}

    # ---- startup-time allocation a trainer does once (engine: pinned ring + writers; this
    # rank's HBM snapshot arena), reported on its own, outside every timed window below
    sync()
    tp = time.perf_counter()
    arena_bytes = dcp.prepare_async(state(), simulate=sim)
    sync()
    t_prepare = time.perf_counter() - tp
    _progress(rank, f"checkpoint: prepared ({arena_bytes / 1e9:.2f} GB arena); async save + {args.overlap_steps} steps")
    # ---- async save overlapped with training steps, as a training loop issues it: between two
    # steps with the device still busy (no host sync before the save - an idle device drops its
    # clocks and the next step pays the ramp).  Each step timed on the device (events between
    # consecutive steps; the first interval also holds the HBM snapshot copy) and on the host.
    cuda = dev.type == "cuda"
    n_ov = max(1, args.overlap_steps)
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(n_ov + 1)] if cuda else []
    for i in range(2):  # back to a busy device after the prepare's sync
        step(i)
    if cuda:
        evs[0].record()
    t0 = time.perf_counter()
    h = dcp.async_save(state(), path, simulate=sim)
    t_resume = time.perf_counter() - t0  # training may continue from here
    t1 = time.perf_counter()
    host_each = []
    for i in range(n_ov):
        th = time.perf_counter()
        step(i)
        if cuda:
            evs[i + 1].record()
        host_each.append((time.perf_counter() - th) * 1e3)
    sync()
    each_ms = [evs[i].elapsed_time(evs[i + 1]) for i in range(n_ov)] if cuda else host_each
    overlap_ms = sum(each_ms) / n_ov if cuda else (time.perf_counter() - t1) / n_ov * 1e3
    _progress(rank, "checkpoint: overlap steps done; waiting for durability")
    local_write = h.wait()
    if dist.is_initialized():
        dist.barrier()
    h._finish()
    if dist.is_initialized():
        dist.barrier()
    t_durable = time.perf_counter() - t0
    nbytes = torch.tensor([float(h.nbytes)], device=dev)
    if dist.is_initialized():
        dist.all_reduce(nbytes)
    if rank == 0:
        shutil.rmtree(path, ignore_errors=True)  # keep one checkpoint on disk at a time
    # ---- blocking save (nothing overlapped) for the pure write bandwidth
    path2 = path + "_sync"
    if rank == 0:
        shutil.rmtree(path2, ignore_errors=True)
    if dist.is_initialized():
        dist.barrier()
    sync()
    _progress(rank, "checkpoint: blocking save")
    t2 = time.perf_counter()
    dcp.save(state(), path2, simulate=sim)
    t_sync = time.perf_counter() - t2
    _progress(rank, "checkpoint: restores")
    # ---- restore into the live model + optimizer: first warm (shards still in the page cache
    # right after the write), then cold (every shard dropped from the page cache with
    # posix_fadvise(DONTNEED) after its fsync, so the bytes come from the device)
    def restore():
        sync()
        if dist.is_initialized():
            dist.barrier()
        t3 = time.perf_counter()
        sd = state()
        dcp.load(sd, path2, simulate=sim)
        # (simulated ZeRO shards are read in place into the optimizer's own state buffers)
        set_state_dict(model, None if zsim else opt, model_state_dict=sd["model"], optim_state_dict=sd.get("optim"))
        sync()
        if dist.is_initialized():
            dist.barrier()
        return time.perf_counter() - t3

    t_restore_warm = restore()
    resident = drop_page_cache(path2)
    if dist.is_initialized():
        dist.barrier()
    t_restore = restore()
    vals = torch.tensor([t_resume, t_durable, t_sync, t_restore, overlap_ms, local_write, t_restore_warm, resident],
                        device=dev, dtype=torch.float64)
    if dist.is_initialized():
        dist.all_reduce(vals, op=dist.ReduceOp.MAX)
    t_resume, t_durable, t_sync, t_restore, overlap_ms, local_write, t_restore_warm, resident = vals.tolist()
    if rank == 0:
        shutil.rmtree(path, ignore_errors=True)
        shutil.rmtree(path2, ignore_errors=True)
    total = nbytes.item()
    out = {
        "ckpt_bytes_total": int(total),
        "ckpt_save_blocking_s": round(t_resume, 4),
        "ckpt_save_durable_s": round(t_durable, 4),
        "ckpt_save_sync_s": round(t_sync, 4),
        "ckpt_restore_s": round(t_restore, 4),
        "ckpt_restore_collectives": dcp.LAST_LOAD_COLLECTIVES,  # coalesced broadcasts of the last restore
        "ckpt_restore_cold": resident < 0.01,
        "ckpt_restore_resident_frac": round(resident, 4),  # measured by mincore before the cold restore
        "ckpt_restore_warm_s": round(t_restore_warm, 4),
        "ckpt_save_plus_restore_s": round(t_sync + t_restore, 4),
        "ckpt_write_GBps": round(total / max(t_sync, 1e-9) / 1e9, 3),
        "ckpt_restore_GBps": round(total / max(t_restore, 1e-9) / 1e9, 3),
        "ms_per_step_during_async_save": round(overlap_ms, 3),  # device time, snapshot copy included
        "ms_per_step_during_async_save_each": [round(x, 3) for x in each_ms],
        "host_ms_per_step_during_async_save_each": [round(x, 3) for x in host_each],
        "ckpt_d2h_drained_s": (round(h.d2h_s, 4) if h.d2h_s else None),  # submit -> last byte in the pinned ring
        "ckpt_d2h_mode": _d2h_mode(),
        "ckpt_prepare_s": round(t_prepare, 4),  # one-time: engine + snapshot arena (startup in a trainer)
        "ckpt_snapshot_arena_bytes": int(arena_bytes),
        "ckpt_format": f"torch.distributed.checkpoint (.metadata + __<rank>_0.distcp x {world}), native engine",
        "ckpt_scope": "model + optimizer + step" if scope == "full" else "model + step",
        "ckpt_fs": _fs_of(base),
    }
    if downgraded:
        out["ckpt_scope_downgraded"] = True
    if sim:
        # one rank's share of a W-rank job: bytes/GBps above are this rank's shard
        out["ckpt_simulated"] = {"world": sim[0], "rank": sim[1], "note": "per-rank shard of a W-rank plan, "
                                 "written and restored by one process; other ranks' shards not written"}
        out["ckpt_format"] = f"torch.distributed.checkpoint (.metadata + __{sim[1]}_0.distcp of {sim[0]}), native engine"
        if zsim:
            out["ckpt_simulated"]["layout"] = "ZeRO-1 owner shards (optimizer state), dedup plan (parameters)"
    return out


def _d2h_mode() -> str:
    from ray_torch_distributed_checkpoint_amd.checkpoint import torchsave

    try:
        return torchsave.get_engine().d2h_mode
    except Exception:  # noqa: BLE001
        return "?"


def drop_page_cache(path: str) -> float:
    """fsync + posix_fadvise(DONTNEED) every shard, then MEASURE how much of the checkpoint is
    still in the page cache (mincore over an mmap of each file): the returned resident
    fraction is what makes the next restore cold or not (0.0 = every byte comes from the
    device).  On tmpfs/ramfs the pages cannot be dropped and the fraction stays ~1.0."""
    from ray_torch_distributed_checkpoint_amd.utils import pagecache

    pagecache.drop(path)
    return pagecache.resident_fraction(path)


def _fs_of(path: str) -> str:
    """Filesystem type of the mount holding `path` (from /proc/mounts)."""
    try:
        best, fs = "", "?"
        p = os.path.realpath(path)
        with open("/proc/mounts") as f:
            for line in f:
                parts = line.split()
                if len(parts) >= 3 and (p == parts[1] or p.startswith(parts[1].rstrip("/") + "/")):
                    if len(parts[1]) > len(best):
                        best, fs = parts[1], parts[2]
        return fs
    except OSError:
        return "?"


if __name__ == "__main__":
    main()

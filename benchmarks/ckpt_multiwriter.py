"""Eight ranks writing and restoring their Llama-3-8B ZeRO-1 train-state shards AT ONCE on one
node (BASELINE config 4's I/O pattern; SURVEY §5.4 item 4: concurrent writers sharing host DRAM,
the pinned rings and the disk).

Every rank holds exactly the shard a W-rank DistributedDataParallel(zero_stage=1) Llama-3-8B
job owns (checkpoint/sharded.py simulated_zero_ranges: the real bucket plan and ZeRO layout over
the model's parameter shapes) for the three fp32 kinds of the train state - master parameters,
AdamW exp_avg, exp_avg_sq - as FlatShardedTensor chunks of the torch-shaped tensors, so each
rank's file is its ~1/W of the 96 GB state.  The compute model is not instantiated (the I/O path
does not depend on it); shard contents are random.  All ranks then:
  1. dcp.save (collective: per-rank `__r_0.distcp` through the native engine - HBM snapshot,
     SDMA drain into the pinned ring, O_DIRECT writers - then rank 0's metadata commit),
  2. drop their file from the page cache (cold restore),
  3. dcp.load into fresh device buffers (each rank reads only its own chunks), verified bitwise.

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 benchmarks/ckpt_multiwriter.py [--layers 32]

On a one-GPU box all ranks share cuda:0 over gloo (8 x ~12 GB of HBM); on an 8-GPU node each
rank uses its own GPU.  When the node's free disk cannot hold the full state, the number of
decoder layers is reduced (reported as `layers`), never the per-rank write pattern.
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import sys
import tempfile
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--layers", type=int, default=0, help="decoder layers (0: the model's, reduced to fit the disk)")
    ap.add_argument("--dir", default=None)
    ap.add_argument("--disk-frac", type=float, default=0.8)
    ap.add_argument("--cpu", action="store_true", help="host tensors over gloo (plumbing test, e.g. llama3-tiny)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.cpu:
        ndev, dev, backend = 0, torch.device("cpu"), "gloo"
    else:
        ndev = torch.cuda.device_count()
        dev = torch.device("cuda", local % ndev)
        torch.cuda.set_device(dev)
        backend = "nccl" if ndev >= world else "gloo"
    sync = torch.cuda.synchronize if dev.type == "cuda" else (lambda: None)
    import datetime

    dist.init_process_group(backend, timeout=datetime.timedelta(seconds=600),
                            **({"device_id": dev} if backend == "nccl" else {}))

    from ray_torch_distributed_checkpoint_amd.checkpoint import dcp
    from ray_torch_distributed_checkpoint_amd.checkpoint.sharded import FlatShardedTensor, simulated_zero_ranges
    from ray_torch_distributed_checkpoint_amd.models import Llama, LlamaConfig
    from ray_torch_distributed_checkpoint_amd.utils import pagecache

    cfg = LlamaConfig.named(args.model)
    base = args.dir or os.environ.get("RTDC_BENCH_CKPT_DIR") or tempfile.gettempdir()
    free = shutil.disk_usage(base).free
    full_layers = cfg.n_layers

    def shapes_for(nl):
        cfg.n_layers = nl
        m = Llama(cfg, device="meta")
        cfg.n_layers = full_layers
        named = [(n, tuple(p.shape)) for n, p in m.named_parameters() if p.requires_grad]
        return list(reversed(named))  # the flat layout order DDP lays out (reverse registration)

    layers = args.layers or full_layers
    order = shapes_for(layers)
    total_bytes = 3 * 4 * sum(int(torch.Size(s).numel()) for _, s in order)
    while not args.layers and total_bytes > free * args.disk_frac and layers > 1:
        layers -= 1
        order = shapes_for(layers)
        total_bytes = 3 * 4 * sum(int(torch.Size(s).numel()) for _, s in order)

    numels = [int(torch.Size(s).numel()) for _, s in order]
    offs, ranges = simulated_zero_ranges(numels, world, 32.0)
    mine = ranges[rank]
    owned = sum(b - a for a, b in mine)
    g = torch.Generator(device=dev) if dev.type == "cuda" else torch.Generator()
    g.manual_seed(1000 + rank)

    def build(fill: bool):
        bufs = {k: torch.empty(owned, dtype=torch.float32, device=dev) for k in ("param", "exp_avg", "exp_avg_sq")}
        if fill:
            for b in bufs.values():
                b.normal_(generator=g)
        else:
            for b in bufs.values():
                b.zero_()
        sd = {"model": {}, "optim": {"state": {}}}
        # compact position of each owned flat range in this rank's buffers
        cpos, c = [], 0
        for a, b in mine:
            cpos.append(c)
            c += b - a
        covered = torch.zeros(owned, dtype=torch.bool, device=dev)
        for (name, shape), lo, n in zip(order, offs, numels):
            hi = lo + n
            per_rank = [[(max(lo, a) - lo, min(hi, b) - lo) for a, b in rr if max(lo, a) < min(hi, b)] for rr in ranges]
            vals = {}
            for k, buf in bufs.items():
                local_ = []
                for (a, b), cp in zip(mine, cpos):
                    s, e = max(lo, a), min(hi, b)
                    if s < e:
                        local_.append((s - lo, buf[cp + (s - a):cp + (e - a)]))
                        covered[cp + (s - a):cp + (e - a)] = True
                vals[k] = FlatShardedTensor(torch.Size(shape), torch.float32, local_, per_rank, rank)
            sd["model"][name] = vals["param"]
            sd["optim"]["state"][name] = {"exp_avg": vals["exp_avg"], "exp_avg_sq": vals["exp_avg_sq"]}
        if fill:  # the ZeRO bucket padding belongs to no parameter: never saved, kept at zero
            for b in bufs.values():
                b.masked_fill_(~covered, 0.0)
        return sd, bufs

    from bench import _checksum

    sd, bufs = build(True)
    sums = [_checksum(bufs[k]) for k in ("param", "exp_avg", "exp_avg_sq")]
    path = os.path.join(base, "rtdc_multiwriter_ckpt")
    if rank == 0:
        shutil.rmtree(path, ignore_errors=True)
        os.makedirs(path, exist_ok=True)
    dcp.prepare_async(sd)  # engine + snapshot arena (startup-time allocation)
    sync()
    dist.barrier()

    # ---- 1. every rank saves its shard at once
    t0 = time.perf_counter()
    h = dcp.async_save(sd, path)
    t_block = time.perf_counter() - t0
    h.wait()
    t_local = time.perf_counter() - t0
    dist.barrier()
    h._finish()
    dist.barrier()
    t_save = time.perf_counter() - t0

    # ---- 2. cold restore (the saved buffers and the snapshot arena are freed first: 8 ranks on
    # one GPU would otherwise hold three copies of their shard)
    from ray_torch_distributed_checkpoint_amd.checkpoint import snapshot

    del sd, bufs, h
    snapshot.clear()
    if dev.type == "cuda":
        torch.cuda.empty_cache()
    pagecache.drop(path)
    resident = pagecache.resident_fraction(path)
    sd2, bufs2 = build(False)
    sync()
    dist.barrier()
    t1 = time.perf_counter()
    dcp.load(sd2, path)
    sync()
    t_local_load = time.perf_counter() - t1
    dist.barrier()
    t_load = time.perf_counter() - t1
    ok = sums == [_checksum(bufs2[k]) for k in ("param", "exp_avg", "exp_avg_sq")]

    mine_bytes = owned * 4 * 3
    vals = torch.tensor([t_block, t_local, t_save, t_local_load, t_load, float(mine_bytes), 0.0 if ok else 1.0,
                         resident], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
    allv = [torch.zeros_like(vals) for _ in range(world)]
    dist.all_gather(allv, vals)
    if rank == 0:
        a = torch.stack(allv).cpu()
        tot = float(a[:, 5].sum())
        out = {
            "bench": "ckpt_multiwriter", "model": args.model, "layers": layers, "layers_full": full_layers,
            "world": world, "backend": backend, "gpus_visible": ndev,
            "layout": "ZeRO-1 owner chunks (simulated_zero_ranges: the real DDP bucket plan), fp32 param + exp_avg + exp_avg_sq",
            "per_rank_GB": [round(x / 1e9, 3) for x in a[:, 5].tolist()],
            "total_GB": round(tot / 1e9, 2),
            "save_blocking_s_max": round(float(a[:, 0].max()), 4),
            "save_local_durable_s": [round(x, 3) for x in a[:, 1].tolist()],
            "save_committed_s": round(float(a[:, 2].max()), 3),
            "save_aggregate_GBps": round(tot / float(a[:, 2].max()) / 1e9, 2),
            "restore_cold": bool(float(a[:, 7].max()) < 0.01), "restore_resident_frac_max": round(float(a[:, 7].max()), 4),
            "restore_local_s": [round(x, 3) for x in a[:, 3].tolist()],
            "restore_s": round(float(a[:, 4].max()), 3),
            "restore_aggregate_GBps": round(tot / float(a[:, 4].max()) / 1e9, 2),
            "save_plus_restore_s": round(float(a[:, 2].max() + a[:, 4].max()), 3),
            "verified_bitwise": bool(float(a[:, 6].max()) == 0.0),
            "fs": _fs_of(base), "free_disk_GB": round(free / 1e9, 1),
        }
        print(json.dumps(out), flush=True)
        shutil.rmtree(path, ignore_errors=True)
    dist.barrier()
    dist.destroy_process_group()


def _fs_of(path: str) -> str:
    best, fs = "", "?"
    p = os.path.realpath(path)
    with open("/proc/mounts") as f:
        for line in f:
            parts = line.split()
            if len(parts) >= 3 and (p == parts[1] or p.startswith(parts[1].rstrip("/") + "/")):
                if len(parts[1]) > len(best):
                    best, fs = parts[1], parts[2]
    return fs


if __name__ == "__main__":
    main()

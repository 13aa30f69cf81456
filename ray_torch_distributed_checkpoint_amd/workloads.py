"""The BASELINE bf16 data-parallel workloads as `TorchTrainer` per-worker loops with periodic
sharded asynchronous checkpoints and exact resume.

This is the reference's product - a per-worker loop that checkpoints and `report`s into
`RunConfig(storage_path)` and can be restored with `--from-run` (R/my_ray_module.py:115-213,
:253-264; R/train_flow.py:65-77) - applied to the BASELINE.json configs beyond the toy MLP:

  config 2  resnet18      DDP bf16, sharded DCP save every N steps
  config 3  gpt2-small    DDP, RCCL all-reduce overlapped with the async checkpoint write
  config 4  llama3-8b     sharded state_dict (per-rank `__<r>_0.distcp` shards, 288 GB sizing)
  config 5  any model     kill at step K (RTDC_FAIL_AT_STEP), restart / --from-run, bit-equal

(+ `gpt2-tiny`, `llama3-tiny`, `resnet18-tiny` with the same code paths for CPU/gloo tests.)

Every `ckpt_every_n_steps` steps the loop calls
    h = dcp.async_save(state, train.get_context().next_checkpoint_dir())
    train.report(metrics, checkpoint=Checkpoint.from_async_save(h))
which returns as soon as the HBM snapshot is enqueued: the native engine drains it through the
pinned ring while the next steps run, and the session commits `checkpoint_NNNNNN/`
(`.metadata` + one `__<rank>_0.distcp` per rank) in the background once every rank's shard is
durable; retention (`CheckpointConfig.num_to_keep`) applies on commit.

The checkpointed state is the full train state - model (incl. BatchNorm buffers), optimizer
(FQN-keyed, torch-compatible), step, epoch, sampler position, and every rank's CPU / device /
Philox / numpy RNG state - so a restart (`train.get_checkpoint()`, FailureConfig) or
`--from-run ... --resume_mode exact` continues with losses bit-identical to an uninterrupted
run (deterministic kernels, fixed bucket order).  `resume_mode="weights"` loads only the model
(the reference's warm start).

Data is synthetic and index-addressed (a sample is a pure function of its index), sharded by
`DistributedSampler`'s seed+epoch permutation contract, and generated on the device.
"""
from __future__ import annotations

import argparse
import json
import time
from dataclasses import asdict, dataclass
from typing import Optional

import numpy as np
import torch
import torch.distributed as dist

from . import ops
from . import train
from .checkpoint import dcp
from .checkpoint.state_dict import get_state_dict, set_state_dict
from .optim import FusedAdamW, FusedSGD
from .parallel.sampler import DistributedSampler
from .utils.profiling import phase


# ---------------------------------------------------------------------------------- config
@dataclass
class WorkloadConfig:
    model: str = "gpt2-tiny"
    steps: int = 20                       # total optimizer steps (global)
    batch_size_per_worker: Optional[int] = None
    seq_len: Optional[int] = None         # tokens (LMs) or image side (ResNet)
    lr: Optional[float] = None
    ckpt_every_n_steps: Optional[int] = None   # None -> CheckpointConfig.ckpt_every_n_steps
    report_every_n_steps: Optional[int] = None  # None -> ckpt interval
    seed: int = 1234
    dataset_size: int = 1 << 20
    resume_mode: str = "exact"            # exact | weights (for an explicit `checkpoint`)
    checkpoint: object = None             # upstream Checkpoint (--from-run / --from-task)
    async_checkpoint: Optional[bool] = None  # None -> CheckpointConfig.async_checkpoint
    num_classes: int = 10

    @classmethod
    def from_dict(cls, d: dict) -> "WorkloadConfig":
        known = {f for f in cls.__dataclass_fields__}
        return cls(**{k: v for k, v in d.items() if k in known})


_DEFAULTS = {
    # name prefix: (batch/worker, seq_len or image side, lr)
    "gpt2-tiny": (4, 64, 1e-3), "gpt2": (16, 1024, 6e-4),
    "llama3-tiny": (2, 64, 1e-3), "llama3": (1, 2048, 3e-4),
    "resnet18-tiny": (8, 32, 0.05), "resnet18": (256, 224, 0.1),
}


def _defaults(name: str):
    for k in sorted(_DEFAULTS, key=len, reverse=True):
        if name.startswith(k):
            return _DEFAULTS[k]
    raise ValueError(f"unknown workload model {name!r}")


# ---------------------------------------------------------------------------------- data
def _mix(x: torch.Tensor, seed: int) -> torch.Tensor:
    """Deterministic integer hash (values stay < 2^31: no signed overflow on any device)."""
    x = (x + (seed * 7919 + 1)) & 0x7FFFFFFF
    for _ in range(3):
        x = ((x ^ (x >> 13)) * 1103515245 + 12345) & 0x7FFFFFFF
    return x


class SyntheticTokens:
    """`n` sequences of `seq_len + 1` random tokens; sequence i is a function of (seed, i)."""

    def __init__(self, n: int, seq_len: int, vocab: int, seed: int = 0):
        self.n, self.seq_len, self.vocab, self.seed = n, seq_len, vocab, seed

    def __len__(self):
        return self.n

    def batch(self, idx: torch.Tensor):
        """(inputs, targets), contiguous [B, seq_len] int64.  On the GPU one native kernel
        (`data_ops.hip` synth_tokens) writes both; the CPU path is the same hash in ATen."""
        if idx.is_cuda:
            from .ops._ext import gpu_ext

            ids = idx.to(torch.int64).contiguous()
            B = ids.numel()
            inp = torch.empty((B, self.seq_len), dtype=torch.int64, device=idx.device)
            tgt = torch.empty_like(inp)
            gpu_ext().synth_tokens(ids, inp, tgt, self.vocab, self.seed * 7919 + 1)
            return inp, tgt
        pos = torch.arange(self.seq_len + 1, device=idx.device, dtype=torch.int64)
        tok = _mix(idx.to(torch.int64)[:, None] * (self.seq_len + 1) + pos, self.seed) % self.vocab
        return tok[:, :-1].contiguous(), tok[:, 1:].contiguous()


class SyntheticImages:
    """`n` labelled images; image i = prototype (i mod P) of a fixed pool, label = its class."""

    def __init__(self, n: int, hw: int, classes: int, device, seed: int = 0, pool: int = 64):
        g = torch.Generator().manual_seed(seed)
        self.n, self.classes = n, classes
        self.x = torch.randn(pool, 3, hw, hw, generator=g).to(device)
        self.y = (torch.arange(pool) % classes).to(device)

    def __len__(self):
        return self.n

    def batch(self, idx: torch.Tensor):
        j = idx % self.x.shape[0]
        return self.x.index_select(0, j), self.y.index_select(0, j)


class ShardedStream:
    """Batches of this rank's shard in sampler order with an exact, checkpointable position
    (epoch, pos): `DistributedSampler`'s seed+epoch permutation, strided by rank."""

    def __init__(self, dataset, batch: int, world: int, rank: int, seed: int, device):
        self.ds, self.B, self.device = dataset, batch, device
        self.sampler = DistributedSampler(dataset, num_replicas=world, rank=rank, shuffle=True, seed=seed,
                                          drop_last=True)
        self.epoch, self.pos, self._ids, self._ids_epoch = 0, 0, None, None

    def _epoch_ids(self):
        if self._ids_epoch != self.epoch:
            self.sampler.set_epoch(self.epoch)
            self._ids = torch.tensor(self.sampler.indices(), dtype=torch.int64, device=self.device)
            self._ids_epoch = self.epoch
        return self._ids

    def next(self):
        ids = self._epoch_ids()
        if self.pos + self.B > ids.numel():
            self.epoch, self.pos = self.epoch + 1, 0
            ids = self._epoch_ids()
        j = ids[self.pos:self.pos + self.B]
        self.pos += self.B
        return self.ds.batch(j)

    def state_dict(self):
        return {"epoch": self.epoch, "pos": self.pos}

    def load_state_dict(self, sd):
        self.epoch, self.pos = int(sd["epoch"]), int(sd["pos"])


# ---------------------------------------------------------------------------------- model
@dataclass
class Workload:
    model: torch.nn.Module
    optimizer: torch.optim.Optimizer
    data: object
    batch: int
    seq_len: int
    tokens_per_sample: int = 0
    flops_per_sample: float = 0.0
    loss_fn: object = None


def build(cfg: WorkloadConfig, device) -> Workload:
    """Model (same random init on every rank: seeded), optimizer, synthetic dataset."""
    B0, S0, lr0 = _defaults(cfg.model)
    B = cfg.batch_size_per_worker or B0
    S = cfg.seq_len or S0
    lr = cfg.lr or lr0
    torch.manual_seed(cfg.seed)
    name = cfg.model
    if name.startswith("resnet18"):
        from .models import ResNet18

        # "-tiny" = the full network on 32x32 images (the GEMM tiles need >= 64 channels)
        model = ResNet18(num_classes=cfg.num_classes).to(device)
        opt = FusedSGD(model.parameters(), lr=lr, momentum=0.9, weight_decay=5e-5)
        data = SyntheticImages(cfg.dataset_size, S, cfg.num_classes, device, seed=cfg.seed)
        return Workload(model, opt, data, B, S, 0, model.flops_per_sample(S),
                        lambda net, x, y: ops.cross_entropy(net(x), y))
    if name.startswith("llama"):
        from .models import Llama, LlamaConfig

        mc = LlamaConfig.named(name)
        S = min(S, mc.max_seq_len)
        model = Llama(mc, device=device)
    elif name.startswith("gpt2"):
        from .models import GPT2, GPT2Config

        mc = GPT2Config.named(name)
        S = min(S, mc.n_positions)
        model = GPT2(mc).to(device)
    else:
        raise ValueError(f"unknown workload model {name!r}")
    opt = FusedAdamW(model.parameters(), lr=lr, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.1)
    data = SyntheticTokens(cfg.dataset_size, S, mc.vocab_size, seed=cfg.seed)
    return Workload(model, opt, data, B, S, S, model.flops_per_token(S) * S, lambda net, x, y: net(x, y))


# ---------------------------------------------------------------------------------- RNG state
def _pack(obj) -> bytes:
    """Deterministic byte encoding of a nested dict of tensors / JSON scalars (a JSON header +
    raw tensor bytes): equal states give equal bytes on every rank, so the replicated,
    deduplicated sharded save stores the value once and any rank may be its writer."""
    tensors = []

    def enc(o):
        if torch.is_tensor(o):
            tensors.append(o.detach().cpu().contiguous())
            return {"__t": len(tensors) - 1, "dtype": str(o.dtype).replace("torch.", ""), "shape": list(o.shape)}
        if isinstance(o, dict):
            return {str(k): enc(v) for k, v in o.items()}
        return o

    head = json.dumps(enc(obj), sort_keys=True).encode()
    body = b"".join(t.reshape(-1).view(torch.uint8).numpy().tobytes() for t in tensors)
    return len(head).to_bytes(8, "little") + head + body


def _unpack(blob: bytes):
    n = int.from_bytes(blob[:8], "little")
    head = json.loads(blob[8:8 + n].decode())
    body = memoryview(blob)[8 + n:]
    metas = []

    def walk(o):
        if isinstance(o, dict):
            if "__t" in o:
                metas.append(o)
            else:
                for v in o.values():
                    walk(v)

    walk(head)
    offs, at = {}, 0
    for m in sorted(metas, key=lambda m: m["__t"]):
        dt = getattr(torch, m["dtype"])
        nb = int(np.prod(m["shape"], dtype=np.int64)) * torch.empty((), dtype=dt).element_size()
        offs[m["__t"]] = (at, nb, dt, m["shape"])
        at += nb

    def dec(o):
        if isinstance(o, dict):
            if "__t" in o:
                off, nb, dt, shape = offs[o["__t"]]
                raw = torch.frombuffer(bytearray(body[off:off + nb]), dtype=torch.uint8)
                return raw.view(dt).reshape(shape)
            return {k: dec(v) for k, v in o.items()}
        return o

    return dec(head)


def _rng_blob(device) -> bytes:
    """Every rank's RNG states (CPU, device, Philox dropout stream, numpy) gathered to all
    ranks and packed into one `bytes` value (identical on every rank)."""
    _, keys, pos, has_gauss, gauss = np.random.get_state()
    mine = {"torch_cpu": torch.get_rng_state(), "philox": ops.default_stream().state_dict(),
            "numpy": {"keys": torch.from_numpy(keys.astype(np.int64)), "pos": int(pos),
                      "has_gauss": int(has_gauss), "gauss": float(gauss)}}
    if device.type == "cuda":
        mine["torch_cuda"] = torch.cuda.get_rng_state(device)
    world = dist.get_world_size() if dist.is_initialized() else 1
    parts = [None] * world
    if world > 1:
        dist.all_gather_object(parts, mine)
    else:
        parts = [mine]
    return _pack({f"rank{r}": p for r, p in enumerate(parts)})


def _set_rng(blob: bytes, rank: int, device) -> bool:
    if not blob:
        return False
    st = _unpack(blob).get(f"rank{rank}")
    if st is None:  # resumed at a different world size: this rank has no recorded stream
        return False
    torch.set_rng_state(st["torch_cpu"].cpu())
    ops.default_stream().load_state_dict(st["philox"])
    n = st["numpy"]
    np.random.set_state(("MT19937", n["keys"].cpu().numpy().astype(np.uint32), n["pos"], n["has_gauss"],
                         n["gauss"]))
    if device.type == "cuda" and "torch_cuda" in st:
        torch.cuda.set_rng_state(st["torch_cuda"].cpu(), device)
    return True


# ---------------------------------------------------------------------------------- loop
def _unwrap(m):
    return m.module if hasattr(m, "module") else m


def _train_state(core, opt, stream, step, rng: bytes):
    msd, osd = get_state_dict(core, opt)
    return {"model": msd, "optim": osd,
            "trainer": {"step": int(step), "epoch": stream.epoch, "pos": stream.pos, "rng": rng}}


def restore(core, opt, stream, checkpoint, mode: str, device, rank: int) -> int:
    """Load a sharded checkpoint into the live model/optimizer; returns the step to resume at
    (0 for a weights-only warm start)."""
    with checkpoint.as_directory() as path:
        if mode == "weights":
            msd, _ = get_state_dict(core, None)
            sd = dcp.load({"model": msd}, path)
            set_state_dict(core, None, model_state_dict=sd["model"])
            step = 0
        else:
            sd = _train_state(core, opt, stream, 0, b"")
            dcp.load(sd, path)
            set_state_dict(core, opt, model_state_dict=sd["model"], optim_state_dict=sd["optim"])
            tr = sd["trainer"]
            stream.load_state_dict(tr)
            if not _set_rng(tr["rng"], rank, device):
                torch.manual_seed(int(tr["step"]) * 1000003 + rank)
            step = int(tr["step"])
    sp = getattr(opt, "flat_space", None) or getattr(core.parameters().__next__(), "_rtdc_space", None)
    if sp is not None:
        sp.refresh_shadows()  # bf16 compute copies of the restored fp32 masters
    return step


def train_loop_per_worker(config: dict):
    cfg = WorkloadConfig.from_dict(config)
    ctx = train.get_context()
    ccfg = ctx.get_checkpoint_config()
    every = cfg.ckpt_every_n_steps or ccfg.ckpt_every_n_steps
    report_every = cfg.report_every_n_steps or every or max(1, cfg.steps)
    use_async = ccfg.async_checkpoint if cfg.async_checkpoint is None else cfg.async_checkpoint
    dev = train.torch.get_device()
    world, rank = ctx.get_world_size(), ctx.get_world_rank()
    train.torch.enable_reproducibility(cfg.seed)

    wl = build(cfg, dev)
    # fused optimizers wait for the deferred last bucket themselves (DDP defer_tail_to_optimizer)
    net = train.torch.prepare_model(wl.model, parallel_strategy_kwargs={"defer_tail_to_optimizer": True})
    core, opt = _unwrap(net), wl.optimizer
    stream = ShardedStream(wl.data, wl.batch, world, rank, cfg.seed, dev)

    start = 0
    restart = train.get_checkpoint()  # set when the trainer restarted this gang after a failure
    if restart is not None:
        start = restore(core, opt, stream, restart, "exact", dev, rank)
        print(f"[workload] rank {rank}: restarted from {restart.path} at step {start}", flush=True)
    elif cfg.checkpoint is not None:
        start = restore(core, opt, stream, cfg.checkpoint, cfg.resume_mode, dev, rank)
        print(f"[workload] rank {rank}: resumed ({cfg.resume_mode}) from {cfg.checkpoint.path} at step {start}",
              flush=True)

    pending = None  # this rank's in-flight async save (at most one: bounded snapshot memory)
    losses = []
    t_last, n_last = time.perf_counter(), 0
    for step in range(start, cfg.steps):
        train.report_progress(step)
        x, y = stream.next()
        with phase("fwd"):
            loss = wl.loss_fn(net, x, y)
        with phase("bwd"):
            loss.backward()
        with phase("opt"):
            opt.step()
            opt.zero_grad(set_to_none=True)
        losses.append(loss.detach())
        n_last += 1
        done = step + 1
        do_ckpt = bool(every) and (done % every == 0 or done == cfg.steps)
        if not (do_ckpt or done % report_every == 0 or done == cfg.steps):
            continue
        vals = torch.stack(losses).float().tolist()  # the one host sync per report
        dt = time.perf_counter() - t_last
        metrics = {"step": done, "loss": vals[-1], "losses": vals, "epoch": stream.epoch,
                   "samples_per_s": round(n_last * wl.batch * world / max(dt, 1e-9), 3)}
        if wl.tokens_per_sample:
            metrics["tokens_per_s"] = round(metrics["samples_per_s"] * wl.tokens_per_sample, 1)
        losses, n_last = [], 0
        ck = None
        if do_ckpt:
            with phase("ckpt"):
                if pending is not None:
                    pending.wait()
                state = _train_state(core, opt, stream, done, _rng_blob(dev))
                if use_async:
                    pending = dcp.async_save(state, ctx.next_checkpoint_dir())
                    ck = train.Checkpoint.from_async_save(pending)
                    metrics["ckpt_snapshot_s"] = round(pending.t_return, 6)
                else:
                    t0 = time.perf_counter()
                    d = ctx.next_checkpoint_dir()
                    dcp.save(state, d)
                    ck = train.Checkpoint.from_directory(d)
                    metrics["ckpt_save_s"] = round(time.perf_counter() - t0, 6)
        train.report(metrics, checkpoint=ck)
        t_last = time.perf_counter()
    if pending is not None:
        pending.wait()


# ---------------------------------------------------------------------------------- driver
def default_zero_stage(model: str, world: int) -> int:
    """ZeRO-1 by default where the replicated optimizer dominates: Llama-3-8B's AdamW streams
    ~241 GB per step (40 of 147 ms on one MI355X); sharded over W ranks each moves 1/W of it,
    and the state checkpoint is written as owner shards with no all-gather.  The small models
    keep the replicated step (their update is < 1 ms)."""
    return 1 if model.startswith("llama") and world > 1 else 0


def train_workload(model: str = "gpt2-tiny", steps: int = 20, num_workers: int = 1, use_gpu: bool = False,
                   batch_size_per_worker: int | None = None, seq_len: int | None = None, lr: float | None = None,
                   ckpt_every_n_steps: int | None = 5, num_checkpoints_to_keep: int | None = 2,
                   checkpoint_storage_path: str | None = None, checkpoint=None, resume_mode: str = "exact",
                   max_failures: int = 0, seed: int = 1234, grad_comm_dtype: str = "fp32",
                   bucket_cap_mb: float = 32.0, zero_stage: int = -1, progress_timeout_s: float | None = 300.0,
                   dataset_size: int = 1 << 20, name: str | None = None, verbose: int = 1,
                   report_every_n_steps: int | None = None):
    """`train_fashion_mnist`'s counterpart for the bf16 workloads (R/my_ray_module.py:216-251).
    zero_stage -1: `default_zero_stage(model, num_workers)`."""
    if zero_stage < 0:
        zero_stage = default_zero_stage(model, num_workers)
    cfg = WorkloadConfig(model=model, steps=steps, batch_size_per_worker=batch_size_per_worker, seq_len=seq_len,
                         lr=lr, ckpt_every_n_steps=ckpt_every_n_steps, seed=seed, resume_mode=resume_mode,
                         checkpoint=checkpoint, dataset_size=dataset_size, report_every_n_steps=report_every_n_steps)
    run_config = train.RunConfig(
        name=name, storage_path=checkpoint_storage_path, verbose=verbose,
        checkpoint_config=train.CheckpointConfig(num_to_keep=num_checkpoints_to_keep,
                                                 ckpt_every_n_steps=ckpt_every_n_steps),
        failure_config=train.FailureConfig(max_failures=max_failures),
        progress_timeout_s=progress_timeout_s)
    trainer = train.TorchTrainer(
        train_loop_per_worker, train_loop_config={k: v for k, v in asdict(cfg).items() if v is not None},
        scaling_config=train.ScalingConfig(num_workers=num_workers, use_gpu=use_gpu),
        torch_config=train.TorchConfig(grad_comm_dtype=grad_comm_dtype, bucket_cap_mb=bucket_cap_mb,
                                       zero_stage=zero_stage),
        run_config=run_config)
    return trainer.fit()


def main(argv=None):
    ap = argparse.ArgumentParser(description="bf16 DDP workload with sharded async checkpoints")
    ap.add_argument("--model", default="gpt2-tiny")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--num-workers", type=int, default=1)
    ap.add_argument("--batch", type=int, default=None)
    ap.add_argument("--seq-len", type=int, default=None)
    ap.add_argument("--ckpt-every", type=int, default=5)
    ap.add_argument("--keep", type=int, default=2)
    ap.add_argument("--storage", default=None)
    ap.add_argument("--max-failures", type=int, default=0)
    ap.add_argument("--grad-comm-dtype", default="fp32")
    ap.add_argument("--zero-stage", type=int, default=-1, choices=[-1, 0, 1],
                    help="-1: ZeRO-1 for llama* at more than one worker, else replicated")
    ap.add_argument("--cpu", action="store_true")
    a = ap.parse_args(argv)
    use_gpu = torch.cuda.is_available() and not a.cpu
    res = train_workload(a.model, a.steps, a.num_workers, use_gpu, a.batch, a.seq_len, None, a.ckpt_every, a.keep,
                         a.storage, max_failures=a.max_failures, grad_comm_dtype=a.grad_comm_dtype,
                         zero_stage=a.zero_stage)
    print(res)


if __name__ == "__main__":
    main()

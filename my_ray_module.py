"""The reference workload (R/my_ray_module.py) on the MI355X-native framework.

Same public surface - `get_dataloaders`, `get_labels_map`, `NeuralNetwork`,
`train_func_per_worker`, `train_fashion_mnist`, `set_weights_from_checkpoint`,
`TorchPredictor`, `BEST_CHECKPOINT_FILENAME`, `LATEST_CHECKPOINT_FILENAME` - and the same
behaviour (per-epoch `latest_model.pt` + `best_model.pt` on improvement with keys `epoch,
model_state_dict, optimizer_state_dict, val_losses, val_accuracy`; report `{val_loss,
accuracy}`; resume = warm start from `best_model.pt` with the `module.` prefix stripped),
with these deliberate fixes of reference quirks:

* validation metrics are all-reduced over ranks (the reference reports rank 0's shard),
  so every rank takes the same best-checkpoint decision;
* only rank 0 writes the checkpoint files (the reference has every rank write identical
  names into one directory); writes go through the native engine (`torch.load`-compatible);
* `latest_model.pt` carries the full training state (optimizer, epoch, sampler position,
  CPU/GPU/Philox RNG) so `resume_mode="exact"` continues bit-exactly; the default
  `resume_mode="best_weights"` keeps the reference's warm-start semantics, and falls back to
  `latest_model.pt` when the newest checkpoint has no `best_model.pt` (reference crash B.1);
* one device->host sync per epoch for the metrics (the reference does two per val batch);
* on one GPU the whole training step (zero_grad, forward, CE, backward, fused SGD) is
  captured once into a hipGraph and replayed per batch (`utils.graphs.CapturedStep`): the
  B=16..32 toy step is launch-bound, one graph launch replaces ~15 kernel launches;
* observability: roctx ranges (`fwd`/`bwd`/`opt`/`val`/`ckpt`, visible in rocprofv3
  --marker-trace), a step counter for the supervisor's stall detection, and per-epoch
  `train_samples_per_s` / `epoch_s` / checkpoint seconds next to `val_loss` / `accuracy`.
"""
from __future__ import annotations

import contextlib
import os
import tempfile
import time
from typing import Dict

import numpy as np
import torch
import torch.distributed as dist

from ray_torch_distributed_checkpoint_amd import ops
from ray_torch_distributed_checkpoint_amd import train
from ray_torch_distributed_checkpoint_amd.checkpoint import torchsave
from ray_torch_distributed_checkpoint_amd.data import get_dataloaders as _get_dataloaders
from ray_torch_distributed_checkpoint_amd.data import get_labels_map as _get_labels_map
from ray_torch_distributed_checkpoint_amd.models import NeuralNetwork as _NeuralNetwork
from ray_torch_distributed_checkpoint_amd.optim import FusedSGD
from ray_torch_distributed_checkpoint_amd.train import (Checkpoint, CheckpointConfig, RunConfig, ScalingConfig,
                                                        TorchTrainer)
from ray_torch_distributed_checkpoint_amd.utils.graphs import CapturedStep
from ray_torch_distributed_checkpoint_amd.utils.profiling import phase

BEST_CHECKPOINT_FILENAME = "best_model.pt"
LATEST_CHECKPOINT_FILENAME = "latest_model.pt"

NeuralNetwork = _NeuralNetwork


def get_dataloaders(batch_size, val_only=False, as_ray_ds=False):
    return _get_dataloaders(batch_size, val_only=val_only, as_ray_ds=as_ray_ds)


def get_labels_map():
    return _get_labels_map()


def _rng_state(dev):
    _, keys, pos, has_gauss, gauss = np.random.get_state()
    st = {"torch_cpu": torch.get_rng_state(), "philox": ops.default_stream().state_dict(),
          "numpy": {"keys": torch.from_numpy(keys.astype(np.int64)), "pos": int(pos), "has_gauss": int(has_gauss),
                    "gauss": float(gauss)}}
    if dev.type == "cuda":
        st["torch_cuda"] = torch.cuda.get_rng_state(dev)
    return st


def _set_rng_state(st, dev):
    # the checkpoint may have been loaded with map_location=<gpu>: RNG states live on the host
    torch.set_rng_state(st["torch_cpu"].cpu())
    ops.default_stream().load_state_dict(st["philox"])
    if "numpy" in st:
        n = st["numpy"]
        np.random.set_state(("MT19937", n["keys"].cpu().numpy().astype(np.uint32), n["pos"], n["has_gauss"],
                             n["gauss"]))
    if dev.type == "cuda" and "torch_cuda" in st:
        torch.cuda.set_rng_state(st["torch_cuda"].cpu(), dev)


def raise_if_poisoned(model) -> None:
    """After a replayed (hipGraph) step: no host code runs inside a replay, so a P2P all-reduce
    that timed out waiting for a late peer has only NaN-poisoned its bucket and set the error
    word - the fused optimizer kernel read it and skipped the update on the device
    (kernels/optim.hip comm_poisoned).  Fail the attempt here, before anything reports or
    checkpoints that step."""
    p2p = getattr(model, "p2p", None)
    if p2p is not None and p2p.error():
        raise RuntimeError("P2P all-reduce timed out waiting for a peer rank during a captured step "
                           "(gradients poisoned with NaN, update skipped)")


def train_func_per_worker(config: Dict):
    lr = config["lr"]
    epochs = config["epochs"]
    batch_size = config["batch_size_per_worker"]
    checkpoint = config.get("checkpoint")
    resume_mode = config.get("resume_mode", "best_weights")
    restart_ckpt = train.get_checkpoint()  # set when the trainer restarted us after a failure
    if restart_ckpt is not None and (checkpoint is None or restart_ckpt.path != checkpoint.path):
        checkpoint, resume_mode = restart_ckpt, "exact"
    seed = config.get("seed")
    device = train.torch.get_device()
    ctx = train.get_context()
    world, rank = ctx.get_world_size(), ctx.get_world_rank()
    if seed is not None:
        train.torch.enable_reproducibility(int(seed))

    print("[my_ray_module] Preparing distributed data loaders...")
    train_dataloader, val_dataloader = get_dataloaders(batch_size=batch_size)
    train_dataloader = train.torch.prepare_data_loader(train_dataloader)
    val_dataloader = train.torch.prepare_data_loader(val_dataloader)

    model = NeuralNetwork()
    start_epoch = 0
    resume_state = None
    if checkpoint is not None:
        print(f"[my_ray_module] Resuming from checkpoint at {checkpoint.path}.")
        if resume_mode == "exact":
            resume_state = load_latest_state(checkpoint, device)
            model.load_state_dict(_strip(resume_state["model_state_dict"]))
        else:
            set_weights_from_checkpoint(model, checkpoint, device)
    model = train.torch.prepare_model(model)
    print("[my_ray_module] Model on-device. Training model...")

    best_val_loss = float("inf")
    val_losses, val_acc = [], []
    optimizer = FusedSGD(model.parameters(), lr=lr, momentum=0.9)
    if resume_state is not None:
        optimizer.load_state_dict(resume_state["optimizer_state_dict"])
        val_losses = list(resume_state["val_losses"])
        val_acc = list(resume_state["val_accuracy"])
        best_val_loss = float(resume_state.get("best_val_loss", min(val_losses) if val_losses else float("inf")))
        start_epoch = int(resume_state["epoch"]) + 1
        if "rng" in resume_state:
            _set_rng_state(resume_state["rng"], device)

    # hipGraph-captured step (every batch full): static input tensors the loader's batches are
    # copied into, one graph launch per step.  With several workers the step includes the
    # gradient all-reduce, so it is captured only when every bucket goes through the one-shot
    # P2P all-reduce (device-resident epochs: graph-capturable, parallel/p2p.py) - the
    # reference's own 2-worker config (R/train_flow.py:17-18) with its 1-2 MB buckets.
    sampler = getattr(train_dataloader, "sampler", None)
    n_train = len(sampler) if (world > 1 and sampler is not None) else (
        len(train_dataloader.dataset) if hasattr(train_dataloader, "dataset") else 0)
    captured = None
    use_graph = (device.type == "cuda" and config.get("hipgraph", True) and n_train > 0
                 and n_train % batch_size == 0 and (world == 1 or _all_buckets_p2p(model)))
    if use_graph:
        from ray_torch_distributed_checkpoint_amd.ops.streams import side_stream

        side = side_stream(device, "capture")
        sx = torch.zeros((batch_size, 1, 28, 28), device=device)
        sy = torch.zeros((batch_size,), dtype=torch.int64, device=device)

        def graph_step():
            optimizer.zero_grad()
            loss_ = ops.cross_entropy(model(sx), sy)
            loss_.backward()
            optimizer.step()
            return loss_

    step_no = 0
    t0_full = time.time()
    for epoch in range(start_epoch, epochs):
        t0 = time.time()
        if world > 1:
            train_dataloader.sampler.set_epoch(epoch)
        model.train()
        nseen = 0
        for X, y in train_dataloader:
            train.report_progress(step_no)
            step_no += 1
            nseen += y.shape[0]
            if use_graph and step_no > 2:
                # the first steps ran eagerly (lazy optimizer state, workspaces); from here one
                # graph launch per step - capture records without executing, then replays
                sx.copy_(X.view_as(sx))
                sy.copy_(y)
                if captured is None:
                    captured = CapturedStep(graph_step, warmup=0)
                with phase("step"):
                    captured.replay()
                if world > 1:
                    raise_if_poisoned(model)
                continue
            # before a capture, run the eager steps on a side stream (as CapturedStep's warm-up
            # does): autograd's AccumulateGrad nodes must not belong to the default stream
            # when the graph is recorded
            warm = use_graph and captured is None
            if warm:
                side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side) if warm else contextlib.nullcontext():
                with phase("fwd"):
                    pred = model(X)
                    loss = ops.cross_entropy(pred, y)
                optimizer.zero_grad()
                with phase("bwd"):
                    loss.backward()
                with phase("opt"):
                    optimizer.step()
            if warm:
                torch.cuda.current_stream().wait_stream(side)
            del pred, loss
        train_time = time.time() - t0

        model.eval()
        tot_loss = torch.zeros((), device=device)
        tot_correct = torch.zeros((), device=device, dtype=torch.int64)
        nb = 0
        nrows = 0
        with torch.no_grad():
            for X, y in val_dataloader:
                pred = model(X)
                ls, nc = ops.xent_metrics(pred, y)
                tot_loss += ls / y.shape[0]  # mean-of-batch-means like the reference
                tot_correct += nc
                nb += 1
                nrows += y.shape[0]
        stats = torch.stack([tot_loss.double(), tot_correct.double(),
                             torch.tensor(float(nb), device=device, dtype=torch.float64),
                             torch.tensor(float(nrows), device=device, dtype=torch.float64)])
        if world > 1:
            dist.all_reduce(stats)
        s = stats.tolist()
        val_loss = s[0] / s[2]
        accuracy = s[1] / s[3]
        val_losses.append(val_loss)
        val_acc.append(accuracy)

        checkpoint_dir = None
        if rank == 0:
            checkpoint_dir = tempfile.mkdtemp(prefix="rtdc_ckpt_")
            base = {
                "epoch": epoch,
                "model_state_dict": model.state_dict(),
                "optimizer_state_dict": optimizer.state_dict(),
                "val_losses": val_losses,
                "val_accuracy": val_acc,
            }
            full = dict(base, best_val_loss=min(best_val_loss, val_loss), rng=_rng_state(device))
            torchsave.save(full, os.path.join(checkpoint_dir, LATEST_CHECKPOINT_FILENAME))
        if val_loss < best_val_loss:
            best_val_loss = val_loss
            if rank == 0:
                torchsave.save(base, os.path.join(checkpoint_dir, BEST_CHECKPOINT_FILENAME))
        ckpt = Checkpoint.from_directory(checkpoint_dir) if checkpoint_dir else None
        train.report({"val_loss": val_loss, "accuracy": accuracy, "epoch": epoch, "epoch_s": round(time.time() - t0, 4),
                      "train_samples_per_s": round(nseen * world / max(train_time, 1e-9), 1)}, checkpoint=ckpt)
        if checkpoint_dir:
            import shutil

            shutil.rmtree(checkpoint_dir, ignore_errors=True)  # reference leaks its mkdtemp dirs
        tf = time.time()
        print(f"[my_ray_module] Model on-device. Last epoch took {round((tf - t0) / 60, 3)} minutes. Training model...")

    if captured is not None:
        captured.close()
    tf_full = time.time()
    print(f"[my_ray_module] Training completed in {round((tf_full - t0_full) / 60, 3)} minutes!")


def _all_buckets_p2p(net) -> bool:
    eng = getattr(net, "_engine", None)
    return getattr(net, "p2p", None) is not None and eng is not None and all(eng.p2p_buckets())


def train_fashion_mnist(
    num_workers=1,
    use_gpu=False,
    global_batch_size=32,
    learning_rate=1e-3,
    epochs=10,
    num_checkpoints_to_keep=2,
    checkpoint_storage_path=None,
    checkpoint=None,
    resume_mode="best_weights",
    max_failures=0,
    seed=None,
    hipgraph=True,
):
    train_config = {
        "lr": learning_rate,
        "epochs": epochs,
        "batch_size_per_worker": global_batch_size // num_workers,
        "resume_mode": resume_mode,
        "hipgraph": hipgraph,
    }
    if seed is not None:
        train_config["seed"] = seed
    if checkpoint is not None:
        train_config["checkpoint"] = checkpoint
    run_config = RunConfig(
        checkpoint_config=CheckpointConfig(num_to_keep=num_checkpoints_to_keep),
        storage_path=checkpoint_storage_path,
        verbose=1,
        failure_config=train.FailureConfig(max_failures=max_failures),
    )
    scaling_config = ScalingConfig(num_workers=num_workers, use_gpu=use_gpu)
    # one node, GPUs: the MLP's two 1-2 MB gradient buckets are latency-bound on a ring, so they
    # take the one-shot hipIpc all-reduce over xGMI (which also lets the step be graph-captured)
    torch_config = train.TorchConfig(p2p_max_kb=4096.0 if use_gpu and 1 < num_workers <= 8 else 0.0)
    trainer = TorchTrainer(
        train_loop_per_worker=train_func_per_worker,
        train_loop_config=train_config,
        scaling_config=scaling_config,
        run_config=run_config,
        torch_config=torch_config,
    )
    return trainer.fit()


def _strip(sd):
    return {k.replace("module.", ""): v for k, v in sd.items()}


def load_latest_state(checkpoint, device):
    with checkpoint.as_directory() as checkpoint_dir:
        return torch.load(os.path.join(checkpoint_dir, LATEST_CHECKPOINT_FILENAME), map_location=device,
                          weights_only=True)


def set_weights_from_checkpoint(model_structure, checkpoint, device):
    with checkpoint.as_directory() as checkpoint_dir:
        path = os.path.join(checkpoint_dir, BEST_CHECKPOINT_FILENAME)
        if not os.path.exists(path):
            path = os.path.join(checkpoint_dir, LATEST_CHECKPOINT_FILENAME)
        checkpoint_dict = torch.load(path, map_location=device, weights_only=True)
        model_structure.load_state_dict(_strip(checkpoint_dict["model_state_dict"]))


class TorchPredictor:
    """Reference predictor (R/my_ray_module.py:266-284).  `__call__` keeps the numpy batch
    contract; `predict_tensors` is the device-side entry the data pipeline uses on a GPU
    (pinned double-buffered input, outputs kept on the device until one final D2H)."""

    input_column = "features"

    def __init__(self, checkpoint: Checkpoint, cpu_only=False, device=None):
        if device is not None:
            self.device = torch.device(device)
        else:
            self.device = torch.device("cpu") if cpu_only else torch.device("cuda")
        self.model = NeuralNetwork()
        set_weights_from_checkpoint(model_structure=self.model, checkpoint=checkpoint, device=self.device)
        self.model.to(self.device)
        self.model.eval()

    @torch.inference_mode()
    def predict_tensors(self, features: torch.Tensor) -> Dict[str, torch.Tensor]:
        if features.dim() == 5 and features.shape[0] == 1:
            features = features.squeeze(0)
        logits = self.model(features)
        return {"logits": logits, "predicted_values": logits.argmax(dim=1)}

    def __call__(self, batch: Dict[str, np.ndarray]) -> Dict[str, np.ndarray]:
        features = batch["features"]
        if features.ndim == 5 and features.shape[0] == 1:
            features = features.squeeze(0)
        tensor = torch.as_tensor(features, dtype=torch.float32)
        if self.device.type == "cuda":
            tensor = tensor.pin_memory().to(self.device, non_blocking=True)
        with torch.inference_mode():
            logits = self.model(tensor).cpu().numpy().astype(np.float32)
            predicted_values = logits.argmax(axis=1)
        return {"logits": logits, "predicted_values": predicted_values}


if __name__ == "__main__":
    train_fashion_mnist(num_workers=min(4, max(1, torch.cuda.device_count())), use_gpu=torch.cuda.is_available())

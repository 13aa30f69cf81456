"""Multi-GPU test matrix: one rank per device over RCCL, world = torch.cuda.device_count() (2..8).

Every distributed path of the framework, with real devices and real RCCL (SURVEY §2.3, §2.6;
reference: the DDP wrap at R/my_ray_module.py:135 over the 2-worker ScalingConfig of
R/train_flow.py:17-18,63, per-worker batch global // N at R/my_ray_module.py:230):

* DDP gradients (native bucket engine, fp32 and bf16 communication) equal the single-process
  gradient of the concatenated batch, identically on every rank;
* ZeRO-1 (reduce-scatter of gradient buckets, owned-shard fused AdamW, parameter all-gather)
  equals the replicated optimizer;
* the one-shot hipIpc P2P all-reduce (parallel/p2p.py) over xGMI: bitwise equal to the RCCL
  all-reduce on exactly representable sums, within fp32 rounding otherwise, bitwise identical
  on every rank; DDP buckets routed over it match the RCCL bucket path;
* an async sharded DCP save of the DDP train state by N ranks restores bitwise at N ranks and
  reshards to N/2 ranks; a ZeRO-1 sharded save (each rank writes only its optimizer shards)
  restores bitwise at N;
* a trainer run with N GPU workers killed at step K restarts from the latest committed
  checkpoint with bit-equal losses.

The "rccl" cases skip on a one-GPU box.  The "gloo" cases run the same worker code with two
processes sharing cuda:0 over gloo - the stand-in that keeps this matrix exercised on one GPU.
"""
import hashlib
import json
import os
import socket
import sys
import traceback

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

pytestmark = pytest.mark.gpu

NGPU = torch.cuda.device_count() if torch.cuda.is_available() else 0
WORLD = min(NGPU, 8)
B, T = 2, 64
needs_multi = pytest.mark.skipif(NGPU < 2, reason="one rank per GPU needs >= 2 GPUs")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _model(dev, seed=0):
    from ray_torch_distributed_checkpoint_amd.models import GPT2, GPT2Config

    torch.manual_seed(seed)
    return GPT2(GPT2Config.named("gpt2-tiny")).to(dev)


def _batch(world, dev, salt=7):
    g = torch.Generator().manual_seed(salt)
    return torch.randint(0, 1000, (world * B, T + 1), generator=g).to(dev)


def _digest(t: torch.Tensor) -> str:
    return hashlib.sha1(t.detach().contiguous().cpu().view(torch.uint8).numpy().tobytes()).hexdigest()


def _state_digests(model, opt) -> dict:
    out = {"p." + n: _digest(p) for n, p in model.named_parameters()}
    for k, st in opt.state_dict()["state"].items():
        for n, v in st.items():
            if torch.is_tensor(v) and v.dim() > 0:
                out[f"o.{k}.{n}"] = _digest(v)
    return out


# ------------------------------------------------------------------------------ scenarios
def _sc_ddp(rank, world, dev):
    from ray_torch_distributed_checkpoint_amd.parallel.ddp import DistributedDataParallel

    out = {}
    for comm in ("fp32", "bf16"):
        model = _model(dev)
        net = DistributedDataParallel(model, grad_comm_dtype=comm, bucket_cap_mb=0.25, first_bucket_mb=0.05)
        data = _batch(world, dev)[rank * B:(rank + 1) * B]
        for _ in range(2):  # the second step reuses the buckets
            net.space.zero_grad(set_to_none=True)
            net(data[:, :-1], data[:, 1:]).backward()
        torch.cuda.synchronize()
        out[comm] = ({n: p.grad.detach().float().cpu().numpy() for n, p in model.named_parameters()},
                     len(net.buckets), net.comm_plan()["grad_comm_dtype"])
    if rank == 0:  # single-process reference of the concatenated batch
        from ray_torch_distributed_checkpoint_amd.optim import FlatParamSpace

        model = _model(dev)
        FlatParamSpace(list(reversed(list(model.parameters()))))
        data = _batch(world, dev)
        model(data[:, :-1], data[:, 1:]).backward()
        out["ref"] = {n: p.grad.detach().float().cpu().numpy() for n, p in model.named_parameters()}
    return out


def _sc_zero(rank, world, dev):
    from ray_torch_distributed_checkpoint_amd.optim import FusedAdamW
    from ray_torch_distributed_checkpoint_amd.parallel.ddp import DistributedDataParallel

    out = {}
    for zero in (0, 1):
        model = _model(dev)
        net = DistributedDataParallel(model, bucket_cap_mb=0.25, first_bucket_mb=0.05, zero_stage=zero)
        opt = FusedAdamW(model.parameters(), lr=1e-3, weight_decay=0.1)
        for k in range(3):
            data = _batch(world, dev, salt=11 + k)[rank * B:(rank + 1) * B]
            net(data[:, :-1], data[:, 1:]).backward()
            opt.step()
            opt.zero_grad()
        sd = opt.state_dict()  # ZeRO: consolidated (collective)
        torch.cuda.synchronize()
        out[zero] = ({n: p.detach().float().cpu().numpy() for n, p in model.named_parameters()},
                     {f"{k}.{n}": v.float().cpu().numpy() for k, st in sd["state"].items() for n, v in st.items()
                      if torch.is_tensor(v) and v.dim() > 0},
                     int(sum(b.numel() for b in opt._bufs.values())))
    return out


def _sc_p2p(rank, world, dev):
    import torch.distributed as dist

    from ray_torch_distributed_checkpoint_amd.parallel.ddp import DistributedDataParallel
    from ray_torch_distributed_checkpoint_amd.parallel.p2p import P2PAllReduce

    p2p = P2PAllReduce(capacity_mb=4.0, device=dev, timeout_s=60.0)
    out = {"exact": [], "rand": [], "rand_ref": [], "err": 0}
    for it, n in enumerate((4096, 65536 + 64, 1 << 19)):
        g = torch.Generator().manual_seed(1000 * it + rank)
        # small integers: every summation order is exact, so P2P must equal RCCL bit for bit
        x = torch.randint(-8, 9, (n,), generator=g).float().to(dev)
        a, b = x.clone(), x.clone()
        p2p.all_reduce_(a, average=False)
        dist.all_reduce(b)
        torch.cuda.synchronize()
        out["exact"].append(bool(torch.equal(a, b)))
        r = torch.randn(n, generator=g).to(dev)
        c, d = r.clone(), r.clone()
        p2p.all_reduce_(c, average=True)
        dist.all_reduce(d)
        d /= world
        torch.cuda.synchronize()
        out["rand"].append(_digest(c))  # identical on every rank
        out["rand_ref"].append(float(((c - d).abs().max() / d.abs().max()).item()))
    out["err"] = p2p.error()
    # DDP buckets over P2P vs over the process group
    grads = {}
    for mode, kb in (("pg", 0.0), ("p2p", 4096.0)):
        model = _model(dev)
        net = DistributedDataParallel(model, bucket_cap_mb=0.25, first_bucket_mb=0.05, p2p_max_kb=kb)
        data = _batch(world, dev)[rank * B:(rank + 1) * B]
        net(data[:, :-1], data[:, 1:]).backward()
        torch.cuda.synchronize()
        grads[mode] = {n: p.grad.detach().float().cpu().numpy() for n, p in model.named_parameters()}
        out["p2p_buckets" if kb else "pg_buckets"] = len(net.comm_plan()["p2p_buckets"])
    out["grad_rel"] = max(float(np.abs(grads["p2p"][n] - grads["pg"][n]).max() /
                                max(np.abs(grads["pg"][n]).max(), 1e-12)) for n in grads["pg"])
    return out


def _train_state(rank, world, dev, zero, steps=2, pg=None):
    from ray_torch_distributed_checkpoint_amd.optim import FusedAdamW
    from ray_torch_distributed_checkpoint_amd.parallel.ddp import DistributedDataParallel

    model = _model(dev, seed=5)
    net = DistributedDataParallel(model, process_group=pg, bucket_cap_mb=0.25, first_bucket_mb=0.05,
                                  zero_stage=zero)
    opt = FusedAdamW(model.parameters(), lr=1e-3, weight_decay=0.1)
    for k in range(steps):
        data = _batch(world, dev, salt=31 + k)[rank * B:(rank + 1) * B]
        net(data[:, :-1], data[:, 1:]).backward()
        opt.step()
        opt.zero_grad()
    if steps == 0:
        opt.init_state()
    return model, net, opt


def _sc_ckpt(rank, world, dev, path):
    import torch.distributed as dist

    from ray_torch_distributed_checkpoint_amd.checkpoint import dcp
    from ray_torch_distributed_checkpoint_amd.checkpoint.state_dict import get_state_dict, set_state_dict

    out = {}
    # replicated train state, async sharded save (dedup: each rank writes a share) at N ranks
    model, net, opt = _train_state(rank, world, dev, zero=0)
    saved = _state_digests(model, opt)
    msd, osd = get_state_dict(model, opt)
    ck = os.path.join(path, "rep")
    h = dcp.async_save({"model": msd, "optim": osd, "step": 2}, ck)
    h.result()
    out["rep_files"] = sorted(os.listdir(ck)) if rank == 0 else None
    out["rep_bytes"] = h.nbytes
    out["state_bytes"] = sum(p.numel() * p.element_size() for p in model.parameters()) + sum(
        v.numel() * v.element_size() for st in opt.state_dict()["state"].values() for v in st.values()
        if torch.is_tensor(v) and v.dim() > 0)

    def restore(pg, zero):
        # (the restoring group's own DDP wrap: a subgroup restore must not run collectives on
        # the world group)
        m2, _n2, o2 = _train_state(rank, world, dev, zero=zero, steps=0, pg=pg)
        ms, os_ = get_state_dict(m2, o2)
        sd = {"model": ms, "optim": os_, "step": 0}
        dcp.load(sd, ck, process_group=pg)
        set_state_dict(m2, o2, model_state_dict=sd["model"], optim_state_dict=sd["optim"])
        torch.cuda.synchronize()
        return _state_digests(m2, o2), sd["step"]

    got, step = restore(None, 0)
    out["rep_restore_equal"] = got == saved and step == 2
    # reshard: the first N/2 ranks read the N-rank checkpoint
    half = max(1, world // 2)
    sub = dist.new_group(ranks=list(range(half)))  # (collective: every rank creates it)
    if rank < half:
        got, step = restore(sub, 0)
        out["rep_reshard_equal"] = got == saved and step == 2
    dist.barrier()
    # ZeRO-1: each rank writes only its optimizer shards (no all-gather); restore at N
    model, net, opt = _train_state(rank, world, dev, zero=1)
    saved_z = _state_digests(model, opt)  # consolidated (collective)
    msd, osd = get_state_dict(model, opt)
    ck = os.path.join(path, "zero")
    h = dcp.async_save({"model": msd, "optim": osd, "step": 2}, ck)
    h.result()
    m2, _n2, o2 = _train_state(rank, world, dev, zero=1, steps=0)
    ms, os_ = get_state_dict(m2, o2)
    sd = {"model": ms, "optim": os_, "step": 0}
    dcp.load(sd, ck)
    set_state_dict(m2, o2, model_state_dict=sd["model"], optim_state_dict=sd["optim"])
    out["zero_restore_equal"] = _state_digests(m2, o2) == saved_z
    return out


def _worker(rank, world, port, backend, path, q):
    try:
        import torch.distributed as dist

        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                          LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(world))
        dev = torch.device("cuda", rank % torch.cuda.device_count())
        torch.cuda.set_device(dev)
        kw = {"device_id": dev} if backend == "nccl" else {}
        dist.init_process_group(backend, rank=rank, world_size=world, **kw)
        res = {}
        for name, fn in (("ddp", _sc_ddp), ("zero", _sc_zero), ("p2p", _sc_p2p)):
            res[name] = fn(rank, world, dev)
            dist.barrier()
            print(f"[multigpu {backend} r{rank}/{world}] {name} done", flush=True)
        res["ckpt"] = _sc_ckpt(rank, world, dev, path)
        print(f"[multigpu {backend} r{rank}/{world}] ckpt done", flush=True)
        q.put((rank, "ok", res))
        dist.barrier()
        dist.destroy_process_group()
    except Exception:
        q.put((rank, "err", traceback.format_exc()))


_cache: dict = {}


def _matrix(backend, tmp_path_factory):
    """One spawn of `world` ranks per backend runs every scenario (process start and RCCL
    initialisation are paid once); the tests below assert on its results."""
    if backend in _cache:
        return _cache[backend]
    import torch.multiprocessing as mp

    world = WORLD if backend == "nccl" else 2
    path = str(tmp_path_factory.mktemp(f"mg_{backend}"))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, backend, path, q)) for r in range(world)]
    # ranks sharing one device (the gloo stand-in): one HIP hardware queue each, or gloo's priority
    # streams oversubscribe the device's queue slots and the scheduler time-slices the two
    # processes (profiles/multiproc_slowdown_r6.md).  Set in the parent: a spawned child
    # initialises HIP when it imports this module.
    old_q = os.environ.get("GPU_MAX_HW_QUEUES")
    if backend == "gloo":
        os.environ["GPU_MAX_HW_QUEUES"] = "1"
    try:
        for p in ps:
            p.start()
    finally:
        if backend == "gloo":
            if old_q is None:
                os.environ.pop("GPU_MAX_HW_QUEUES", None)
            else:
                os.environ["GPU_MAX_HW_QUEUES"] = old_q
    out = {}
    try:
        for _ in range(world):
            r, st, v = q.get(timeout=600)
            if st != "ok":
                _cache[backend] = (world, None, f"rank {r}:\n{v}")
                return _cache[backend]
            out[r] = v
    finally:
        for p in ps:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    _cache[backend] = (world, out, None)
    return _cache[backend]


BACKENDS = [pytest.param("nccl", marks=needs_multi, id="rccl"), pytest.param("gloo", id="gloo_standin")]


@pytest.fixture
def mx(request, tmp_path_factory):
    world, out, err = _matrix(request.param, tmp_path_factory)
    assert err is None, err
    return request.param, world, out


@pytest.mark.parametrize("mx", BACKENDS, indirect=True)
def test_ddp_gradients_equal_concatenated_batch(mx):
    _backend, world, out = mx
    ref = out[0]["ddp"]["ref"]
    for comm, tol in (("fp32", 5e-3), ("bf16", 5e-3)):
        g0, nb, dt = out[0]["ddp"][comm]
        assert dt == comm and nb > 3
        for r in range(world):  # every rank holds the same averaged gradient
            for n, v in g0.items():
                assert np.array_equal(out[r]["ddp"][comm][0][n], v), (comm, r, n)
        for n, v in ref.items():
            err = np.linalg.norm(g0[n] - v) / max(np.linalg.norm(v), 1e-12)
            assert err < tol, (comm, n, err)


@pytest.mark.parametrize("mx", BACKENDS, indirect=True)
def test_zero1_equals_replicated_optimizer(mx):
    """gloo sums in a fixed order, so ZeRO-1 is bitwise the replicated optimizer there.  RCCL
    reduce-scatters the padded ZeRO buckets and all-reduces the unpadded ones, so element sums
    can associate differently; there the check is fp32 rounding (and bitwise across ranks)."""
    backend, world, out = mx
    rep, z = out[0]["zero"][0], out[0]["zero"][1]
    assert z[2] * world <= rep[2] * 1.05 + (1 << 17)  # ZeRO keeps ~1/world of the optimizer state
    for r in range(world):
        zr = out[r]["zero"][1]
        for n, v in rep[0].items():
            if backend == "gloo":
                assert np.array_equal(zr[0][n], v), (r, n)
            else:
                np.testing.assert_allclose(zr[0][n], v, rtol=2e-5, atol=2e-6, err_msg=f"rank {r} {n}")
            assert np.array_equal(zr[0][n], z[0][n]), (r, n)  # identical on every rank
        for n, v in rep[1].items():
            if backend == "gloo":
                assert np.array_equal(zr[1][n], v), (r, n)
            else:
                np.testing.assert_allclose(zr[1][n], v, rtol=1e-4, atol=1e-7, err_msg=f"rank {r} {n}")


@pytest.mark.parametrize("mx", BACKENDS, indirect=True)
def test_p2p_oneshot_matches_collective(mx):
    _backend, world, out = mx
    for r in range(world):
        p = out[r]["p2p"]
        assert p["err"] == 0, "a P2P wait timed out"
        assert all(p["exact"]), "P2P != collective on exactly representable sums"
        assert p["rand"] == out[0]["p2p"]["rand"], f"rank {r}: P2P result differs across ranks"
        assert max(p["rand_ref"]) < 1e-5
        assert p["grad_rel"] < 1e-5
        assert p["p2p_buckets"] > 0 and p["pg_buckets"] == 0  # the P2P arm really routed buckets


@pytest.mark.parametrize("mx", BACKENDS, indirect=True)
def test_sharded_save_restore_and_reshard(mx):
    _backend, world, out = mx
    files = out[0]["ckpt"]["rep_files"]
    assert ".metadata" in files and sum(f.endswith(".distcp") for f in files) >= 1
    half = max(1, world // 2)
    for r in range(world):
        c = out[r]["ckpt"]
        assert c["rep_restore_equal"], f"rank {r}: N-rank restore differs"
        if r < half:
            assert c["rep_reshard_equal"], f"rank {r}: N/2-rank reshard differs"
        assert c["zero_restore_equal"], f"rank {r}: ZeRO-1 restore differs"
    # dedup: the ranks together write one copy of the replicated state, not N
    total = sum(out[r]["ckpt"]["rep_bytes"] for r in range(world))
    state = out[0]["ckpt"]["state_bytes"]
    assert 0.9 * state <= total <= 1.1 * state + (1 << 20), (total, state)


def _losses(path):
    out = {}
    for line in open(os.path.join(path, "result.json")):
        row = json.loads(line)
        for i, v in enumerate(reversed(row["losses"])):
            k = row["step"] - i
            assert out.get(k, v) == v
            out[k] = v
    return out


@needs_multi
@pytest.mark.parametrize("zero", [0, 1])
def test_trainer_n_gpu_kill_restart_bit_equal(tmp_path, monkeypatch, zero):
    """TorchTrainer with one worker per GPU (RCCL): SIGKILL at step 3, supervisor restart from the
    latest committed async checkpoint, losses bit-equal to the uninterrupted run."""
    from ray_torch_distributed_checkpoint_amd import workloads as W

    for k in ("RTDC_FAIL_AT_STEP", "RTDC_HANG_AT_STEP", "RTDC_FORCE_CPU"):
        monkeypatch.delenv(k, raising=False)
    kw = dict(steps=6, num_workers=WORLD, use_gpu=True, ckpt_every_n_steps=2, verbose=0, zero_stage=zero)
    a = W.train_workload("gpt2-tiny", checkpoint_storage_path=str(tmp_path / "a"), **kw)
    monkeypatch.setenv("RTDC_FAIL_AT_STEP", "3")
    b = W.train_workload("gpt2-tiny", checkpoint_storage_path=str(tmp_path / "b"), max_failures=1, **kw)
    la, lb = _losses(a.path), _losses(b.path)
    assert sorted(la) == list(range(1, 7))
    assert la == lb
    files = sorted(os.listdir(b.checkpoint.path))
    assert ".metadata" in files and any(f.endswith(".distcp") for f in files)

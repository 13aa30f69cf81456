"""Step time after each part of the bench's checkpoint phase (2 gloo ranks sharing one GPU):
which part leaves the training step slower.

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 scripts/diag_postckpt.py
"""
import os
import sys
import tempfile
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    nodist = os.environ.get("DIAG_NODIST") == "1"  # independent processes on the same GPU, no gloo
    if nodist:
        rank = int(os.environ["RANK"])
        dist.barrier = lambda: None
        dist.destroy_process_group = lambda: None
    else:
        dist.init_process_group("gloo")
        rank = dist.get_rank()
    torch.cuda.set_device(0)
    from ray_torch_distributed_checkpoint_amd.checkpoint import dcp
    from ray_torch_distributed_checkpoint_amd.checkpoint.state_dict import get_state_dict, set_state_dict
    from ray_torch_distributed_checkpoint_amd.models import GPT2, GPT2Config
    from ray_torch_distributed_checkpoint_amd.optim import FusedAdamW
    from ray_torch_distributed_checkpoint_amd.parallel.ddp import DistributedDataParallel

    torch.manual_seed(0)
    model = GPT2(GPT2Config.named("gpt2-small")).cuda()
    opt = FusedAdamW(model.parameters(), lr=1e-4)
    cur = {"net": model if nodist else DistributedDataParallel(model, bucket_cap_mb=32, defer_tail_to_optimizer=True)}
    d = torch.randint(0, 50257, (4, 1025), device="cuda")
    x, y = d[:, :-1].contiguous(), d[:, 1:].contiguous()
    seed = torch.ones((), device="cuda")

    def steps(tag, n=int(os.environ.get("DIAG_N", "4"))):
        torch.cuda.synchronize()
        dist.barrier()
        t = time.perf_counter()
        for _ in range(n):
            cur["net"](x, y).backward(seed)
            opt.step()
            opt.zero_grad()
        torch.cuda.synchronize()
        dist.barrier()
        if rank == 0 or nodist:
            print(f"r{rank} {tag:28s} {(time.perf_counter() - t) / n * 1e3:9.1f} ms/step", flush=True)

    def state():
        msd, osd = get_state_dict(model, opt)
        return {"model": msd, "optim": osd, "step": 1}

    base = os.path.join(tempfile.gettempdir(), "diag_postckpt")
    steps("warm", 2)
    steps("baseline")
    mode = os.environ.get("DIAG_MODE", "")
    if mode:  # one ingredient of prepare_async at a time
        from ray_torch_distributed_checkpoint_amd.checkpoint import snapshot, torchsave

        if mode == "plan":
            dcp._plan_save(state(), None, True, None)
        elif mode == "engine":
            torchsave.get_engine()
        elif mode == "reserve":
            _w, r, _i, _m, per = dcp._plan_save(state(), None, True, None)
            snapshot.reserve([it.tensor for it in per[r] if it.kind == "tensor"])
        elif mode == "bevents":
            keep = [torch.cuda.Event(blocking=True) for _ in range(8)]
        elif mode == "engine_small":
            from ray_torch_distributed_checkpoint_amd.ops import _ext

            keep = _ext.ext().CkptEngine(1, 4096, 1, 0, stream=torch.cuda.Stream().cuda_stream)
        elif mode in ("ev_block", "ev_plain"):
            import ctypes

            hip = ctypes.CDLL("libamdhip64.so", mode=ctypes.RTLD_GLOBAL)
            evs = [ctypes.c_void_p() for _ in range(8)]
            flags = 0x3 if mode == "ev_block" else 0x2  # hipEventBlockingSync | hipEventDisableTiming
            rcs = [hip.hipEventCreateWithFlags(ctypes.byref(e), ctypes.c_uint(flags)) for e in evs]
            if rank == 0:
                print(f"{mode} rc={rcs}", flush=True)
        elif mode == "engine_nowriter":
            from ray_torch_distributed_checkpoint_amd.ops import _ext

            keep = _ext.ext().CkptEngine(1, 4096, 0, 0, stream=torch.cuda.Stream().cuda_stream)
        elif mode in ("rawstream", "rawstream0", "hostmalloc"):
            import ctypes

            hip = ctypes.CDLL("libamdhip64.so", mode=ctypes.RTLD_GLOBAL)
            h = ctypes.c_void_p()
            if mode == "rawstream":
                rc = hip.hipStreamCreateWithFlags(ctypes.byref(h), ctypes.c_uint(1))
            elif mode == "rawstream0":
                rc = hip.hipStreamCreate(ctypes.byref(h))
            else:
                rc = hip.hipHostMalloc(ctypes.byref(h), ctypes.c_size_t(4096), ctypes.c_uint(0))
            if rank == 0:
                print(f"{mode} rc={rc}", flush=True)
        elif mode == "pythread":
            import threading

            ev = threading.Event()

            def idle():
                torch.cuda.set_device(0)
                ev.wait()

            threading.Thread(target=idle, daemon=True).start()
        elif mode == "stream":
            keep = [torch.cuda.Stream(), torch.empty(512 << 20, dtype=torch.uint8, pin_memory=True)]
        steps(f"after {mode}")
        steps(f"after {mode} (2)")
        dist.destroy_process_group()
        return
    dcp.prepare_async(state())
    steps("after prepare_async")
    h = dcp.async_save(state(), base + "_a")
    steps("during async save", 2)
    h.wait()
    dist.barrier()
    h._finish()
    dist.barrier()
    steps("after async save")
    dcp.save(state(), base + "_b")
    steps("after blocking save")
    sd = state()
    dcp.load(sd, base + "_b")
    steps("after dcp.load")
    set_state_dict(model, opt, model_state_dict=sd["model"], optim_state_dict=sd["optim"])
    steps("after set_state_dict")
    cur["net"].detach()
    cur["net"] = DistributedDataParallel(model, bucket_cap_mb=32, defer_tail_to_optimizer=True)
    steps("after DDP re-wrap", 2)
    steps("after DDP re-wrap (2)")
    dist.destroy_process_group()


if __name__ == "__main__":
    main()

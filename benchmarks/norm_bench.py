"""LayerNorm forward at the GPT-2 shape (16384 x 768, bf16): the native row kernel vs ATen's,
plus the HBM bandwidth it reaches (the backward is timed inside the model profile:
scripts/gpu.sh prof).  python benchmarks/norm_bench.py"""
from __future__ import annotations

import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from ray_torch_distributed_checkpoint_amd.ops import norm  # noqa: E402


def timeit(fn, reps=50):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    fn()
    torch.cuda.synchronize()
    ev[0].record()
    for _ in range(reps):
        fn()
    ev[1].record()
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]) / reps * 1e3


def main():
    dev = torch.device("cuda", 0)
    M, D = 16384, 768
    x = torch.randn(M, D, device=dev).bfloat16()
    w = torch.nn.Parameter(torch.ones(D, device=dev))
    b = torch.nn.Parameter(torch.zeros(D, device=dev))
    nb = M * D * 2

    def ours_fwd():
        return norm.layer_norm(x, w, b)

    def aten_fwd():
        return F.layer_norm(x, (D,), w.bfloat16(), b.bfloat16())

    r = {"M": M, "D": D}
    r["ours_fwd_us"] = round(timeit(ours_fwd), 1)
    r["ours_fwd_TBps"] = round(2 * nb / r["ours_fwd_us"] / 1e6, 2)
    r["aten_fwd_us"] = round(timeit(aten_fwd), 1)
    ref = F.layer_norm(x.float(), (D,), w, b)
    r["ours_fwd_max_err"] = float((ours_fwd().float() - ref).abs().max())
    r["RTDC_NORM_FWD2R"] = os.environ.get("RTDC_NORM_FWD2R", "0")
    print(json.dumps(r), flush=True)

    # backward at the GPT-2 form (residual-stream gradient added in the kernel, column sums of
    # dx for the residual projection's bias, dgamma / dbeta partial rows) and the Llama RMSNorm
    # form; bytes = read x, dy, dres + write dx
    from ray_torch_distributed_checkpoint_amd.ops._ext import gpu_ext
    from ray_torch_distributed_checkpoint_amd.ops.norm import _bwd_waves, _bwd_ws_elems

    ext = gpu_ext()
    for name, M2, D2, rms in (("gpt2_ln", 16384, 768, False), ("llama_rms", 2048, 4096, True)):
        x2 = torch.randn(M2, D2, device=dev).bfloat16()
        dy = torch.randn(M2, D2, device=dev).bfloat16()
        dres = torch.randn(M2, D2, device=dev).bfloat16()
        g2 = torch.ones(D2, device=dev).bfloat16()
        mean = torch.zeros(M2, device=dev)
        rstd = torch.ones(M2, device=dev)
        dx = torch.empty_like(x2)
        nw = _bwd_waves(M2)
        ws = torch.empty(_bwd_ws_elems(nw, D2), device=dev)
        dg, db, dxs = (torch.empty(D2, device=dev) for _ in range(3))
        if rms:
            fn = lambda: ext.rmsnorm_bwd(dy, x2, g2, rstd, dres, dx, ws, dg, None, nw, False)  # noqa: E731
        else:
            fn = lambda: ext.layernorm_bwd(dy, x2, g2, mean, rstd, dres, dx, ws, dg, db, dxs, nw, False,  # noqa: E731
                                           False)
        us = timeit(fn)
        print(json.dumps({"bwd": name, "M": M2, "D": D2, "us": round(us, 1),
                          "TBps": round(4 * M2 * D2 * 2 / us / 1e6, 2)}), flush=True)


if __name__ == "__main__":
    main()

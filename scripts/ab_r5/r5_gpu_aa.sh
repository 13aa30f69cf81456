#!/bin/bash
# (the RTDC_ADAMW variant kernel was removed after this A/B: profiles/adamw_two_group_ab_r5.txt)
# AdamW: one 4-element group per lane (RTDC_ADAMW=1) vs two groups (2) vs two groups with
# non-temporal stores (3) - isolated on the GPT-2 parameter count, then the GPT-2 step
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "adamw or fused_optimizers" > gpurun_out/aa_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/aa_tests.log; exit 1; }
tail -n 1 gpurun_out/aa_tests.log
timeout -k 10 180 python - <<'PY'
import os, torch
from ray_torch_distributed_checkpoint_amd.optim import FusedAdamW
torch.manual_seed(0)
# GPT-2 small parameter shapes (124.4M fp32 master weights)
shapes = [(50304, 768), (1024, 768)] + [(768,), (768,), (2304, 768), (2304,), (768, 768), (768,),
          (768,), (768,), (3072, 768), (3072,), (768, 3072), (768,)] * 12 + [(768,), (768,)]
ps = [torch.randn(*s, device="cuda", requires_grad=True) for s in shapes]
for p in ps: p.grad = torch.randn_like(p)
opt = FusedAdamW(ps, lr=1e-4, weight_decay=0.1)
n = sum(p.numel() for p in ps)
for arm in ("1", "2", "3", "1", "2", "3"):
    os.environ["RTDC_ADAMW"] = arm
    for _ in range(3): opt.step()
    torch.cuda.synchronize()
    e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    e[0].record()
    for _ in range(20): opt.step()
    e[1].record(); torch.cuda.synchronize()
    us = e[0].elapsed_time(e[1]) / 20 * 1e3
    print(f"RTDC_ADAMW={arm}: {us:.1f} us per step over {n/1e6:.1f}M params ({30*n/us/1e6:.2f} TB/s at 30 B/param)")
PY
for r in 1 2; do for arm in 1 2 3; do
  RTDC_ADAMW=$arm timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-ckpt > gpurun_out/aa_bench_${arm}_$r.log 2>&1 || { echo "bench failed"; exit 1; }
  echo "ADAMW=$arm $r $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/aa_bench_${arm}_$r.log)"
done; done

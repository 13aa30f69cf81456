#!/bin/bash
# token-id sort: register-resident segments (default) vs the chunk loop (RTDC_SORT_REG=0)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "sort_ids or embedding" > gpurun_out/s_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/s_tests.log; exit 1; }
tail -n 1 gpurun_out/s_tests.log
timeout -k 10 120 python - <<'PY'
import os, torch
from ray_torch_distributed_checkpoint_amd.ops.embedding import sort_ids
ids = torch.randint(0, 50257, (16384,), device="cuda")
for arm in ("1", "0", "1", "0"):
    os.environ["RTDC_SORT_REG"] = arm
    for _ in range(3): sort_ids(ids, 50257)
    torch.cuda.synchronize()
    e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    e[0].record()
    for _ in range(50): sort_ids(ids, 50257)
    e[1].record(); torch.cuda.synchronize()
    print(f"RTDC_SORT_REG={arm}: {e[0].elapsed_time(e[1]) / 50 * 1e3:.1f} us per sort of 16384 ids")
PY
for r in 1 2; do for arm in 1 0; do
  RTDC_SORT_REG=$arm timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-ckpt > gpurun_out/s_bench_${arm}_$r.log 2>&1 || { echo "bench failed"; exit 1; }
  echo "SORT_REG=$arm $r $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/s_bench_${arm}_$r.log)"
done; done

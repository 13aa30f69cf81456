#!/bin/bash
# flash attention: (row & 7) LDS swizzle at Dh 64 (in-tree) vs the round-4 (row >> 1) & 7 (abv/_C_oldswz.so)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python scripts/ab_r5/attn_dump.py gpurun_out/attn_new.pt > gpurun_out/o_dump1.log 2>&1 || { echo dump1 failed; tail gpurun_out/o_dump1.log; exit 1; }
RTDC_EXT_SO=abv/_C_oldswz.so timeout -k 10 120 python scripts/ab_r5/attn_dump.py gpurun_out/attn_old.pt > gpurun_out/o_dump2.log 2>&1 || { echo dump2 failed; exit 1; }
python3 -c "
import torch
a=torch.load('gpurun_out/attn_new.pt', weights_only=True); b=torch.load('gpurun_out/attn_old.pt', weights_only=True)
for k in a: print(k, 'fwd bitwise', torch.equal(a[k][0], b[k][0]), 'bwd bitwise', torch.equal(a[k][1], b[k][1]))
"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "flash or attention" > gpurun_out/o_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/o_tests.log; exit 1; }
tail -n 1 gpurun_out/o_tests.log
for r in 1 2 3; do for arm in new old; do
  if [ $arm = old ]; then e="RTDC_EXT_SO=abv/_C_oldswz.so"; else e="RTDC_EXT_SO="; fi
  env $e timeout -k 10 120 python benchmarks/attn_bench.py --reps 30 > gpurun_out/o_attn_${arm}_$r.log 2>&1 || { echo "attn $arm failed"; exit 1; }
  echo "$arm $r $(python3 -c "
import json
for l in open('gpurun_out/o_attn_${arm}_$r.log'):
    if l.startswith('{'):
        d=json.loads(l); print(d['shape'], d['kernel_fwd_us'], d['kernel_bwd_us'], end=' | ')
")"
done; done
for r in 1 2; do for arm in new old; do
  if [ $arm = old ]; then e="RTDC_EXT_SO=abv/_C_oldswz.so"; else e="RTDC_EXT_SO="; fi
  env $e timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-ckpt > gpurun_out/o_bench_${arm}_$r.log 2>&1 || { echo "bench $arm failed"; exit 1; }
  echo "$arm $r $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/o_bench_${arm}_$r.log)"
done; done

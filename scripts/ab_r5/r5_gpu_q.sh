#!/bin/bash
# flash attention Dh 128: 2 (row & 7) LDS swizzle (in-tree) vs round 4's (row & 15) (abv/_C_old128.so)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out /tmp/dump
timeout -k 10 120 python scripts/ab_r5/attn_dump.py /tmp/dump/attn_new.pt > gpurun_out/q_dump1.log 2>&1 || { echo dump1 failed; tail gpurun_out/q_dump1.log; exit 1; }
RTDC_EXT_SO=abv/_C_old128.so timeout -k 10 120 python scripts/ab_r5/attn_dump.py /tmp/dump/attn_old.pt > gpurun_out/q_dump2.log 2>&1 || { echo dump2 failed; exit 1; }
python3 -c "
import torch
a=torch.load('/tmp/dump/attn_new.pt', weights_only=True); b=torch.load('/tmp/dump/attn_old.pt', weights_only=True)
for k in a: print(k, 'fwd bitwise', torch.equal(a[k][0], b[k][0]), 'bwd bitwise', torch.equal(a[k][1], b[k][1]))
"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "flash or attention" > gpurun_out/q_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/q_tests.log; exit 1; }
tail -n 1 gpurun_out/q_tests.log
for r in 1 2 3; do for arm in new old; do
  if [ $arm = old ]; then e="RTDC_EXT_SO=abv/_C_old128.so"; else e="RTDC_EXT_SO="; fi
  env $e timeout -k 10 120 python benchmarks/attn_bench.py --reps 30 > gpurun_out/q_attn_${arm}_$r.log 2>&1 || { echo "attn $arm failed"; exit 1; }
  echo "$arm $r $(python3 -c "
import json
for l in open('gpurun_out/q_attn_${arm}_$r.log'):
    if l.startswith('{'):
        d=json.loads(l); print(d['shape'], d['kernel_fwd_us'], d['kernel_bwd_us'], end=' | ')
")"
done; done

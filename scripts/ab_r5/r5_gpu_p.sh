#!/bin/bash
# BatchNorm reduce kernels with a channel-major (conflict-free) LDS layout (in-tree) vs round 4's (abv/_C_oldbn.so)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out /tmp/dump
timeout -k 10 180 python scripts/ab_r5/resnet_dump.py /tmp/dump/new.pt > gpurun_out/p_dump1.log 2>&1 || { echo dump1 failed; tail gpurun_out/p_dump1.log; exit 1; }
RTDC_EXT_SO=abv/_C_oldbn.so timeout -k 10 180 python scripts/ab_r5/resnet_dump.py /tmp/dump/old.pt > gpurun_out/p_dump2.log 2>&1 || { echo dump2 failed; exit 1; }
python3 -c "
import torch
a=torch.load('/tmp/dump/new.pt', weights_only=True); b=torch.load('/tmp/dump/old.pt', weights_only=True)
bad=[k for k in a if not torch.equal(a[k], b[k])]
print('resnet step tensors', len(a), 'bitwise differing', len(bad), bad[:5])
"
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_cnn_gpu.py > gpurun_out/p_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/p_tests.log; exit 1; }
tail -n 1 gpurun_out/p_tests.log
for r in 1 2 3; do for arm in new old; do
  if [ $arm = old ]; then e="RTDC_EXT_SO=abv/_C_oldbn.so"; else e="RTDC_EXT_SO="; fi
  env $e timeout -k 10 240 python bench.py --model resnet18 --steps 20 --warmup 5 --no-ckpt > gpurun_out/p_bench_${arm}_$r.log 2>&1 || { echo "bench $arm failed"; exit 1; }
  echo "$arm $r $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/p_bench_${arm}_$r.log)"
done; done

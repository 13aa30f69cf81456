#!/bin/bash
# norm backward combine: half-major 16-B LDS slots (in-tree) vs chunk-major (abv/_C_oldnorm.so)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out /tmp/dump
timeout -k 10 120 python scripts/ab_r5/norm_dump.py /tmp/dump/n_new.pt > gpurun_out/w_dump1.log 2>&1 || { echo dump1 failed; tail gpurun_out/w_dump1.log; exit 1; }
RTDC_EXT_SO=abv/_C_oldnorm.so timeout -k 10 120 python scripts/ab_r5/norm_dump.py /tmp/dump/n_old.pt > gpurun_out/w_dump2.log 2>&1 || { echo dump2 failed; exit 1; }
python3 -c "
import torch
a=torch.load('/tmp/dump/n_new.pt', weights_only=True); b=torch.load('/tmp/dump/n_old.pt', weights_only=True)
for k in a: print(k, 'bitwise', all(torch.equal(u, v) for u, v in zip(a[k], b[k])))
"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "norm" > gpurun_out/w_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/w_tests.log; exit 1; }
tail -n 1 gpurun_out/w_tests.log
for r in 1 2 3; do for arm in new old; do
  if [ $arm = old ]; then e="RTDC_EXT_SO=abv/_C_oldnorm.so"; else e="RTDC_EXT_SO="; fi
  env $e timeout -k 10 120 python benchmarks/norm_bench.py > gpurun_out/w_norm_${arm}_$r.log 2>&1 || { echo "norm_bench failed"; exit 1; }
  echo "$arm $r $(grep '"bwd"' gpurun_out/w_norm_${arm}_$r.log | tr '\n' ' ')"
done; done

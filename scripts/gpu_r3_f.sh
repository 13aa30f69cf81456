#!/bin/bash
# Round 3 GPU pass F: DDP trainer tests after the enable_reproducibility fix, the copy-source
# profile, and the product path without the deterministic-mode NaN fill.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_ddp_gpu.py tests/test_faulttol_gpu.py -x -v --timeout 150 \
  --timeout-method thread > gpurun_out/r3f_ddp_tests.log 2>&1
rc=$?; echo "DDP TESTS EXIT $rc"; tail -n 2 gpurun_out/r3f_ddp_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/debug_copies_r3.py > gpurun_out/r3f_copies.txt 2>&1
rc=$?; echo "COPIES EXIT $rc"
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_product_r3.sh

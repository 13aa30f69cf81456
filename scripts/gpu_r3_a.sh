#!/bin/bash
# Round 3, first GPU pass: full GPU test suite (ZeRO compact state, native token sort /
# synthesis, P2P timeout poisoning), then the product-path run with the native data kernel.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread \
  > gpurun_out/r3a_tests.log 2>&1
rc=$?; echo "TESTS EXIT $rc"; tail -n 5 gpurun_out/r3a_tests.log
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_product_r3.sh

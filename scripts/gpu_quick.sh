#!/bin/bash
# quick loop: GEMM / MLP / attention / model numerics, then the headline bench + kernel profile
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q --timeout 120 \
  --timeout-method thread -k "${TESTK:-gemm or mlp or attention or gpt2 or gelu}" > gpurun_out/t_quick.log 2>&1
rc=$?; echo "TESTS EXIT $rc"; tail -n 4 gpurun_out/t_quick.log
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_prof.sh

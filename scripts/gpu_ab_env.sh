#!/bin/bash
# A/B one environment knob on the GPT-2-small bench: GPT-2 model/fault-tolerance GPU tests
# first, then alternating runs VAR=A, VAR=B, VAR=A, VAR=B (same process order every call).
#   bash scripts/gpu_ab_env.sh VAR A B [extra bench args]
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
var=$1; a=$2; b=$3; shift 3
timeout -k 10 400 python -u -m pytest tests/test_models_gpu.py tests/test_gpt2_parity_gpu.py tests/test_faulttol_gpu.py \
  -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_tests.log 2>&1
rc=$?; echo "TESTS EXIT $rc"; tail -n 3 gpurun_out/ab_tests.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in $a $b; do
    env "$var=$v" timeout -k 10 240 python bench.py --steps 30 --warmup 5 --no-ckpt "$@" > gpurun_out/ab_${v}_$i.log 2>&1
    rc=$?
    ms=$(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_${v}_$i.log)
    echo "$var=$v run $i EXIT $rc $ms"
    [ $rc -eq 0 ] || exit $rc
  done
done

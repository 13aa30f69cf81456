#!/bin/bash
# A/B of two native builds: ab/_C_old.so (RTDC_EXT_SO) vs the in-tree _C, GPT-2 then ResNet-18
# bench runs alternating old/new; optional pytest selection first ($1, e.g. "tests/test_optim.py").
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -n "$1" ]; then
  timeout -k 10 400 python -u -m pytest $1 -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/abso_tests.log 2>&1
  rc=$?; echo "TESTS EXIT $rc"; tail -n 2 gpurun_out/abso_tests.log; [ $rc -eq 0 ] || exit $rc
fi
OLD=/root/repo/ab/_C_old.so
for model in gpt2-small resnet18; do
  for arm in old new old new; do
    if [ $arm = old ]; then export RTDC_EXT_SO=$OLD; else unset RTDC_EXT_SO; fi
    timeout -k 10 240 python bench.py --model $model --steps 30 --warmup 5 --no-ckpt > gpurun_out/abso_${model}_$arm.log 2>&1
    rc=$?; echo "$model $arm EXIT $rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/abso_${model}_$arm.log)"
    [ $rc -eq 0 ] || exit $rc
  done
done

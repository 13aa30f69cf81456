#!/bin/bash
# attention numerics on the new build, then A/B old (ab/_C_old.so) vs new: attention bench on
# the GPT-2 shapes and the headline bench
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q --timeout 120 \
  --timeout-method thread -k "attention or flash or gpt2 or llama" > gpurun_out/t_aba.log 2>&1
rc=$?; echo "TESTS EXIT $rc"; tail -n 3 gpurun_out/t_aba.log
[ $rc -eq 0 ] || exit $rc
OLD=/root/repo/ab/_C_old.so
for arm in old new; do
  if [ $arm = old ]; then export RTDC_EXT_SO=$OLD; else unset RTDC_EXT_SO; fi
  timeout -k 10 200 python benchmarks/attn_bench.py --only gpt2 > gpurun_out/aba_attn_$arm.jsonl 2>&1
  rc=$?; echo "ATTN $arm EXIT $rc"; grep shape gpurun_out/aba_attn_$arm.jsonl | cut -c1-300
  [ $rc -eq 0 ] || exit $rc
done
for arm in old new old new; do
  if [ $arm = old ]; then export RTDC_EXT_SO=$OLD; else unset RTDC_EXT_SO; fi
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-ckpt > gpurun_out/aba_bench_$arm.log 2>&1
  rc=$?; echo "BENCH $arm EXIT $rc"; tail -n 1 gpurun_out/aba_bench_$arm.log | cut -c1-150
  [ $rc -eq 0 ] || exit $rc
done

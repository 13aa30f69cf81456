#!/bin/bash
# quick A/B old (ab/_C_old.so) vs new on one GEMM shape + the headline bench
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
OLD=/root/repo/ab/_C_old.so
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k gemm > gpurun_out/t_abq.log 2>&1
rc=$?; echo "TESTS EXIT $rc"; tail -n 2 gpurun_out/t_abq.log; [ $rc -eq 0 ] || exit $rc
for arm in old new; do
  if [ $arm = old ]; then export RTDC_EXT_SO=$OLD; else unset RTDC_EXT_SO; fi
  timeout -k 10 300 python benchmarks/gemm_bench.py --only ${SHAPE:-fc} > gpurun_out/abq_gemm_${arm}.jsonl 2>&1
  rc=$?; echo "GEMM $arm EXIT $rc"; [ $rc -eq 0 ] || exit $rc
done
for arm in old new; do
  if [ $arm = old ]; then export RTDC_EXT_SO=$OLD; else unset RTDC_EXT_SO; fi
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-ckpt > gpurun_out/abq_bench_$arm.log 2>&1
  rc=$?; echo "BENCH $arm EXIT $rc"; tail -n 1 gpurun_out/abq_bench_$arm.log | cut -c1-150
  [ $rc -eq 0 ] || exit $rc
done

#!/bin/bash
# A/B of two native builds on one box: ab/_C_old.so (RTDC_EXT_SO) vs the in-tree _C
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
OLD=/root/repo/ab/_C_old.so
for arm in old new old new; do
  if [ $arm = old ]; then export RTDC_EXT_SO=$OLD; else unset RTDC_EXT_SO; fi
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-ckpt > gpurun_out/ab_bench_$arm.log 2>&1
  rc=$?; echo "BENCH $arm EXIT $rc"; tail -n 1 gpurun_out/ab_bench_$arm.log | cut -c1-200
  [ $rc -eq 0 ] || exit $rc
done
for arm in old new; do
  if [ $arm = old ]; then export RTDC_EXT_SO=$OLD; else unset RTDC_EXT_SO; fi
  timeout -k 10 300 python benchmarks/gemm_bench.py ${GEMM_ARGS:-} > gpurun_out/ab_gemm_$arm.jsonl 2>&1
  rc=$?; echo "GEMM $arm EXIT $rc"; [ $rc -eq 0 ] || exit $rc
done
for arm in old new; do
  if [ $arm = old ]; then export RTDC_EXT_SO=$OLD; else unset RTDC_EXT_SO; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ab_prof_$arm -o run -- python3 bench.py --steps 5 --warmup 2 --no-ckpt > gpurun_out/ab_prof_$arm.log 2>&1
  rc=$?; echo "PROF $arm EXIT $rc"; [ $rc -eq 0 ] || exit $rc
done

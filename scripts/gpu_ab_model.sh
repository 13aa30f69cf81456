#!/bin/bash
# A/B old (ab/_C_old.so) vs new: GEMM bench at model-like magnitudes + in-model kernel trace
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
OLD=/root/repo/ab/_C_old.so
for arm in old new; do
  if [ $arm = old ]; then export RTDC_EXT_SO=$OLD; else unset RTDC_EXT_SO; fi
  GEMM_BENCH_XSCALE=0.05 timeout -k 10 300 python benchmarks/gemm_bench.py --only fc > gpurun_out/abm_gemm_${arm}.jsonl 2>&1
  rc=$?; echo "GEMM $arm EXIT $rc"; [ $rc -eq 0 ] || exit $rc
done
for arm in old new; do
  if [ $arm = old ]; then export RTDC_EXT_SO=$OLD; else unset RTDC_EXT_SO; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/abm_prof_$arm -o run -- python3 bench.py --steps 5 --warmup 2 --no-ckpt > gpurun_out/abm_prof_$arm.log 2>&1
  rc=$?; echo "PROF $arm EXIT $rc"; [ $rc -eq 0 ] || exit $rc
done

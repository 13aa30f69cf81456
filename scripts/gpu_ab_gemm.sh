#!/bin/bash
# GEMM numerics on the new build, then A/B old (ab/_C_old.so) vs new: GEMM bench with and
# without the persistent kernel, and the headline bench
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q --timeout 120 \
  --timeout-method thread -k "${TESTK:-gemm or mlp or attention or gpt2 or gelu or llama}" > gpurun_out/t_abg.log 2>&1
rc=$?; echo "TESTS EXIT $rc"; tail -n 4 gpurun_out/t_abg.log
[ $rc -eq 0 ] || exit $rc
OLD=/root/repo/ab/_C_old.so
for persist in 0 1; do
  for arm in old new; do
    if [ $arm = old ]; then export RTDC_EXT_SO=$OLD; else unset RTDC_EXT_SO; fi
    RTDC_GEMM_PERSIST=$persist timeout -k 10 300 python benchmarks/gemm_bench.py > gpurun_out/abg_gemm_${arm}_p$persist.jsonl 2>&1
    rc=$?; echo "GEMM $arm persist=$persist EXIT $rc"; [ $rc -eq 0 ] || exit $rc
  done
done
for arm in old new old new; do
  if [ $arm = old ]; then export RTDC_EXT_SO=$OLD; else unset RTDC_EXT_SO; fi
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-ckpt > gpurun_out/abg_bench_$arm.log 2>&1
  rc=$?; echo "BENCH $arm EXIT $rc"; tail -n 1 gpurun_out/abg_bench_$arm.log | cut -c1-160
  [ $rc -eq 0 ] || exit $rc
done
unset RTDC_EXT_SO
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/abg_prof_new -o run -- python3 bench.py --steps 5 --warmup 2 --no-ckpt > gpurun_out/abg_prof_new.log 2>&1
echo "PROF EXIT $?"

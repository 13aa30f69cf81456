#!/bin/bash
# A/B: 8-wave GEMM main-loop schedule (RTDC_GEMM_STAGGER 0 = one barrier per phase,
# 1 = two barriers per phase with waves 4-7 one barrier behind)
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
RTDC_GEMM_STAGGER=1 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 \
  --timeout-method thread -k "gemm" > gpurun_out/t_stag.log 2>&1
rc=$?; echo "TESTS EXIT $rc"; tail -n 3 gpurun_out/t_stag.log
[ $rc -eq 0 ] || exit $rc
for sg in 0 1; do
  RTDC_GEMM_STAGGER=$sg timeout -k 10 300 python benchmarks/gemm_bench.py --sweep --cfgs 6,7,8 > gpurun_out/gemm_stag$sg.jsonl 2>&1
  rc=$?; echo "GEMM STAG=$sg EXIT $rc"; grep shape gpurun_out/gemm_stag$sg.jsonl
  [ $rc -eq 0 ] || exit $rc
done
for sg in 0 1; do
  RTDC_GEMM_STAGGER=$sg timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-ckpt > gpurun_out/bench_stag$sg.log 2>&1
  rc=$?; echo "BENCH STAG=$sg EXIT $rc"; tail -n 1 gpurun_out/bench_stag$sg.log
  [ $rc -eq 0 ] || exit $rc
done

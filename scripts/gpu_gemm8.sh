#!/bin/bash
# 8-phase GEMM: numerics (all tile configs) then the shape sweep vs hipBLASLt
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q -k "gemm" > gpurun_out/gemm_tests.log 2>&1
rc=$?; echo "TESTS EXIT $rc"; tail -n 25 gpurun_out/gemm_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python benchmarks/gemm_bench.py --sweep --cfgs 0,6 > gpurun_out/gemm_bench8.jsonl 2>&1
rc=$?; echo "BENCH EXIT $rc"; cat gpurun_out/gemm_bench8.jsonl
exit $rc

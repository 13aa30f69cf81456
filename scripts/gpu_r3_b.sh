#!/bin/bash
# Round 3 GPU pass B: GEMM numerics (incl. the 4-wave cfg 10) -> GEMM A/B sweep -> full GPU
# suite -> product path.  Every GPU step has its own time limit; the chain stops at a failure.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -v -k "gemm or sort or synth" --timeout 120 \
  --timeout-method thread > gpurun_out/r3b_gemm_tests.log 2>&1
rc=$?; echo "GEMM TESTS EXIT $rc"; tail -n 3 gpurun_out/r3b_gemm_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u benchmarks/gemm_bench.py --reps 20 --sweep --cfgs 6,8,10 > gpurun_out/r3b_gemm_bench.jsonl 2>&1
rc=$?; echo "GEMM BENCH EXIT $rc"; tail -n 2 gpurun_out/r3b_gemm_bench.jsonl
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread \
  > gpurun_out/r3b_tests.log 2>&1
rc=$?; echo "TESTS EXIT $rc"; tail -n 5 gpurun_out/r3b_tests.log
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_product_r3.sh

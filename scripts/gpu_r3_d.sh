#!/bin/bash
# Round 3 GPU pass D: 4-wave GEMM numerics + A/B sweep, then pass C (full suite, product path,
# Llama-3-8B shard + trainer).
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v -k "gemm" --timeout 120 \
  --timeout-method thread > gpurun_out/r3d_gemm_tests.log 2>&1
rc=$?; echo "GEMM TESTS EXIT $rc"; tail -n 3 gpurun_out/r3d_gemm_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u benchmarks/gemm_bench.py --reps 20 --sweep --cfgs 6,8,10 > gpurun_out/r3d_gemm_bench.jsonl 2>&1
rc=$?; echo "GEMM BENCH EXIT $rc"
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_r3_c.sh

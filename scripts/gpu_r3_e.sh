#!/bin/bash
# Round 3 GPU pass E: interleaved 4-wave GEMM (numerics + A/B), P2P/DDP tests (graph-captured
# 2-worker toy step, timeout poisoning, tightened DDP tolerance), the copy-source profile, and
# the product path again (trainer without the deterministic-mode NaN fill).
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v -k "gemm" --timeout 120 \
  --timeout-method thread > gpurun_out/r3e_gemm_tests.log 2>&1
rc=$?; echo "GEMM TESTS EXIT $rc"; tail -n 2 gpurun_out/r3e_gemm_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u benchmarks/gemm_bench.py --reps 20 --sweep --cfgs 6,10 > gpurun_out/r3e_gemm_bench.jsonl 2>&1
rc=$?; echo "GEMM BENCH EXIT $rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_p2p_gpu.py tests/test_ddp_gpu.py -x -v --timeout 150 \
  --timeout-method thread > gpurun_out/r3e_p2p_ddp_tests.log 2>&1
rc=$?; echo "P2P/DDP TESTS EXIT $rc"; tail -n 2 gpurun_out/r3e_p2p_ddp_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/debug_copies_r3.py > gpurun_out/r3e_copies.txt 2>&1
rc=$?; echo "COPIES EXIT $rc"
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_product_r3.sh

#!/bin/bash
# GEMM epilogue change: numerics, GEMM bench (GPT-2 shapes), headline bench + kernel profile
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q --timeout 120 \
  --timeout-method thread -k "${TESTK:-gemm or mlp or attention or gpt2 or gelu or llama}" > gpurun_out/t_epi.log 2>&1
rc=$?; echo "TESTS EXIT $rc"; tail -n 4 gpurun_out/t_epi.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python benchmarks/gemm_bench.py > gpurun_out/gemm_epi.jsonl 2>&1
rc=$?; echo "GEMM EXIT $rc"; grep shape gpurun_out/gemm_epi.jsonl
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_prof.sh

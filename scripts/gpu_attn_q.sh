#!/bin/bash
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q --timeout 120 \
  --timeout-method thread -k "attention or flash or gpt2 or llama" > gpurun_out/t_attn.log 2>&1
rc=$?; echo "TESTS EXIT $rc"; tail -n 3 gpurun_out/t_attn.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python benchmarks/attn_bench.py > gpurun_out/attn_bench.jsonl 2>&1
rc=$?; echo "ATTN EXIT $rc"; grep shape gpurun_out/attn_bench.jsonl
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-ckpt > gpurun_out/bench_gpt2.log 2>&1
rc=$?; echo "BENCH EXIT $rc"; tail -n 1 gpurun_out/bench_gpt2.log

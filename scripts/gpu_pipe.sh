#!/bin/bash
# DMA-pipelined attention + persistent GEMM: numerics, microbenchmarks, headline bench, profile
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q --timeout 120 \
  --timeout-method thread -k "gemm or attention or flash or gpt2" > gpurun_out/t_pipe.log 2>&1
rc=$?; echo "TESTS EXIT $rc"; tail -n 15 gpurun_out/t_pipe.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python benchmarks/attn_bench.py > gpurun_out/attn_bench.jsonl 2>&1
rc=$?; echo "ATTN EXIT $rc"; cat gpurun_out/attn_bench.jsonl
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python benchmarks/gemm_bench.py --sweep --cfgs 6,7,8,9 > gpurun_out/gemm_bench.jsonl 2>&1
rc=$?; echo "GEMM EXIT $rc"; cat gpurun_out/gemm_bench.jsonl
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_gpt2.log 2>&1
rc=$?; echo "BENCH EXIT $rc"; tail -n 1 gpurun_out/bench_gpt2.log
[ $rc -eq 0 ] || exit $rc
RTDC_GEMM_PERSIST=0 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-ckpt > gpurun_out/bench_gpt2_nopersist.log 2>&1
rc=$?; echo "BENCH0 EXIT $rc"; tail -n 1 gpurun_out/bench_gpt2_nopersist.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_gpt2 -o run -- python3 bench.py --steps 5 --warmup 2 --no-ckpt > gpurun_out/prof_gpt2.log 2>&1
echo "PROF EXIT $?"

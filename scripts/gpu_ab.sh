#!/bin/bash
# A/B: attention ring depth (RTDC_FA_NS), GEMM asm-transposed reads + persistent form
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q --timeout 120 \
  --timeout-method thread -k "gemm or attention or flash or gpt2" > gpurun_out/t_ab.log 2>&1
rc=$?; echo "TESTS EXIT $rc"; tail -n 4 gpurun_out/t_ab.log
[ $rc -eq 0 ] || exit $rc
for ns in 2 3 4; do
  RTDC_FA_NS=$ns timeout -k 10 200 python benchmarks/attn_bench.py --only gpt2 > gpurun_out/attn_ns$ns.jsonl 2>&1
  rc=$?; echo "ATTN NS=$ns EXIT $rc"; grep shape gpurun_out/attn_ns$ns.jsonl
  [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 200 python benchmarks/attn_bench.py --only llama8b > gpurun_out/attn_llama.jsonl 2>&1
rc=$?; echo "ATTN LLAMA EXIT $rc"; grep shape gpurun_out/attn_llama.jsonl
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python benchmarks/gemm_bench.py --sweep --cfgs 6,7,8 > gpurun_out/gemm_bench.jsonl 2>&1
rc=$?; echo "GEMM EXIT $rc"; grep shape gpurun_out/gemm_bench.jsonl
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-ckpt > gpurun_out/bench_gpt2.log 2>&1
rc=$?; echo "BENCH EXIT $rc"; tail -n 1 gpurun_out/bench_gpt2.log

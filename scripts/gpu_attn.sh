#!/bin/bash
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q -k attention > gpurun_out/attn_tests.log 2>&1
rc=$?; echo "TESTS EXIT $rc"; tail -n 3 gpurun_out/attn_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python benchmarks/attn_bench.py > gpurun_out/attn_bench.jsonl 2>&1
rc=$?; cat gpurun_out/attn_bench.jsonl | grep shape; exit $rc

#!/bin/bash
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "cross or lm_head" > gpurun_out/xent_tests.log 2>&1
rc=$?; echo "TESTS EXIT $rc"; tail -n 3 gpurun_out/xent_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python benchmarks/xent_bench.py > gpurun_out/xent_bench.log 2>&1
rc=$?; echo "XBENCH EXIT $rc"; tail -n 1 gpurun_out/xent_bench.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-ckpt > gpurun_out/bench_nockpt.log 2>&1
rc=$?; echo "BENCH EXIT $rc"; tail -n 1 gpurun_out/bench_nockpt.log | cut -c1-400
exit $rc

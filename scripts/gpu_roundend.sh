#!/bin/bash
# Round-end rehearsal of what the driver runs: GPU test suite, smoke(), default bench (with the
# checkpoint phase), then the 2-rank gloo rehearsal of the multi-GPU bench path.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread \
  > gpurun_out/re_tests.log 2>&1
rc=$?; echo "TESTS EXIT $rc"; tail -n 5 gpurun_out/re_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/re_smoke.log 2>&1
rc=$?; echo "SMOKE EXIT $rc"; tail -n 2 gpurun_out/re_smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/re_bench.log 2>&1
rc=$?; echo "BENCH EXIT $rc"; tail -n 1 gpurun_out/re_bench.log
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_multirank.sh

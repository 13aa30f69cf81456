#!/bin/bash
# GPU test suite + default headline bench (+ optional extra bench args as $@)
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread \
  > gpurun_out/tests.log 2>&1
rc=$?; echo "TESTS EXIT $rc"; tail -n 5 gpurun_out/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py "$@" > gpurun_out/bench.log 2>&1
rc=$?; echo "BENCH EXIT $rc"; tail -n 3 gpurun_out/bench.log
exit $rc

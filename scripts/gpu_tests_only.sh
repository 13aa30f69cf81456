#!/bin/bash
# Run a subset of GPU tests: scripts/gpu_tests_only.sh <pytest args>
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread "$@" > gpurun_out/tests_sub.log 2>&1
rc=$?; echo "TESTS EXIT $rc"; tail -n 15 gpurun_out/tests_sub.log
exit $rc

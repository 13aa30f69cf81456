#!/bin/bash
# run the given GPU test files (default: all GPU tests) under one pytest process
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
FILES=${@:-tests}
timeout -k 10 900 python -m pytest $FILES -x -q -m gpu > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "TESTS EXIT $rc"; tail -n 40 gpurun_out/gpu_tests.log
exit $rc

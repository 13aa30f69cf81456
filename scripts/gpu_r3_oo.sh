#!/bin/bash
# Round-3 pass OO: full GPU suite with the 3x3 weight-gradient kernel, then the ResNet-18 kernel
# statistics (on / off).
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/oo_tests.log 2>&1
rc=$?; echo "TESTS EXIT $rc"; tail -n 3 gpurun_out/oo_tests.log
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_r3_nn.sh

#!/bin/bash
# kernel/model GPU tests, then the GPT-2 headline bench + kernel profile
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "TESTS EXIT $rc"; tail -n 25 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_gpt2_prof.sh

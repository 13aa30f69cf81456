#!/bin/bash
# Round-3 pass I (re-entry): full GPU test suite on the rebuilt extension, then pass H
# (GPT-2 step kernel trace with the native LM head + 2-rank gloo rehearsal).
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "TESTS EXIT $rc"; tail -n 5 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_prof_gpt2.sh && bash scripts/gpu_multirank.sh

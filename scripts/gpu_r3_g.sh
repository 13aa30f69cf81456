#!/bin/bash
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -u scripts/debug_copies_r3.py > gpurun_out/r3g_copies.txt 2>&1
rc=$?; echo "COPIES EXIT $rc"; head -20 gpurun_out/r3g_copies.txt
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_gemm_diag_r3.sh

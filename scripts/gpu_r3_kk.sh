#!/bin/bash
# Round-3 pass KK: which parameters differ in the 1-rank forced-collective RCCL DDP test, and
# under which deferral knobs.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -u scripts/diag_ddp_rccl.py fp32 > gpurun_out/kk_default.log 2>&1
rc=$?; echo "DEFAULT EXIT $rc"; grep -E "DIFF|differ" gpurun_out/kk_default.log | head -20
[ $rc -eq 0 ] || exit $rc
RTDC_COLSUM_DEFER=0 timeout -k 10 200 python -u scripts/diag_ddp_rccl.py fp32 > gpurun_out/kk_defer0.log 2>&1
rc=$?; echo "DEFER0 EXIT $rc"; grep -E "DIFF|differ" gpurun_out/kk_defer0.log | head -20
[ $rc -eq 0 ] || exit $rc
RTDC_WGRAD_SIDE=0 timeout -k 10 200 python -u scripts/diag_ddp_rccl.py fp32 > gpurun_out/kk_side0.log 2>&1
rc=$?; echo "SIDE0 EXIT $rc"; grep -E "DIFF|differ" gpurun_out/kk_side0.log | head -20

#!/bin/bash
# Round-3 pass QQ: Cout = 64 conv tile knobs re-measured on this build (stem + layer 1):
# RTDC_CONV64WG_W8 (8-wave 64x256 weight-gradient tile: now only the stem's) and RTDC_CONV64_W8.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
  for cfg in "RTDC_CONV64WG_W8=0" "RTDC_CONV64WG_W8=1" "RTDC_CONV64_W8=0"; do
    tag=$(echo $cfg | tr '=' '_')
    env $cfg timeout -k 10 200 python bench.py --model resnet18 --steps 30 --warmup 5 --no-ckpt > gpurun_out/resnet_qq_${tag}_r$r.log 2>&1
    rc=$?; echo "RESNET $cfg r$r EXIT $rc $(tail -n 1 gpurun_out/resnet_qq_${tag}_r$r.log | grep -o '"ms_per_step": [0-9.]*')"
    [ $rc -eq 0 ] || exit $rc
  done
done

#!/bin/bash
# Round-3 pass HH: BatchNorm statistics-pass grid (RTDC_BN_LOADS 16-B loads per thread: 32 / 16 / 8)
# on ResNet-18, alternating, two rounds.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
  for v in 32 16 8; do
    RTDC_BN_LOADS=$v timeout -k 10 200 python bench.py --model resnet18 --steps 30 --warmup 5 --no-ckpt > gpurun_out/resnet_hh_${v}_r$r.log 2>&1
    rc=$?; echo "RESNET BN_LOADS=$v r$r EXIT $rc $(tail -n 1 gpurun_out/resnet_hh_${v}_r$r.log | grep -o '"ms_per_step": [0-9.]*')"
    [ $rc -eq 0 ] || exit $rc
  done
done

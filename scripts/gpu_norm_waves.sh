#!/bin/bash
# LayerNorm backward grid size A/B (RTDC_NORM_BWD_WAVES) on the headline bench + kernel times
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
for nw in 4096 3072 2048; do
  RTDC_NORM_BWD_WAVES=$nw timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/nw_prof_$nw -o run -- python3 bench.py --steps 5 --warmup 2 --no-ckpt > gpurun_out/nw_prof_$nw.log 2>&1
  rc=$?; echo "PROF $nw EXIT $rc"; [ $rc -eq 0 ] || exit $rc
done

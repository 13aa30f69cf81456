#!/bin/bash
# per-kernel time of the column reductions, two-launch vs wide one-launch (RTDC_COLSUM_WIDE)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in 0 1; do
  RTDC_COLSUM_WIDE=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/cs_$v -o run -- python3 bench.py --steps 10 --warmup 3 --no-ckpt > gpurun_out/cs_$v.log 2>&1
  rc=$?; echo "PROF $v EXIT $rc"; [ $rc -eq 0 ] || exit $rc
  f=$(find gpurun_out/cs_$v -name '*kernel_stats.csv' | head -1)
  python3 scripts/kstats.py "$f" 13 40 | grep -E "total|colsum|norm_bwd" 
done

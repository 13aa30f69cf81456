#!/bin/bash
# per-kernel time of the GPT-2 step under two values of one knob: bash scripts/gpu_env_prof.sh VAR A B [grep]
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
var=$1; a=$2; b=$3; pat=${4:-gemm8}
for v in $a $b; do
  env "$var=$v" timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ep_$v -o run -- python3 bench.py --steps 10 --warmup 3 --no-ckpt > gpurun_out/ep_$v.log 2>&1
  rc=$?; echo "PROF $var=$v EXIT $rc"; [ $rc -eq 0 ] || exit $rc
  f=$(find gpurun_out/ep_$v -name '*kernel_stats.csv' | head -1)
  python3 scripts/kstats.py "$f" 13 40 | grep -E "total|$pat"
done

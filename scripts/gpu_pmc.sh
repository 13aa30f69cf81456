#!/bin/bash
# One rocprofv3 --pmc pass per counter group (kernel trace only; never combined with other
# traces).  usage: gpu_pmc.sh <label> "<counters>" -- <program args...>
set -o pipefail
label=$1; counters=$2; shift 3
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmc_$label -o run \
  --pmc $counters -- "$@" > gpurun_out/pmc_$label.log 2>&1
rc=$?; echo "PMC $label EXIT $rc"
[ $rc -eq 0 ] || exit $rc
f=$(find gpurun_out/pmc_$label -name '*counter_collection.csv' | head -1)
python3 scripts/pmc_summary.py "$f" rtdc > gpurun_out/pmc_${label}_summary.txt
cat gpurun_out/pmc_${label}_summary.txt

#!/bin/bash
# roctx phase ranges (fwd / bwd / opt) of the GPT-2 bench step: rocprofv3 marker + kernel trace
# (no counters in this run)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --marker-trace --kernel-trace --output-format csv -d gpurun_out/marker -o run \
  -- python3 bench.py --steps 5 --warmup 2 --no-ckpt > gpurun_out/marker.log 2>&1
rc=$?; echo "MARKER EXIT $rc"
[ $rc -eq 0 ] || exit $rc
ls gpurun_out/marker

#!/bin/bash
# Two gloo ranks on one GPU, each under its own rocprofv3 --hip-trace --kernel-trace (the program
# directly after `--`; no launcher that re-execs), running scripts/diag_postckpt.py with
# DIAG_MODE (default rawstream).  Summaries: scripts/diag_trace.py gpurun_out/diag_r0.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1 MASTER_PORT=${MASTER_PORT:-29631} WORLD_SIZE=2
export DIAG_MODE=${DIAG_MODE-rawstream} DIAG_N=${DIAG_N:-3}
mkdir -p gpurun_out
pids=()
for r in 0 1; do
  rm -rf gpurun_out/diag_r$r
  RANK=$r LOCAL_RANK=$r timeout -k 10 ${DIAG_TIMEOUT:-300} rocprofv3 --hip-trace --kernel-trace --output-format csv \
    -d gpurun_out/diag_r$r -o run -- python3 scripts/diag_postckpt.py > gpurun_out/diag_r$r.log 2>&1 &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait "$p" || rc=$?; done
echo "[diag_trace] EXIT $rc"
tail -n 8 gpurun_out/diag_r0.log
[ $rc -eq 0 ] && python3 scripts/diag_trace.py gpurun_out/diag_r0 gpurun_out/diag_r0.log > gpurun_out/diag_trace_summary.txt
exit $rc

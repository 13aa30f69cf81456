#!/bin/bash
# One gpurun batch (edit the step list per call): each GPU step runs under its own timeout and
# the batch stops at the first step that ends by signal / timeout (rc > 1); test failures
# (rc 1) do not stop it.  Logs: gpurun_out/<step>.log.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # step <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[$name] EXIT $rc"; tail -n 2 "gpurun_out/$name.log"
  if [ $rc -gt 1 ]; then echo "stopping after $name"; exit $rc; fi
}
step snap_tests 200 python -u -m pytest tests/test_snapshot_gpu.py -x -v -s --timeout 150 --timeout-method thread
GPU_MAX_HW_QUEUES=2 DIAG_TIMEOUT=250 step diag_trace_q2 300 bash scripts/diag_trace.sh
cp gpurun_out/diag_trace_summary.txt gpurun_out/diag_trace_summary_q2.txt 2>/dev/null
step gpu_tests 900 python -u -m pytest tests -m gpu -x -v -s --timeout 200 --timeout-method thread
step bench_gpt2 400 python bench.py --steps 20 --warmup 5

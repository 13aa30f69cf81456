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
  echo "[$name] EXIT $rc"; tail -n 2 "gpurun_out/$name.log" | cut -c1-300
  if [ $rc -gt 1 ]; then echo "stopping after $name"; exit $rc; fi
}
step final3_gpu_tests 700 python -u -m pytest tests -x -v -m gpu --timeout 200 --timeout-method thread
step final3_smoke 240 python -c 'import __graft_entry__ as g; g.smoke()'
step final3_bench_gpt2 500 python bench.py

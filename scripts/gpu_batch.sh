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
  echo "[$name] EXIT $rc"; tail -n 3 "gpurun_out/$name.log"
  if [ $rc -gt 1 ]; then echo "stopping after $name"; exit $rc; fi
}
step resume_test 300 python -u -m pytest tests/test_resume_fullsize_gpu.py -v -s --timeout 240 --timeout-method thread
step gpu_tests 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread
step product 1100 python3 scripts/product_path.py gpurun_out/product

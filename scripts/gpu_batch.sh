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
step attn_def 300 python -u benchmarks/attn_bench.py --only gpt2
step attn_fwd2 300 env RTDC_FA_FWD=2 python -u benchmarks/attn_bench.py --only gpt2
step attn_fwd3 300 env RTDC_FA_FWD=3 python -u benchmarks/attn_bench.py --only gpt2
step attn_dq1 300 env RTDC_FA_DQ=1 python -u benchmarks/attn_bench.py --only gpt2
step attn_dkdv1 300 env RTDC_FA_DKDV=1 python -u benchmarks/attn_bench.py --only gpt2
step attn_ns3 300 env RTDC_FA_NS=3 python -u benchmarks/attn_bench.py --only gpt2
step attn_def2 300 python -u benchmarks/attn_bench.py --only gpt2

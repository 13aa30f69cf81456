#!/bin/bash
# ResNet-18 step as captured hipGraph replays (bench --graph auto) vs eager launches
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_models_gpu.py -k "hipgraph or captured" > gpurun_out/r_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r_tests.log; exit 1; }
tail -n 1 gpurun_out/r_tests.log
for r in 1 2; do for arm in graph eager; do
  if [ $arm = graph ]; then g=auto; else g=0; fi
  timeout -k 10 300 python bench.py --model resnet18 --graph $g > gpurun_out/r_bench_${arm}_$r.log 2>&1 || { echo "bench $arm failed"; tail -20 gpurun_out/r_bench_${arm}_$r.log; exit 1; }
  echo "$arm $r $(grep '^{' gpurun_out/r_bench_${arm}_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d.get("ms_per_step_during_async_save"), d.get("step_launch"), d.get("ckpt_save_plus_restore_s"))')"
done; done

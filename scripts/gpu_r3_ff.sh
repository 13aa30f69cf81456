#!/bin/bash
# Round-3 pass FF (round-end rehearsal of this build): the whole GPU test suite, smoke(), the
# default bench (GPT-2-small, with checkpoint) and a PMC pass over the GPT-2 step.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/ff_tests.log 2>&1
rc=$?; echo "TESTS EXIT $rc"; tail -n 3 gpurun_out/ff_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/ff_smoke.log 2>&1
rc=$?; echo "SMOKE EXIT $rc"; tail -n 1 gpurun_out/ff_smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/ff_bench.log 2>&1
rc=$?; echo "BENCH EXIT $rc $(tail -n 1 gpurun_out/ff_bench.log | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' | tr '\n' ' ')"
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_pmc_step.sh > gpurun_out/ff_pmc.out 2>&1
rc=$?; echo "PMC EXIT $rc"; head -14 gpurun_out/pmc_step_summary.txt

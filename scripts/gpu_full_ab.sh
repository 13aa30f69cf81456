#!/bin/bash
# full GPU test suite on the new build, then A/B headline bench old (ab/_C_old.so) vs new,
# then the new build's kernel profile
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
[ -n "$SKIP_TESTS" ] || timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_full.log 2>&1
rc=$?; echo "TESTS EXIT $rc"; tail -n 4 gpurun_out/t_full.log
[ $rc -eq 0 ] || exit $rc
OLD=/root/repo/ab/_C_old.so
for arm in ${ARMS:-old new old new}; do
  if [ $arm = old ]; then export RTDC_EXT_SO=$OLD; else unset RTDC_EXT_SO; fi
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-ckpt > gpurun_out/fab_bench_$arm.log 2>&1
  rc=$?; echo "BENCH $arm EXIT $rc"; tail -n 1 gpurun_out/fab_bench_$arm.log | cut -c1-150
  [ $rc -eq 0 ] || exit $rc
done
unset RTDC_EXT_SO
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fab_prof_new -o run -- python3 bench.py --steps 5 --warmup 2 --no-ckpt > gpurun_out/fab_prof_new.log 2>&1
echo "PROF EXIT $?"

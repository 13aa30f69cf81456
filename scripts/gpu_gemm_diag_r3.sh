#!/bin/bash
# Where does the 8-wave GEMM main loop lose time?  Timing-only builds (ab/_C_diag<N>.so, see
# scripts/build_diag_so.sh) vs the shipped build, cfg 6 forced, two alternating rounds.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
  for N in 0 1 2 4 5; do
    if [ $N = 0 ]; then unset RTDC_EXT_SO; else export RTDC_EXT_SO=/root/repo/ab/_C_diag$N.so; fi
    for shp in sq4096 fc; do
      timeout -k 10 120 python -u benchmarks/gemm_bench.py --reps 20 --only $shp --sweep --cfgs 6 > gpurun_out/diag_${N}_${shp}_$r.jsonl 2>&1
      rc=$?; echo "diag$N $shp r$r EXIT $rc"
      [ $rc -eq 0 ] || exit $rc
      python3 -c "import json; d=[json.loads(l) for l in open('gpurun_out/diag_${N}_${shp}_$r.jsonl') if l.startswith('{')][0]; print('   ', {k: v for k, v in d.items() if 'cfg' in k})"
    done
  done
done

#!/bin/bash
# Round-3 pass S: Cout = 64 weight gradients on 8-wave 64x256 tiles (RTDC_CONV64WG_W8) - CNN tests
# under it, ResNet-18 benches interleaved 1,0,1,0, then a kernel trace of the default build.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
RTDC_CONV64WG_W8=1 timeout -k 10 300 python -u -m pytest tests/test_cnn_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/cnn_tests_wg8.log 2>&1
rc=$?; echo "CNN TESTS WG8 EXIT $rc"; tail -n 3 gpurun_out/cnn_tests_wg8.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for w in 1 0; do
    RTDC_CONV64WG_W8=$w timeout -k 10 200 python bench.py --model resnet18 --steps 20 --warmup 5 --no-ckpt > gpurun_out/resnet_wg8_${w}_r$r.log 2>&1
    rc=$?; echo "RESNET WG8=$w r$r EXIT $rc $(tail -n 1 gpurun_out/resnet_wg8_${w}_r$r.log | grep -o '"ms_per_step": [0-9.]*')"
    [ $rc -eq 0 ] || exit $rc
  done
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_resnet -o run -- python3 bench.py --model resnet18 --steps 5 --warmup 2 --no-ckpt > gpurun_out/prof_resnet.log 2>&1
rc=$?; echo "PROF EXIT $rc"
[ $rc -eq 0 ] || exit $rc
f=$(find gpurun_out/prof_resnet -name '*kernel_stats.csv' | head -1)
python3 scripts/kstats.py "$f" 7 40 > gpurun_out/prof_resnet_summary.txt
t=$(find gpurun_out/prof_resnet -name '*kernel_trace.csv' | head -1)
python3 scripts/kstep.py "$t" --marker sgd_kernel > gpurun_out/prof_resnet_step.txt
head -24 gpurun_out/prof_resnet_summary.txt

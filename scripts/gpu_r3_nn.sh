#!/bin/bash
# Round-3 pass NN: ResNet-18 kernel statistics with the 3x3 weight-gradient kernel on and off.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in 1 0; do
  RTDC_CONV3_WGRAD=$v timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/nn_prof$v -o run -- python3 bench.py --model resnet18 --steps 10 --warmup 3 --no-ckpt > gpurun_out/nn_prof$v.log 2>&1
  rc=$?; echo "PROF $v EXIT $rc"
  [ $rc -eq 0 ] || exit $rc
  f=$(find gpurun_out/nn_prof$v -name '*kernel_stats.csv' | head -1)
  head -16 "$f" | cut -c1-200
done

#!/bin/bash
# Checkpoint engine sweep on the GPT-2-small train state (1.49 GB): writer threads x pinned
# slot size x slot count; sync save / cold restore wall-clock from bench.py
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
df -h /tmp | tail -1
for r in 1 2; do
  for cfg in "8 64 8" "16 64 16" "8 128 8" "16 128 8" "4 64 8"; do
    set -- $cfg
    RTDC_CKPT_WRITERS=$1 RTDC_CKPT_SLOT_MB=$2 RTDC_CKPT_SLOTS=$3 timeout -k 10 200 python bench.py --steps 3 --warmup 2 \
      > gpurun_out/ck_$1_$2_$3_$r.log 2>&1
    rc=$?
    echo "w=$1 slot=$2 n=$3 r$r EXIT $rc $(tail -1 gpurun_out/ck_$1_$2_$3_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print({k: d.get(k) for k in ["ckpt_save_blocking_s","ckpt_save_durable_s","ckpt_save_sync_s","ckpt_write_GBps","ckpt_restore_s","ckpt_restore_warm_s","ckpt_restore_GBps"]})')"
    [ $rc -eq 0 ] || exit $rc
  done
done

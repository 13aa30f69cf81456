#!/bin/bash
# checkpoint writers: PCLMUL CRC-32 (default) vs the system zlib table CRC (RTDC_CRC_ZLIB=1),
# GPT-2-small train state, one process, alternating arms
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2 3; do for arm in pclmul zlib; do
  if [ $arm = zlib ]; then e="RTDC_CRC_ZLIB=1"; else e="RTDC_CRC_ZLIB=0"; fi
  env $e timeout -k 10 240 python bench.py --steps 5 --warmup 2 > gpurun_out/crc_${arm}_$r.log 2>&1 || { echo "$arm failed"; tail -5 gpurun_out/crc_${arm}_$r.log; exit 1; }
  echo "$arm $r $(grep '^{' gpurun_out/crc_${arm}_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ("ckpt_save_durable_s","ckpt_save_sync_s","ckpt_write_GBps","ckpt_restore_s","ms_per_step_during_async_save","ms_per_step")})')"
done; done

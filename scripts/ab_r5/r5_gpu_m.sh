#!/bin/bash
# restore: native batch zip-record locator (default) vs the per-item Python parser (RTDC_ZIP_PARSE=py)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2 3; do for arm in native py; do
  RTDC_ZIP_PARSE=$arm timeout -k 10 240 python bench.py --steps 5 --warmup 2 > gpurun_out/zip_${arm}_$r.log 2>&1 || { echo "$arm failed"; tail -5 gpurun_out/zip_${arm}_$r.log; exit 1; }
  echo "$arm $r $(grep '^{' gpurun_out/zip_${arm}_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ("ckpt_restore_s","ckpt_restore_warm_s","ckpt_save_sync_s","ckpt_save_durable_s","ckpt_save_plus_restore_s")})')"
done; done

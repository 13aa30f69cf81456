#!/bin/bash
# Round-3 pass K: what does hipBLASLt's kernel look like on the GPT-2 shapes?  Kernel trace of
# gemm_bench (plain fwd / dgrad of fc, mlp_proj, lm_head, sq4096): per-kernel VGPR / AGPR /
# LDS / workgroup size / grid of the Cijk kernels next to ours.
set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_blaslt -o run -- python3 benchmarks/gemm_bench.py --reps 3 > gpurun_out/prof_blaslt.log 2>&1
rc=$?; echo "PROF EXIT $rc"; tail -3 gpurun_out/prof_blaslt.log
[ $rc -eq 0 ] || exit $rc
t=$(find gpurun_out/prof_blaslt -name '*kernel_trace.csv' | head -1)
python3 - "$t" > gpurun_out/blaslt_kernels.txt <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
print(list(rows[0].keys()))
seen = collections.OrderedDict()
for r in rows:
    k = (r["Kernel_Name"][:150], r.get("Grid_Size"), r.get("Workgroup_Size"))
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    if k not in seen:
        seen[k] = [r, []]
    seen[k][1].append(d)
for (name, grid, wg), (r, ds) in seen.items():
    if "gemm" not in name and "Cijk" not in name:
        continue
    ds.sort()
    print(f"{ds[len(ds)//2]:9.1f} us  grid {grid:>9} wg {wg:>4} vgpr {r.get('VGPR_Count')} agpr {r.get('Accum_VGPR_Count')} sgpr {r.get('SGPR_Count')} lds {r.get('LDS_Block_Size')} scratch {r.get('Scratch_Size')}  {name}")
PY
cat gpurun_out/blaslt_kernels.txt | cut -c1-260 | head -80

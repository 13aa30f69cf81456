"""Per-kernel-family MFMA utilisation, LDS bank-conflict rate and HBM bytes from rocprofv3
--pmc counter_collection.csv files of a bench run.

MFMA utilisation = SQ_VALU_MFMA_BUSY_CYCLES / (GPU cycles x 4 SIMDs x #CUs): the share of
SIMD-cycles the matrix pipe was busy while the kernel ran (busy cycles are summed over SIMDs;
a v_mfma_f32_16x16x32_bf16 counts 16).  GPU cycles = GRBM_GUI_ACTIVE / 8: rocprofv3 sums the
counter over the 8 XCDs (checked on the hipBLASLt LM-head GEMM: 1.27 TFLOP in 1.07 ms at
~2.1 GHz is 54 % of the 16x16x32 rate, the counters give 54.4 %).  LDS conflicts are
SQ_LDS_BANK_CONFLICT cycles per LDS instruction; bytes read are FETCH_SIZE (KiB)."""
import csv
import sys
from collections import defaultdict

NCU = 256
NXCD = 8


def load(path):
    per = defaultdict(lambda: defaultdict(float))
    for r in csv.DictReader(open(path)):
        key = (r["Dispatch_Id"], r["Kernel_Name"])
        per[key][r["Counter_Name"]] += float(r["Counter_Value"])
    return per


def family(name: str) -> str:
    n = name.replace("void ", "")
    return n.split("(")[0][:80]


def main():
    fam = defaultdict(lambda: defaultdict(float))
    cnt = defaultdict(int)
    for i, path in enumerate(sys.argv[1:]):
        for (_d, k), cs in load(path).items():
            f = family(k)
            if i == 0:
                cnt[f] += 1
            for c, v in cs.items():
                fam[f][c + ("" if i == 0 else "#2")] += v
    rows = sorted(fam.items(), key=lambda kv: -kv[1].get("GRBM_GUI_ACTIVE", 0))
    tot_active = sum(v.get("GRBM_GUI_ACTIVE", 0) for _, v in rows) / NXCD
    tot_mfma = sum(v.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) for _, v in rows)
    print(f"all kernels: GPU-active cycles {tot_active:.3e}, MFMA utilisation "
          f"{100 * tot_mfma / max(1, tot_active * 4 * NCU):.1f} % (busy SIMD-cycles / active cycles x 4 x {NCU})")
    print(f"{'kernel family':80s} {'disp':>5s} {'time%':>6s} {'mfma%':>6s} {'conf/lds':>8s} {'GB rd':>7s}")
    for f, v in rows:
        act = v.get("GRBM_GUI_ACTIVE", 0) / NXCD
        mf = v.get("SQ_VALU_MFMA_BUSY_CYCLES", 0)
        lds = v.get("SQ_INSTS_LDS", 0)
        conf = v.get("SQ_LDS_BANK_CONFLICT", 0)
        rd = v.get("FETCH_SIZE#2", 0) * 1024 / 1e9
        print(f"{f:80s} {cnt[f]:5d} {100 * act / max(1, tot_active):6.1f} {100 * mf / max(1, act * 4 * NCU):6.1f} "
              f"{conf / max(1, lds):8.2f} {rd:7.2f}")


if __name__ == "__main__":
    main()

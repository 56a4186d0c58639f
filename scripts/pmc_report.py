"""Per-kernel summary of rocprofv3 counter passes (pmc_sq.sh / pmc_ta.sh output dirs):
per-wave instruction mix, VALU-issue time share, TA/TD busy, LDS bank conflicts.
usage: python scripts/pmc_report.py <dir> [<dir> ...]"""
import collections
import csv
import glob
import sys

agg = collections.defaultdict(lambda: collections.defaultdict(float))
for d in sys.argv[1:]:
    for f in glob.glob(f"{d}/**/run_counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("cdb::", "").replace("(anonymous namespace)::", "")
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, c in agg.items():
    w = c.get("SQ_WAVES", 0)
    print(k)
    if w:
        per = {n: c[n] / w for n in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD",
                                     "SQ_INSTS_VMEM_WR", "SQ_INSTS_BRANCH", "SQ_INSTS_SMEM") if n in c}
        print("   per wave:", {n.replace("SQ_INSTS_", ""): round(v, 1) for n, v in per.items()}, "waves", int(w))
    g = c.get("GRBM_GUI_ACTIVE", 0)
    for n in sorted(c):
        print(f"   {n:34s} {c[n]:.4g}" + (f"   ({c[n] / g / 256:.3f} per CU-cycle)" if g and n.startswith(("TA_", "TD_")) else ""))

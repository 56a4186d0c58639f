"""Counters of the LAST dispatch of each kernel matching a regex (the bench's timed merge: the
setup merges run the same kernels before it), summed over the passes of a pmc_sq.sh run.
Usage: python3 scripts/pmc_last.py gpurun_out/pmc_<tag> [regex]"""
import collections
import csv
import glob
import re
import sys

root, rx = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "bucket_wave_pipe")
last = {}
for f in sorted(glob.glob(f"{root}/pass*/**/*counter_collection.csv", recursive=True)):
    rows = [r for r in csv.DictReader(open(f)) if re.search(rx, r["Kernel_Name"])]
    if not rows:
        continue
    disp = max(int(r["Dispatch_Id"]) for r in rows)
    acc = collections.defaultdict(float)
    for r in rows:
        if int(r["Dispatch_Id"]) == disp:
            acc[r["Counter_Name"]] += float(r["Counter_Value"])
    last.update(acc)
for k in sorted(last):
    print(f"{k:28s} {last[k]:18.6g}")
w = last.get("SQ_WAVE_CYCLES")
if w:
    for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS"):
        if k in last:
            print(f"{k} / SQ_WAVE_CYCLES = {last[k] / w:.3f}")

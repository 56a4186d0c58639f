"""Sums rocprofv3 --pmc counter values per kernel over every pass directory given:
python3 scripts/pmc_sum.py <dir>... -> one line per kernel with each counter's total (and per wave)."""
import collections
import csv
import glob
import os
import sys

tot = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for d in sys.argv[1:]:
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0][:48]
            tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[k].add(r.get("Dispatch_Id", ""))
for k, c in sorted(tot.items(), key=lambda kv: -kv[1].get("SQ_WAVES", 0)):
    w = c.get("SQ_WAVES", 0)
    print(f"{k}  dispatches={len(disp[k])}")
    for n, v in sorted(c.items()):
        print(f"    {n:34s} {v:16.4g}" + (f"   per wave {v / w:10.1f}" if w and n != "SQ_WAVES" else ""))

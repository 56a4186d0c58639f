"""Prints a rocprofv3 kernel_stats.csv compactly: short kernel name (+ template args), calls, avg us."""
import csv
import sys

pat = sys.argv[2].split(",") if len(sys.argv) > 2 else None
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"].replace("(anonymous namespace)::", "")
    base = n.split("(")[0].split("::")[-1]
    if n.startswith("void "):
        base = n[5:].split("(")[0]
        base = base.split("::")[-1] if "<" not in base else base[base.rfind("::", 0, base.index("<")) + 2:]
    base = base.replace("cdb::(anonymous namespace)::", "")
    if pat and not any(p in base for p in pat):
        continue
    print(f"{base[:70]:70s} {int(r['Calls']):5d} {float(r['AverageNs']) / 1e3:10.1f} us")

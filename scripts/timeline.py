"""Kernel timeline of the last merge step in a rocprofv3 kernel trace (between the last
merge_begin_marker and the merge_end_marker after it): start / end / duration in ms from the
step's first merge kernel."""
import csv
import glob
import sys

f = sys.argv[1]
if not f.endswith(".csv"):
    f = glob.glob(f + "/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
begins = [i for i, r in enumerate(rows) if "merge_begin_marker" in r["Kernel_Name"]]
i0 = begins[-1]
i1 = next(i for i in range(i0, len(rows)) if "merge_end_marker" in rows[i]["Kernel_Name"])
t0 = int(rows[i0]["Start_Timestamp"])
for r in rows[i0:i1 + 1]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"].replace("cdb::", "").replace("(anonymous namespace)::", "")
    print(f"{(s - t0) / 1e6:8.3f} {(e - t0) / 1e6:8.3f} {(e - s) / 1e6:7.3f}  {name[:70]}")

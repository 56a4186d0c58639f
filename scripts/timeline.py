"""Kernel timeline of the last merge step in a rocprofv3 kernel trace (between the last
merge_begin_marker and the merge_end_marker after it): start / end / duration in ms from the
step's first merge kernel.

--stats OUT.csv [--last K]: also write step-only kernel statistics -- the kernels of the last K
marker-bracketed merges (the bench's K timed steps when the traced command ran no merge after
them), per kernel name: calls, total / average / min / max duration -- the same columns as
rocprofv3's whole-run kernel_stats.csv, which also counts setup merges."""
import argparse
import csv
import glob

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--stats")
ap.add_argument("--last", type=int, default=1)
args = ap.parse_args()
f = args.trace
if not f.endswith(".csv"):
    f = glob.glob(f + "/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
begins = [i for i, r in enumerate(rows) if "merge_begin_marker" in r["Kernel_Name"]]


def step(i0):
    i1 = next(i for i in range(i0, len(rows)) if "merge_end_marker" in rows[i]["Kernel_Name"])
    return rows[i0:i1 + 1]


def clean(name):
    return name.replace("cdb::", "").replace("(anonymous namespace)::", "")


last = step(begins[-1])
t0 = int(last[0]["Start_Timestamp"])
for r in last:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"{(s - t0) / 1e6:8.3f} {(e - t0) / 1e6:8.3f} {(e - s) / 1e6:7.3f}  {clean(r['Kernel_Name'])[:70]}")

if args.stats:
    agg = {}
    steps = begins[-args.last:]
    for i0 in steps:
        for r in step(i0):
            d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            a = agg.setdefault(clean(r["Kernel_Name"]), [0, 0, None, 0])
            a[0] += 1
            a[1] += d
            a[2] = d if a[2] is None else min(a[2], d)
            a[3] = max(a[3], d)
    with open(args.stats, "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["Name", "Calls", "Steps", "TotalDurationNs", "AverageNs", "PerStepNs", "MinNs", "MaxNs",
                     "Percentage"])
        tot = sum(a[1] for a in agg.values()) or 1
        for name, a in sorted(agg.items(), key=lambda kv: -kv[1][1]):
            w.writerow([name, a[0], len(steps), a[1], a[1] // a[0], a[1] // len(steps), a[2], a[3],
                        f"{100.0 * a[1] / tot:.3f}"])

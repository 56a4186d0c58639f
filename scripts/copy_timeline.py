"""Decode-call timeline from a rocprofv3 --kernel-trace --memory-copy-trace directory: the
host-to-device copies over 1 ms (span and busy union) and, per kernel, first start, last end and
busy time, relative to the first large copy."""
import collections
import csv
import glob
import sys

d = glob.glob(sys.argv[1] + "/**/run_kernel_trace.csv", recursive=True)[0].rsplit("/", 1)[0]
K = list(csv.DictReader(open(d + "/run_kernel_trace.csv")))
M = list(csv.DictReader(open(d + "/run_memory_copy_trace.csv")))
ev = [(int(k["Start_Timestamp"]), int(k["End_Timestamp"]), k["Kernel_Name"][:48]) for k in K]
h2d = [(int(m["Start_Timestamp"]), int(m["End_Timestamp"]), "H2D stream %s" % m["Stream_Id"]) for m in M
       if m["Direction"] == "MEMORY_COPY_HOST_TO_DEVICE"]
big = sorted((a, b) for a, b, _ in h2d if b - a > 1e6)
t0 = big[0][0]
busy, cur = 0, None
for a, b in big:
    if cur is None or a > cur[1]:
        busy += (cur[1] - cur[0]) if cur else 0
        cur = [a, b]
    else:
        cur[1] = max(cur[1], b)
busy += cur[1] - cur[0]
print("large H2D copies: first %.1f ms, last end %.1f ms, busy (union) %.1f ms" % (0.0, (big[-1][1] - t0) / 1e6, busy / 1e6))
first, last, tot, n = {}, {}, collections.Counter(), collections.Counter()
for a, b, k in sorted(ev + h2d):
    if a < t0 - 5e6:
        continue
    first.setdefault(k, (a - t0) / 1e6)
    last[k] = (b - t0) / 1e6
    tot[k] += (b - a) / 1e6
    n[k] += 1
for k, v in sorted(first.items(), key=lambda x: x[1])[: int(sys.argv[2]) if len(sys.argv) > 2 else 40]:
    print(f"{v:9.2f} {last[k]:9.2f}  n={n[k]:4d} busy {tot[k]:8.2f}  {k}")

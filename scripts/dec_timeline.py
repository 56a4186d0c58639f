"""Timeline of the largest decode call in a rocprofv3 kernel + memory-copy trace directory:
per kernel (and copy direction) busy time, first start and last end relative to the call."""
import collections
import csv
import sys

d = sys.argv[1]
K = list(csv.DictReader(open(f"{d}/run_kernel_trace.csv")))
M = list(csv.DictReader(open(f"{d}/run_memory_copy_trace.csv")))
ev = [(int(k["Start_Timestamp"]), int(k["End_Timestamp"]), k["Kernel_Name"][:44]) for k in K]
ev += [(int(m["Start_Timestamp"]), int(m["End_Timestamp"]), m["Direction"][12:]) for m in M]
ev.sort()
segs, cur = [], [ev[0]]
for e in ev[1:]:
    if e[0] - max(x[1] for x in cur[-50:]) > 20e6:
        segs.append(cur)
        cur = [e]
    else:
        cur.append(e)
segs.append(cur)
s = max(segs, key=len)
a = s[0][0]
print("call: %.2f ms" % ((max(x[1] for x in s) - a) / 1e6))
by, first, last, cnt = collections.defaultdict(float), {}, {}, collections.Counter()
for x in s:
    by[x[2]] += (x[1] - x[0]) / 1e6
    cnt[x[2]] += 1
    first.setdefault(x[2], (x[0] - a) / 1e6)
    last[x[2]] = (x[1] - a) / 1e6
for k, v in sorted(by.items(), key=lambda kv: -kv[1])[: int(sys.argv[2]) if len(sys.argv) > 2 else 12]:
    print("   %-46s n=%4d busy %7.2f ms  first %7.2f last %7.2f" % (k, cnt[k], v, first[k], last[k]))
if len(sys.argv) > 3:
    for x in s:
        if sys.argv[3] in x[2]:
            print("      %8.2f +%6.2f" % ((x[0] - a) / 1e6, (x[1] - x[0]) / 1e6))

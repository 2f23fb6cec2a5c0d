"""Per-kernel mean duration over launch-index windows of a rocprofv3 kernel
trace (one row per dispatch): python tools/trace_phases.py TRACE.csv A:B [C:D ...]
Windows count each kernel's launches in dispatch order (e.g. the bench's
pipelined frames, then its one-at-a-time frames)."""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Dispatch_Id"]))
by = collections.defaultdict(list)
for r in rows:
    n = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("jxg::", "")
    by[n].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
for win in sys.argv[2:]:
    a, b = (int(x) for x in win.split(":"))
    print("== launches [%d, %d) of each kernel" % (a, b))
    tot = 0.0
    for n, d in sorted(by.items(), key=lambda kv: -sum(kv[1][a:b])):
        w = d[a:b]
        if not w or n in ("synth_kernel",):
            continue
        m = sum(w) / len(w)
        tot += m
        print("  %-28s n=%3d mean %8.4f ms  min %8.4f" % (n, len(w), m, min(w)))
    print("  sum of means %.4f ms" % tot)

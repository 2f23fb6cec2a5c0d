"""Busy fractions of a rocprofv3 kernel trace over a time window given by
launch indices of one kernel: python tools/trace_busy.py TRACE.csv KERNEL A B
Window = [start of KERNEL's launch A, end of its launch B); reports the union
of all kernels' intervals and of each kernel's own intervals as fractions."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
name = lambda r: r["Kernel_Name"].split("(")[0].replace("void ", "").replace("jxg::", "")
iv = collections.defaultdict(list)
for r in rows:
    iv[name(r)].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
for k in iv:
    iv[k].sort()
K, A, B = sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
t0, t1 = iv[K][A][0], iv[K][B][1]


def union(ints):
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(ints):
        s, e = max(s, t0), min(e, t1)
        if e <= s:
            continue
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


W = t1 - t0
print("window %.3f ms (%s launches %d..%d)" % (W / 1e6, K, A, B))
allk = [x for v in iv.values() for x in v]
print("  any kernel     %.3f" % (union(allk) / W))
nonchain = [x for k, v in iv.items() if not k.startswith("ans_encode") for x in v]
print("  any non-chain  %.3f" % (union(nonchain) / W))
for k, v in sorted(iv.items(), key=lambda kv: -union(kv[1])):
    u = union(v)
    if u:
        print("  %-26s %.3f" % (k, u / W))

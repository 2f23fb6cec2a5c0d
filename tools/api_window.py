"""Main-thread HIP API time per frame over the middle of a rocprofv3 run
(window: front_kernel launches with grid z == Z, the middle 60 %):
  python tools/api_window.py DIR [Z]"""
import collections
import csv
import sys

d, Z = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "4")
ks = [r for r in csv.DictReader(open(d + "/run_kernel_trace.csv"))
      if "front_kernel" in r["Kernel_Name"] and r["Grid_Size_Z"] == Z]
ks.sort(key=lambda r: int(r["Start_Timestamp"]))
i0, i1 = len(ks) // 5, len(ks) * 4 // 5
a, b = int(ks[i0]["Start_Timestamp"]), int(ks[i1]["Start_Timestamp"])
nfr = sum(int(k["Grid_Size_Z"]) for k in ks[i0:i1])
rows = [r for r in csv.DictReader(open(d + "/run_hip_api_trace.csv")) if a <= int(r["Start_Timestamp"]) < b]
main = collections.Counter(r["Thread_Id"] for r in rows).most_common(1)[0][0]
for tag in ("main", "helpers"):
    th = collections.defaultdict(lambda: [0, 0])
    for r in rows:
        if (r["Thread_Id"] == main) != (tag == "main"):
            continue
        e = th[r["Function"]]
        e[0] += 1
        e[1] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    print("%s: window %.2f ms, %d frames -> %.3f ms/frame; API %.3f ms/frame"
          % (tag, (b - a) / 1e6, nfr, (b - a) / 1e6 / nfr, sum(v[1] for v in th.values()) / 1e6 / nfr))
    for f, (n, t) in sorted(th.items(), key=lambda kv: -kv[1][1])[:10]:
        print("  %-28s per frame n=%5.2f  %.4f ms  avg %.1f us" % (f, n / nfr, t / 1e6 / nfr, t / 1e3 / n))

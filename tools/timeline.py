"""Per-frame kernel timeline with idle gaps from a rocprofv3 kernel trace:
python3 tools/timeline.py PROF_DIR [first-kernel substring]"""
import csv, glob, sys
p = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
first = sys.argv[2] if len(sys.argv) > 2 else "front_kernel"
rows = sorted(csv.DictReader(open(p)), key=lambda r: int(r["Start_Timestamp"]))
fi = [i for i, r in enumerate(rows) if first in r["Kernel_Name"]]
seq = rows[fi[-3]:fi[-2] + 1]
t0 = int(seq[0]["Start_Timestamp"])
prev = None
idle = 0.0
for r in seq:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev) / 1000 if prev else 0.0
    idle += max(gap, 0)
    print("%8.1f gap %7.1f dur %7.1f %s" % ((s - t0) / 1000, gap, (e - s) / 1000, r["Kernel_Name"][:50]))
    prev = e
print("idle between kernels: %.1f us" % idle)

"""Experiment: summarize a rocprofv3 kernel trace of the streaming bench.

python tools/trace_pipe.py gpurun_out/TAG/<lib>/.../run_kernel_trace.csv [nlast]

Over the last `nlast` frames (ans_encode launches): frame period, per-kernel
average duration, and the time fractions during which (a) some chain runs,
(b) some transform kernel (front / merge / statistics / emission) runs,
(c) neither -- the GPU waiting on the host."""
import csv
import sys
from collections import defaultdict


def short(name):
    n = name.split("(")[0].replace("void ", "").replace("jxg::", "")
    return n.split("<")[0]


def main():
    path = sys.argv[1]
    nlast = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((short(r["Kernel_Name"]), int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    rows.sort(key=lambda x: x[1])
    chains = [r for r in rows if r[0] == "ans_encode_kernel"]
    if len(chains) < nlast + 1:
        nlast = len(chains) - 1
    t0 = chains[-nlast - 1][1]
    t1 = chains[-1][1]
    win = [r for r in rows if r[1] >= t0 and r[1] < t1]
    print("frames %d  period %.3f ms" % (nlast, (t1 - t0) / nlast / 1e6))
    dur = defaultdict(list)
    for n, a, b in win:
        dur[n].append((b - a) / 1e6)
    for n, d in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
        print("  %-28s n %4d avg %.3f ms  sum/frame %.3f ms" % (n, len(d), sum(d) / len(d), sum(d) / nlast))
    # time fractions on a 10 us grid
    step = 10_000
    nb = (t1 - t0) // step + 1
    ch = bytearray(nb)
    tr = bytearray(nb)
    for n, a, b in rows:
        if b < t0 or a > t1:
            continue
        lo, hi = max(0, (a - t0) // step), min(nb - 1, (b - t0) // step)
        tgt = ch if n == "ans_encode_kernel" else tr
        for i in range(lo, hi + 1):
            tgt[i] = 1
    both = sum(1 for i in range(nb) if ch[i] and tr[i]) / nb
    onlyc = sum(1 for i in range(nb) if ch[i] and not tr[i]) / nb
    onlyt = sum(1 for i in range(nb) if tr[i] and not ch[i]) / nb
    idle = sum(1 for i in range(nb) if not ch[i] and not tr[i]) / nb
    print("time: chain+transform %.2f  chain only %.2f  transform only %.2f  idle %.2f" %
          (both, onlyc, onlyt, idle))


if __name__ == "__main__":
    main()

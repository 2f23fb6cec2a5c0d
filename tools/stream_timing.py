"""Experiment: host-side time per jxg_submit_rgb8_device / jxg_receive call for
a stream of device-resident frames (default 64 x 1080p, ANS)."""
import os, sys, time
os.environ["GPU_MAX_HW_QUEUES"] = "16"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "jpeg-xl-lossy-image-compression-thesis_amd"))
import numpy as np
import torch
import jxg
from jxg.synth import synth_rgb8_device
w, h, n = (int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 3 else (1920, 1080, 64)
flags = jxg.FLAG_ANS if (len(sys.argv) <= 4 or sys.argv[4] == "ans") else 0
nd = int(os.environ.get("NDISTINCT", "8"))
frames = [synth_rgb8_device(w, h, 0x4A584C03 + f) for f in range(nd)]
torch.cuda.synchronize()
enc = jxg.Encoder(distance=1.0, effort=7, flags=flags)
for rep in range(2):
    ts, tr = [], []
    t0 = time.perf_counter()
    for k in range(n):
        a = time.perf_counter()
        enc.submit_device(frames[k % nd].data_ptr(), w, h)
        ts.append(time.perf_counter() - a)
        while enc.pending() > 16:
            a = time.perf_counter(); enc.receive(copy=False); tr.append(time.perf_counter() - a)
    while enc.pending():
        a = time.perf_counter(); enc.receive(copy=False); tr.append(time.perf_counter() - a)
    dt = time.perf_counter() - t0
    st = enc.stats()
    print("rep", rep, "MPix/s %.0f" % (w * h * n / dt / 1e6), "ms/frame %.3f" % (dt * 1e3 / n),
          "submit ms p50 %.3f p90 %.3f max %.3f" % tuple(np.percentile(np.array(ts) * 1e3, [50, 90, 100])),
          "receive ms p50 %.3f max %.3f" % tuple(np.percentile(np.array(tr) * 1e3, [50, 100])) if tr else "",
          "codes %.3f layout %.3f" % (st["ms_host_codes"], st["ms_host_layout"]))
enc.close()

"""One-at-a-time 8K encodes (the bench frame, device input) through the
library JXG_LIB_PATH selects: median stage times (front kernel, AQ, merge,
statistics, emission = rANS chains + bit placement + LF coding) and the
codestream hash, per preset -- same-box A/B of builds:
  for l in a b; do JXG_LIB_PATH=tools/ab/libjxg_$l.so python tools/chain_probe.py; done"""
import hashlib
import os
import sys

os.environ.setdefault("GPU_MAX_HW_QUEUES", "16")
import numpy as np  # noqa: E402
import torch  # noqa: E402  (one HIP runtime)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "jpeg-xl-lossy-image-compression-thesis_amd"))
import jxg  # noqa: E402
from jxg.synth import synth_rgb8_device  # noqa: E402

n = int(os.environ.get("N", "12"))
t = synth_rgb8_device(7680, 4320, 0x4A584C02)
torch.cuda.synchronize()
lib = os.path.basename(os.environ.get("JXG_LIB_PATH", "") or "libjxg.so")
ALL = {"cjxl": jxg.FLAGS_CJXL_DEFAULTS, "plain": jxg.FLAG_ANS,
       "gab": jxg.FLAG_ANS | jxg.FLAG_GABORISH, "epf": jxg.FLAG_ANS | jxg.FLAG_EPF,
       "aqm": jxg.FLAG_ANS | jxg.FLAG_AQ_MASKING}
for preset in os.environ.get("PRESETS", "cjxl,plain").split(","):
    flags = ALL[preset]
    with jxg.Encoder(distance=1.0, effort=int(os.environ.get("EFFORT", "7")), flags=flags) as enc:
        rows, shas = [], set()
        for i in range(n + 2):
            b = enc.encode_device(t.data_ptr(), 7680, 4320)
            st = enc.stats()
            shas.add(hashlib.sha256(b).hexdigest()[:16])
            if i >= 2:
                rows.append((st["ms_front_kernel"], st.get("ms_aq", 0.0),
                             st["ms_front"] - st["ms_front_kernel"] - st.get("ms_aq", 0.0),
                             st["ms_histogram"], st["ms_emit"], st["ms_total"]))
        m = np.median(np.array(rows), axis=0)
        print("%-16s %-5s front %.4f aq %.4f merge %.4f hist %.4f emit %.4f total %.4f  %d B sha %s"
              % (lib, preset, *m, len(b), ",".join(sorted(shas))), flush=True)

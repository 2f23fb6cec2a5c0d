"""Front-kernel phase split (JXG_FRONT_PROFILE builds: JXG_LIB_PATH=tools/ab/libjxg_fprof.so):
N one-at-a-time 8K encodes at the given effort / preset; the library prints the
per-phase shader-clock sums of thread 0 of every workgroup at context destroy.
Usage: JXG_LIB_PATH=... python tools/front_phase_probe.py EFFORT PRESET(cjxl|plain) [N]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "jpeg-xl-lossy-image-compression-thesis_amd"))
import torch  # noqa: F401  (one HIP runtime per process: torch first)

import jxg
from jxg.synth import synth_rgb8_device

e = int(sys.argv[1])
preset = sys.argv[2]
n = int(sys.argv[3]) if len(sys.argv) > 3 else 5
flags = jxg.FLAGS_CJXL_DEFAULTS if preset == "cjxl" else 0
w, h = 7680, 4320
t = synth_rgb8_device(w, h, 0x4A584C02)
torch.cuda.synchronize()
enc = jxg.Encoder(distance=1.0, effort=e, flags=flags)
enc.encode_device(t.data_ptr(), w, h)  # warm (counted too)
fk = []
mk = []
for _ in range(n):
    enc.encode_device(t.data_ptr(), w, h)
    fk.append(enc.timings()[0])
    if os.environ.get("PROBE_MERGE"):
        st = enc.stats()
        mk.append(st["ms_front"] - st["ms_front_kernel"])
print("effort %d preset %s: front kernel ms per launch %s (the profile sums %d launches)"
      % (e, preset, [round(x, 4) for x in fk], n + 1), flush=True)
if mk:
    print("effort %d preset %s: merge stage ms per encode %s" % (e, preset, [round(x, 4) for x in mk]), flush=True)
enc.close()

"""One-at-a-time 8K encodes at effort 8 (the bench frame, device input), for a
kernel trace of the 128 / 256 px merge levels (tools: rocprofv3 --kernel-trace --stats)."""
import os
import sys

os.environ.setdefault("GPU_MAX_HW_QUEUES", "16")
import torch  # noqa: E402,F401  (one HIP runtime)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "jpeg-xl-lossy-image-compression-thesis_amd"))
import jxg  # noqa: E402
from jxg.synth import natural_rgb8, synth_rgb8_device  # noqa: E402

n = int(os.environ.get("N", "3"))
kind = os.environ.get("FRAME", "synth")
if kind == "synth":
    t = synth_rgb8_device(7680, 4320, 0x4A584C02)
else:
    t = torch.from_numpy(natural_rgb8(7680, 4320, 3)).cuda()
torch.cuda.synchronize()
with jxg.Encoder(distance=1.0, effort=8, flags=jxg.FLAGS_CJXL_DEFAULTS) as enc:
    for i in range(n):
        b = enc.encode_device(t.data_ptr(), 7680, 4320)
        st = enc.stats()
        print("e8 %s: %d B, front %.3f ms, front+merge %.3f ms, emit %.3f ms"
              % (kind, len(b), st["ms_front_kernel"], st["ms_front"], st["ms_emit"]), flush=True)

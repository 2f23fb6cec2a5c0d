#!/bin/bash
# Round-2 first call: probe the box for a JPEG XL codec (djxl/cjxl/libjxl),
# host core count, then GPU tests + default bench + rocprof kernel stats.
set -e
export TMPDIR=/tmp
R=$PWD
O=gpurun_out/${1:-r02a}
mkdir -p $O
python3 - > $O/probe.txt 2>&1 <<'PY'
import ctypes.util, os, shutil, subprocess
for t in ("djxl", "cjxl", "jxlinfo", "benchmark_xl"):
    print(t, shutil.which(t))
for l in ("jxl", "jxl_threads", "jxl_dec"):
    print("lib" + l, ctypes.util.find_library(l))
try:
    out = subprocess.run(["ldconfig", "-p"], capture_output=True, text=True).stdout
    print("ldconfig jxl entries:", [x.strip() for x in out.splitlines() if "jxl" in x])
except Exception as e:
    print("ldconfig failed", e)
for mod in ("imagecodecs", "PIL", "pillow_jxl", "jxlpy"):
    try:
        m = __import__(mod)
        print(mod, getattr(m, "__version__", "?"))
        if mod == "imagecodecs":
            print("imagecodecs jpegxl:", hasattr(m, "jpegxl_encode"))
        if mod == "PIL":
            from PIL import features
            print("PIL jxl:", features.check("jpegxl") if "jpegxl" in features.get_supported() else "n/a")
    except Exception as e:
        print(mod, "absent:", type(e).__name__)
print("nproc", os.cpu_count(), "affinity", len(os.sched_getaffinity(0)))
PY
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
timeout -k 10 300 python bench.py > $O/bench.log 2>&1
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --alt-ans-streams 0 --alt-thesis 0 > $R/$O/bench_prof.log 2>&1

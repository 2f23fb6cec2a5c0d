"""Static checks of the gfx950 code objects (CPU only: hipcc cross-compiles).

Every kernel must be one flat body: an outlined device function (s_swappc)
passes the LDS image by a generic pointer and runs on a call stack in scratch
-- round 3's two-plane merge rewrite had its whole transform + quantization
outlined from merge_write_kernel that way, and that build faulted on the GPU.
The kernels' register / scratch budgets are checked too, so a change that
makes the compiler spill heavily or outline shows up here before it reaches
the GPU."""
import os
import re
import shutil
import subprocess
from concurrent.futures import ThreadPoolExecutor

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "jpeg-xl-lossy-image-compression-thesis_amd", "csrc")
HIPCC = "/opt/rocm/bin/hipcc"
SOURCES = sorted(f for f in os.listdir(CSRC) if f.endswith(".hip"))


@pytest.fixture(scope="module")
def isa(tmp_path_factory):
    if not os.path.exists(HIPCC):
        pytest.skip("no hipcc")
    d = tmp_path_factory.mktemp("isa")

    def one(src):
        out = d / (src + ".s")
        subprocess.check_call([HIPCC, "-O3", "-std=c++17", "-ffp-contract=off",
                               "--offload-arch=gfx950", "--offload-device-only", "-S",
                               "-o", str(out), os.path.join(CSRC, src)],
                              stderr=subprocess.DEVNULL)
        return src, out.read_text()

    with ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:
        return dict(ex.map(one, SOURCES))


def kernels(text):
    """(name, vgprs, vgpr spills, private segment bytes) per kernel (metadata)."""
    out = []
    meta = text[text.find(".amdgpu_metadata"):]
    names = list(re.finditer(r"\.name:\s+(\S+)", meta))
    for i, m in enumerate(names):
        # a kernel's metadata entry: from the key list before its .name (the
        # entry's earlier keys) to the next entry's .name
        start = meta.rfind("- .", 0, m.start())
        end = names[i + 1].start() if i + 1 < len(names) else len(meta)
        body = meta[start:end]

        def num(key):
            k = re.search(r"\.%s:\s+(\d+)" % key, body)
            return int(k.group(1)) if k else 0
        if ".symbol:" in body:
            out.append((m.group(1), num("vgpr_count"), num("vgpr_spill_count"),
                        num("private_segment_fixed_size")))
    return out


@pytest.mark.parametrize("src", SOURCES)
def test_no_device_calls(isa, src):
    calls = re.findall(r"s_swappc_b64", isa[src])
    assert not calls, "%s: %d outlined device-function calls" % (src, len(calls))


@pytest.mark.parametrize("src", SOURCES)
def test_register_budgets(isa, src):
    ks = kernels(isa[src])
    assert ks, "no kernel metadata in %s" % src
    for name, vgpr, spill, priv in ks:
        assert vgpr <= 256, (name, vgpr)
        assert spill <= 32, "%s spills %d VGPRs" % (name, spill)
        assert priv <= 128, "%s uses %d bytes of scratch" % (name, priv)

"""RD of the masking quant field (JXO_OPT_AQ_MASKING / JXG_FLAG_AQ_MASKING)
against the activity heuristic, at equal rate (oracle encoder == GPU bytes,
oracle decoder): bpp / PSNR curves over distances and the
Bjontegaard rate difference (PSNR-domain, cubic fit in log-rate) between them.
Usage: python tools/aq_rd.py [--jobs 4] > profiles/.../aq_rd.log"""
import argparse
import os
import sys
import time
from multiprocessing import Pool

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "jpeg-xl-lossy-image-compression-thesis_amd")]

DISTANCES = (0.5, 0.75, 1.0, 1.5, 2.0, 3.0)
AQ_MASKING = 4
FILTERS = ((0, "none"), (3, "gab+epf"))


def frames():
    from jxg.synth import config_image, natural_rgb8
    return [("natural_rgb8(1920,1080,3)", lambda: natural_rgb8(1920, 1080, 3)),
            ("bench crop 1920x1080", lambda: config_image(2)[:1080, :1920])]


def one(job):
    fi, d, fl = job
    import jxl_decode
    import oracle_ffi
    import jxg
    name, make = frames()[fi]
    img = make()
    t = time.time()
    r = oracle_ffi.encode(img, d, 7, 0, 1, fl)
    dec = jxl_decode.decode(r.bytes)
    psnr = jxg.calculate_psnr(jxg.calculate_mse(img, dec.rgb))
    return fi, d, fl, len(r.bytes) * 8 / img.shape[0] / img.shape[1], psnr, time.time() - t


def bd_rate(r1, p1, r2, p2):
    """average rate difference of curve 2 vs curve 1 (percent) over the
    overlapping PSNR interval: cubic fits of log(rate) in PSNR"""
    l1, l2 = np.log(r1), np.log(r2)
    f1, f2 = np.polyfit(p1, l1, 3), np.polyfit(p2, l2, 3)
    lo, hi = max(min(p1), min(p2)), min(max(p1), max(p2))
    i1, i2 = np.polyint(f1), np.polyint(f2)
    a1 = (np.polyval(i1, hi) - np.polyval(i1, lo)) / (hi - lo)
    a2 = (np.polyval(i2, hi) - np.polyval(i2, lo)) / (hi - lo)
    return (np.exp(a2 - a1) - 1) * 100, lo, hi


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--jobs", type=int, default=4)
    args = ap.parse_args()
    os.environ.setdefault("OMP_NUM_THREADS", "2")
    jobs = [(fi, d, fl | aq) for fi in range(len(frames())) for fl, _n in FILTERS
            for aq in (0, AQ_MASKING) for d in DISTANCES]
    with Pool(args.jobs) as pool:
        res = pool.map(one, jobs, chunksize=1)
    names = [n for n, _ in frames()]
    table = {}
    for fi, d, fl, bpp, psnr, dt in res:
        table[(fi, fl, d)] = (bpp, psnr)
        print("%-26s d%-4g %-8s %-8s %.4f bpp  %.3f dB  (%.0f s)" % (
            names[fi], d, dict(FILTERS)[fl & 3], "masking" if fl & AQ_MASKING else "activity",
            bpp, psnr, dt), flush=True)
    print()
    for fi in range(len(names)):
        for fl, fname in FILTERS:
            c = [np.array([table[(fi, fl | aq, d)] for d in DISTANCES]) for aq in (0, AQ_MASKING)]
            bd, lo, hi = bd_rate(c[0][:, 0], c[0][:, 1], c[1][:, 0], c[1][:, 1])
            print("BD-rate masking vs activity  %-26s %-8s %+.1f %%  (PSNR %.2f-%.2f dB)" % (
                names[fi], fname, bd, lo, hi))


if __name__ == "__main__":
    main()

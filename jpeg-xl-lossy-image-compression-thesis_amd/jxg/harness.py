"""Harness counterpart: the benchmark-jpegxl comparison
records, their CSV files and the A/B comparison, with the GPU encoder behind
``execute_cjxl`` and the GPU quality kernels (jxg_compare_rgb8) behind the
metrics.

Mirrors pscoro/JPEG-XL-Lossy-Image-Compression-Thesis benchmark-jpegxl:

* ``ComparisonResult`` / ``ComparisonResultDiff`` -- csv_writer.rs:23-63
  (17 columns each, same order and header text, csv_writer.rs:113-142 and
  :178-196); values formatted as Rust's ``to_string`` (f32 distance, f64
  metrics, integer sizes).
* ``write_csv_header`` writes the header only to a missing or empty file
  (csv_writer.rs:113-121); ``write_csv`` appends (csv_writer.rs:82-86).
* ``compare_results`` -- JXLCompressionBenchmark::compare_results
  (benchmark.rs:727-864): sort both runs by original image name, assert the
  rows pair up, diff = run 2 - run 1 per column, summary = mean of the diffs,
  written to ``comparison_diffs.csv`` and ``summary.csv`` next to results_1.
* ``compare_to_orig`` -- JXLCompressionBenchmark::compare_to_orig
  (benchmark.rs:895-972): file-size ratios (metrics.rs:15-26), MSE / PSNR /
  SSIM on the GPU; MS-SSIM is 0.0 as in the reference (benchmark.rs:933);
  Butteraugli and SSIMULACRA2 need libjxl's tools (Docker) and are 0.0 here.
* ``file_size_ratio`` -- metrics.rs:15-26.
"""
import csv
import os
from dataclasses import dataclass, fields

import numpy as np

from . import rust_f32, rust_f64

RESULT_HEADER = [
    "Original Image Name", "Compressed Image Name", "Distance", "Effort",
    "Original File Size", "Compressed File Size", "Original Raw Size", "Compressed Raw Size",
    "File Size Ratio", "Raw Size Ratio", "MSE", "PSNR", "SSIM", "MS-SSIM", "Butteraugli",
    "Butteraugli 3-Norm", "SSIMULACRA2",
]
DIFF_HEADER = [
    "Original Image Name", "Compressed Image Name", "Distance", "Effort",
    "Diff Original File Size", "Diff Compressed File Size", "Diff Original Raw Size",
    "Diff Compressed Raw Size", "Diff File Size Ratio", "Diff Raw Size Ratio", "Diff MSE",
    "Diff PSNR", "Diff SSIM", "Diff MS-SSIM", "Diff Butteraugli", "Diff Butteraugli 3-Norm",
    "Diff SSIMULACRA2",
]


@dataclass
class ComparisonResult:
    orig_image_name: str
    comp_image_name: str
    distance: float  # f32
    effort: int
    orig_file_size: int
    comp_file_size: int
    orig_raw_size: int
    comp_raw_size: int
    comp_file_size_ratio: float
    raw_file_size_ratio: float
    mse: float
    psnr: float
    ssim: float
    ms_ssim: float
    butteraugli: float
    butteraugli_pnorm: float
    ssimulacra2: float

    def row(self):
        return [self.orig_image_name, self.comp_image_name, rust_f32(self.distance),
                str(self.effort), str(self.orig_file_size), str(self.comp_file_size),
                str(self.orig_raw_size), str(self.comp_raw_size)] + [
                    rust_f64(getattr(self, f.name)) for f in fields(self)[8:]]

    @classmethod
    def parse(cls, rec):
        """csv_writer.rs:200-226 (read_csv): f32 distance, u32 effort, u64 sizes."""
        return cls(rec[0], rec[1], float(np.float32(rec[2])), int(rec[3]), int(rec[4]),
                   int(rec[5]), int(rec[6]), int(rec[7]), *[float(v) for v in rec[8:17]])


@dataclass
class ComparisonResultDiff:
    orig_image_name: str
    comp_image_name: str
    distance: float
    effort: int
    diff_orig_file_size: float
    diff_comp_file_size: float
    diff_orig_raw_size: float
    diff_comp_raw_size: float
    diff_comp_file_size_ratio: float
    diff_raw_file_size_ratio: float
    diff_mse: float
    diff_psnr: float
    diff_ssim: float
    diff_ms_ssim: float
    diff_butteraugli: float
    diff_butteraugli_pnorm: float
    diff_ssimulacra2: float

    def row(self):
        return [self.orig_image_name, self.comp_image_name, rust_f32(self.distance),
                str(self.effort)] + [rust_f64(getattr(self, f.name)) for f in fields(self)[4:]]


def write_csv_header(file_name: str, header) -> None:
    if os.path.exists(file_name) and os.path.getsize(file_name) > 0:
        return
    parent = os.path.dirname(file_name)
    if parent:
        os.makedirs(parent, exist_ok=True)
    with open(file_name, "w", newline="") as f:
        csv.writer(f, lineterminator="\n").writerow(header)


def write_csv(records, file_name: str) -> None:
    with open(file_name, "a", newline="") as f:
        w = csv.writer(f, lineterminator="\n")
        for r in records:
            w.writerow(r.row())


def read_csv(file_name: str):
    with open(file_name, newline="") as f:
        rows = list(csv.reader(f))
    return [ComparisonResult.parse(r) for r in rows[1:] if r]


def file_size_ratio(orig: int, comp: int, denom: str) -> float:
    if (orig == 0 and denom == "orig") or (comp == 0 and denom == "comp"):
        return 0.0
    if denom == "orig":
        return float(comp) / float(orig)
    if denom == "comp":
        return float(orig) / float(comp)
    raise ValueError("Invalid denominator for file size ratio")


_DIFF_FIELDS = [f.name for f in fields(ComparisonResult)[4:]]


def compare_results(results_1: str, results_2: str):
    """benchmark.rs:727-864; returns (diffs, summary) and writes the CSVs."""
    r1 = sorted(read_csv(results_1), key=lambda r: r.orig_image_name)
    r2 = sorted(read_csv(results_2), key=lambda r: r.orig_image_name)
    assert len(r1) == len(r2)
    diffs = []
    for a, b in zip(r1, r2):
        assert a.orig_image_name == b.orig_image_name
        assert a.comp_image_name == b.comp_image_name
        assert a.distance == b.distance
        assert a.effort == b.effort
        vals = [float(getattr(b, n)) - float(getattr(a, n)) for n in _DIFF_FIELDS]
        diffs.append(ComparisonResultDiff(a.orig_image_name, a.comp_image_name, a.distance,
                                          a.effort, *vals))
    acc = [0.0] * len(_DIFF_FIELDS)
    for d in diffs:
        for i, f in enumerate(fields(ComparisonResultDiff)[4:]):
            acc[i] += getattr(d, f.name)
    n = float(len(diffs))
    summary = ComparisonResultDiff("Summary", "Summary", 0.0, 0, *[v / n for v in acc])
    out_dir = os.path.dirname(os.path.abspath(results_1))
    diff_file = os.path.join(out_dir, "comparison_diffs.csv")
    write_csv_header(diff_file, DIFF_HEADER)
    write_csv(diffs, diff_file)
    summary_file = os.path.join(out_dir, "summary.csv")
    write_csv_header(summary_file, DIFF_HEADER)
    write_csv([summary], summary_file)
    return diffs, summary


def compare_to_orig(encoder, orig_name: str, orig_rgb: np.ndarray, orig_file_size: int,
                    comp_name: str, comp_rgb: np.ndarray, comp_file_size: int,
                    distance: float, effort: int, result_file: str | None = None,
                    ssim: bool = True) -> ComparisonResult:
    """benchmark.rs:895-972 with the metrics on the GPU.  ``encoder`` is a
    jxg.Encoder (its context runs jxg_compare_rgb8); ``comp_rgb`` is the
    decoded image (stock djxl where present, any decoder otherwise).  Raw
    sizes are width * height * 3 (image_reader.rs:523-540, Rgb8)."""
    h, w = orig_rgb.shape[:2]
    raw = w * h * 3
    q = encoder.compare(orig_rgb, comp_rgb, ssim=ssim)
    res = ComparisonResult(
        orig_name, comp_name, float(np.float32(distance)), int(effort), int(orig_file_size),
        int(comp_file_size), raw, raw,
        file_size_ratio(orig_file_size, comp_file_size, "comp"),
        file_size_ratio(raw, comp_file_size, "comp"),
        q["mse"], q["psnr"], q["ssim"] if ssim else 0.0, 0.0, 0.0, 0.0, 0.0)
    if result_file:
        write_csv_header(result_file, RESULT_HEADER)
        write_csv([res], result_file)
    return res

"""ORACLE — test infrastructure only (never imported by the product path).

Pure-Python restatement of datago's aspect-ratio bucket logic, used by tests/ to
check the product's C++ bucket table (datago_amd/csrc/host/buckets.cpp) through
the C ABI.  Every function cites the reference code it restates.

Parity is pinned by the reference's own known answers
(/root/reference/src/image_processing.rs:441-478, 602-608, 681-725) which are
replayed in tests/test_buckets.py.
"""
from __future__ import annotations

import bisect
import math
from typing import Dict, List, Optional, Tuple


def build_image_size_list(default_image_size: int, downsampling_ratio: int,
                          min_aspect_ratio: float, max_aspect_ratio: float) -> List[Tuple[int, int]]:
    """image_processing.rs:188-219 (u32 integer division, f64 sqrt/ceil/floor)."""
    patch_size = default_image_size // downsampling_ratio
    patch_size_sq = float((patch_size * patch_size) & 0xFFFFFFFF)
    sizes: List[Tuple[int, int]] = []
    min_patch_w = int(math.ceil(math.sqrt(patch_size_sq * min_aspect_ratio)))
    max_patch_w = int(math.floor(math.sqrt(patch_size_sq * max_aspect_ratio)))
    for patch_w in range(min_patch_w, max_patch_w + 1):
        patch_h = int(math.floor(patch_size_sq / float(patch_w)))
        sizes.append((patch_w * downsampling_ratio, patch_h * downsampling_ratio))
    min_patch_h = int(math.ceil(math.sqrt(patch_size_sq / max_aspect_ratio)))
    max_patch_h = int(math.floor(math.sqrt(patch_size_sq / min_aspect_ratio)))
    for patch_h in range(min_patch_h, max_patch_h + 1):
        patch_w = int(math.floor(patch_size_sq / float(patch_h)))
        sizes.append((patch_w * downsampling_ratio, patch_h * downsampling_ratio))
    return sizes


def aspect_ratio_to_str(size: Tuple[int, int]) -> str:
    """image_processing.rs:130-133 — Rust `format!("{:.3}", w as f64 / h as f64)`.

    Rust and CPython both print the correctly rounded decimal of the exact
    binary value (ties-to-even), so '%.3f' is the same function.
    """
    return "%.3f" % (float(size[0]) / float(size[1]))


class ARAwareTransform:
    """image_processing.rs:77-128 (`get_ar_aware_transform` + the struct)."""

    def __init__(self, default_image_size: int, downsampling_ratio: int,
                 min_aspect_ratio: float, max_aspect_ratio: float):
        # asserts at image_processing.rs:78-93
        assert default_image_size > 0 and downsampling_ratio > 0
        assert min_aspect_ratio > 0.0 and max_aspect_ratio >= min_aspect_ratio
        sizes = build_image_size_list(default_image_size, downsampling_ratio,
                                      min_aspect_ratio, max_aspect_ratio)
        # HashMap insert: last insert wins per key (:104-108)
        self.aspect_ratio_to_size: Dict[str, Tuple[int, int]] = {}
        for s in sizes:
            self.aspect_ratio_to_size[aspect_ratio_to_str(s)] = s
        # parsed keys sorted by value (:110-114)
        self.aspect_ratios: List[Tuple[float, str]] = sorted(
            ((float(k), k) for k in self.aspect_ratio_to_size), key=lambda t: t[0])

    def get_closest_aspect_ratio(self, image_width: int, image_height: int) -> str:
        """image_processing.rs:222-252; ties go to the right neighbour."""
        if not self.aspect_ratios:
            raise RuntimeError("Aspect ratio to size map is empty")
        target = float(image_width) / float(image_height)
        vals = [a for a, _ in self.aspect_ratios]
        idx = bisect.bisect_left(vals, target)
        if idx < len(vals) and vals[idx] == target:
            return self.aspect_ratios[idx][1]
        if idx == 0:
            return self.aspect_ratios[0][1]
        if idx == len(vals):
            return self.aspect_ratios[-1][1]
        left = abs(target - vals[idx - 1])
        right = abs(vals[idx] - target)
        return self.aspect_ratios[idx - 1][1] if left < right else self.aspect_ratios[idx][1]

    def target_size(self, w: int, h: int, forced_key: Optional[str] = None) -> Tuple[int, int]:
        key = forced_key if forced_key else self.get_closest_aspect_ratio(w, h)
        if key not in self.aspect_ratio_to_size:
            raise KeyError("Aspect ratio not found in aspect ratio to size map")  # :334-336
        return self.aspect_ratio_to_size[key]


def rust_round(x: float) -> float:
    """f64::round — half away from zero (image_processing.rs:285-286)."""
    return math.floor(x + 0.5) if x >= 0 else -math.floor(-x + 0.5)


def scaled_size(w: int, h: int, tw: int, th: int) -> Tuple[int, int]:
    """image_processing.rs:278-286: scale = max(tw/W, th/H); round(W*s), round(H*s)."""
    sx = float(tw) / float(w)
    sy = float(th) / float(h)
    s = max(sx, sy)
    return int(rust_round(float(w) * s)), int(rust_round(float(h) * s))


def fit_crop_box(src_w: int, src_h: int, dst_w: int, dst_h: int,
                 centering=(0.5, 0.5)) -> Tuple[float, float, float, float]:
    """fast_image_resize 5.5.0 `CropBox::fit_src_into_dst_size` (called at
    image_processing.rs:304-310; crate not vendored — restated from its
    published source, itself a copy of Pillow's ImageOps.fit)."""
    if src_w == 0 or src_h == 0 or dst_w == 0 or dst_h == 0:
        return 0.0, 0.0, float(src_w), float(src_h)
    width = float(src_w)
    height = float(src_h)
    image_ratio = width / height
    required_ratio = float(dst_w) / float(dst_h)
    eps = 2.220446049250313e-16
    if abs(image_ratio - required_ratio) < eps:
        cw, ch = width, height
    elif image_ratio >= required_ratio:
        cw, ch = required_ratio * height, height
    else:
        cw, ch = width, width / required_ratio
    return (width - cw) * centering[0], (height - ch) * centering[1], cw, ch


CONFIGS = {
    # BASELINE.json configs and the reference's own test configs
    "224/16": (224, 16, 0.5, 2.0),
    "256/16": (256, 16, 0.5, 2.0),
    "512/16": (512, 16, 0.5, 2.0),
    "512/32": (512, 32, 0.5, 2.0),
    "1024/32": (1024, 32, 0.5, 2.0),
}

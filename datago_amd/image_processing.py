"""Host-side mirror of datago's image-processing interface, backed by the HIP
library through the C ABI (no CPU pixel path).

Same names, argument meaning and error behaviour as the reference
(/root/reference/src/image_processing.rs, structs.rs), so tests read like the
reference's own:

    ImageTransformConfig          image_processing.rs:43-74 (serde defaults)
    .get_ar_aware_transform()     :77-121  (asserts -> AssertionError here)
    ARAwareTransform              :123-128, get_closest_aspect_ratio :222-252
    aspect_ratio_to_str           :130-133
    EncodeFormat / ImageEncoding  :14-41
    image_to_payload              :341-431 (decode + crop_and_resize on the GPU)
    ImagePayload                  structs.rs:52-71

Differences (documented, not silent): the payload comes from coded bytes (the
GPU decodes them), not from a decoded DynamicImage; an unknown forced aspect
ratio raises KeyError where the reference panics (:334-336).
"""
from __future__ import annotations

import enum
import json
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

import numpy as np

from . import _lib

DEFAULT_JPEG_QUALITY = 92


class EncodeFormat(enum.IntEnum):
    PNG = 0
    JPEG = 1


@dataclass
class ImageEncoding:
    encode_images: bool = False
    img_to_rgb8: bool = False
    encode_format: EncodeFormat = EncodeFormat.PNG
    jpeg_quality: int = DEFAULT_JPEG_QUALITY


@dataclass
class ImageTransformConfig:
    crop_and_resize: bool
    default_image_size: int = 0
    downsampling_ratio: int = 0
    min_aspect_ratio: float = 0.0
    max_aspect_ratio: float = 0.0
    pre_encode_images: bool = False
    image_to_rgb8: bool = False
    encode_format: EncodeFormat = EncodeFormat.PNG
    jpeg_quality: int = DEFAULT_JPEG_QUALITY

    @classmethod
    def from_json(cls, s: str) -> "ImageTransformConfig":
        d = json.loads(s) if isinstance(s, str) else dict(s)
        if "crop_and_resize" not in d:  # required field (serde)
            raise ValueError("missing field `crop_and_resize`")
        fmt = d.get("encode_format", "png")
        return cls(crop_and_resize=bool(d["crop_and_resize"]),
                   default_image_size=int(d.get("default_image_size", 0)),
                   downsampling_ratio=int(d.get("downsampling_ratio", 0)),
                   min_aspect_ratio=float(d.get("min_aspect_ratio", 0.0)),
                   max_aspect_ratio=float(d.get("max_aspect_ratio", 0.0)),
                   pre_encode_images=bool(d.get("pre_encode_images", False)),
                   image_to_rgb8=bool(d.get("image_to_rgb8", False)),
                   encode_format=EncodeFormat.JPEG if str(fmt).lower() == "jpeg" else EncodeFormat.PNG,
                   jpeg_quality=int(d.get("jpeg_quality", DEFAULT_JPEG_QUALITY)))

    def get_ar_aware_transform(self) -> "ARAwareTransform":
        assert self.crop_and_resize, "Crop and resize must be enabled to create ARAwareTransform"
        assert self.default_image_size > 0, "Default image size must be greater than 0"
        assert self.downsampling_ratio > 0, "Downsampling ratio must be greater than 0"
        assert self.min_aspect_ratio > 0.0 and self.max_aspect_ratio >= self.min_aspect_ratio, \
            "Aspect ratio constraints are invalid"
        return ARAwareTransform(self)

    def encoding(self) -> ImageEncoding:
        return ImageEncoding(self.pre_encode_images, self.image_to_rgb8, self.encode_format, self.jpeg_quality)


class ARAwareTransform:
    """Bucket table + the device context that applies it."""

    def __init__(self, cfg: ImageTransformConfig, device: int = 0):
        self.cfg = cfg
        self.table = _lib.BucketTable(cfg.default_image_size, cfg.downsampling_ratio, cfg.min_aspect_ratio,
                                      cfg.max_aspect_ratio)
        bl = self.table.buckets()
        self.aspect_ratio_to_size: Dict[str, Tuple[int, int]] = {k: (w, h) for (w, h, k) in bl}
        self.aspect_ratios: List[Tuple[float, str]] = [(float(k), k) for (_, _, k) in bl]
        self.device = device
        self._ctx: Dict[bool, _lib.Context] = {}

    def get_closest_aspect_ratio(self, image_width: int, image_height: int) -> str:
        return self.table.get(self.table.closest(image_width, image_height))[2]

    def context(self, encoding: "ImageEncoding" = None) -> "_lib.Context":
        enc = encoding if encoding is not None else ImageEncoding()
        key = (enc.img_to_rgb8, enc.encode_images, int(enc.encode_format), enc.jpeg_quality)
        if key not in self._ctx:
            c = self.cfg
            self._ctx[key] = _lib.Context(self.device, crop_and_resize=True,
                                          default_image_size=c.default_image_size,
                                          downsampling_ratio=c.downsampling_ratio,
                                          min_aspect_ratio=c.min_aspect_ratio,
                                          max_aspect_ratio=c.max_aspect_ratio,
                                          image_to_rgb8=enc.img_to_rgb8, pre_encode_images=enc.encode_images,
                                          encode_format=int(enc.encode_format), jpeg_quality=enc.jpeg_quality)
        return self._ctx[key]


def aspect_ratio_to_str(size: Tuple[int, int]) -> str:
    return _lib.aspect_ratio_to_str(int(size[0]), int(size[1]))


@dataclass
class ImagePayload:
    """structs.rs:52-71.  data: HWC row-major, tightly packed (or encoded bytes)."""
    data: bytes = b""
    original_height: int = 0
    original_width: int = 0
    height: int = 0
    width: int = 0
    channels: int = 0
    bit_depth: int = 0
    is_encoded: bool = False

    def to_numpy_array(self) -> np.ndarray:
        """structs.rs:154-188 equivalent."""
        a = np.frombuffer(self.data, np.uint8)
        if self.channels == 1:
            return a.reshape(self.height, self.width)
        return a.reshape(self.height, self.width, self.channels)

    def to_pil_image(self):
        from PIL import Image
        return Image.fromarray(self.to_numpy_array())


_plain_ctx: Dict[tuple, _lib.Context] = {}


def _decode_ctx(device: int, enc: "ImageEncoding") -> _lib.Context:
    key = (device, enc.img_to_rgb8, enc.encode_images, int(enc.encode_format), enc.jpeg_quality)
    if key not in _plain_ctx:
        _plain_ctx[key] = _lib.Context(device, image_to_rgb8=enc.img_to_rgb8, pre_encode_images=enc.encode_images,
                                       encode_format=int(enc.encode_format), jpeg_quality=enc.jpeg_quality)
    return _plain_ctx[key]


def images_to_payloads(datas: List[bytes], img_tfm: Optional[ARAwareTransform], aspect_ratios: List[str],
                       encoding: ImageEncoding = ImageEncoding(), device: int = 0
                       ) -> List[Tuple[int, Optional[ImagePayload]]]:
    """Batched image_to_payload over coded bytes: one GPU batch.  Returns
    (status, payload) per image; status != 0 means the reference would have
    returned an ImageError (CORRUPT) or the format is outside the GPU path
    (UNSUPPORTED, the caller's CPU path keeps it)."""
    if img_tfm is not None:
        ctx = img_tfm.context(encoding)
        forced = []
        for ar in aspect_ratios:
            if not ar:
                forced.append(-1)
                continue
            k = img_tfm.table.find_key(ar)
            if k < 0:
                raise KeyError("Aspect ratio not found in aspect ratio to size map")  # :334-336
            forced.append(k)
    else:
        ctx = _decode_ctx(device, encoding)
        forced = [-1] * len(datas)
    out = []
    for st, arr, m in ctx.decode_batch(datas, forced):
        if st != _lib.DG_OK:
            out.append((st, None))
            continue
        out.append((st, ImagePayload(data=arr.tobytes(), original_height=m.original_height,
                                     original_width=m.original_width, height=m.height, width=m.width,
                                     channels=m.channels, bit_depth=m.bit_depth, is_encoded=bool(m.is_encoded))))
    return out


def image_to_payload(data: bytes, img_tfm: Optional[ARAwareTransform], aspect_ratio: str = "",
                     encoding: ImageEncoding = ImageEncoding(), device: int = 0) -> ImagePayload:
    """image_processing.rs:341-431 for one coded image.  Raises
    ValueError (the reference's ImageError) on undecodable input."""
    st, p = images_to_payloads([data], img_tfm, [aspect_ratio], encoding, device)[0]
    if st != _lib.DG_OK:
        raise ValueError(f"image decode failed: {_lib.STATUS_NAMES.get(st, st)}")
    return p


def images_to_tensors(datas: List[bytes], img_tfm: Optional[ARAwareTransform], aspect_ratios: List[str],
                      encoding: ImageEncoding = ImageEncoding(), device: int = 0):
    """images_to_payloads for a GPU training loop: the
    payload data stays in HBM as torch uint8 tensors written by the kernels,
    without the D2H copy and the two to three host copies of the Python
    hand-off (structs.rs:103-188).  Returns (status, tensor, meta) per image."""
    if img_tfm is not None:
        ctx = img_tfm.context(encoding)
        forced = []
        for ar in aspect_ratios:
            k = img_tfm.table.find_key(ar) if ar else -1
            if ar and k < 0:
                raise KeyError("Aspect ratio not found in aspect ratio to size map")  # :334-336
            forced.append(k)
    else:
        ctx = _decode_ctx(device, encoding)
        forced = [-1] * len(datas)
    return ctx.decode_batch_torch(datas, forced)


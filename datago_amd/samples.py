"""Multi-payload samples over the GPU path: the reference-first aspect-ratio
propagation of datago's workers, with every payload of a sample decoded,
bucket-resized (and re-encoded) in one GPU batch.

    process_sample      worker_wds.rs:19-171 (WebDataset members of one sample)
    process_db_sample   worker_http.rs:113-264 (image + masks + additional images)

The bucket of every payload after the reference one is the key
aspect_ratio_to_str(reference output size) (worker_wds.rs:68-76,
worker_http.rs:138-141); dg_sample_align derives it from the headers, so the
whole sample goes to the GPU at once.  A reference payload whose body turns
out corrupt (known only after decoding) is skipped as the reference skips a
failed load (worker_wds.rs:134-137) and the remaining payloads are re-run
against the next reference.  Payloads outside the GPU path
(DG_ERR_UNSUPPORTED: 16-bit PNG, CMYK JPEG, progressive JPEG unless the
context option is set ...) are
returned with that status for the caller's CPU path; there is no CPU pixel
path here.
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

from . import _lib
from .image_processing import ARAwareTransform, EncodeFormat, ImageEncoding, ImagePayload, aspect_ratio_to_str

TEXT_TYPES = ("cls", "json", "txt")   # worker_wds.rs:10
IMG_TYPES = ("jpg", "jpeg", "png")    # worker_wds.rs:11


def is_supported_type(ext: str) -> bool:
    """worker_wds.rs:13-17 (case-insensitive here; the callers compare the raw extension)."""
    e = ext.lower()
    return e in TEXT_TYPES or e in IMG_TYPES


@dataclass
class BinaryFile:          # structs.rs:396-399
    filename: str
    buffer: bytes


@dataclass
class TarballSample:       # structs.rs:401-424
    name: str
    content: List[BinaryFile] = field(default_factory=list)


@dataclass
class Sample:              # structs.rs:242-280 (the fields this path fills)
    id: str
    source: str
    image: ImagePayload
    attributes: Dict[str, str] = field(default_factory=dict)
    masks: Dict[str, ImagePayload] = field(default_factory=dict)
    additional_images: Dict[str, ImagePayload] = field(default_factory=dict)
    unsupported: Dict[str, int] = field(default_factory=dict)  # payloads left to the CPU path


def _ctx(img_tfm: Optional[ARAwareTransform], encoding: ImageEncoding, device: int) -> _lib.Context:
    from .image_processing import _decode_ctx
    return img_tfm.context(encoding) if img_tfm is not None else _decode_ctx(device, encoding)


def _payload(arr, m) -> ImagePayload:
    return ImagePayload(data=arr.tobytes(), original_height=m.original_height, original_width=m.original_width,
                        height=m.height, width=m.width, channels=m.channels, bit_depth=m.bit_depth,
                        is_encoded=bool(m.is_encoded))


def _aligned_batch(datas: List[bytes], img_tfm: Optional[ARAwareTransform], encodings: List[ImageEncoding],
                   device: int = 0) -> List[Tuple[int, Optional[ImagePayload]]]:
    """Decode/transform a sample's payloads in order with reference-first
    alignment.  encodings[i] may differ per payload (DB masks)."""
    n = len(datas)
    out: List[Tuple[int, Optional[ImagePayload]]] = [(_lib.DG_ERR_CORRUPT, None)] * n
    table = img_tfm.table if img_tfm is not None else None
    key_idx = None
    todo = list(range(n))
    while todo:
        forced = _lib.sample_align(table, [datas[i] for i in todo]) if key_idx is None else [key_idx] * len(todo)
        # one GPU batch per distinct encoding
        groups: Dict[tuple, List[int]] = {}
        for j, i in enumerate(todo):
            e = encodings[i]
            groups.setdefault((e.encode_images, e.img_to_rgb8, int(e.encode_format), e.jpeg_quality), []).append(j)
        res: Dict[int, tuple] = {}
        for js in groups.values():
            ctx = _ctx(img_tfm, encodings[todo[js[0]]], device)
            for j, r in zip(js, ctx.decode_batch([datas[todo[j]] for j in js], [forced[j] for j in js])):
                res[j] = r
        if key_idx is not None or table is None:
            for j, i in enumerate(todo):
                st, arr, m = res[j]
                out[i] = (st, _payload(arr, m) if st == _lib.DG_OK else None)
            break
        # the reference: the first payload that decoded
        ref = next((j for j in range(len(todo)) if res[j][0] == _lib.DG_OK), None)
        for j in range(len(todo) if ref is None else ref + 1):
            st, arr, m = res[j]
            out[todo[j]] = (st, _payload(arr, m) if st == _lib.DG_OK else None)
        if ref is None:
            break
        if forced[ref] != -1:  # decoded against a reference that failed: align again from here
            todo = todo[ref:]
            continue
        m = res[ref][2]
        key_idx = table.find_key(aspect_ratio_to_str((m.width, m.height)))
        redo = []
        for j in range(ref + 1, len(todo)):
            if forced[j] == key_idx:
                st, arr, mm = res[j]
                out[todo[j]] = (st, _payload(arr, mm) if st == _lib.DG_OK else None)
            else:
                redo.append(todo[j])
        todo = redo
    return out


def process_sample(sample: TarballSample, img_tfm: Optional[ARAwareTransform], encoding: ImageEncoding,
                   extension_reference_image: str = "jpg", device: int = 0) -> Optional[Sample]:
    """worker_wds.rs:19-171 for one tarball sample (members sorted
    reference-first by the generator, generator_wds.rs:154-166).  Returns
    None where the reference returns Err(())."""
    if not sample.content:
        return None
    sample_id = os.path.splitext(os.path.basename(sample.content[0].filename))[0]
    if not sample_id:
        return None
    attributes: Dict[str, str] = {}
    imgs: List[BinaryFile] = []
    for item in sample.content:
        ext = os.path.splitext(item.filename)[1].lstrip(".")
        if not is_supported_type(ext):
            continue
        if ext in IMG_TYPES:
            imgs.append(item)
        elif ext in TEXT_TYPES:
            attributes[ext] = item.buffer.decode("utf-8", errors="replace")
    res = _aligned_batch([f.buffer for f in imgs], img_tfm, [encoding] * len(imgs), device)
    final: Optional[Sample] = None
    for item, (st, p) in zip(imgs, res):
        if st == _lib.DG_ERR_UNSUPPORTED:
            if final is None:
                final = Sample(sample_id, sample.name, ImagePayload())
            final.unsupported[item.filename] = st
            continue
        if st != _lib.DG_OK:
            continue  # load_from_memory failed: member skipped (worker_wds.rs:134-137)
        ext = os.path.splitext(item.filename)[1].lstrip(".")
        if final is None:
            final = Sample(sample_id, sample.name, ImagePayload())
        if ext == extension_reference_image:
            final.image = p
        else:
            final.additional_images[item.filename] = p
    if final is None:
        return None
    final.attributes = attributes
    return final


def process_db_sample(sample_id: str, image: bytes, masks: Dict[str, bytes], additional_images: Dict[str, bytes],
                      img_tfm: Optional[ARAwareTransform], encoding: ImageEncoding,
                      device: int = 0) -> Optional[Sample]:
    """worker_http.rs:113-264: the image first (its output size fixes the
    aspect ratio), then the image-type latents with the same encoding and the
    masks as PNG without RGB conversion (:186-192).  Any failure fails the
    sample (None)."""
    mask_enc = ImageEncoding(encode_images=encoding.encode_images, img_to_rgb8=False,
                             encode_format=EncodeFormat.PNG, jpeg_quality=encoding.jpeg_quality)
    names = ["image"] + list(additional_images) + list(masks)
    datas = [image] + list(additional_images.values()) + list(masks.values())
    encs = [encoding] * (1 + len(additional_images)) + [mask_enc] * len(masks)
    res = _aligned_batch(datas, img_tfm, encs, device)
    if any(st not in (_lib.DG_OK, _lib.DG_ERR_UNSUPPORTED) for st, _ in res):
        return None
    s = Sample(sample_id, "db", res[0][1] if res[0][0] == _lib.DG_OK else ImagePayload())
    for k, name in enumerate(names):
        st, p = res[k]
        if st == _lib.DG_ERR_UNSUPPORTED:  # e.g. masks re-encoded as PNG: the caller's CPU path
            s.unsupported[name] = st
        elif k == 0:
            continue
        elif k <= len(additional_images):
            s.additional_images[name] = p
        else:
            s.masks[name] = p
    return s

"""Multi-payload samples on the GPU (datago_amd/samples.py): every payload of
a sample lands in the reference payload's bucket (worker_wds.rs:68-76,
worker_http.rs:138-214) and equals the oracle's crop_and_resize to that
bucket bit for bit."""
import numpy as np
import pytest

from datago_amd import synth
from datago_amd.image_processing import ImageEncoding, ImageTransformConfig
from datago_amd.samples import BinaryFile, TarballSample, process_db_sample, process_sample
from oracle import buckets as B
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _tfm(size=512, ratio=16):
    return ImageTransformConfig(True, size, ratio, 0.5, 2.0).get_ar_aware_transform()


def _check(payload, data, target):
    _, dec = O.decode_any(data)
    exp = O.crop_and_resize(dec, target[0], target[1], O.MODE_FIR) if (dec.shape[1], dec.shape[0]) != target else dec
    assert (payload.width, payload.height) == target
    assert np.frombuffer(payload.data, np.uint8).tobytes() == exp.tobytes()


def test_wds_sample_alignment():
    tfm = _tfm()
    ob = B.ARAwareTransform(512, 16, 0.5, 2.0)
    img = synth.make_jpeg(1, 640, 480, 90)
    mask = synth.make_png(2, 640, 470, "L")        # a slightly different AR: forced to the image's bucket
    other = synth.make_jpeg(3, 300, 900, 90, "4:4:4")
    s = TarballSample("shard-0.tar", [BinaryFile("k1.jpg", img), BinaryFile("k1.png", mask),
                                      BinaryFile("k1.extra.jpeg", other), BinaryFile("k1.cls", b"7")])
    out = process_sample(s, tfm, ImageEncoding(), "jpg")
    assert out is not None and out.id == "k1" and out.attributes == {"cls": "7"}
    target = ob.aspect_ratio_to_size[ob.get_closest_aspect_ratio(640, 480)]
    _check(out.image, img, target)
    _check(out.additional_images["k1.png"], mask, target)
    _check(out.additional_images["k1.extra.jpeg"], other, target)


def test_wds_corrupt_reference_is_skipped():
    tfm = _tfm()
    ob = B.ARAwareTransform(512, 16, 0.5, 2.0)
    bad = synth.make_jpeg(4, 640, 480, 90)[:700]   # header fine, entropy data truncated
    nxt = synth.make_jpeg(5, 300, 900, 90)
    last = synth.make_jpeg(6, 800, 800, 90)
    # only the ".jpg" member is the reference image; ".jpeg" members are additional images
    s = TarballSample("shard", [BinaryFile("k2.jpg", bad), BinaryFile("k2.b.jpeg", nxt),
                                BinaryFile("k2.c.jpeg", last)])
    out = process_sample(s, tfm, ImageEncoding(), "jpg")
    assert out is not None and out.image.width == 0  # the reference member failed to load
    target = ob.aspect_ratio_to_size[ob.get_closest_aspect_ratio(300, 900)]
    _check(out.additional_images["k2.b.jpeg"], nxt, target)
    _check(out.additional_images["k2.c.jpeg"], last, target)


def test_db_sample_masks_and_reencode():
    tfm = _tfm(1024, 32)
    ob = B.ARAwareTransform(1024, 32, 0.5, 2.0)
    img = synth.make_png(7, 1000, 700, "RGB")
    mask = synth.make_png(8, 1000, 700, "L")
    s = process_db_sample("id", img, {"mask": mask}, {"masked_image": synth.make_jpeg(9, 1000, 700, 90)}, tfm,
                          ImageEncoding())
    target = ob.aspect_ratio_to_size[ob.get_closest_aspect_ratio(1000, 700)]
    _check(s.image, img, target)
    _check(s.masks["mask"], mask, target)
    assert (s.additional_images["masked_image"].width, s.additional_images["masked_image"].height) == target
    # pre_encode_images: the image is JPEG-encoded and the mask PNG-encoded on the GPU
    # (worker_http.rs:186-192 forces PNG for masks); the mask decodes to the same pixels
    s = process_db_sample("id", img, {"mask": mask}, {}, tfm, ImageEncoding(encode_images=True, encode_format=1))
    assert s.image.is_encoded and s.image.channels == -1
    assert s.unsupported == {}
    m = s.masks["mask"]
    assert m.is_encoded and m.channels == -1
    plain = process_db_sample("id", img, {"mask": mask}, {}, tfm, ImageEncoding()).masks["mask"]
    st, dec = O.png_decode(bytes(m.data))
    assert st == 0 and dec.shape == (plain.height, plain.width, 1)
    assert np.array_equal(dec.reshape(-1), np.frombuffer(bytes(plain.data), np.uint8))


def test_torch_handoff_equals_host_path():
    """images_to_tensors: outputs written into CUDA tensors (no D2H) equal the host path."""
    import torch
    from datago_amd.image_processing import images_to_payloads, images_to_tensors
    tfm = _tfm()
    datas = [synth.make_jpeg(40 + i, 300 + 50 * i, 200 + 70 * i, 90) for i in range(6)]
    datas.append(synth.make_png(99, 333, 222, "RGBA"))
    host = images_to_payloads(datas, tfm, [""] * len(datas))
    dev = images_to_tensors(datas, tfm, [""] * len(datas))
    for (st, p), (st2, t, m) in zip(host, dev):
        assert st == 0 and st2 == 0 and t.is_cuda
        assert t.cpu().numpy().tobytes() == p.data and (m.width, m.height) == (p.width, p.height)
    enc = images_to_tensors(datas[:2], tfm, ["", ""], ImageEncoding(encode_images=True, encode_format=1))
    ref = images_to_payloads(datas[:2], tfm, ["", ""], ImageEncoding(encode_images=True, encode_format=1))
    for (st, t, m), (_, p) in zip(enc, ref):
        assert st == 0 and m.is_encoded and t.cpu().numpy().tobytes() == p.data

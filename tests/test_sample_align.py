"""Multi-payload alignment (worker_wds.rs:68-76, worker_http.rs:138-214):
dg_sample_align (header-only, runs on the CPU) against the oracle's bucket
restatement (pinned to the reference's known answers)."""
import numpy as np

from datago_amd import _lib as L
from datago_amd import synth
from oracle import buckets as B


def test_align_forces_reference_bucket():
    t = L.BucketTable(512, 16, 0.5, 2.0)
    ob = B.ARAwareTransform(512, 16, 0.5, 2.0)
    ref = synth.make_jpeg(1, 640, 480, 90)
    others = [synth.make_jpeg(2, 100, 900, 90), synth.make_png(3, 300, 100, "L"), synth.make_jpeg(4, 640, 480, 90)]
    forced = L.sample_align(t, [ref] + others)
    key = ob.get_closest_aspect_ratio(640, 480)
    w, h = ob.aspect_ratio_to_size[key]
    exp_key = B.aspect_ratio_to_str((w, h))  # aspect_ratio_to_str(output size)
    assert forced[0] == -1
    assert all(t.get(f)[2] == exp_key for f in forced[1:])


def test_align_skips_unparseable_reference_and_no_config():
    t = L.BucketTable(1024, 32, 0.5, 2.0)
    good = synth.make_jpeg(5, 400, 800, 90)
    forced = L.sample_align(t, [b"not an image", good, synth.make_jpeg(6, 800, 400, 90)])
    assert forced[:2] == [-1, -1]
    assert t.get(forced[2])[2] == t.get(t.closest(400, 800))[2]
    assert L.sample_align(None, [good, good]) == [-1, -1]


def test_align_forced_first():
    t = L.BucketTable(512, 32, 0.5, 2.0)
    d = [synth.make_jpeg(7, 640, 480, 90), synth.make_jpeg(8, 640, 480, 90)]
    k = t.find_key("2.000")
    assert L.sample_align(t, d, k) == [k, k]


def test_align_grid_matches_oracle():
    rng = np.random.default_rng(0)
    for cfg in ((512, 16), (1024, 32), (512, 32)):
        t = L.BucketTable(cfg[0], cfg[1], 0.5, 2.0)
        ob = B.ARAwareTransform(cfg[0], cfg[1], 0.5, 2.0)
        for _ in range(10):
            w, h = int(rng.integers(1, 3000)), int(rng.integers(1, 3000))
            d = synth.make_jpeg(int(rng.integers(0, 1 << 30)), min(w, 64), min(h, 64), 90)
            # probe reports the header dims; use a real header of the drawn size cheaply: 1-colour image
            from PIL import Image
            import io
            buf = io.BytesIO()
            Image.new("RGB", (w, h), (10, 20, 30)).save(buf, "JPEG", quality=50)
            f = L.sample_align(t, [buf.getvalue(), d])
            bw, bh = ob.aspect_ratio_to_size[ob.get_closest_aspect_ratio(w, h)]
            assert t.get(f[1])[2] == B.aspect_ratio_to_str((bw, bh))

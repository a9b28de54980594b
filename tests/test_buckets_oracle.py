"""Bucket oracle vs the reference's own known answers (image_processing.rs)."""
import json
import os

import pytest

from oracle import buckets as B

HERE = os.path.dirname(os.path.abspath(__file__))


def test_reference_known_answers_224():
    # image_processing.rs:441-478
    t = B.ARAwareTransform(224, 16, 0.5, 2.0)
    assert t.get_closest_aspect_ratio(100, 100) == "1.000"
    assert t.get_closest_aspect_ratio(200, 100) == "1.900"
    assert t.get_closest_aspect_ratio(100, 200) == "0.526"
    assert t.target_size(300, 200, "1.000") == (224, 224)
    assert t.target_size(300, 200, "1.900") == (304, 160)
    assert t.target_size(400, 200) == (304, 160)


def test_aspect_ratio_to_str():
    # image_processing.rs:602-608
    assert B.aspect_ratio_to_str((100, 100)) == "1.000"
    assert B.aspect_ratio_to_str((200, 100)) == "2.000"
    assert B.aspect_ratio_to_str((100, 200)) == "0.500"
    assert B.aspect_ratio_to_str((150, 100)) == "1.500"


def test_size_list_invariants():
    # image_processing.rs:480-494, 727-759
    for (w, h) in B.build_image_size_list(224, 16, 0.5, 2.0):
        assert 0.5 <= w / h <= 2.0 and w % 16 == 0 and h % 16 == 0
    for (w, h) in B.build_image_size_list(256, 16, 1.0, 1.0):
        assert w == h and w % 16 == 0
    s = B.build_image_size_list(512, 32, 0.25, 4.0)
    ars = [w / h for w, h in s]
    assert min(ars) <= 0.3 and max(ars) >= 3.5
    assert all(w % 32 == 0 and h % 32 == 0 for w, h in s)


def test_sorted_and_edge_clamp():
    # image_processing.rs:653-679, 701-725
    t = B.ARAwareTransform(224, 16, 0.5, 2.0)
    vals = [a for a, _ in t.aspect_ratios]
    assert vals == sorted(vals) and min(vals) >= 0.5 and max(vals) <= 2.0
    assert float(t.get_closest_aspect_ratio(1000, 100)) <= 2.0
    assert float(t.get_closest_aspect_ratio(100, 1000)) >= 0.5


def test_survey_appendix_a_tables():
    t = B.ARAwareTransform(1024, 32, 0.5, 2.0)
    assert len(t.aspect_ratios) == 27
    assert len(B.build_image_size_list(1024, 32, 0.5, 2.0)) == 46
    assert t.aspect_ratio_to_size["0.489"] == (704, 1440)
    assert t.aspect_ratio_to_size["1.370"] == (1184, 864)
    assert t.aspect_ratio_to_size["2.045"] == (1440, 704)
    t = B.ARAwareTransform(512, 16, 0.5, 2.0)
    assert t.get_closest_aspect_ratio(640, 480) == "1.370"
    assert t.aspect_ratio_to_size["1.370"] == (592, 432)
    assert B.scaled_size(640, 480, 592, 432) == (592, 444)
    t = B.ARAwareTransform(512, 32, 0.5, 2.0)
    assert t.get_closest_aspect_ratio(640, 480) == "1.286"
    assert len(t.aspect_ratios) == 13


def test_golden_bucket_file_matches_oracle():
    with open(os.path.join(HERE, "golden", "buckets.json")) as f:
        g = json.load(f)
    for cfg, d in g.items():
        t = B.ARAwareTransform(*d["params"])
        assert [k for _, k in t.aspect_ratios] == d["keys"]
        for w, h, k in d["closest"]:
            assert t.get_closest_aspect_ratio(w, h) == k

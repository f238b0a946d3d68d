"""CPU-only: the oracle (oracle/liborc.so, the C restatement) against the
reference's golden fixtures and known-answer vectors.  This is what pins the
checker that the GPU parity tests rely on."""
import hashlib
import math

import pytest

import orc
from conftest import golden_rgb, manifest, scene_path

NAMES = sorted(manifest().keys())


def p3_text(rgb: bytes, w: int, h: int) -> bytes:
    out = [b"P3\n%d %d\n255\n" % (w, h)]
    for i in range(0, len(rgb), 3):
        out.append(b"%d %d %d\n" % (rgb[i], rgb[i + 1], rgb[i + 2]))
    return b"".join(out)


@pytest.mark.parametrize("name", NAMES)
def test_golden_fixture_matches_reference_sha(name):
    """The committed RGB8 fixture re-serialises to the reference's exact P3 bytes."""
    m = manifest()[name]
    rgb = golden_rgb(name)
    assert hashlib.sha256(rgb).hexdigest() == m["sha256_rgb"]
    assert hashlib.sha256(p3_text(rgb, m["width"], m["height"])).hexdigest() == m["sha256_p3"]


SURVEY_SHA = {  # reference ray_serial / restatement, g++ 11.4 -O3
    "simple_1280x720_d10": "1e1bfcd02c13536f07de0d90e76ded18d962f98ff157b4bc34fbea85bf0d205f",
    "medium_1280x720_d10": "aa0c8d69e98b45f3d389d5294fa1874940c0ece55104a7bb684ced7428c214af",
    "complex_1280x720_d10": "3ac688c6930a96f50d29d8395b75a55b30dd1fe7053de0852d23fc085d03a818",
    "simple_800x600_d10": "ed31b25f71372c4be99c17c712419b3a518b2011f7952c494bf9f8ca08125eec",
    "medium_1920x1080_d2": "5fba5b5b0ea41a22b0011c24316c45330e87c905b0fb5ddab6e008bc9e589072",
    "complex_1920x1080_d4": "a036103e08278188cbef5d39297b0dceb6fd0a51f87c5fce45700209f7fc4c8a",
}


@pytest.mark.parametrize("name", sorted(SURVEY_SHA))
def test_fixtures_agree_with_survey(name):
    assert manifest()[name]["sha256_p3"] == SURVEY_SHA[name]


SURVEY_RAYS = {  # SURVEY.md section 6 / BASELINE.md section 2
    "simple_1280x720_d10": (921600, 21522, 1030528),
    "complex_1280x720_d10": (921600, 169217, 3052855),
    "simple_800x600_d10": (480000, 11198, 536668),
    "medium_1920x1080_d2": (2073600, 400614, 4777134),
    "complex_1920x1080_d4": (2073600, 378178, 6862485),
}


@pytest.mark.parametrize("name", sorted(SURVEY_RAYS))
def test_ray_counts_agree_with_survey(name):
    r = manifest()[name]["rays"]
    assert (r["primary"], r["reflect"], r["shadow"]) == SURVEY_RAYS[name]


@pytest.mark.parametrize("name", NAMES)
def test_oracle_reproduces_golden(name):
    m = manifest()[name]
    rgb, counts, _ = orc.OracleScene(scene_path(m["scene"])).render(m["width"], m["height"], m["depth"], threads=8)
    assert rgb == golden_rgb(name)
    assert {k: counts[k] for k in ("primary", "shadow", "reflect")} == m["rays"]


def test_oracle_row_subsets_match_full_frame():
    m = manifest()["complex_97x61_d4"]
    full = golden_rgb("complex_97x61_d4")
    W, H = m["width"], m["height"]
    sc = orc.OracleScene(scene_path("complex"))
    band, G = 8, 3
    nb = -(-H // band)
    R = -(-nb // G) * band
    for r in range(G):
        rgb, _, _ = sc.render(W, H, 4, band=band, first=r, stride=G, count=R)
        for k in range(R):
            y = (k // band) * band * G + r * band + k % band
            if y < H:
                assert rgb[k * W * 3:(k + 1) * W * 3] == full[y * W * 3:(y + 1) * W * 3]


# populi-files/demo1_intersection.cpp:36-40: unit sphere at the origin.
@pytest.mark.parametrize("origin,direction,hit,t", [
    ((5, 0, 0), (-1, 0, 0), True, 4.0),     # along X: roots 4, 6 -> nearest 4
    ((5, 5, 0), (-1, 0, 0), False, None),   # disc = -96
    ((5, 1, 0), (-1, 0, 0), True, 5.0),     # grazing: disc == 0, t = 5
    ((0, 0, 5), (0, 0, -1), True, 4.0),     # along Z
])
def test_intersect_known_answers(origin, direction, hit, t):
    h, tt = orc.intersect((0, 0, 0), 1.0, origin, direction)
    assert h == hit
    if hit:
        assert tt == t


def test_intersect_semantics_quirks():
    # origin inside the sphere: nearest root negative -> far root (sphere.h:55-57)
    h, t = orc.intersect((0, 0, 0), 2.0, (0, 0, 0), (1, 0, 0))
    assert h and t == 2.0
    # sphere entirely behind: both roots negative -> miss (sphere.h:51-53)
    h, _ = orc.intersect((0, 0, 0), 1.0, (5, 0, 0), (1, 0, 0))
    assert not h
    # tangent behind the origin: disc == 0 keeps the NEGATIVE root (sphere.h:43-47)
    h, t = orc.intersect((0, 0, 0), 1.0, (5, 1, 0), (1, 0, 0))
    assert h and t == -5.0


def test_quantizer():
    # int(255.99 * std::min(1.0, c)), main.cpp:85
    assert orc.quantize(1.0) == 255
    assert orc.quantize(7.5) == 255
    assert orc.quantize(0.0) == 0
    assert orc.quantize(0.5) == 127
    assert orc.quantize(math.nan) == 255  # std::min(1.0, NaN) returns 1.0
    assert orc.quantize(-0.001) == 0      # truncation toward zero
    assert orc.quantize(-0.5) == -127     # no lower clamp upstream


def test_oracle_antialias_single_sample_is_the_serial_path():
    """orc_render_aa(samples=1) == orc_render; samples=4 renders 4x the primary rays
    and averages in sample order (main_gpu.cu:249-333 restated in fp64)."""
    import orc

    o = orc.OracleScene(scene_path("complex"))
    a, ca, _ = o.render(97, 61, 4, threads=2)
    b, cb, _ = o.render_aa(97, 61, 4, samples=1, threads=2)
    assert a == b and ca == cb
    _, c4, _ = o.render_aa(9, 7, 3, samples=4, threads=1)
    assert c4["primary"] == 4 * 9 * 7

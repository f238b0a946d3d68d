"""CPU-only: the oracle (oracle/liborc.so, the C restatement the GPU parity
tests check against) pinned to the REFERENCE itself on random scenes, not
only on the committed fixtures.  Each scene of tests/fuzz_gen.py's general,
near-light and EPSILON-margin generators (the ones the GPU fuzz uses) is
rendered by oracle/_ref/ref_render -- the reference's own trace_ray /
load_scene / Camera / write_ppm (src/main.cpp:16-91, scene.h, sphere.h,
scene_loader.h) compiled from /root/reference by oracle/Makefile, unmodified
-- and by the oracle; the P3 bytes must be identical.  The GPU fuzz then
compares the device against the oracle on the same generators, so the chain
device == oracle == reference holds on random inputs.  Skipped where the
reference build is absent (the GPU box: /root/reference is not there)."""
import os
import random
import subprocess

import pytest

import fuzz_gen
import orc

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.path.join(REPO, "oracle", "_ref", "ref_render")

pytestmark = pytest.mark.skipif(not os.access(REF, os.X_OK), reason="oracle/_ref not built (no /root/reference)")


def p3(rgb: bytes, w: int, h: int) -> bytes:
    out = [b"P3\n%d %d\n255\n" % (w, h)]
    for i in range(0, len(rgb), 3):
        out.append(b"%d %d %d\n" % (rgb[i], rgb[i + 1], rgb[i + 2]))
    return b"".join(out)


# (generator, seed, scenes)
CASES = [("scene", 501, 120), ("near", 502, 80), ("margin", 503, 160)]


@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_oracle_equals_reference_on_random_scenes(case, tmp_path):
    gen, seed, count = case
    rng = random.Random(seed)
    done = 0
    for k in range(count):
        text = fuzz_gen.margin_scene(rng) if gen == "margin" else fuzz_gen.scene(rng, near=(gen == "near"))
        W, H = rng.choice(fuzz_gen.ODD_SIZES if gen == "margin" else fuzz_gen.SIZES)
        W, H = min(W, 64), min(H, 48)  # the reference's serial brute force: keep each render well under a second
        D = rng.choice([1, 2, 4, 8])
        path = tmp_path / ("s%d.txt" % k)
        path.write_text(text)
        out = tmp_path / ("s%d.ppm" % k)
        r = subprocess.run([REF, str(path), str(W), str(H), str(D), "--out", str(out)], capture_output=True,
                           text=True, timeout=120)
        assert r.returncode == 0, r.stderr[-2000:]
        ref = out.read_bytes()
        got, _, _ = orc.OracleScene(text=text).render(W, H, D, threads=4)
        assert p3(got, W, H) == ref, "%s seed %d scene %d (%dx%d d%d)\n%s" % (gen, seed, k, W, H, D, text)
        done += 1
    assert done == count

#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ (run HERE, never on the GPU box).

Sources of truth, in order:
  * oracle/_ref/ray_serial  -- the reference's unmodified src/main.cpp, built by
    oracle/Makefile with the reference's makefile:28 flags.  Native 1280x720 d10.
  * oracle/_ref/ref_render  -- the reference's own trace_ray/Camera/load_scene/
    write_ppm (src/main.cpp, include/*.h) behind a size-parameterised driver
    (oracle/ref_driver.cpp).  All BASELINE.json sizes.
Every fixture is also rendered by the C restatement (oracle/oracle_cli) and the
two must be byte-identical, which pins the oracle.

Scenes with a fractional shininess (the parser takes any double,
scene_loader.h:66-70; pow(rdv, shininess) at scene.h:113 then leaves the
integer exponents every shipped scene has) are written by frac_scenes() into
tests/golden/scenes/: complex.txt with each shininess s -> 0.73 s + 0.5 (3
decimals), and a camera inside a cloud of mirrors with shininess drawn from
[0.5, 2000).

  python tests/golden/make_golden.py [NAME ...]   (default: every config;
  named configs are re-rendered and merged into the existing manifest)

Committed output per config: <name>.ppm.xz (binary P6 of the RGB8 bytes) and an
entry in manifest.json with the SHA-256 of the reference's P3 text, the SHA-256
of the RGB8 bytes, and the oracle's ray counts.
"""
import hashlib
import json
import lzma
import os
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
ORACLE = os.path.join(REPO, "oracle")
SCENES = os.path.join(REPO, "cs420-ray-tracer_amd", "scenes")
GSCENES = os.path.join(HERE, "scenes")  # generated test scenes (frac_scenes)

# name, scene, W, H, depth, source
CONFIGS = [
    ("simple_1280x720_d10", "simple", 1280, 720, 10, "ray_serial"),
    ("medium_1280x720_d10", "medium", 1280, 720, 10, "ray_serial"),
    ("complex_1280x720_d10", "complex", 1280, 720, 10, "ray_serial"),
    ("simple_800x600_d10", "simple", 800, 600, 10, "ref_render"),      # BASELINE cfg 1
    ("medium_1920x1080_d2", "medium", 1920, 1080, 2, "ref_render"),    # cfg 2
    ("complex_1920x1080_d4", "complex", 1920, 1080, 4, "ref_render"),  # cfg 3 (north star)
    ("synth200_1920x1080_d4", "synth200", 1920, 1080, 4, "ref_render"),  # cfg 3' (the metric)
    ("synth10k_384x216_d6", "synth10k", 384, 216, 6, "ref_render"),    # cfg 5 at 1/100 pixels
    ("complex_97x61_d4", "complex", 97, 61, 4, "ref_render"),          # ragged small case
    ("simple_2x2_d10", "simple", 2, 2, 10, "ref_render"),              # tiny case
    ("simple_1x1_d10", "simple", 1, 1, 10, "ref_render"),              # W-1 = 0: NaN camera ray
    # the hybrid driver's fixed size (src/main_hybrid.cpp:41-42, max_depth 3 at :736)
    ("simple_1080x720_d3", "simple", 1080, 720, 3, "ref_render"),
    ("medium_1080x720_d3", "medium", 1080, 720, 3, "ref_render"),
    ("complex_1080x720_d3", "complex", 1080, 720, 3, "ref_render"),
    # fractional shininess: pow(rdv, shininess) off the integer exponents
    ("complexfrac_960x540_d4", "complexfrac", 960, 540, 4, "ref_render"),
    ("mirrorfrac_320x240_d6", "mirrorfrac", 320, 240, 6, "ref_render"),
]


def frac_scenes():
    """Writes tests/golden/scenes/{complexfrac,mirrorfrac}.txt (deterministic)."""
    import random

    os.makedirs(GSCENES, exist_ok=True)
    out = []
    for line in open(os.path.join(SCENES, "complex.txt")):
        t = line.split()
        if t and t[0] == "sphere" and len(t) >= 11:
            t[10] = "%.3f" % (0.73 * float(t[10]) + 0.5)
            line = " ".join(t) + "\n"
        out.append(line)
    with open(os.path.join(GSCENES, "complexfrac.txt"), "w") as f:
        f.write("# complex.txt with shininess s -> 0.73 s + 0.5 (tests/golden/make_golden.py)\n" + "".join(out))
    rng = random.Random(2026)
    lines = ["# camera inside a cloud of mirrors, fractional shininess (tests/golden/make_golden.py)"]
    for _ in range(300):
        lines.append("sphere %.4f %.4f %.4f %.4f %.3f %.3f %.3f %.2f 0.5 %.3f" % (
            rng.uniform(-14, 14), rng.uniform(-14, 14), rng.uniform(-14, 14), rng.uniform(0.6, 2.2), rng.random(),
            rng.random(), rng.random(), rng.choice([0.0, 0.5, 0.8, 0.9, 1.0]), rng.uniform(0.5, 2000.0)))
    lines += ["light 0 30 0 1 1 1 1", "light 20 -10 25 0.6 0.5 0.4 1", "light -3 2 1 0.9 0.9 0.7 1",
              "ambient 0.1 0.1 0.1", "camera 0.3 0.2 0.1 5 1 -7 80"]
    with open(os.path.join(GSCENES, "mirrorfrac.txt"), "w") as f:
        f.write("\n".join(lines) + "\n")


def scene_file(scene: str) -> str:
    p = os.path.join(SCENES, scene + ".txt")
    return p if os.path.exists(p) else os.path.join(GSCENES, scene + ".txt")


def parse_p3(data: bytes):
    toks = data.split()
    assert toks[0] == b"P3"
    w, h, mx = int(toks[1]), int(toks[2]), int(toks[3])
    assert mx == 255
    vals = [int(t) for t in toks[4:]]
    assert len(vals) == w * h * 3
    assert all(0 <= v <= 255 for v in vals)
    return w, h, bytes(vals)


def p3_bytes(rgb: bytes, w: int, h: int) -> bytes:
    out = [b"P3\n%d %d\n255\n" % (w, h)]
    for i in range(0, len(rgb), 3):
        out.append(b"%d %d %d\n" % (rgb[i], rgb[i + 1], rgb[i + 2]))
    return b"".join(out)


def main():
    subprocess.check_call(["make", "-s", "-C", ORACLE])
    frac_scenes()
    only = set(sys.argv[1:])
    manifest = {}
    if only:
        with open(os.path.join(HERE, "manifest.json")) as f:
            manifest = json.load(f)
    tmp = tempfile.mkdtemp(prefix="golden_")
    for name, scene, w, h, d, src in CONFIGS:
        if only and name not in only:
            continue
        scene_path = scene_file(scene)
        if src == "ray_serial":
            assert (w, h, d) == (1280, 720, 10)
            subprocess.check_call([os.path.join(ORACLE, "_ref", "ray_serial"), scene_path],
                                  cwd=tmp, stdout=subprocess.DEVNULL)
            ref_ppm = os.path.join(tmp, "output_serial.ppm")
        else:
            ref_ppm = os.path.join(tmp, name + ".ref.ppm")
            subprocess.check_call([os.path.join(ORACLE, "_ref", "ref_render"), scene_path,
                                   str(w), str(h), str(d), "--out", ref_ppm], stdout=subprocess.DEVNULL)
        ref = open(ref_ppm, "rb").read()
        rw, rh, rgb = parse_p3(ref)
        assert (rw, rh) == (w, h)
        assert p3_bytes(rgb, w, h) == ref, "P3 re-serialisation mismatch"
        orc_p6 = os.path.join(tmp, name + ".orc.ppm")
        out = subprocess.check_output([os.path.join(ORACLE, "oracle_cli"), scene_path, str(w), str(h), str(d),
                                       "--threads", "8", "--p6", orc_p6])
        counts = json.loads(out)
        orc = open(orc_p6, "rb").read()
        hdr = b"P6\n%d %d\n255\n" % (w, h)
        assert orc.startswith(hdr)
        if orc[len(hdr):] != rgb:
            sys.exit(f"ORACLE MISMATCH on {name}")
        with open(os.path.join(HERE, name + ".ppm.xz"), "wb") as f:
            f.write(lzma.compress(hdr + rgb, preset=9 | lzma.PRESET_EXTREME))
        manifest[name] = {
            "scene": scene, "width": w, "height": h, "depth": d,
            "source": "reference " + ("src/main.cpp (ray_serial)" if src == "ray_serial"
                                      else "trace_ray via oracle/ref_driver.cpp"),
            "sha256_p3": hashlib.sha256(ref).hexdigest(),
            "sha256_rgb": hashlib.sha256(rgb).hexdigest(),
            "rays": {k: counts[k] for k in ("primary", "shadow", "reflect")},
        }
        print(name, manifest[name]["sha256_p3"], counts, flush=True)
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()

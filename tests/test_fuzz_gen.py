"""CPU: the fuzz generators (tests/fuzz_gen.py) the GPU campaign draws from
produce what they claim -- deterministic scenes the parser and the oracle
take, with exact negative-root tangents behind the camera (sphere.h:43-47)
and geometry within 2 EPSILON of surfaces."""
import random

import fuzz_gen


def _spheres(text):
    out = []
    for ln in text.splitlines():
        f = ln.split()
        if f and f[0] == "sphere":
            out.append(([float(v) for v in f[1:4]], float(f[4])))
    return out


def test_generators_are_deterministic():
    a = [fuzz_gen.margin_scene(random.Random(5)) for _ in range(3)]
    b = [fuzz_gen.margin_scene(random.Random(5)) for _ in range(3)]
    assert a == b
    assert fuzz_gen.scene(random.Random(9), near=True) == fuzz_gen.scene(random.Random(9), near=True)


def test_margin_scenes_parse_and_render_in_the_oracle():
    import orc
    import rt_hip

    rng = random.Random(4242)
    for _ in range(40):
        text = fuzz_gen.margin_scene(rng)
        sc = rt_hip.Scene.parse(text)
        o = orc.OracleScene(text=text)
        assert sc.num_spheres == o.s.num_spheres and sc.num_lights == o.s.num_lights
        assert sc.warnings == 0
        rgb, cnt, _ = o.render(7, 5, 2, threads=4)
        assert len(rgb) == 7 * 5 * 3 and cnt["primary"] == 35


def test_margin_scenes_hold_exact_tangents_and_eps_contacts():
    """Among the margin scenes: centre rays exactly tangent to a sphere behind
    the camera (the reference's disc == 0 branch returns t < 0), and contact
    pairs whose surfaces are within 2 EPSILON."""
    import orc

    rng = random.Random(4242)
    tangents = contacts = 0
    for _ in range(200):
        text = fuzz_gen.margin_scene(rng)
        cam = [ln.split() for ln in text.splitlines() if ln.startswith("camera")][0]
        P, L = [float(v) for v in cam[1:4]], [float(v) for v in cam[4:7]]
        sph = _spheres(text)
        if L[0] == P[0] and L[1] == P[1] and L[2] == P[2] - 5.0:
            for c, r in sph:
                hit, t = orc.intersect(c, r, P, (0.0, 0.0, -1.0))
                if hit and t < 0 and c[2] > P[2]:
                    tangents += 1
        for i in range(len(sph) - 12, len(sph)):
            if i < 1:
                continue
            for j in range(max(0, i - 1200), i):
                (ci, ri), (cj, rj) = sph[i], sph[j]
                d = sum((ci[k] - cj[k]) ** 2 for k in range(3)) ** 0.5
                if abs(d - abs(ri) - abs(rj)) <= 2.0 * fuzz_gen.EPS + 1e-9 * d:
                    contacts += 1
                    break
    assert tangents >= 10, tangents
    assert contacts >= 50, contacts

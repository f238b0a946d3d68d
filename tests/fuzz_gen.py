"""Random scene generators and the per-scene parity check of the randomised
sweeps -- shared by tests/test_gpu_fuzz.py (the driver-run, fixed-seed,
time-bounded suite) and scripts/gpu_fuzz.py (the open-ended builder's sweep).
TEST INFRASTRUCTURE: the oracle (oracle/orc.py) is the checker.

Three generators, each a function of a random.Random stream only, so a
(seed, index) names a scene exactly (scripts/fuzz_repro.py replays one):

* ``scene(rng, near)`` -- round 2-5's sweep: 1 to 1,500 spheres (cull sweeps,
  the BVH, the uniform grid above 1,024), radii 1e-4 .. 400, mirror clouds,
  0-6 lights, whole or fractional shininess (int_pow / dd_pow), cameras
  anywhere; ``near``: half the lights just outside a sphere, within or near
  a shadow ray's EPSILON overshoot past the light (scene.h:72-82, the defect
  round 5's sweep found in the light grids).
* ``margin_scene(rng)`` -- geometry placed within 2 EPSILON of every culling
  structure's margin (the reference's EPSILON = 0.001 offsets:
  scene.h:76-82 for shadow rays, main.cpp:46-48 for reflection rays):
  sphere pairs whose surfaces are -EPSILON .. +2 EPSILON apart, so a
  reflection's origin hit + n EPSILON lands inside, on or just outside a
  neighbour (the sphere grids' origin ball and their "within R + rho" global
  lists); cameras within +-2 EPSILON of a sphere surface (the camera grid's
  containing-sphere lists); lights within 2 EPSILON of a surface (the light
  grids' overshoot list); axis-aligned views whose centre ray (odd W, H) is
  EXACTLY tangent to a sphere behind the camera, and whose reflection off a
  head-on mirror is exactly tangent to a sphere behind its origin (disc == 0
  in the reference's arithmetic, sphere.h:43-47: the negative root the camera
  grid's, the sphere grids' and the uniform grid's behind-origin lists must
  keep); whole scenes moved 1e3 .. 1e6 from the origin (the fp32 BVH boxes
  and grid cells relative to the scene centre); up to 1,100 spheres (the
  uniform grid).
* ``SIZES`` / ``LARGE_SIZES`` / ``ODD_SIZES`` -- image sizes: small, 1,024+
  tiles (the heavy-first tile order with single, merged and tail groups), and
  odd sizes whose centre pixel ray is the camera's forward axis exactly.
"""
import random

EPS = 1e-3  # ray_math_constants.h:22 EPSILON

SIZES = [(1, 1), (7, 5), (64, 48), (96, 64), (160, 90)]
LARGE_SIZES = [(256, 256), (320, 240), (400, 300), (96, 64)]
ODD_SIZES = [(1, 1), (7, 5), (33, 17), (65, 49), (97, 61)]


def scene(rng: random.Random, near: bool = False) -> str:
    n = rng.choice([1, 2, 5, 30, 200, 700, 1100, 1500])
    spread = rng.choice([0.5, 5.0, 20.0, 1000.0])
    mirror = rng.random() < 0.3
    frac = rng.random() < 0.4  # fractional shininess: dd_pow (rt_pow.h) instead of int_pow

    def shin():
        if frac and rng.random() < 0.8:
            return "%.4f" % rng.choice([0.5, 7.5, 33.3, 1500.25, rng.uniform(0.01, 2000.0)])
        return "%d" % rng.choice([0, 1, 5, 20, 100, 200])

    lines = []
    for _ in range(n):
        r = rng.choice([1e-3, 0.05, 0.3, 1.0, 4.0]) * rng.uniform(0.5, 1.5) * spread / 10
        refl = rng.choice([0.8, 0.9, 1.0]) if mirror else rng.choice([0.0, 0.0, 0.3, 0.7, 1.0])
        lines.append("sphere %.9g %.9g %.9g %.9g %.3f %.3f %.3f %.2f 0.5 %s" % (
            rng.uniform(-spread, spread), rng.uniform(-spread, spread), rng.uniform(-3 * spread, spread), r,
            rng.random(), rng.random(), rng.random(), refl, shin()))
    for _ in range(rng.randint(0, 6)):
        pos = (rng.uniform(-2 * spread, 2 * spread), rng.uniform(-spread, 3 * spread), rng.uniform(-3 * spread, spread))
        if near and n > 0 and rng.random() < 0.5:
            # a light just outside a sphere, within or near a shadow ray's
            # EPSILON overshoot past it (scene.h:72-82)
            f = lines[rng.randrange(n)].split()
            c, rad = [float(v) for v in f[1:4]], abs(float(f[4]))
            u = [rng.gauss(0, 1) for _ in range(3)]
            norm = sum(v * v for v in u) ** 0.5 or 1.0
            gap = rng.choice([0.0002, 0.0008, 0.00099, 0.0012, 0.003]) * rng.uniform(0.9, 1.1)
            pos = tuple(c[k] + u[k] / norm * (rad + gap) for k in range(3))
        lines.append("light %.9g %.9g %.9g %.3f %.3f %.3f 1" % (*pos, rng.random(), rng.random(), rng.random()))
    lines.append("ambient %.3f %.3f %.3f" % (rng.random() * 0.3, rng.random() * 0.3, rng.random() * 0.3))
    cam = [rng.uniform(-spread, spread) * 0.3 for _ in range(3)]
    look = [rng.uniform(-spread, spread) * 0.5, rng.uniform(-spread, spread) * 0.5, -2 * spread]
    lines.append("camera %.6g %.6g %.6g %.6g %.6g %.6g %d" % (*cam, *look, rng.choice([20, 45, 60, 90, 140])))
    return "\n".join(lines) + "\n"


def _unit(rng):
    while True:
        u = [rng.gauss(0, 1) for _ in range(3)]
        n = sum(v * v for v in u) ** 0.5
        if n > 1e-3:
            return [v / n for v in u]


def margin_scene(rng: random.Random) -> str:
    """Geometry within 2 EPSILON of the culling structures' margins (module
    docstring).  Coordinates are printed with 17 significant digits, so the
    parser (istream >> double) reads back exactly the doubles built here."""
    off = [rng.choice([0.0, 0.0, 1e3, -1e5, 1e6]) for _ in range(3)] if rng.random() < 0.5 else [0.0] * 3
    scale = rng.choice([0.05, 1.0, 30.0])
    n = rng.choice([2, 8, 40, 200, 1100])
    mirror = rng.random() < 0.5
    sph = []  # (centre, radius, reflectivity)

    def add(c, r, refl=None):
        if refl is None:
            refl = rng.choice([0.7, 0.9, 1.0]) if mirror else rng.choice([0.0, 0.0, 0.3, 0.9])
        sph.append(([c[k] for k in range(3)], r, refl))

    for _ in range(n):
        c = [off[0] + scale * rng.uniform(-10, 10), off[1] + scale * rng.uniform(-6, 6),
             off[2] + scale * rng.uniform(-30, -2)]
        r = scale * rng.choice([0.02, 0.3, 1.0, 2.5]) * rng.uniform(0.7, 1.3)
        add(c, -r if rng.random() < 0.05 else r)  # the parser accepts negative radii
    # contact pairs: surfaces -EPSILON .. +2 EPSILON apart, so a reflection
    # leaving s near the contact starts (hit + n EPSILON, main.cpp:46) inside,
    # on or just outside the neighbour
    for _ in range(min(len(sph), rng.choice([2, 6, 12]))):
        c, r, _ = sph[rng.randrange(len(sph))]
        u = _unit(rng)
        r2 = scale * rng.choice([0.3, 1.0, 2.0]) * rng.uniform(0.7, 1.3)
        gap = rng.choice([-1.0, -0.5, 0.0, 0.5, 0.999, 1.0, 1.001, 1.5, 2.0]) * EPS
        add([c[k] + u[k] * (abs(r) + r2 + gap) for k in range(3)], r2)
    # the camera: free, within +-2 EPSILON of a sphere surface, or an axis-aligned
    # view with exact tangents behind the camera and behind a reflection's origin
    kind = rng.choice(["free", "surface", "surface", "tangent"])
    fov = rng.choice([30, 60, 90])
    if kind == "tangent":
        # integer coordinates (exact in fp64 at every offset used): forward is
        # (0, 0, -1) exactly, and with odd W, H the centre pixel's ray is too
        P = [float(round(off[k])) + rng.randint(-3, 3) for k in range(3)]
        R = float(rng.randint(1, 3))
        k2 = float(rng.randint(2, 9))
        # the centre ray's line is tangent to this sphere at t = -k2: disc == 0
        add([P[0], P[1] + R, P[2] + k2], R, 0.0)
        m = float(rng.randint(4, 9))
        # a mirror hit head on at P - (m - 1) z; its reflection leaves along +z
        # from P - (m - 1 - EPS) z and is tangent to a sphere behind that origin
        add([P[0], P[1], P[2] - m], 1.0, 0.9)
        R2 = float(rng.randint(1, 2))
        add([P[0] + R2, P[1], P[2] - m - float(rng.randint(4, 9))], R2, 0.2)
        cam, look = P, [P[0], P[1], P[2] - 5.0]
    elif kind == "surface":
        c, r, _ = sph[rng.randrange(len(sph))]
        u = _unit(rng)
        g = rng.choice([-2.0, -1.0, -0.5, 0.0, 0.5, 1.0, 2.0]) * EPS
        cam = [c[k] + u[k] * (abs(r) + g) for k in range(3)]
        look = [c[k] + u[k] * (abs(r) + 10 * scale) + rng.uniform(-3, 3) * scale for k in range(3)]
        if rng.random() < 0.5:  # looking back across the sphere
            look = [c[k] + rng.uniform(-1, 1) * scale for k in range(3)]
    else:
        cam = [off[0] + scale * rng.uniform(-3, 3), off[1] + scale * rng.uniform(-3, 3), off[2] + scale * 5]
        look = [off[0], off[1], off[2] - 15 * scale]
    lights = []
    for _ in range(rng.randint(1, 5)):
        if rng.random() < 0.6:  # within 2 EPSILON of a surface (the light grids' overshoot list)
            c, r, _ = sph[rng.randrange(len(sph))]
            u = _unit(rng)
            g = rng.choice([0.0, 0.5, 0.999, 1.0, 1.001, 1.5, 2.0]) * EPS
            lights.append([c[k] + u[k] * (abs(r) + g) for k in range(3)])
        else:
            lights.append([off[0] + scale * rng.uniform(-15, 15), off[1] + scale * rng.uniform(0, 20),
                           off[2] + scale * rng.uniform(-30, 10)])
    frac = rng.random() < 0.3
    out = []
    for c, r, refl in sph:
        shin = ("%.4f" % rng.uniform(0.5, 300.0)) if frac and rng.random() < 0.7 else "%d" % rng.choice([0, 5, 20, 100])
        out.append("sphere %.17g %.17g %.17g %.17g %.3f %.3f %.3f %.2f 0.5 %s" % (
            c[0], c[1], c[2], r, rng.random(), rng.random(), rng.random(), refl, shin))
    for p in lights:
        out.append("light %.17g %.17g %.17g %.3f %.3f %.3f 1" % (*p, rng.random(), rng.random(), rng.random()))
    out.append("ambient %.3f %.3f %.3f" % (rng.random() * 0.2, rng.random() * 0.2, rng.random() * 0.2))
    out.append("camera %.17g %.17g %.17g %.17g %.17g %.17g %d" % (*cam, *look, fov))
    return "\n".join(out) + "\n"


class Mismatch(AssertionError):
    pass


def check_scene(r, text, W, H, D, rng, k, threads=16, torch=None, orc=None, rt_hip=None):
    """Renders one scene on cuda:0 through the C-ABI and compares it with the
    oracle byte for byte and ray count for ray count; for k % 3 == 2 also as
    three frames of one launch (rt_render_frames_async: the deferred kernel,
    the XCD frame mapping) and three frames from three camera positions (a
    device camera grid per frame).  Consumes rng exactly as scripts/gpu_fuzz.py
    always has (three camera jitters per moving launch), so (seed, index)
    replays.  Returns (pixels, frames, moving frames); raises Mismatch."""
    sc = rt_hip.Scene.parse(text)
    r.upload(sc)
    rgb, st = r.render(sc.camera(), W, H, D)
    ref, cnt, _ = orc.OracleScene(text=text).render(W, H, D, threads=threads)
    rgb = bytes(rgb)
    if rgb != ref:
        bad = sum(a != b for a, b in zip(rgb, ref))
        raise Mismatch("one-frame launch: %d bytes differ (%dx%d d%d, %d spheres)" % (bad, W, H, D, sc.num_spheres))
    if (st.rays_primary, st.rays_shadow, st.rays_reflect) != (cnt["primary"], cnt["shadow"], cnt["reflect"]):
        raise Mismatch("one-frame launch: ray counts %s vs oracle %s" % (
            (st.rays_primary, st.rays_shadow, st.rays_reflect), cnt))
    frames = moving = 0
    if k % 3 == 2:
        F, stride = 3, W * H * 3
        buf = torch.full((F * stride,), 77, dtype=torch.uint8, device="cuda:0")
        torch.cuda.synchronize()
        r.render_frames_async([sc.camera()] * F, W, H, D, None, buf.data_ptr(), stride)
        r.stats()
        host = bytes(buf.cpu().numpy())
        for f in range(F):
            if host[f * stride:(f + 1) * stride] != ref:
                raise Mismatch("three frames at one position: frame %d differs" % f)
        frames += F
        cams = []
        for f in range(F):
            c = rt_hip.rt_camera.from_buffer_copy(sc.camera())
            for a in range(3):
                c.position[a] += rng.uniform(-1.0, 1.0) * rng.choice([1e-3, 0.1, 1.0])
            cams.append(c)
        buf.fill_(77)
        torch.cuda.synchronize()
        r.render_frames_async(cams, W, H, D, None, buf.data_ptr(), stride)
        st3 = r.stats()
        host = bytes(buf.cpu().numpy())
        oref = orc.OracleScene(text=text)
        tot = [0, 0, 0]
        for f in range(F):
            want, c3, _ = oref.render(W, H, D, threads=threads, camera=cams[f])
            if host[f * stride:(f + 1) * stride] != want:
                raise Mismatch("three frames at three positions: frame %d differs" % f)
            tot = [tot[0] + c3["primary"], tot[1] + c3["shadow"], tot[2] + c3["reflect"]]
        if [st3.rays_primary, st3.rays_shadow, st3.rays_reflect] != tot:
            raise Mismatch("three positions: ray counts differ")
        moving += F
    return W * H, frames, moving

"""Replays scripts/gpu_fuzz.py's random stream up to one scene and runs that
scene's checks one by one with details (a debugging tool, not a test): the
single launch, three frames of one launch at one position, three frames from
three positions -- each frame's differing bytes and the ray counts against the
oracle.
  python scripts/fuzz_repro.py SEED INDEX   (INDEX: the mismatch line's scene number - 1)
  python scripts/fuzz_repro.py SEED INDEX "default;RT_HIP_WIDE=0;..."   (knob settings, tuning build)"""
import os
import random
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "scripts"))
import gpu_fuzz  # noqa: E402  (its scene generator, torch, orc, rt_hip)

torch, orc, rt_hip = gpu_fuzz.torch, gpu_fuzz.orc, gpu_fuzz.rt_hip


def replay(seed, index):
    rng = random.Random(seed)
    for k in range(index + 1):
        text = gpu_fuzz.scene(rng)
        W, H, D = rng.choice(gpu_fuzz.SIZES) + (rng.choice([0, 1, 2, 4, 8]),)
        cams = None
        if k % 3 == 2:
            sc = rt_hip.Scene.parse(text)
            cams = []
            for f in range(3):
                c = rt_hip.rt_camera.from_buffer_copy(sc.camera())
                for a in range(3):
                    c.position[a] += rng.uniform(-1.0, 1.0) * rng.choice([1e-3, 0.1, 1.0])
                cams.append(c)
    return text, W, H, D, cams


def diff(got, want, W):
    bad = [i for i in range(len(want)) if got[i] != want[i]]
    if not bad:
        return "equal"
    px = sorted({i // 3 for i in bad})
    return "%d bytes differ, %d pixels, first (x %d, row %d): got %s want %s" % (
        len(bad), len(px), px[0] % W, px[0] // W, tuple(got[3 * px[0]:3 * px[0] + 3]),
        tuple(want[3 * px[0]:3 * px[0] + 3]))


def main():
    seed, index = int(sys.argv[1]), int(sys.argv[2])
    text, W, H, D, cams = replay(seed, index)
    with open(os.path.join(REPO, "gpurun_out", "fuzz_repro_scene.txt"), "w") as f:
        f.write("%d %d %d\n%s" % (W, H, D, text))
    sc = rt_hip.Scene.parse(text)
    print("scene %d: %dx%d d%d, %d spheres, %d lights" % (index, W, H, D, sc.num_spheres, sc.num_lights), flush=True)
    r = rt_hip.Renderer(0, variant=os.environ.get("FUZZ_VARIANT") or None)
    try:
        r.upload(sc)
        print("info", {k: v for k, v in r.info().as_dict().items() if k != "reserved0"}, flush=True)
        rgb, st = r.render(sc.camera(), W, H, D)
        ref, cnt, _ = orc.OracleScene(text=text).render(W, H, D, threads=16)
        print("single:", diff(bytes(rgb), ref, W), "counts", (st.rays_primary, st.rays_shadow, st.rays_reflect),
              "oracle", (cnt["primary"], cnt["shadow"], cnt["reflect"]), flush=True)
        F, stride = 3, W * H * 3
        for rep in range(3):
            buf = torch.full((F * stride,), 77, dtype=torch.uint8, device="cuda:0")
            torch.cuda.synchronize()
            r.render_frames_async([sc.camera()] * F, W, H, D, None, buf.data_ptr(), stride)
            s3 = r.stats()
            host = bytes(buf.cpu().numpy())
            print("3 frames, one position, rep %d:" % rep, [diff(host[f * stride:(f + 1) * stride], ref, W)
                                                           for f in range(F)],
                  "counts", (s3.rays_primary, s3.rays_shadow, s3.rays_reflect), flush=True)
        if cams:
            oref = orc.OracleScene(text=text)
            wants = [oref.render(W, H, D, threads=16, camera=c) for c in cams]
            tot = [sum(w[1][k] for w in wants) for k in ("primary", "shadow", "reflect")]
            for rep in range(3):
                buf = torch.full((F * stride,), 77, dtype=torch.uint8, device="cuda:0")
                torch.cuda.synchronize()
                r.render_frames_async(cams, W, H, D, None, buf.data_ptr(), stride)
                s3 = r.stats()
                host = bytes(buf.cpu().numpy())
                print("3 frames, three positions, rep %d:" % rep,
                      [diff(host[f * stride:(f + 1) * stride], wants[f][0], W) for f in range(F)],
                      "counts", (s3.rays_primary, s3.rays_shadow, s3.rays_reflect), "oracle", tuple(tot),
                      "grid", bool(r.info().cam_grid_last), flush=True)
    finally:
        r.close()


def settings_sweep(seed, index, settings):
    """The scene's frame from its second moved camera, one launch of that
    frame alone and the three-position launch, on the tuning build under
    each knob setting ("K=V+K2=V2;..." , "default")."""
    text, W, H, D, cams = replay(seed, index)
    sc = rt_hip.Scene.parse(text)
    oref = orc.OracleScene(text=text)
    wants = [oref.render(W, H, D, threads=16, camera=c)[0] for c in cams]
    F, stride = 3, W * H * 3
    for spec in settings.split(";"):
        env = {} if spec == "default" else dict(kv.split("=") for kv in spec.split("+"))
        os.environ.update(env)
        r = rt_hip.Renderer(0, variant="tuning")
        try:
            r.upload(sc)
            one = [diff(bytes(r.render(c, W, H, D)[0]), wants[f], W) for f, c in enumerate(cams)]
            buf = torch.full((F * stride,), 77, dtype=torch.uint8, device="cuda:0")
            torch.cuda.synchronize()
            r.render_frames_async(cams, W, H, D, None, buf.data_ptr(), stride)
            r.stats()
            host = bytes(buf.cpu().numpy())
            three = [diff(host[f * stride:(f + 1) * stride], wants[f], W) for f in range(F)]
            print(spec, "| one frame per launch:", one, "| three per launch:", three,
                  "grid", bool(r.info().cam_grid_last), flush=True)
        finally:
            r.close()
            for k in env:
                del os.environ[k]


if __name__ == "__main__":
    if len(sys.argv) > 3:
        settings_sweep(int(sys.argv[1]), int(sys.argv[2]), sys.argv[3])
    else:
        main()

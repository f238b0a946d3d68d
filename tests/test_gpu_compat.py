"""The reference's hybrid GPU interface, link-compatible (include/rt_hip_compat.h;
src/kernel.cu:185-207 as src/main_hybrid.cpp:104-109, 170-171 calls it):
upload_lights_and_ambience + launch_gpu_kernel over the hybrid driver's 64x64
tiles, round-robin over 3 streams, into a device float3 framebuffer.

The caller hands over fp32 GPUSphere / GPULight / GPUCamera data; the scene
here is exactly representable in fp32 and the camera looks straight down -z,
so the fp32 hand-over loses nothing and the result must be the serial fp64
path's framebuffer (the oracle, rounded to float on store) -- and bit-identical
to rt_render_tile's RT_FB_F32X3 output of the same scene."""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SCENE = """\
sphere 0 0 -5 1  0.75 0.25 0.25  0.5 0.5 32
sphere 2 0.5 -6 1.5  0.25 0.75 0.25  0 0.5 16
sphere -2.5 0.25 -4 0.75  0.25 0.25 0.75  0.25 0.5 64
sphere 0 -101 -5 100  0.5 0.5 0.5  0 1 8
sphere 1 2 -9 0.5  1 1 1  0.75 0.5 100
light 5 10 5  1 1 1  1
light -6 8 2  0.5 0.75 1  1
ambient 0.125 0.125 0.125
camera 0 1 6  0 1 -20  60
"""
W, H, D, TILE = 160, 100, 3, 64  # main_hybrid.cpp: max_depth 3, 64x64 tiles


def _gpu_scene(rt_hip, torch, sc):
    n, nl = sc.num_spheres, sc.num_lights
    sph = (rt_hip.rt_gpu_sphere * n)()
    for i in range(n):
        s = sc.sphere(i)
        sph[i].center = rt_hip.rt_float3(*s["center"])
        sph[i].radius = s["radius"]
        sph[i].material.albedo = rt_hip.rt_float3(*s["color"])
        sph[i].material.metallic = s["reflectivity"]
        sph[i].material.shininess = s["shininess"]
    lights = (rt_hip.rt_gpu_light * nl)()
    for i in range(nl):
        L = sc.light(i)
        lights[i].position = rt_hip.rt_float3(*L["position"])
        lights[i].color = rt_hip.rt_float3(*L["color"])
        lights[i].intensity = L["intensity"]
    cam = rt_hip.rt_gpu_camera()
    cam.origin = rt_hip.rt_float3(0, 1, 6)
    cam.forward = rt_hip.rt_float3(0, 0, -1)
    cam.fov = 60.0
    d_sph = torch.frombuffer(bytearray(bytes(sph)), dtype=torch.uint8).to("cuda:0")
    d_cam = torch.frombuffer(bytearray(bytes(cam)), dtype=torch.uint8).to("cuda:0")
    return d_sph, d_cam, lights


def _launch_all(rt_hip, torch, fb, d_sph, d_cam, n, nl, streams):
    L = rt_hip.lib()
    k = 0
    for ty in range(0, H, TILE):
        for tx in range(0, W, TILE):
            s = streams[k % len(streams)]
            k += 1
            L.launch_gpu_kernel(C.cast(fb.data_ptr(), C.POINTER(rt_hip.rt_float3)),
                                C.cast(d_sph.data_ptr(), C.POINTER(rt_hip.rt_gpu_sphere)), n, nl,
                                C.cast(d_cam.data_ptr(), C.POINTER(rt_hip.rt_gpu_camera)), tx, ty, TILE, TILE, W, H, D,
                                C.c_void_p(s.cuda_stream))
            assert L.rt_compat_status() == 0, rt_hip.status_string(L.rt_compat_status())
    for s in streams:
        s.synchronize()


def test_hybrid_interface_matches_oracle_and_render_tile():
    import orc
    import rt_hip
    import torch

    sc = rt_hip.Scene.parse(SCENE)
    n, nl = sc.num_spheres, sc.num_lights
    d_sph, d_cam, lights = _gpu_scene(rt_hip, torch, sc)
    L = rt_hip.lib()
    L.upload_lights_and_ambience(lights, nl, rt_hip.rt_float3(0.125, 0.125, 0.125))
    assert L.rt_compat_status() == 0
    fb = torch.full((H * W * 3,), float("nan"), dtype=torch.float32, device="cuda:0")
    torch.cuda.synchronize()
    streams = [torch.cuda.Stream() for _ in range(3)]  # NUM_STREAMS, main_hybrid.cpp:41
    _launch_all(rt_hip, torch, fb, d_sph, d_cam, n, nl, streams)
    got = fb.cpu().numpy().reshape(H, W, 3).astype(np.float64)
    assert np.isfinite(got).all()

    # the serial fp64 path on the same scene (oracle), fb in PPM order -> y = 0 bottom
    _, _, _, ref_fb = orc.OracleScene(text=SCENE).render(W, H, D, threads=4, want_fb=True)
    ref = np.array(ref_fb, dtype=np.float64).reshape(H, W, 3)[::-1]
    err = np.abs(got - ref) - (np.abs(ref) * 2.0**-23 + 2.0**-125)
    assert (err <= 0).all(), (float(err.max()), np.argwhere(err > 0)[:3].tolist())

    # bit-identical to the library's own tile entry on the same scene
    r = rt_hip.Renderer(0)
    try:
        r.upload(sc)
        f2 = torch.full((H * W * 3,), float("nan"), dtype=torch.float32, device="cuda:0")
        torch.cuda.synchronize()
        for ty in range(0, H, TILE):
            for tx in range(0, W, TILE):
                r.render_tile(sc.camera(), W, H, D, tx, ty, TILE, TILE, rt_hip.RT_FB_F32X3, f2.data_ptr())
        r.stats()
        assert torch.equal(fb, f2)
    finally:
        r.close()


def test_hybrid_interface_errors_never_exit():
    import rt_hip
    import torch

    sc = rt_hip.Scene.parse(SCENE)
    n, nl = sc.num_spheres, sc.num_lights
    d_sph, d_cam, lights = _gpu_scene(rt_hip, torch, sc)
    L = rt_hip.lib()
    L.upload_lights_and_ambience(lights, nl, rt_hip.rt_float3(0.125, 0.125, 0.125))
    fb = torch.full((H * W * 3,), 7.0, dtype=torch.float32, device="cuda:0")
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    args = (C.cast(fb.data_ptr(), C.POINTER(rt_hip.rt_float3)), C.cast(d_sph.data_ptr(), C.POINTER(rt_hip.rt_gpu_sphere)))
    cam = C.cast(d_cam.data_ptr(), C.POINTER(rt_hip.rt_gpu_camera))
    # more lights than uploaded: the reference would read past its __constant__ array
    L.launch_gpu_kernel(*args, n, nl + 1, cam, 0, 0, W, H, W, H, D, C.c_void_p(s.cuda_stream))
    assert L.rt_compat_status() == 1  # RT_ERR_INVALID_ARG
    L.launch_gpu_kernel(*args, -1, nl, cam, 0, 0, W, H, W, H, D, C.c_void_p(s.cuda_stream))
    assert L.rt_compat_status() == 1
    L.upload_lights_and_ambience(None, 2, rt_hip.rt_float3(0, 0, 0))
    assert L.rt_compat_status() == 1
    s.synchronize()
    assert (fb == 7.0).all()  # nothing rendered
    # a tile entirely outside the image renders nothing and succeeds (kernel.cu:103)
    L.launch_gpu_kernel(*args, n, nl, cam, W + 5, 0, 8, 8, W, H, D, C.c_void_p(s.cuda_stream))
    assert L.rt_compat_status() == 0
    s.synchronize()
    assert (fb == 7.0).all()


def _hip_runtime():
    """The HIP runtime torch loaded (the one librt_hip.so is bound to), for raw
    hipStreamCreate / hipStreamDestroy calls."""
    with open("/proc/self/maps") as f:
        paths = {line.split()[-1] for line in f if "libamdhip64" in line}
    assert paths, "no HIP runtime loaded"
    hip = C.CDLL(sorted(paths)[0])
    hip.hipStreamCreate.argtypes = [C.POINTER(C.c_void_p)]
    hip.hipStreamDestroy.argtypes = [C.c_void_p]
    hip.hipStreamSynchronize.argtypes = [C.c_void_p]
    return hip


def test_hybrid_interface_streams_destroyed_between_calls():
    """render_hybrid creates three streams per call and destroys them at its end
    (main_hybrid.cpp:407-409, 489-491; COMPARE_MODES calls it twice, :817): the
    per-device default context must not keep a destroyed stream.  Two rounds of
    launch_gpu_kernel over the tiles on raw HIP streams, destroyed after each
    round, the second with moved spheres (the re-upload waits for the context's
    stream): both framebuffers bit-identical to rt_render_tile's."""
    import rt_hip
    import torch

    hip = _hip_runtime()
    L = rt_hip.lib()
    for rnd, shift in enumerate((0.0, 0.5)):
        text = SCENE.replace("sphere 0 0 -5 1 ", "sphere %g 0 -5 1 " % shift)
        sc = rt_hip.Scene.parse(text)
        n, nl = sc.num_spheres, sc.num_lights
        d_sph, d_cam, lights = _gpu_scene(rt_hip, torch, sc)
        L.upload_lights_and_ambience(lights, nl, rt_hip.rt_float3(0.125, 0.125, 0.125))
        assert L.rt_compat_status() == 0
        fb = torch.full((H * W * 3,), float("nan"), dtype=torch.float32, device="cuda:0")
        torch.cuda.synchronize()
        raw = [C.c_void_p() for _ in range(3)]
        for s in raw:
            assert hip.hipStreamCreate(C.byref(s)) == 0
        k = 0
        for ty in range(0, H, TILE):
            for tx in range(0, W, TILE):
                L.launch_gpu_kernel(C.cast(fb.data_ptr(), C.POINTER(rt_hip.rt_float3)),
                                    C.cast(d_sph.data_ptr(), C.POINTER(rt_hip.rt_gpu_sphere)), n, nl,
                                    C.cast(d_cam.data_ptr(), C.POINTER(rt_hip.rt_gpu_camera)), tx, ty, TILE, TILE,
                                    W, H, D, raw[k % 3])
                k += 1
                assert L.rt_compat_status() == 0, (rnd, rt_hip.status_string(L.rt_compat_status()))
        for s in raw:
            assert hip.hipStreamSynchronize(s) == 0
            assert hip.hipStreamDestroy(s) == 0
        r = rt_hip.Renderer(0)
        try:
            r.upload(sc)
            f2 = torch.full((H * W * 3,), float("nan"), dtype=torch.float32, device="cuda:0")
            torch.cuda.synchronize()
            for ty in range(0, H, TILE):
                for tx in range(0, W, TILE):
                    r.render_tile(sc.camera(), W, H, D, tx, ty, TILE, TILE, rt_hip.RT_FB_F32X3, f2.data_ptr())
            r.stats()
            assert torch.equal(fb, f2), rnd
        finally:
            r.close()

"""Where the drop-in path's time goes (a builder's probe, not a test): the
ray_serial sequence of bench.py's e2e (parse, rt_create, rt_upload_scene, one
synchronous render to host memory, rt_write_ppm P3) in fresh contexts, each
step timed, plus the render split into its host parts: the render enqueued
into a device buffer (rt_render_async), its completion (rt_render_stats), and
the device-to-host copy.
  python scripts/e2e_probe.py [SCENE] [RUNS]"""
import os
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "cs420-ray-tracer_amd"))
import rt_hip  # noqa: E402


def main():
    scene = sys.argv[1] if len(sys.argv) > 1 else "complex"
    runs = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    W, H, D = 1920, 1080, 4
    path = os.path.join(REPO, "cs420-ray-tracer_amd", "scenes", scene + ".txt")
    with tempfile.TemporaryDirectory() as tmp:
        out = os.path.join(tmp, "output_gpu.ppm")
        for k in range(runs):
            t = [time.perf_counter()]
            sc = rt_hip.Scene.load(path)
            cam = sc.camera()
            t.append(time.perf_counter())
            r = rt_hip.Renderer(0)
            t.append(time.perf_counter())
            r.upload(sc)
            t.append(time.perf_counter())
            rgb, st = r.render(cam, W, H, D)
            t.append(time.perf_counter())
            rt_hip.write_ppm(out, rgb, W, H)
            t.append(time.perf_counter())
            # the same render again in this context (warm)
            rgb2, st2 = r.render(cam, W, H, D)
            t.append(time.perf_counter())
            r.close()
            names = ["parse", "create", "upload", "render", "write_p3", "render_again"]
            print("run %d: " % k + " ".join("%s %.3f" % (n, (b - a) * 1e3) for n, a, b in zip(names, t, t[1:])) +
                  " | kernel %.3f / %.3f ms, total %.3f ms, %d rays, %.0f Mrays/s, p3 %d B" % (
                      st.kernel_ms, st2.kernel_ms, (t[5] - t[0]) * 1e3, st.rays, st.rays / (t[5] - t[0]) / 1e6,
                      os.path.getsize(out)), flush=True)


def split():
    """The render split: enqueue into device memory, completion, and the
    device-to-host copy into pageable vs pinned memory, in a fresh context."""
    import torch

    scene = sys.argv[1] if len(sys.argv) > 1 else "complex"
    W, H, D = 1920, 1080, 4
    path = os.path.join(REPO, "cs420-ray-tracer_amd", "scenes", scene + ".txt")
    pinned = torch.empty(W * H * 3, dtype=torch.uint8, pin_memory=True)
    page = bytearray(W * H * 3)
    for k in range(3):
        sc = rt_hip.Scene.load(path)
        r = rt_hip.Renderer(0)
        r.upload(sc)
        dev = torch.empty(W * H * 3, dtype=torch.uint8, device="cuda:0")
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r.render_async(sc.camera(), W, H, D, None, dev.data_ptr())
        t1 = time.perf_counter()
        st = r.stats()
        t2 = time.perf_counter()
        pinned.copy_(dev)
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        host = dev.cpu()
        t4 = time.perf_counter()
        import ctypes
        ctypes.memmove((ctypes.c_char * len(page)).from_buffer(page), host.data_ptr(), len(page))
        t5 = time.perf_counter()
        r.close()
        print("split %d: enqueue %.3f, to completion %.3f (kernel %.3f), D2H pinned %.3f, D2H pageable %.3f, "
              "memcpy %.3f ms" % (k, (t1 - t0) * 1e3, (t2 - t1) * 1e3, st.kernel_ms, (t3 - t2) * 1e3,
                                  (t4 - t3) * 1e3, (t5 - t4) * 1e3), flush=True)


def pin_costs():
    """What pinning the output costs in a process: hipHostMalloc / hipHostFree
    of a 1080p RGB8 buffer, hipHostRegister / Unregister of a pageable one."""
    import ctypes

    hip = ctypes.CDLL("libamdhip64.so")
    nbytes = 1920 * 1080 * 3
    for k in range(3):
        p = ctypes.c_void_p()
        t0 = time.perf_counter()
        assert hip.hipHostMalloc(ctypes.byref(p), ctypes.c_size_t(nbytes), 0) == 0
        t1 = time.perf_counter()
        ctypes.memset(p, 0, nbytes)
        t2 = time.perf_counter()
        hip.hipHostFree(p)
        t3 = time.perf_counter()
        buf = (ctypes.c_char * nbytes)()
        t4 = time.perf_counter()
        assert hip.hipHostRegister(buf, ctypes.c_size_t(nbytes), 0) == 0
        t5 = time.perf_counter()
        hip.hipHostUnregister(buf)
        t6 = time.perf_counter()
        print("pin %d: hipHostMalloc %.3f, first touch %.3f, hipHostFree %.3f, hipHostRegister %.3f, "
              "Unregister %.3f ms" % (k, (t1 - t0) * 1e3, (t2 - t1) * 1e3, (t3 - t2) * 1e3, (t5 - t4) * 1e3,
                                      (t6 - t5) * 1e3), flush=True)


if __name__ == "__main__":
    main()
    if os.environ.get("E2E_SPLIT", "1") == "1":
        split()
        pin_costs()

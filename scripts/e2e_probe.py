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


if __name__ == "__main__":
    main()

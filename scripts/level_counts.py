"""Reflection rays and kernel time per depth for one scene (a design probe,
not a test): renders the scene's camera at W x H for depth 1..D on cuda:0
through the C-ABI and prints the ray counts and kernel ms of each depth, so
the rays and time each reflection level adds can be read off.
  python scripts/level_counts.py SCENE W H D"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "cs420-ray-tracer_amd"))
import rt_hip as rt  # noqa: E402


def main():
    path, W, H, D = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
    sc = rt.Scene.load(path)
    r = rt.Renderer(0)
    r.upload(sc)
    cam = sc.camera()
    prev = None
    for d in range(1, D + 1):
        best = None
        for _ in range(3):
            _, st = r.render(cam, W, H, d)
            best = st.kernel_ms if best is None else min(best, st.kernel_ms)
        s = st.as_dict()
        line = "depth %d: primary %d shadow %d reflect %d exact %d cull %d kernel %.3f ms" % (
            d, s["primary"], s["shadow"], s["reflect"], s["tests_exact"], s["tests_cull"], best)
        if prev:
            line += " | level %d: +%d reflect rays, +%d shadow, +%.3f ms, +%d exact, +%d cull" % (
                d - 1, s["reflect"] - prev["reflect"], s["shadow"] - prev["shadow"], best - prev["ms"],
                s["tests_exact"] - prev["tests_exact"], s["tests_cull"] - prev["tests_cull"])
        print(line, flush=True)
        prev = dict(s, ms=best)


if __name__ == "__main__":
    main()

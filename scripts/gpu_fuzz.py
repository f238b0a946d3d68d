"""Randomised parity sweep, open-ended (a builder's tool; the driver-run,
fixed-seed form is tests/test_gpu_fuzz.py): random scenes from
tests/fuzz_gen.py -- the general generator (FUZZ_NEAR_LIGHTS=1: half the
lights just outside a sphere; FUZZ_MARGIN=1: the EPSILON-margin generator,
odd sizes) -- rendered on cuda:0 through the C-ABI and compared with the
oracle byte for byte and ray count for ray count; every third scene also as
three frames of one launch and three frames from three camera positions.
FUZZ_LARGE=1: images of 1,024 tiles and more.  Knobs (RT_HIP_*) apply as set
in the environment (FUZZ_VARIANT=tuning for the tuning build's).  Prints a
line every 25 scenes and a summary; exits non-zero on the first mismatch
(the scene goes to gpurun_out/fuzz_mismatch.txt).
  python scripts/gpu_fuzz.py [SECONDS] [SEED]"""
import os
import random
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "cs420-ray-tracer_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import torch  # noqa: E402  (torch's HIP runtime first; frame buffers)
import orc  # noqa: E402  (the checker)
import rt_hip  # noqa: E402
import fuzz_gen  # noqa: E402

MARGIN = os.environ.get("FUZZ_MARGIN") == "1"
SIZES = fuzz_gen.LARGE_SIZES if os.environ.get("FUZZ_LARGE") == "1" else (
    fuzz_gen.ODD_SIZES if MARGIN else fuzz_gen.SIZES)


def scene(rng):
    if MARGIN:
        return fuzz_gen.margin_scene(rng)
    return fuzz_gen.scene(rng, near=os.environ.get("FUZZ_NEAR_LIGHTS") == "1")


def main():
    budget = float(sys.argv[1]) if len(sys.argv) > 1 else 300.0
    rng = random.Random(int(sys.argv[2]) if len(sys.argv) > 2 else 20261016)
    r = rt_hip.Renderer(0, variant=os.environ.get("FUZZ_VARIANT") or None)
    t0, k, px, frames, moving = time.time(), 0, 0, 0, 0
    try:
        while time.time() - t0 < budget:
            text = scene(rng)
            W, H, D = rng.choice(SIZES) + (rng.choice([0, 1, 2, 4, 8]),)
            try:
                p, f, m = fuzz_gen.check_scene(r, text, W, H, D, rng, k, torch=torch, orc=orc, rt_hip=rt_hip)
            except fuzz_gen.Mismatch as e:
                print("MISMATCH scene %d (%dx%d d%d): %s" % (k + 1, W, H, D, e), flush=True)
                os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
                with open(os.path.join(REPO, "gpurun_out", "fuzz_mismatch.txt"), "w") as fh:
                    fh.write("%d %d %d\n%s" % (W, H, D, text))
                return 1
            k += 1
            px, frames, moving = px + p, frames + f, moving + m
            if k % 25 == 0:
                print("%d scenes ok (%d pixels), %.0f s" % (k, px, time.time() - t0), flush=True)
    finally:
        r.close()
    print("fuzz: %d scenes, %d pixels (+ %d frames of 3-frame launches at one position, %d frames of 3-frame "
          "launches at three positions), all byte-identical to the oracle" % (k, px, frames, moving))
    return 0


if __name__ == "__main__":
    sys.exit(main())

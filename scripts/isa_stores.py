"""Global-memory store kinds per render kernel in the device assembly (the
north star's "coalesced stores to the RGB framebuffer": the default kernels
must carry no byte stores).  python scripts/isa_stores.py [k.s] -- without an
argument compiles rt_kernel.hip for gfx950 first."""
import collections
import os
import re
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def asm() -> str:
    if len(sys.argv) > 1:
        return open(sys.argv[1]).read()
    with tempfile.TemporaryDirectory() as t:
        out = os.path.join(t, "k.s")
        subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17",
                               "-ffp-contract=off", "-I" + os.path.join(REPO, "include"), "--cuda-device-only",
                               "-S", "-o", out, os.path.join(REPO, "cs420-ray-tracer_amd", "csrc", "rt_kernel.hip")],
                              stderr=subprocess.DEVNULL)
        return open(out).read()


def main():
    txt = asm()
    cur, counts = None, collections.OrderedDict()
    for line in txt.splitlines():
        m = re.match(r"^(_Z\S*render\S*):", line)
        if m:
            cur = m.group(1)
            counts[cur] = collections.Counter()
            continue
        if cur and line.startswith("\t.size"):
            cur = None
        if cur:
            m = re.match(r"\s+((?:global|flat|buffer)_(?:store|atomic)_\w+)", line)
            if m:
                counts[cur][m.group(1)] += 1
    for k, c in counts.items():
        print(f"{k[:64]:64s} {dict(sorted(c.items()))}")


if __name__ == "__main__":
    main()

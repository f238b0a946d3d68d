#!/usr/bin/env python3
"""Register budget of the render kernels from the code object's own metadata
(hipcc -S of rt_kernel.hip for gfx950, the Makefile's flags): arch VGPRs (.vgpr_count), AGPRs
(.agpr_count; accum_offset = where they would start), SGPRs, spills, and the
allocation the hardware makes -- VGPRs in granules of 8 on gfx950, 512 per
SIMD lane, so waves per SIMD = floor(512 / roundup8(vgprs)).  rocprofv3's
kernel trace prints the dispatch's VGPR field decoded with a granule of 4,
i.e. half the allocation: 84 for a kernel that allocates 168.
  python scripts/regs.py [extra hipcc flags]"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "cs420-ray-tracer_amd", "csrc", "rt_kernel.hip")
with tempfile.TemporaryDirectory() as tmp:
    out = os.path.join(tmp, "k.s")
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
                    "-I" + os.path.join(ROOT, "include"), "-mllvm", "--amdgpu-sched-strategy=max-memory-clause",
                    "--cuda-device-only", "-S", "-o", out, SRC] + sys.argv[1:],
                   check=True, stderr=subprocess.DEVNULL)
    txt = open(out).read()
meta = txt[txt.rfind("amdhsa.kernels"):]
print(f"{'kernel':58s} {'vgpr':>4s} {'agpr':>4s} {'alloc':>5s} {'w/SIMD':>6s} {'rocprof':>7s} {'vspill':>6s} "
      f"{'sgpr':>4s} {'sspill':>6s}")
for blk in meta.split("  - .")[1:]:
    name = re.search(r"\.name:\s+(\S+)", blk)
    if not name or "render" not in name.group(1):
        continue
    g = lambda k: int((re.search(r"\.%s:\s+(\d+)" % k, blk) or [None, "0"])[1])
    v, a = g("vgpr_count"), g("agpr_count")
    alloc = (max(v, 1) + 7) // 8 * 8 + ((a + 7) // 8 * 8 if a else 0)
    dem = subprocess.run(["c++filt"], input=name.group(1), capture_output=True, text=True).stdout.strip()
    dem = dem.replace("rtk::", "").replace("(rtk::RenderArgs)", "").replace("(RenderArgs)", "")
    print(f"{dem[:58]:58s} {v:4d} {a:4d} {alloc:5d} {512 // alloc:6d} {alloc // 2:7d} {g('vgpr_spill_count'):6d} "
          f"{g('sgpr_count'):4d} {g('sgpr_spill_count'):6d}")

"""CPU: the product library's configuration surface.  librt_hip.so reads only
the RT_HIP_* knobs a user of the drop-in needs (the north star's LDS-staged
scene, the camera-grid policy); the layout and grid knobs the parity tests
sweep live in the tuning build (variants/librt_hip_tuning.so), and no ablation
branch is left in the kernel sources."""
import os
import re

from conftest import PKG, PRODUCT_KNOBS

CSRC = os.path.join(PKG, "csrc")


def _knobs(path):
    with open(path, "rb") as f:
        return {m.decode() for m in re.findall(rb"RT_HIP_[A-Z0-9_]+", f.read())}


def test_product_library_reads_few_knobs():
    got = _knobs(os.path.join(PKG, "librt_hip.so"))
    assert got <= PRODUCT_KNOBS - {"RT_HIP_LIB"}, sorted(got)
    assert len(got) <= 10


def test_tuning_build_reads_the_test_knobs():
    got = _knobs(os.path.join(PKG, "variants", "librt_hip_tuning.so"))
    assert {"RT_HIP_DEFER", "RT_HIP_STACK", "RT_HIP_SHADOW_GRID_N", "RT_HIP_SPHERE_GRID_N"} <= got


def test_no_ablation_branches_in_kernel_sources():
    for name in os.listdir(CSRC):
        if name.endswith((".hip", ".h", ".cpp")):
            with open(os.path.join(CSRC, name)) as f:
                assert "RT_ABL" not in f.read(), name

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


# Every knob the tuning build reads (the parity tests sweep each non-default
# layout a scene or launch can reach); rejected paths are deleted with their
# knobs (round 6: RT_HIP_PAIR_CLASS, RT_HIP_LG_ORDER, RT_HIP_DEFER_GRID and the
# render_deferred_grid kernel), so this list only shrinks.
TUNING_KNOBS = {
    "RT_HIP_BEHIND_GRID", "RT_HIP_BVH", "RT_HIP_BVH4", "RT_HIP_BVH_ALWAYS", "RT_HIP_BVH_GROUPS", "RT_HIP_BVH_LEAF",
    "RT_HIP_BVH_MIN", "RT_HIP_BVH_ORDERED", "RT_HIP_CAM_GRID_BUDGET", "RT_HIP_CAM_GRID_MAXP", "RT_HIP_CAM_GRID_N",
    "RT_HIP_DEFER", "RT_HIP_DEFER_DIV", "RT_HIP_DEFER_LEVEL", "RT_HIP_DEFER_WALK", "RT_HIP_GRID_CELLS",
    "RT_HIP_GRID_CLOSEST", "RT_HIP_MERGE_Q", "RT_HIP_SCHED", "RT_HIP_SHADOW_GRID", "RT_HIP_SHADOW_GRID_N",
    "RT_HIP_SINGLE_CLASS", "RT_HIP_SPHERE_GRID", "RT_HIP_SPHERE_GRID_N", "RT_HIP_STACK", "RT_HIP_TAIL",
    "RT_HIP_TAIL_WAVES", "RT_HIP_WIDE", "RT_HIP_XCD_FRAMES",
}


def test_tuning_build_reads_exactly_the_test_knobs():
    got = _knobs(os.path.join(PKG, "variants", "librt_hip_tuning.so"))
    assert got == TUNING_KNOBS | (PRODUCT_KNOBS - {"RT_HIP_LIB"}), sorted(got ^ (TUNING_KNOBS | PRODUCT_KNOBS))


def test_rejected_kernels_are_gone():
    with open(os.path.join(CSRC, "rt_kernel.hip")) as f:
        src = f.read()
    for name in ("render_deferred_grid", "pair_class", "defer_grid"):
        assert name not in src, name


def test_no_ablation_branches_in_kernel_sources():
    for name in os.listdir(CSRC):
        if name.endswith((".hip", ".h", ".cpp")):
            with open(os.path.join(CSRC, name)) as f:
                assert "RT_ABL" not in f.read(), name

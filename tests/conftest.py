import json
import lzma
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "cs420-ray-tracer_amd")
ORACLE = os.path.join(REPO, "oracle")
GOLDEN = os.path.join(REPO, "tests", "golden")
SCENES = os.path.join(PKG, "scenes")
for p in (PKG, ORACLE):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs on the GPU box)")


def scene_path(name: str) -> str:
    """A shipped scene, or a generated test scene (tests/golden/scenes, make_golden.py)."""
    p = os.path.join(SCENES, name + ".txt")
    return p if os.path.exists(p) else os.path.join(GOLDEN, "scenes", name + ".txt")


def manifest() -> dict:
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        return json.load(f)


def golden_rgb(name: str) -> bytes:
    """RGB8 bytes (PPM row order) of a committed golden fixture."""
    with open(os.path.join(GOLDEN, name + ".ppm.xz"), "rb") as f:
        data = lzma.decompress(f.read())
    m = manifest()[name]
    hdr = b"P6\n%d %d\n255\n" % (m["width"], m["height"])
    assert data.startswith(hdr)
    return data[len(hdr):]


def diff_summary(a: bytes, b: bytes) -> str:
    import numpy as np

    x = np.frombuffer(a, np.uint8).astype(np.int16)
    y = np.frombuffer(b, np.uint8).astype(np.int16)
    d = np.abs(x - y)
    return f"{int((d > 0).sum())} channels differ, {int((d > 1).sum())} by >1, max {int(d.max()) if d.size else 0}"


# RT_HIP_* knobs the product library reads itself (rt_create); every other
# layout / grid knob is read only by the tuning build (variants/librt_hip_tuning.so)
PRODUCT_KNOBS = {"RT_HIP_LDS_SCENE", "RT_HIP_CAM_GRID", "RT_HIP_LIB"}


def knob_variant():
    """The library a test context must use for the RT_HIP_* knobs now set: the
    product's when only its own knobs are set, else the tuning build."""
    tuning = [k for k in os.environ if k.startswith("RT_HIP_") and k not in PRODUCT_KNOBS]
    return "tuning" if tuning else None


@pytest.fixture(scope="session")
def gpu_renderer():
    import rt_hip

    r = rt_hip.Renderer(0)
    yield r
    r.close()


# GPU suite order: the default-path parity tests (goldens, ray counts, shards,
# multi-frame launches, the CLI) run first, alternative kernel layouts and
# diagnostic knobs (fresh contexts with RT_HIP_* set) last, so under `-x` a
# failure in a non-default path cannot hide the default path's results.
_KNOB_FIXTURES = {"bvh_renderer", "stack_renderer", "grid_renderer", "monkeypatch"}


def _gpu_rank(item) -> int:
    if item.get_closest_marker("gpu") is None:
        return 0
    name = item.nodeid
    if "test_golden_byte_identical" in name or "test_ray_counts_match_oracle" in name:
        return 1
    if _KNOB_FIXTURES & set(getattr(item, "fixturenames", ())):
        return 4
    if "test_gpu_parity.py" in name or "test_gpu_frames.py" in name or "test_gpu_cli.py" in name:
        return 2
    return 3


def pytest_collection_modifyitems(session, config, items):
    items.sort(key=_gpu_rank)  # stable: file order within a rank

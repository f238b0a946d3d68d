"""rtk::renormalized (the second normalisation's fast path, rt_device.h) on the
GPU against rtk::normalized (sqrt + three IEEE divisions as the compiler lowers
them): bit-identical on 4 x 4M operands -- renormalised unit vectors,
reflections of unit vectors, unit vectors with their length moved by -8..8
ulps, and special components (tests/native/renorm_gpu_check.hip)."""
import ctypes as C
import os

import pytest

from conftest import REPO

LIB = os.path.join(REPO, "tests", "native", "librenormcheck.so")


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [3, 20261016])
def test_renormalized_bit_identical_on_device(seed):
    import torch  # noqa: F401  (brings up the HIP runtime the way the product does)

    lib = C.CDLL(LIB)
    lib.renormcheck_run.argtypes = [C.c_ulonglong, C.c_ulonglong, C.POINTER(C.c_ulonglong)]
    counts = (C.c_ulonglong * 14)()
    n = 1 << 22
    assert lib.renormcheck_run(seed, n, counts) == 0
    c = list(counts)
    for kind in range(4):
        tested, fast, bad = c[3 * kind:3 * kind + 3]
        assert tested == n
        assert bad == 0, f"kind {kind}: {bad} mismatches, last a.x={c[12]:#x} a.y={c[13]:#x}"
    # the renormalised directions nearly always take the fast path
    assert c[1] > 0.99 * n and 0 < c[7] < n

"""rtk::div3 (normalized()'s shared-reciprocal division, rt_device.h) against
three IEEE divisions on the GPU: bit-identical on 4 x 4M operand triples
(scene vectors, near-unit vectors, the whole double range, edge values)."""
import ctypes as C
import os

import pytest

from conftest import REPO

LIB = os.path.join(REPO, "tests", "native", "libdivcheck.so")


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [1, 20260215])
def test_div3_bit_identical(seed):
    import torch  # noqa: F401  (brings up the HIP runtime the way the product does)

    lib = C.CDLL(LIB)
    lib.divcheck_run.argtypes = [C.c_ulonglong, C.c_ulonglong, C.POINTER(C.c_ulonglong)]
    counts = (C.c_ulonglong * 14)()
    n = 1 << 22
    assert lib.divcheck_run(seed, n, counts) == 0
    c = list(counts)
    for kind in range(4):
        tested, fast, bad = c[3 * kind:3 * kind + 3]
        assert tested == n
        assert bad == 0, f"kind {kind}: {bad} mismatches, last a.x={c[12]:#x} b={c[13]:#x}"
    # the fast path is what the renderer's operands take
    assert c[1] == n and c[4] == n
    assert 0 < c[7] < n and 0 < c[10] < n

"""Host side of the nibble-row list layout (include/qba.h "packed lists"):
unpack_nibbles against a direct restatement, odd counts, and the argument
checks of the packed entry points (no GPU: they fail before any device work)."""
import ctypes as C

import numpy as np
import pytest

from conftest import sub


def test_unpack_nibbles_matches_definition():
    rng = np.random.default_rng(7)
    for count in (1, 2, 3, 8, 1001):
        L = rng.integers(0, 16, (12, count)).astype(np.uint8)
        nb = (count + 1) // 2
        P = np.zeros((12, nb + 5), np.uint8)
        for g in range(12):
            for c in range(count):
                P[g, c // 2] |= L[g, c] << (4 * (c % 2))
        assert np.array_equal(sub("engine").unpack_nibbles(P, count), L)


@pytest.mark.parametrize("name", ["qba_sample_packed", "qba_sample_check_packed", "qba_check_counts_packed"])
def test_packed_entry_points_reject_null_ctx(name):
    lib = sub("_lib").lib()
    f = getattr(lib, name)
    f.restype = C.c_int
    if name == "qba_check_counts_packed":
        rc = f(None, 11, None, C.c_uint64(10), C.c_uint64(8), None, None, None, 0, None)
    elif name == "qba_sample_packed":
        rc = f(None, 11, C.c_uint64(0), C.c_uint64(0), C.c_uint64(10), None, C.c_uint64(8), None)
    else:
        rc = f(None, 11, C.c_uint64(0), C.c_uint64(0), C.c_uint64(10), None, C.c_uint64(8), None, None, None,
               0, None)
    assert rc == -1  # QBA_EINVAL

"""CPU: the host arithmetic of mte_gather_summaries' multi-rank path (fluidframework_amd/csrc/gather_plan.hpp:
all-gather of the counts, each rank's records padded to the largest count, the gathered blocks
concatenated in rank order without the padding), driven through a fake all-gather
(tests/native/gather_test.cpp). The RCCL transport itself runs in the GPU suite (tests/test_gpu_c4.py)."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

_NATIVE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "native")


@pytest.fixture(scope="module")
def lib():
    subprocess.run(["make", "-s", "-C", _NATIVE], check=True)
    L = ctypes.CDLL(os.path.join(_NATIVE, "_build", "libgathertest.so"))
    L.gather_selftest.restype = ctypes.c_int
    L.gather_selftest.argtypes = [ctypes.c_void_p, ctypes.c_int]
    return L


@pytest.mark.parametrize("counts", [
    [5], [3, 3], [7, 2], [0, 4], [4, 0], [0, 0], [1, 0, 0, 9],
    [32768, 32767, 32769, 1, 0, 100, 65536, 2],  # C4's 262 144 documents over 8 ranks, unequal
])
def test_gather_count_pad_concat(lib, counts):
    c = np.array(counts, dtype=np.uint64)
    assert lib.gather_selftest(c.ctypes.data, len(counts)) == 0

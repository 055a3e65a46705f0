"""The C-ABI library loads and exports every symbol include/*.h declares (no GPU needed)."""
import ctypes
import os
import re

from fluidframework_amd import mte

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols(header="mte.h"):
    with open(os.path.join(ROOT, "include", header)) as f:
        text = f.read()
    return sorted(set(re.findall(r"\b(mte_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_header_symbols():
    L = ctypes.CDLL(mte.LIB_PATH)
    syms = declared_symbols()
    assert len(syms) >= 18
    for s in syms:
        assert hasattr(L, s), f"libmte.so lacks {s}"
    assert set(syms) == set(mte.EXPORTS)


def test_library_exports_diag_symbols():
    L = ctypes.CDLL(mte.LIB_PATH)
    syms = declared_symbols("mte_diag.h")
    assert len(syms) == 7
    for s in syms:
        assert hasattr(L, s), f"libmte.so lacks {s}"


def test_abi_version_and_info():
    L = mte.lib()
    assert L.mte_abi_version() == 2
    assert b"gfx950" in L.mte_build_info()


def test_library_targets_gfx950_only():
    # the code object bundled in libmte.so is built for gfx950 and nothing else
    data = open(mte.LIB_PATH, "rb").read()
    assert b"gfx950" in data
    for other in (b"gfx90a", b"gfx942", b"gfx1100"):
        assert other not in data


def test_op_record_layout():
    assert mte.OP_DTYPE.itemsize == 32
    assert ctypes.sizeof(mte.mte_doc_summary) == 32

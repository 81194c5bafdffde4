"""The C-ABI library loads and exports every entry point include/*.h declares
(CPU: no compute calls)."""
import ctypes
import os
import re

import pytest

from ompi_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    syms = set()
    inc = os.path.join(ROOT, "include")
    for name in os.listdir(inc):
        if not name.endswith(".h"):
            continue
        text = open(os.path.join(inc, name)).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        for m in re.finditer(r"\b(ompi_amd_[a-z0-9_]+)\s*\(", text):
            syms.add(m.group(1))
    # typedef'd function-pointer names are not symbols
    return {s for s in syms if not s.endswith("_fn_t")}


def test_library_exports_every_declared_symbol():
    lib = _lib.load()
    missing = [s for s in sorted(declared_symbols()) if not hasattr(lib, s)]
    assert not missing, missing


def test_prototypes_cover_header():
    names = {p[0] for p in _lib.PROTOTYPES}
    assert declared_symbols() <= names, declared_symbols() - names


def test_no_cpu_fallback_when_missing(tmp_path):
    with pytest.raises(ImportError):
        _lib._lib_saved = _lib._lib
        try:
            _lib._lib = None
            _lib.load(str(tmp_path / "nope.so"))
        finally:
            _lib._lib = _lib._lib_saved


def test_handler_tables_match_reference_pattern():
    """Rows have OMPI_OP_BASE_TYPE_MAX (41) slots; NULL where op/base has no
    handler (op_base_op_select.c:182-204 requires the same pattern)."""
    lib = _lib.load()
    assert lib.ompi_amd_op_handler_row(15) is not None
    row = lib.ompi_amd_op_handler_row(3)  # SUM
    assert row[15] and row[16] and row[4]          # float, double, int32
    assert not row[35] and not row[30]             # DOUBLE_INT, BYTE
    row = lib.ompi_amd_op_handler_row(11)          # MAXLOC
    assert row[35] and not row[15]
    assert not ctypes.cast(lib.ompi_amd_op_handler_row(99), ctypes.c_void_p).value


def test_type_extents():
    lib = _lib.load()
    assert lib.ompi_amd_type_extent(35) == 16   # DOUBLE_INT
    assert lib.ompi_amd_type_extent(38) == 8    # SHORT_INT
    assert lib.ompi_amd_type_extent(15) == 4
    assert lib.ompi_amd_type_extent(14) == 0    # short float: not provided

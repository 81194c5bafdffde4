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
    assert lib.ompi_amd_type_extent(14) == 2    # short float (_Float16)
    assert lib.ompi_amd_type_extent(26) == 4    # short float complex (_Float16[2])
    assert lib.ompi_amd_type_extent(24) == 0    # long double: not provided


def test_argument_checks_before_any_device_call():
    """Validation paths that return before touching HIP (CPU-safe): a bad op
    or type index, an undefined (op, type) slot, NULL buffers with count > 0,
    and count == 0 (MPI_Reduce_local with count 0 is a no-op even on NULL)."""
    lib = _lib.load()
    SUCCESS, UNSUPPORTED, BAD_PARAM = 0, -1, -2
    assert lib.ompi_amd_op_reduce(99, 15, None, None, 0, None) == BAD_PARAM
    assert lib.ompi_amd_op_reduce(3, 99, None, None, 0, None) == BAD_PARAM
    assert lib.ompi_amd_op_reduce(3, 35, None, None, 0, None) == UNSUPPORTED   # SUM DOUBLE_INT
    assert lib.ompi_amd_op_reduce_3buff(11, 15, None, None, None, 0, None) == UNSUPPORTED
    assert lib.ompi_amd_op_reduce(3, 15, None, None, 0, None) == SUCCESS
    assert lib.ompi_amd_op_reduce_3buff(3, 15, None, None, None, 0, None) == SUCCESS
    assert lib.ompi_amd_op_reduce(3, 15, None, None, 4, None) == BAD_PARAM
    assert lib.ompi_amd_op_reduce_3buff(3, 15, None, None, None, 4, None) == BAD_PARAM
    assert lib.ompi_amd_op_supported(3, 15) == 1
    assert lib.ompi_amd_op_supported(3, 35) == 0
    assert lib.ompi_amd_op_supported(-1, 15) == 0


@pytest.mark.parametrize("count", [0, -5])
def test_handler_nonpositive_count_is_noop(count):
    """op/base's loops run `for (i = 0; i < *count; ++i)` (op_base_functions.c:
    40-51), so count <= 0 touches nothing; the device handler returns before
    classifying the buffers."""
    from ompi_amd import op as mop
    fn = mop.handler(mop.MPI_SUM, mop.MPI_FLOAT)
    c = ctypes.c_int(count)
    fn(None, None, ctypes.byref(c), None, None)
    mop.handler3(mop.MPI_SUM, mop.MPI_FLOAT)(None, None, None, ctypes.byref(c), None, None)

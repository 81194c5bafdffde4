"""Host-side checks of the point-to-point and one-sided surface (CPU, no
compute calls): the constants the MCA glue passes straight through have the
reference's values, and the C headers and the Python mirrors agree."""
import os
import re

from ompi_amd import _lib, osc, pml
from ompi_amd import op as mop

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_defines(name):
    text = open(os.path.join(ROOT, "include", name)).read()
    return {m.group(1): int(m.group(2)) for m in
            re.finditer(r"#define\s+(OMPI_AMD_\w+)\s+\(?(-?\d+)\)?", text)}


def test_send_modes_match_reference_enum():
    # mca_pml_base_send_mode_t, ompi/mca/pml/pml_constants.h:30-37
    d = header_defines("ompi_amd_p2p.h")
    assert [d["OMPI_AMD_SEND_SYNCHRONOUS"], d["OMPI_AMD_SEND_COMPLETE"],
            d["OMPI_AMD_SEND_BUFFERED"], d["OMPI_AMD_SEND_READY"],
            d["OMPI_AMD_SEND_STANDARD"]] == [0, 1, 2, 3, 4]
    assert (pml.SEND_SYNCHRONOUS, pml.SEND_BUFFERED, pml.SEND_STANDARD) == (0, 2, 4)


def test_wildcards_and_truncate():
    d = header_defines("ompi_amd_p2p.h")
    assert d["OMPI_AMD_ANY_SOURCE"] == pml.ANY_SOURCE == -1      # MPI_ANY_SOURCE
    assert d["OMPI_AMD_ANY_TAG"] == pml.ANY_TAG == -1            # MPI_ANY_TAG
    assert d["OMPI_AMD_ERR_TRUNCATE"] == _lib.ERR_TRUNCATE


def test_lock_constants_match_mpi_h():
    # ompi/include/mpi.h.in:542, 548-549
    d = header_defines("ompi_amd_osc.h")
    assert d["OMPI_AMD_LOCK_EXCLUSIVE"] == osc.LOCK_EXCLUSIVE == 1
    assert d["OMPI_AMD_LOCK_SHARED"] == osc.LOCK_SHARED == 2
    assert d["OMPI_AMD_MODE_NOCHECK"] == osc.MODE_NOCHECK == 1


def test_replace_and_no_op_codes():
    # OMPI_OP_BASE_FORTRAN_REPLACE / _NO_OP, ompi/mca/op/op.h:232-235
    assert (mop.MPI_REPLACE.index, mop.MPI_NO_OP.index) == (13, 14)


def test_status_struct_layout():
    import ctypes
    assert ctypes.sizeof(_lib.Status) == 24
    assert _lib.Status.bytes.offset == 16

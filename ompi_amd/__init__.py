"""ompi_amd — MI355X-native reduction-collective hot path for Open MPI.

Product = libompi_amd.so (HIP kernels for gfx950 + C ABI, include/ompi_amd.h).
This package is the host-side mirror of the reference's interface for the
path: MPI_Op reduce_local (op.py), datatype pack/unpack (datatype.py) and
the device-buffer collectives (coll.py).
"""
from ._lib import OmpiAmdError, load  # noqa: F401
from .op import *  # noqa: F401,F403

__all__ = ["OmpiAmdError", "load"]

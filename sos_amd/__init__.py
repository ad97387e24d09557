"""sos_amd -- MI355X-native SOS (Sandia OpenSHMEM) team-reduction path.

The product is the native library ``sos_amd/libsos_amd.so`` (C ABI: include/shmem.h,
include/shmemx.h, include/sosx.h).  This package holds its sources (``csrc/``) and a
ctypes binding for Python callers (``_lib``, ``shmem``).
"""
from . import _lib  # noqa: F401

__all__ = ["_lib"]

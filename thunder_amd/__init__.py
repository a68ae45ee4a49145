"""thunder_amd -- MI355X (gfx950) particle-filter expectation / Fourier-insert engine.

Drop-in for THUNDER's GPU plugin surface (gpu/interface/Interface.h): the
kernels live in libthunder_amd.so behind the C-ABI of include/thunder_amd.h;
this package is the thin torch/ctypes front end used by the tests and bench.
"""
from ._lib import ThxError, lib  # noqa: F401
from .build import LIB as LIBRARY_PATH  # noqa: F401

__all__ = ["lib", "ThxError", "LIBRARY_PATH"]

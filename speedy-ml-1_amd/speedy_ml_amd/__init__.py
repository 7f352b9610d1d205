"""speedy_ml_amd -- MI355X-native SPEEDY-ML hybrid hot path (host-side mirror).

The compute lives in libspeedyml.so (hand-written gfx950 HIP kernels behind the C
ABI of include/speedy_ml.h).  This package is the Python host layer used by the
tests and bench.py; the Fortran host binding lives in ../fortran/.
"""
from ._lib import SmlError, build, lib  # noqa: F401
from . import domain, synthetic  # noqa: F401

__all__ = ["SmlError", "build", "lib", "domain", "synthetic"]

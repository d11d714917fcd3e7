"""nusiprop_amd -- MI355X-native nuSIprop cascade solver.

The hot path of quarkquartet/nuSIprop, calculate_flux::evolve() (nuSIprop.hpp:
176-337), as hand-written HIP kernels for gfx950 behind a C ABI (include/nusi.h,
libnusi.so), with the reference's Python surface (``pyprop``) on top.
"""
from ._lib import (NusiError, NusiParams, SOURCE_DSNB, SOURCE_POWER_LAW, WARN_ALPHA, WARN_ALPHATILDE,  # noqa: F401
                   WARN_GAMMA, make_params, load)
from .plan import Plan, unpack_alpha  # noqa: F401
from .pyprop import pyprop  # noqa: F401

__all__ = ["pyprop", "Plan", "unpack_alpha", "NusiError", "NusiParams", "make_params", "load",
           "SOURCE_DSNB", "SOURCE_POWER_LAW"]

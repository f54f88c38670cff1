"""mkfhe_amd -- MI355X-native multi-key blind-rotation accumulator engine.

Drop-in for the SKLC-FHE/MKFHE accumulator plugin seam
(UniEncAccumulator::EvalAcc, reference src/binfhe/include/mk-acc.h:55-80),
implemented as hand-written HIP kernels for gfx950 behind the C ABI in
include/mkfhe_amd.h.  See DESIGN.md.
"""
from ._lib import LIB_PATH, MkaccError, MkaccParams  # noqa: F401
from .accumulator import (  # noqa: F401
    MKNTRU,
    MKNTRU_B,
    MKNTRU_LWE,
    PARAMSETS,
    MKAccumulatorEngine,
    MKAccumulatorGroup,
    UniEncAccumulator,
    UniEncAccumulatorXZW,
    UniEncAccumulatorXZW_B,
    accumulator_for,
    make_params,
    paramset,
)

__all__ = [
    "LIB_PATH", "MkaccError", "MkaccParams", "MKNTRU", "MKNTRU_B", "MKNTRU_LWE", "PARAMSETS",
    "MKAccumulatorEngine", "MKAccumulatorGroup", "UniEncAccumulator", "UniEncAccumulatorXZW", "UniEncAccumulatorXZW_B",
    "accumulator_for", "make_params", "paramset",
]

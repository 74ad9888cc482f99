"""lime_amd -- MI355X-native engine for LIME's genomic set-theory hot path.

Intersection, merge (union), subtract (difference) and complement over
ReferenceRegion-keyed interval sets, as hand-written HIP kernels for gfx950
behind the C-ABI in include/lime_amd.h.  See DESIGN.md.
"""
from ._ffi import LimeError, SUBTRACT_LIME, SUBTRACT_SET, load  # noqa: F401
from .engine import (Context, IntervalSet, PAIR_DTYPE, Pairs, Result, Space,  # noqa: F401
                     java_string_order, read_bed)

__version__ = "0.1.0"

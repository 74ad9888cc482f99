"""ctypes binding of the C-ABI in include/lime_amd.h (liblime_amd.so).

The shared library is built in-tree (``make`` / ``__graft_entry__.build()``)
and loaded from this package directory.  There is no fallback: if the
library is missing or a symbol is absent, import fails loudly.
"""
import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "liblime_amd.so")
# tuning experiments only (tools/): load a variant build instead
if os.environ.get("LIME_AMD_LIB_VARIANT"):
    LIB_PATH = os.environ["LIME_AMD_LIB_VARIANT"]

LIME_OK = 0
ERRORS = {
    1: "LIME_ERR_ARG",
    2: "LIME_ERR_RANGE",
    3: "LIME_ERR_DEVICE",
    4: "LIME_ERR_NOMEM",
    5: "LIME_ERR_CONTIG",
    6: "LIME_ERR_IO",
    7: "LIME_ERR_OVERFLOW",
}
# the C-ABI contract this binding is written against (include/lime_amd.h
# LIME_ABI_VERSION): checked at load, so a stale library fails loudly
ABI_VERSION = 6
SUBTRACT_LIME = 0
SUBTRACT_SET = 1


class LimeError(RuntimeError):
    """A non-zero status from the engine; ``code`` is the LIME_ERR_* value."""

    def __init__(self, code, msg):
        super().__init__(f"{ERRORS.get(code, code)}: {msg}")
        self.code = code


class Pair(C.Structure):
    _fields_ = [("start", C.c_uint32), ("end", C.c_uint32), ("a_row", C.c_uint32),
                ("b_row", C.c_uint32)]


vp = C.c_void_p
i32, i64, u32, u64 = C.c_int32, C.c_int64, C.c_uint32, C.c_uint64
P = C.POINTER
pp = P(vp)

# name -> (restype, argtypes); every symbol include/lime_amd.h declares
SIGNATURES = {
    "lime_last_error": (C.c_char_p, []),
    "lime_abi_version": (C.c_int, []),
    "lime_ctx_create": (C.c_int, [C.c_int, pp]),
    "lime_ctx_destroy": (C.c_int, [vp]),
    "lime_ctx_set_stream": (C.c_int, [vp, vp]),
    "lime_ctx_synchronize": (C.c_int, [vp]),
    "lime_ctx_pool_bytes": (i64, [vp]),
    "lime_ctx_pool_live_bytes": (i64, [vp, C.c_int32, P(i64)]),
    "lime_space_create": (C.c_int, [i32, P(i64), pp]),
    "lime_space_destroy": (C.c_int, [vp]),
    "lime_space_contigs": (i32, [vp]),
    "lime_space_span": (i64, [vp]),
    "lime_space_offset": (i64, [vp, i32]),
    "lime_set_create_host": (C.c_int, [vp, vp, i64, P(i32), P(i64), P(i64), pp]),
    "lime_set_create_host_stranded": (C.c_int, [vp, vp, i64, P(i32), P(i64), P(i64),
                                                P(C.c_int8), pp]),
    "lime_set_create_device": (C.c_int, [vp, vp, i64, vp, vp, vp, pp]),
    "lime_set_create_device_stranded": (C.c_int, [vp, vp, i64, vp, vp, vp, vp, pp]),
    "lime_set_create_global": (C.c_int, [vp, vp, i64, vp, vp, vp, pp]),
    "lime_set_create_global_stranded": (C.c_int, [vp, vp, i64, vp, vp, vp, vp, pp]),
    "lime_set_destroy": (C.c_int, [vp]),
    "lime_set_size": (i64, [vp]),
    "lime_set_lower_bound": (i64, [vp, u32]),
    "lime_set_first_reaching": (i64, [vp, u32]),
    "lime_set_lower_bounds": (C.c_int, [vp, C.c_int32, P(u32), P(i64)]),
    "lime_set_first_reachings": (C.c_int, [vp, C.c_int32, P(u32), P(i64)]),
    "lime_set_copy_rows_device": (C.c_int, [vp, i64, i64, vp, vp, vp]),
    "lime_set_stats": (C.c_int, [vp, P(u32), P(u32), P(i32)]),
    "lime_set_extend_sorted": (C.c_int, [vp, vp, i64, vp, vp, vp, u32, u32, i32, pp]),
    "lime_set_concat_sorted": (C.c_int, [vp, vp, i64, vp, vp, vp, i64, vp, vp, vp, u32, u32, i32,
                                         pp]),
    "lime_sample_starts": (C.c_int, [vp, vp, i64, vp, vp, i32, vp]),
    "lime_result_copy_range": (C.c_int, [vp, i64, i64, P(u32), P(u32)]),
    "lime_set_device_arrays": (C.c_int, [vp, pp, pp, pp]),
    "lime_set_fill_host": (C.c_int, [vp, P(i32), P(i64), P(i64), P(i64)]),
    "lime_intersect_count": (C.c_int, [vp, vp, vp, i64, pp, P(i64)]),
    "lime_intersect_count_owned": (C.c_int, [vp, vp, vp, i64, i64, i64, pp, P(i64)]),
    "lime_window_count": (C.c_int, [vp, vp, vp, i64, pp, P(i64)]),
    "lime_closest_count": (C.c_int, [vp, vp, vp, C.c_int, pp, P(i64)]),
    "lime_closest_rounds": (C.c_int, [vp, P(C.c_int32), P(C.c_int32)]),
    "lime_closest_count_chained": (C.c_int, [vp, vp, vp, C.c_int, C.c_int32, P(C.c_int32), pp,
                                             P(i64)]),
    "lime_intersect_fill_device": (C.c_int, [vp, i64, i64, vp]),
    "lime_intersect_fill_host": (C.c_int, [vp, i64, i64, vp]),
    "lime_intersect_checksum": (C.c_int, [vp, P(u64), P(u64)]),
    "lime_pairs_checksum_device": (C.c_int, [vp, vp, i64, P(u64), P(u64)]),
    "lime_pairs_destroy": (C.c_int, [vp]),
    "lime_merge": (C.c_int, [vp, vp, pp, P(i64)]),
    "lime_subtract": (C.c_int, [vp, vp, vp, i64, C.c_int, pp, P(i64)]),
    "lime_complement": (C.c_int, [vp, vp, vp, pp, P(i64)]),
    "lime_complement_runs": (C.c_int, [vp, vp, i64, vp, vp, i64, i64, pp, P(i64)]),
    "lime_result_size": (i64, [vp]),
    "lime_result_fill_host": (C.c_int, [vp, P(i32), P(i64), P(i64), P(i64), P(i64)]),
    "lime_result_run_of_row": (C.c_int, [vp, P(i64)]),
    "lime_result_copy_run_ids_device": (C.c_int, [vp, vp, vp]),
    "lime_result_copy_rows_device": (C.c_int, [vp, i64, i64, vp, vp]),
    "lime_result_run_strands": (C.c_int, [vp, i64, i64, P(C.c_int8)]),
    "lime_result_device_arrays": (C.c_int, [vp, pp, pp]),
    "lime_result_destroy": (C.c_int, [vp]),
    "lime_result_checksum": (C.c_int, [vp, P(u64), P(u64), P(u64), P(u64)]),
    "lime_bitset_from_set": (C.c_int, [vp, vp, pp]),
    "lime_bitset_from_device": (C.c_int, [vp, vp, i64, vp, vp, vp, pp]),
    "lime_bitset_from_global": (C.c_int, [vp, vp, i64, i64, i64, vp, vp, pp]),
    "lime_bitset_and_from_device": (C.c_int, [vp, vp, C.c_int32, P(i64), P(vp), P(vp), P(vp), pp]),
    "lime_bitset_and_from_global": (C.c_int, [vp, vp, i64, i64, C.c_int32, P(i64), P(vp), P(vp),
                                              pp]),
    "lime_bitset_window": (C.c_int, [vp, P(i64), P(i64)]),
    "lime_route_rows": (C.c_int, [vp, vp, i64, vp, vp, vp, u32, i32, P(u32), C.c_int, i64, vp,
                                  vp, vp, P(i64), vp, vp]),
    "lime_route_rows_interleaved": (C.c_int, [vp, vp, i64, vp, vp, vp, u32, i32, P(u32), C.c_int,
                                              i64, i32, vp, P(i64)]),
    "lime_deinterleave_u32": (C.c_int, [vp, i64, i32, vp, vp, vp, vp]),
    "lime_bitset_runs": (C.c_int, [vp, C.c_int, vp, vp, pp, P(i64)]),
    "lime_bitset_and_runs": (C.c_int, [vp, C.c_int, P(vp), pp, P(i64)]),
    "lime_bitset_popcount": (i64, [vp, vp]),
    "lime_bitset_drop_bins": (C.c_int, [vp, vp]),
    "lime_bitset_destroy": (C.c_int, [vp]),
    "lime_synth_uniform": (C.c_int, [vp, vp, i64, u64, u32, u32, vp, vp, vp]),
    "lime_synth_pileup": (C.c_int, [vp, vp, i64, u64, i64, u32, u32, u32, vp, vp, vp]),
    "lime_synth_uniform_rows": (C.c_int, [vp, vp, i64, i64, u64, u32, u32, vp, vp, vp]),
    "lime_synth_pileup_rows": (C.c_int, [vp, vp, i64, i64, u64, i64, u32, u32, u32, vp, vp, vp]),
    "lime_contig_rank": (C.c_int, [i32, P(C.c_char_p), P(i32)]),
    "lime_bed_read": (C.c_int, [C.c_char_p, pp]),
    "lime_bed_rows": (i64, [vp]),
    "lime_bed_contigs": (i32, [vp]),
    "lime_bed_contig_name": (C.c_char_p, [vp, i32]),
    "lime_bed_contig_ids": (P(i32), [vp]),
    "lime_bed_starts": (P(i64), [vp]),
    "lime_bed_ends": (P(i64), [vp]),
    "lime_bed_strands": (P(C.c_int8), [vp]),
    "lime_bed_name": (C.c_char_p, [vp, i64]),
    "lime_bed_free": (None, [vp]),
    "lime_bed_parse_device": (C.c_int, [vp, C.c_char_p, i64, pp]),
    "lime_dbed_rows": (i64, [vp]),
    "lime_dbed_contigs": (i32, [vp]),
    "lime_dbed_contig_name": (C.c_char_p, [vp, i32]),
    "lime_dbed_device_arrays": (C.c_int, [vp, pp, pp, pp, pp]),
    "lime_dbed_fill_host": (C.c_int, [vp, P(i32), P(i64), P(i64), P(C.c_int8), P(i64), P(i32)]),
    "lime_dbed_remap_contigs": (C.c_int, [vp, P(i32), i32]),
    "lime_dbed_free": (None, [vp]),
    "lime_set_format_bed": (C.c_int, [vp, P(C.c_char_p), C.c_char_p, i64, P(i64)]),
    "lime_result_format_bed": (C.c_int, [vp, P(C.c_char_p), C.c_char_p, i64, P(i64)]),
    "lime_genome_read": (C.c_int, [C.c_char_p, P(i32), P(P(C.c_char_p)), P(P(i64))]),
    "lime_genome_free": (None, [i32, P(C.c_char_p), P(i64)]),
    "lime_pair_hash": (u64, [u32, u32, u32, u32]),
}

_lib = None


def load(path=LIB_PATH):
    """Load liblime_amd.so and attach prototypes (raises if absent)."""
    global _lib
    if _lib is not None:
        return _lib
    # PyTorch-ROCm bundles its own HIP runtime with the same soname
    # (libamdhip64.so.7).  Loading torch first makes this library bind to that
    # already-loaded runtime, so the process holds ONE HIP runtime and device
    # pointers / streams are shared with torch; loading ours first would make
    # torch pull in a second runtime that no longer sees the GPU.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    if not os.path.exists(path):
        raise ImportError(
            f"{path} is missing: build the HIP engine first (make, or "
            "__graft_entry__.build()); there is no CPU fallback")
    lib = C.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)  # AttributeError if the symbol is missing
        fn.restype = res
        fn.argtypes = args
    if lib.lime_abi_version() != ABI_VERSION:
        raise ImportError(f"{path}: C-ABI version {lib.lime_abi_version()}, this binding "
                          f"needs {ABI_VERSION}: rebuild the engine")
    _lib = lib
    return lib


def check(status):
    if status != LIME_OK:
        msg = _lib.lime_last_error().decode(errors="replace")
        raise LimeError(status, msg)
    return status

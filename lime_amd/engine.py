"""Pythonic handles over the C-ABI: Context, Space, IntervalSet, results.

This is plumbing for tests, benchmarks and the multi-GPU driver; the
operator mirror of lime-core lives in :mod:`lime_amd.set_theory`.
All compute goes through liblime_amd.so (HIP, gfx950); nothing here falls
back to the CPU.
"""
import ctypes as C

import numpy as np

from . import _ffi
from ._ffi import check, i32, i64, u32, u64, vp

P = C.POINTER

PAIR_DTYPE = np.dtype([("start", "<u4"), ("end", "<u4"), ("a_row", "<u4"), ("b_row", "<u4")])


def _lib():
    return _ffi.load()


def _ptr(a, ct):
    return a.ctypes.data_as(P(ct))


def java_string_order(names):
    """Ranks of `names` in java.lang.String.compareTo order (via the C-ABI)."""
    lib = _lib()
    n = len(names)
    arr = (C.c_char_p * max(n, 1))(*[s.encode() for s in names])
    out = np.zeros(max(n, 1), dtype=np.int32)
    check(lib.lime_contig_rank(n, arr, _ptr(out, i32)))
    return out[:n]


def _format_bed(fn, handle, space):
    """two-call device BED writer -> bytes"""
    names = (C.c_char_p * max(len(space.names), 1))(*[n.encode() for n in space.names])
    n = i64()
    check(fn(handle, names, None, 0, C.byref(n)))
    buf = C.create_string_buffer(max(n.value, 1))
    check(fn(handle, names, buf, n.value, C.byref(n)))
    return buf.raw[:n.value]


class Space:
    """Contigs in Java String order with their lengths (the coordinate space)."""

    def __init__(self, names, lengths):
        names = list(names)
        lengths = [int(x) for x in lengths]
        if len(set(names)) != len(names):
            raise ValueError("duplicate contig names")
        rank = java_string_order(names) if names else np.zeros(0, np.int32)
        order = np.argsort(rank, kind="stable")
        self.names = [names[i] for i in order]
        self.lengths = np.array([lengths[i] for i in order], dtype=np.int64)
        self.index = {n: i for i, n in enumerate(self.names)}
        lib = _lib()
        h = vp()
        check(lib.lime_space_create(len(self.names), _ptr(self.lengths, i64), C.byref(h)))
        self._h = h
        self.offsets = np.array(
            [lib.lime_space_offset(h, c) for c in range(len(self.names) + 1)], dtype=np.int64)

    @property
    def handle(self):
        return self._h

    @property
    def span(self):
        return int(_lib().lime_space_span(self._h))

    @classmethod
    def from_genome_file(cls, path):
        lib = _lib()
        n = i32()
        names = P(C.c_char_p)()
        lens = P(i64)()
        check(lib.lime_genome_read(path.encode(), C.byref(n), C.byref(names), C.byref(lens)))
        try:
            nm = [names[i].decode() for i in range(n.value)]
            ln = [lens[i] for i in range(n.value)]
        finally:
            lib.lime_genome_free(n.value, names, lens)
        return cls(nm, ln)

    def contig_ids(self, names):
        return np.array([self.index[n] for n in names], dtype=np.int32)

    def __del__(self):
        try:
            if getattr(self, "_h", None):
                _lib().lime_space_destroy(self._h)
                self._h = None
        except Exception:
            pass


class IntervalSet:
    """A sorted, device-resident interval set (lime_set)."""

    def __init__(self, ctx, handle, space):
        self.ctx, self._h, self.space = ctx, handle, space

    @property
    def n(self):
        return int(_lib().lime_set_size(self._h))

    def device_arrays(self):
        gs, ge, row = vp(), vp(), vp()
        check(_lib().lime_set_device_arrays(self._h, C.byref(gs), C.byref(ge), C.byref(row)))
        return gs.value, ge.value, row.value

    def to_bed(self):
        """the sorted rows as BED3 text, formatted on the device"""
        return _format_bed(_lib().lime_set_format_bed, self._h, self.space)

    def lower_bound(self, gkey):
        """first sorted row with global start >= gkey"""
        r = _lib().lime_set_lower_bound(self._h, int(gkey))
        if r < 0:
            check(int(-r))
        return int(r)

    def first_reaching(self, gkey):
        """first sorted row from which rows may end past gkey (none before)"""
        r = _lib().lime_set_first_reaching(self._h, int(gkey))
        if r < 0:
            check(int(-r))
        return int(r)

    def lower_bounds(self, gkeys):
        """lower_bound of every key in one launch and one read-back"""
        return self._bounds(_lib().lime_set_lower_bounds, gkeys)

    def first_reachings(self, gkeys):
        """first_reaching of every key in one launch and one read-back"""
        return self._bounds(_lib().lime_set_first_reachings, gkeys)

    def _bounds(self, fn, gkeys):
        k = len(gkeys)
        if k == 0:
            return []
        keys = (C.c_uint32 * k)(*[int(x) for x in gkeys])
        out = (i64 * k)()
        check(fn(self._h, k, keys, out))
        return list(out)

    def stats(self):
        """(min width, max width, has a zero-width row)"""
        lo, hi, z = u32(), u32(), i32()
        check(_lib().lime_set_stats(self._h, C.byref(lo), C.byref(hi), C.byref(z)))
        return lo.value, hi.value, bool(z.value)

    def copy_rows_device(self, first, count, d_gs, d_ge, d_row):
        check(_lib().lime_set_copy_rows_device(self._h, int(first), int(count), d_gs, d_ge,
                                               d_row))

    def to_host(self):
        n = self.n
        out = {k: np.zeros(n, dtype=np.int64) for k in ("start", "end", "row")}
        out["contig"] = np.zeros(n, dtype=np.int32)
        check(_lib().lime_set_fill_host(self._h, _ptr(out["contig"], i32), _ptr(out["start"], i64),
                                        _ptr(out["end"], i64), _ptr(out["row"], i64)))
        return out

    def close(self):
        if self._h and self.ctx.handle:  # a closed context already freed its pool
            _lib().lime_set_destroy(self._h)
        self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Result:
    """merge / subtract / complement / bitset output (lime_result)."""

    def __init__(self, ctx, handle, space, keep=()):
        # `keep`: the inputs whose device arrays this handle still reads
        self.ctx, self._h, self.space, self._keep = ctx, handle, space, keep

    @property
    def n(self):
        return int(_lib().lime_result_size(self._h))

    def to_host(self):
        n = self.n
        out = {k: np.zeros(n, dtype=np.int64) for k in ("start", "end", "a_row", "b_row")}
        out["contig"] = np.zeros(n, dtype=np.int32)
        check(_lib().lime_result_fill_host(self._h, _ptr(out["contig"], i32),
                                           _ptr(out["start"], i64), _ptr(out["end"], i64),
                                           _ptr(out["a_row"], i64), _ptr(out["b_row"], i64)))
        return out

    def to_bed(self):
        """the result's regions as BED3 text, formatted on the device"""
        return _format_bed(_lib().lime_result_format_bed, self._h, self.space)

    def checksum(self):
        """(reg_sum, reg_xor, grp_sum, grp_xor): order-independent checksums of
        the regions and (merge) of the row -> run grouping, on the device"""
        v = [u64() for _ in range(4)]
        check(_lib().lime_result_checksum(self._h, *[C.byref(x) for x in v]))
        return tuple(x.value for x in v)

    def run_of_row(self, n_rows):
        out = np.zeros(n_rows, dtype=np.int64)
        check(_lib().lime_result_run_of_row(self._h, _ptr(out, i64)))
        return out

    def device_arrays(self):
        gs, ge = vp(), vp()
        check(_lib().lime_result_device_arrays(self._h, C.byref(gs), C.byref(ge)))
        return gs.value, ge.value

    def copy_run_ids_device(self, d_run, d_row):
        """merge results: (run of every sorted input row, that row's id) into
        caller device buffers (u32, as many as the merged set has rows)"""
        check(_lib().lime_result_copy_run_ids_device(self._h, vp(d_run), vp(d_row)))

    def copy_rows_device(self, first, count, d_gs, d_ge):
        """regions [first, first + count) (global) into caller device buffers"""
        check(_lib().lime_result_copy_rows_device(self._h, int(first), int(count), vp(d_gs),
                                                  vp(d_ge)))

    def run_strands(self, first, count):
        """stranded merges: strand codes of runs [first, first + count)"""
        out = np.zeros(max(int(count), 1), dtype=np.int8)
        check(_lib().lime_result_run_strands(self._h, int(first), int(count),
                                             _ptr(out, C.c_int8)))
        return out[:count]

    def copy_range(self, first, count):
        """host copy of regions [first, first+count) in GLOBAL coordinates"""
        gs = np.zeros(count, dtype=np.uint32)
        ge = np.zeros(count, dtype=np.uint32)
        check(_lib().lime_result_copy_range(self._h, int(first), int(count),
                                            gs.ctypes.data_as(P(C.c_uint32)),
                                            ge.ctypes.data_as(P(C.c_uint32))))
        return gs, ge

    def close(self):
        if self._h and self.ctx.handle:  # a closed context already freed its pool
            _lib().lime_result_destroy(self._h)
        self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Pairs:
    """Intersect plan: exact pair count plus chunked fill (lime_pairs)."""

    def __init__(self, ctx, handle, n, keep=()):
        # the plan reads A's and B's device arrays: keep both alive
        self.ctx, self._h, self.n, self._keep = ctx, handle, n, keep

    def fill_host(self, first=0, count=None):
        if count is None:
            count = self.n - first
        out = np.zeros(count, dtype=PAIR_DTYPE)
        check(_lib().lime_intersect_fill_host(self._h, first, count, out.ctypes.data))
        return out

    def fill_device(self, first, count, d_out):
        check(_lib().lime_intersect_fill_device(self._h, first, count, d_out))

    def closest_rounds(self):
        """closest plans: (Jacobi rounds run, whether the in-order recursion
        finished the cache-head fixed point)"""
        r, q = C.c_int32(), C.c_int32()
        check(_lib().lime_closest_rounds(self._h, C.byref(r), C.byref(q)))
        return r.value, bool(q.value)

    def checksum(self):
        s, x = u64(), u64()
        check(_lib().lime_intersect_checksum(self._h, C.byref(s), C.byref(x)))
        return s.value, x.value

    def close(self):
        if self._h and self.ctx.handle:  # a closed context already freed its pool
            _lib().lime_pairs_destroy(self._h)
        self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Bitset:
    def __init__(self, ctx, handle, space, keep=()):
        # `keep`: the inputs whose device arrays this handle still reads
        self.ctx, self._h, self.space, self._keep = ctx, handle, space, keep

    def popcount(self):
        return int(_lib().lime_bitset_popcount(self.ctx.handle, self._h))

    def drop_bins(self):
        """paint the words and free the binned rows a bitset from rows keeps
        (4 B per row per input set): same bits, window bits / 8 bytes held"""
        check(_lib().lime_bitset_drop_bins(self.ctx.handle, self._h))
        return self

    def window(self):
        """(lo, n_words): the global bits this bitset covers start at lo"""
        lo, nw = i64(), i64()
        check(_lib().lime_bitset_window(self._h, C.byref(lo), C.byref(nw)))
        return lo.value, nw.value

    def close(self):
        if self._h and self.ctx.handle:  # a closed context already freed its pool
            _lib().lime_bitset_destroy(self._h)
        self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Context:
    """One device, one HIP stream, one memory pool (lime_ctx)."""

    def __init__(self, device=0):
        lib = _lib()
        h = vp()
        check(lib.lime_ctx_create(int(device), C.byref(h)))
        self._h = h
        self.device = device

    @property
    def handle(self):
        return self._h

    def set_stream(self, hip_stream_ptr):
        check(_lib().lime_ctx_set_stream(self._h, hip_stream_ptr))

    def synchronize(self):
        check(_lib().lime_ctx_synchronize(self._h))

    def pool_bytes(self):
        return int(_lib().lime_ctx_pool_bytes(self._h))

    def pool_live_bytes(self, reset_peak=False):
        """(live bytes, their peak since the last reset) of the device pool"""
        peak = i64()
        live = _lib().lime_ctx_pool_live_bytes(self._h, int(bool(reset_peak)), C.byref(peak))
        return int(live), int(peak.value)

    # ------------------------------------------------------------ sets
    def set_from_host(self, space, contig, start, end):
        contig = np.ascontiguousarray(contig, dtype=np.int32)
        start = np.ascontiguousarray(start, dtype=np.int64)
        end = np.ascontiguousarray(end, dtype=np.int64)
        h = vp()
        check(_lib().lime_set_create_host(self._h, space.handle, len(contig), _ptr(contig, i32),
                                          _ptr(start, i64), _ptr(end, i64), C.byref(h)))
        return IntervalSet(self, h, space)

    def set_from_host_stranded(self, space, contig, start, end, strand):
        """Stranded set: sorted by (start, end, strand); merge breaks runs at
        strand changes (the reference fold)."""
        contig = np.ascontiguousarray(contig, dtype=np.int32)
        start = np.ascontiguousarray(start, dtype=np.int64)
        end = np.ascontiguousarray(end, dtype=np.int64)
        strand = np.ascontiguousarray(strand, dtype=np.int8)
        h = vp()
        check(_lib().lime_set_create_host_stranded(self._h, space.handle, len(contig),
                                                   _ptr(contig, i32), _ptr(start, i64),
                                                   _ptr(end, i64), _ptr(strand, C.c_int8),
                                                   C.byref(h)))
        return IntervalSet(self, h, space)

    def set_from_device(self, space, n, d_contig, d_start, d_end):
        h = vp()
        check(_lib().lime_set_create_device(self._h, space.handle, int(n), d_contig, d_start,
                                            d_end, C.byref(h)))
        return IntervalSet(self, h, space)

    def set_from_device_stranded(self, space, n, d_contig, d_start, d_end, d_strand=None):
        """device rows in full RegionOrdering (int8 strand codes in HBM, or
        None = every row independent)"""
        h = vp()
        check(_lib().lime_set_create_device_stranded(self._h, space.handle, int(n), d_contig,
                                                     d_start, d_end, d_strand, C.byref(h)))
        return IntervalSet(self, h, space)

    def set_from_global(self, space, n, d_gs, d_ge, d_row):
        """rows already in the space's global coordinates (u32 device arrays)"""
        h = vp()
        check(_lib().lime_set_create_global(self._h, space.handle, int(n), d_gs, d_ge, d_row,
                                            C.byref(h)))
        return IntervalSet(self, h, space)

    def set_concat_sorted(self, before, s, after, min_width, max_width, has_zero):
        """rows `before` (n, d_gs, d_ge, d_row), then s, then rows `after` --
        a shard's left halo, own rows and right halo, which the caller
        guarantees to be in canonical order -- copied without a sort, a
        validation or a read-back; the added rows' widths bounded by the
        caller's (min, max, any zero)"""
        h = vp()
        nb, bg, be, br = before
        na, ag, ae, ar = after
        check(_lib().lime_set_concat_sorted(self._h, s._h, int(nb), vp(bg), vp(be), vp(br),
                                            int(na), vp(ag), vp(ae), vp(ar), int(min_width),
                                            int(max_width), int(bool(has_zero)), C.byref(h)))
        return IntervalSet(self, h, s.space)

    def sample_starts(self, space, n, d_contig, d_start, k, d_out):
        """k evenly spaced rows' global starts into the device array d_out
        (u32; d_contig None: d_start already global), stream-ordered"""
        check(_lib().lime_sample_starts(self._h, space.handle, int(n), vp(d_contig), vp(d_start),
                                        int(k), vp(d_out)))

    def set_extend_sorted(self, s, n, d_gs, d_ge, d_row, min_width, max_width, has_zero):
        """s's rows followed by n device rows that the caller guarantees to be
        in canonical order past s's last row (a shard's right halo), copied
        without a sort, a validation or a read-back; the widths of the added
        rows are bounded by the caller's (min, max, any zero)"""
        h = vp()
        check(_lib().lime_set_extend_sorted(self._h, s._h, int(n), vp(d_gs), vp(d_ge), vp(d_row),
                                            int(min_width), int(max_width), int(bool(has_zero)),
                                            C.byref(h)))
        return IntervalSet(self, h, s.space)

    def set_from_global_stranded(self, space, n, d_gs, d_ge, d_row, d_strand):
        """global rows with int8 strand codes in HBM: full RegionOrdering, merge
        breaks runs at strand changes"""
        h = vp()
        check(_lib().lime_set_create_global_stranded(self._h, space.handle, int(n), d_gs, d_ge,
                                                     d_row, vp(d_strand), C.byref(h)))
        return IntervalSet(self, h, space)

    # ------------------------------------------------------------- ops
    def intersect(self, a, b, threshold=0, a_owned=-1, b_owned=-1):
        h, n = vp(), i64()
        check(_lib().lime_intersect_count_owned(self._h, a._h, b._h, int(threshold),
                                                int(a_owned), int(b_owned), C.byref(h),
                                                C.byref(n)))
        return Pairs(self, h, n.value, keep=(a, b))

    def window(self, a, b, distance=1000):
        """DistributedWindow: pairs (a, b) with a.isNearby(b, distance); the
        pair records carry a's own region."""
        h, n = vp(), i64()
        check(_lib().lime_window_count(self._h, a._h, b._h, int(distance), C.byref(h),
                                       C.byref(n)))
        return Pairs(self, h, n.value, keep=(a, b))

    def closest(self, a, b, mode=0):
        """SingleClosest (mode 0, Closest.scala:34-214) or
        SingleClosestSingleOverlap (mode 1, :216-268) on one partition: for
        each left row, the cached right rows at the current closest's
        distance.  Both sets must be in RegionOrdering (set_from_host_stranded
        / set_from_device_stranded)."""
        return self.closest_chained(a, b, mode)[0]

    def closest_chained(self, a, b, mode=0, alive_in=True):
        """closest over one of several chained spaces (a genome whose span
        needs more than one space): -> (Pairs, alive_out)"""
        h, n, live = vp(), i64(), C.c_int32()
        check(_lib().lime_closest_count_chained(self._h, a._h, b._h, int(mode), int(bool(alive_in)),
                                                C.byref(live), C.byref(h), C.byref(n)))
        return Pairs(self, h, n.value, keep=(a, b)), bool(live.value)

    def parse_bed(self, text):
        """Parse BED text (bytes) on the device -> DeviceBed (arrays in HBM)."""
        h = vp()
        text = bytes(text)
        check(_lib().lime_bed_parse_device(self._h, text, len(text), C.byref(h)))
        return DeviceBed(self, h, text)

    def merge(self, a):
        h, n = vp(), i64()
        check(_lib().lime_merge(self._h, a._h, C.byref(h), C.byref(n)))
        return Result(self, h, a.space, keep=(a,))

    def subtract(self, a, b, threshold=0, mode=_ffi.SUBTRACT_LIME):
        h, n = vp(), i64()
        check(_lib().lime_subtract(self._h, a._h, b._h, int(threshold), int(mode), C.byref(h),
                                   C.byref(n)))
        return Result(self, h, a.space, keep=(a, b))

    def complement(self, genome_space, a):
        h, n = vp(), i64()
        check(_lib().lime_complement(self._h, genome_space.handle, a._h, C.byref(h), C.byref(n)))
        return Result(self, h, a.space, keep=(a,))

    def complement_runs(self, genome_space, n, d_gs, d_ge, lo=0, hi=None):
        """gaps of sorted disjoint runs in HBM (global coordinates) over the
        genome, only those starting in [lo, hi) (a shard's share)"""
        h, k = vp(), i64()
        hi = genome_space.span if hi is None else hi
        check(_lib().lime_complement_runs(self._h, genome_space.handle, int(n), vp(d_gs),
                                          vp(d_ge), int(lo), int(hi), C.byref(h), C.byref(k)))
        return Result(self, h, genome_space)

    def bitset(self, a):
        h = vp()
        check(_lib().lime_bitset_from_set(self._h, a._h, C.byref(h)))
        return Bitset(self, h, a.space)

    def bitset_from_device(self, space, n, d_contig, d_start, d_end):
        """bit-per-base set straight from UNSORTED device rows (binned paint)"""
        h = vp()
        check(_lib().lime_bitset_from_device(self._h, space.handle, int(n), vp(d_contig),
                                             vp(d_start), vp(d_end), C.byref(h)))
        return Bitset(self, h, space)

    def bitset_from_global(self, space, lo, hi, n, d_gs, d_ge):
        """a coordinate shard's bitset: global bits [lo, hi) from device rows in
        global coordinates (clipped to the window)"""
        h = vp()
        check(_lib().lime_bitset_from_global(self._h, space.handle, int(lo), int(hi), int(n),
                                             vp(d_gs), vp(d_ge), C.byref(h)))
        return Bitset(self, h, space)

    def bitset_and_from_device(self, space, rows):
        """the AND of k row sets' bits straight from their UNSORTED device rows
        (lime_bitset_and_from_device): rows = [(n, d_contig, d_start, d_end)]"""
        k = len(rows)
        ns = (i64 * k)(*[int(r[0]) for r in rows])
        cs, ss, es = ((vp * k)(*[vp(r[j]) for r in rows]) for j in (1, 2, 3))
        h = vp()
        check(_lib().lime_bitset_and_from_device(self._h, space.handle, k, ns, cs, ss, es,
                                                 C.byref(h)))
        return Bitset(self, h, space)

    def bitset_and_from_global(self, space, lo, hi, rows):
        """the same over a shard's window [lo, hi) from GLOBAL rows:
        rows = [(n, d_gs, d_ge)]"""
        k = len(rows)
        ns = (i64 * k)(*[int(r[0]) for r in rows])
        ss, es = ((vp * k)(*[vp(r[j]) for r in rows]) for j in (1, 2))
        h = vp()
        check(_lib().lime_bitset_and_from_global(self._h, space.handle, int(lo), int(hi), k, ns,
                                                 ss, es, C.byref(h)))
        return Bitset(self, h, space)

    def route_rows(self, space, n, d_contig, d_start, d_end, splits, clip=False, cap=-1,
                   d_gs=None, d_ge=None, d_row=None, row_base=0, d_strand=None,
                   d_strand_out=None):
        """Rows -> coordinate shards (lime_route_rows): returns the per-shard
        counts; when their total <= cap the rows are written, grouped by
        shard, to d_gs / d_ge (global) and d_row (row_base + input index),
        their strand codes (d_strand, per input row) to d_strand_out.
        d_contig None: d_start / d_end are already global."""
        k = len(splits) - 1
        sp = (C.c_uint32 * (k + 1))(*[int(x) for x in splits])
        counts = (i64 * k)()
        check(_lib().lime_route_rows(self._h, space.handle, int(n), vp(d_contig), vp(d_start),
                                     vp(d_end), int(row_base) & 0xFFFFFFFF, k, sp, int(bool(clip)),
                                     int(cap), vp(d_gs), vp(d_ge), vp(d_row), counts,
                                     vp(d_strand), vp(d_strand_out)))
        return list(counts)

    def route_rows_interleaved(self, space, n, d_contig, d_start, d_end, splits, k, d_rows,
                               clip=False, cap=-1, row_base=0):
        """lime_route_rows_interleaved: the per-shard counts; when their total
        <= cap the pieces are written to d_rows as k (2: gs, ge; 3: + row id)
        consecutive u32 words each, grouped by shard -- the all_to_all send
        buffer as it stands"""
        nsh = len(splits) - 1
        sp = (C.c_uint32 * (nsh + 1))(*[int(x) for x in splits])
        counts = (i64 * nsh)()
        check(_lib().lime_route_rows_interleaved(self._h, space.handle, int(n), vp(d_contig),
                                                 vp(d_start), vp(d_end),
                                                 int(row_base) & 0xFFFFFFFF, nsh, sp,
                                                 int(bool(clip)), int(cap), int(k), vp(d_rows),
                                                 counts))
        return list(counts)

    def deinterleave(self, n, k, d_src, d_dst0, d_dst1, d_dst2=None):
        """n interleaved rows of k u32 words -> k device columns (one pass,
        stream-ordered)"""
        check(_lib().lime_deinterleave_u32(self._h, int(n), int(k), vp(d_src), vp(d_dst0),
                                           vp(d_dst1), vp(d_dst2)))

    def bitset_runs(self, op, a, b=None):
        h, n = vp(), i64()
        check(_lib().lime_bitset_runs(self._h, int(op), a._h, b._h if b is not None else None,
                                      C.byref(h), C.byref(n)))
        return Result(self, h, a.space, keep=(a, b))

    def bitset_and(self, sets):
        arr = (vp * len(sets))(*[s._h for s in sets])
        h, n = vp(), i64()
        check(_lib().lime_bitset_and_runs(self._h, len(sets), arr, C.byref(h), C.byref(n)))
        return Result(self, h, sets[0].space)

    def pairs_checksum_device(self, d_pairs, count):
        """(sum, xor) of pair_hash over `count` 16-B records already stored in
        a device buffer (e.g. a chunk fill_device wrote)"""
        s, x = u64(), u64()
        check(_lib().lime_pairs_checksum_device(self._h, vp(d_pairs), int(count), C.byref(s),
                                                C.byref(x)))
        return s.value, x.value

    # ----------------------------------------------------------- synth
    def synth_uniform(self, space, n, seed, len_lo, len_hi, d_contig, d_start, d_end):
        check(_lib().lime_synth_uniform(self._h, space.handle, int(n), int(seed), int(len_lo),
                                        int(len_hi), d_contig, d_start, d_end))

    def synth_uniform_rows(self, space, first, n, seed, len_lo, len_hi, d_contig, d_start,
                           d_end):
        """rows [first, first + n) of lime_synth_uniform's sequence"""
        check(_lib().lime_synth_uniform_rows(self._h, space.handle, int(first), int(n), int(seed),
                                             int(len_lo), int(len_hi), d_contig, d_start, d_end))

    def synth_pileup_rows(self, space, first, n, seed, n_centres, sigma, len_lo, len_hi,
                          d_contig, d_start, d_end):
        """rows [first, first + n) of lime_synth_pileup's sequence"""
        check(_lib().lime_synth_pileup_rows(self._h, space.handle, int(first), int(n), int(seed),
                                            int(n_centres), int(sigma), int(len_lo), int(len_hi),
                                            d_contig, d_start, d_end))

    def synth_pileup(self, space, n, seed, n_centres, sigma, len_lo, len_hi, d_contig, d_start,
                     d_end):
        check(_lib().lime_synth_pileup(self._h, space.handle, int(n), int(seed), int(n_centres),
                                       int(sigma), int(len_lo), int(len_hi), d_contig, d_start,
                                       d_end))

    def close(self):
        if getattr(self, "_h", None):
            _lib().lime_ctx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class DeviceBed:
    """lime_dbed: BED records parsed on the device (ADAM loadBed replacement)."""

    def __init__(self, ctx, handle, text):
        self.ctx, self._h, self.text = ctx, handle, text

    @property
    def n(self):
        return int(_lib().lime_dbed_rows(self._h))

    @property
    def names(self):
        lib = _lib()
        return [lib.lime_dbed_contig_name(self._h, i).decode()
                for i in range(lib.lime_dbed_contigs(self._h))]

    def device_arrays(self):
        c, s, e, st = vp(), vp(), vp(), vp()
        check(_lib().lime_dbed_device_arrays(self._h, C.byref(c), C.byref(s), C.byref(e),
                                             C.byref(st)))
        return c.value, s.value, e.value, st.value

    def to_host(self):
        n = self.n
        out = {"contig": np.zeros(n, np.int32), "start": np.zeros(n, np.int64),
               "end": np.zeros(n, np.int64), "strand": np.zeros(n, np.int8),
               "name_off": np.zeros(n, np.int64), "name_len": np.zeros(n, np.int32)}
        check(_lib().lime_dbed_fill_host(self._h, _ptr(out["contig"], i32),
                                         _ptr(out["start"], i64), _ptr(out["end"], i64),
                                         _ptr(out["strand"], C.c_int8),
                                         _ptr(out["name_off"], i64), _ptr(out["name_len"], i32)))
        out["name"] = [self.text[o:o + k].decode() for o, k in zip(out["name_off"].tolist(),
                                                                   out["name_len"].tolist())]
        return out

    def to_set(self, space):
        """Remap contig ids to `space` on the device and build the sorted set
        from the device arrays (no host round trip of the records)."""
        ids = np.array([space.index[nm] for nm in self.names], dtype=np.int32)
        check(_lib().lime_dbed_remap_contigs(self._h, _ptr(ids, i32), len(ids)))
        c, s, e, _ = self.device_arrays()
        return self.ctx.set_from_device(space, self.n, c, s, e)

    def close(self):
        if self._h:
            _lib().lime_dbed_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def read_bed(path):
    """Parse a BED file with the engine's host reader -> dict of numpy arrays."""
    lib = _lib()
    h = vp()
    check(lib.lime_bed_read(path.encode(), C.byref(h)))
    try:
        n = lib.lime_bed_rows(h)
        nc = lib.lime_bed_contigs(h)
        names = [lib.lime_bed_contig_name(h, i).decode() for i in range(nc)]
        ids = np.ctypeslib.as_array(lib.lime_bed_contig_ids(h), shape=(n,)).copy() if n else \
            np.zeros(0, np.int32)
        s = np.ctypeslib.as_array(lib.lime_bed_starts(h), shape=(n,)).copy() if n else \
            np.zeros(0, np.int64)
        e = np.ctypeslib.as_array(lib.lime_bed_ends(h), shape=(n,)).copy() if n else \
            np.zeros(0, np.int64)
        st = np.ctypeslib.as_array(lib.lime_bed_strands(h), shape=(n,)).copy() if n else \
            np.zeros(0, np.int8)
        nm = [lib.lime_bed_name(h, i).decode() for i in range(n)]
    finally:
        lib.lime_bed_free(h)
    return {"names": names, "contig": ids, "chrom": [names[i] for i in ids], "start": s,
            "end": e, "strand": st, "name": nm}

"""ctypes wrapper of oracle/lime_oracle.c -- TEST INFRASTRUCTURE ONLY.

The C file restates LIME's per-partition algorithms line by line (see its
header for the file:line map into /root/reference).  Parity pin: the
reference's own golden vectors (IntersectionSuite, SubtractSuite,
MergeSuite, ComplementSuite), checked in tests/test_oracle.py.
This module is imported only by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg.
"""
import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(_HERE, "lime_oracle.c")
LIB = os.path.join(_HERE, "build", "liblime_oracle.so")

P = C.POINTER
i32, i64, i8 = C.c_int32, C.c_int64, C.c_int8
_lib = None

SUB_LIME, SUB_SET = 0, 1


def build():
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(SRC):
        subprocess.check_call(["gcc", "-O2", "-fPIC", "-shared", "-std=c99", "-pthread", "-o", LIB,
                               SRC])


def lib():
    global _lib
    if _lib is None:
        build()
        L = C.CDLL(LIB)
        pair_args = [i64, P(i32), P(i64), P(i64), P(i8), i64, P(i32), P(i64), P(i64), P(i8), i64]
        L.lo_intersect.restype = i64
        L.lo_intersect.argtypes = pair_args + [i64, P(i32), P(i64), P(i64), P(i64), P(i64)]
        L.lo_subtract.restype = i64
        L.lo_subtract.argtypes = pair_args + [C.c_int, i64, P(i32), P(i64), P(i64), P(i64),
                                              P(i64)]
        L.lo_window.restype = i64
        L.lo_window.argtypes = pair_args + [i64, P(i32), P(i64), P(i64), P(i64), P(i64)]
        L.lo_closest.restype = i64
        L.lo_closest.argtypes = pair_args[:-1] + [C.c_int, i64, P(i32), P(i64), P(i64),
                                                  P(i64), P(i64)]
        L.lo_merge.restype = i64
        L.lo_merge.argtypes = [i64, P(i32), P(i64), P(i64), P(i8), i64, P(i32), P(i64), P(i64),
                               P(i8), P(i64)]
        L.lo_complement.restype = i64
        L.lo_complement.argtypes = [i64, P(i32), P(i64), P(i64), i32, P(i64), i64, P(i32),
                                    P(i64), P(i64)]
        u32p, u64p = P(C.c_uint32), P(C.c_uint64)
        L.lo_intersect_mt.restype = i64
        L.lo_intersect_mt.argtypes = [i32, i64, P(i32), u32p, u32p, i64, P(i32), u32p, u32p, i64,
                                      C.c_int, i64, P(i32), P(i64), P(i64), P(i64), P(i64), u64p,
                                      u64p]
        L.lo_merge_mt.restype = i64
        L.lo_merge_mt.argtypes = [i32, i64, P(i32), u32p, u32p, C.c_int, i64, P(i32), P(i64),
                                  P(i64), P(i64), u64p, u64p]
        L.lo_subtract_mt.restype = i64
        L.lo_subtract_mt.argtypes = [i32, i64, P(i32), u32p, u32p, i64, P(i32), u32p, u32p, i64,
                                     C.c_int, C.c_int, u64p, u64p]
        L.lo_complement_mt.restype = i64
        L.lo_complement_mt.argtypes = [i32, P(i64), i64, P(i32), u32p, u32p, C.c_int, u64p, u64p]
        L.lo_pair_hash.restype = C.c_uint64
        L.lo_pair_hash.argtypes = [C.c_uint32] * 4
        _lib = L
    return _lib


def _p(a, t):
    return None if a is None else a.ctypes.data_as(P(t))


def _in(contig, start, end, strand=None):
    c = np.ascontiguousarray(contig, dtype=np.int32)
    s = np.ascontiguousarray(start, dtype=np.int64)
    e = np.ascontiguousarray(end, dtype=np.int64)
    st = None if strand is None else np.ascontiguousarray(strand, dtype=np.int8)
    return len(c), c, s, e, st


def _out(n):
    return (np.zeros(n, np.int32), np.zeros(n, np.int64), np.zeros(n, np.int64),
            np.zeros(n, np.int64), np.zeros(n, np.int64))


def _result(arrs):
    c, s, e, l, r = arrs
    return {"contig": c, "start": s, "end": e, "a_row": l, "b_row": r}


def intersect(a, b, threshold=0):
    """a, b: (contig, start, end[, strand]) arrays.  Returns dict of arrays in
    the reference's emission order (left sorted order, then cache order)."""
    L = lib()
    na, ac, as_, ae, ast = _in(*a)
    nb, bc, bs, be, bst = _in(*b)
    args = [na, _p(ac, i32), _p(as_, i64), _p(ae, i64), _p(ast, i8), nb, _p(bc, i32),
            _p(bs, i64), _p(be, i64), _p(bst, i8), int(threshold)]
    n = L.lo_intersect(*args, 0, None, None, None, None, None)
    o = _out(n)
    L.lo_intersect(*args, n, *[_p(x, t) for x, t in zip(o, (i32, i64, i64, i64, i64))])
    return _result(o)


def window(a, b, distance=1000):
    """Window.scala sweep restated (lo_window): pairs (a, b) with
    a.isNearby(b, distance); start / end are a's own region.  Reference
    emission order (left sorted order, then cache order)."""
    L = lib()
    na, ac, as_, ae, ast = _in(*a)
    nb, bc, bs, be, bst = _in(*b)
    args = [na, _p(ac, i32), _p(as_, i64), _p(ae, i64), _p(ast, i8), nb, _p(bc, i32),
            _p(bs, i64), _p(be, i64), _p(bst, i8), int(distance)]
    n = L.lo_window(*args, 0, None, None, None, None, None)
    o = _out(n)
    L.lo_window(*args, n, *[_p(x, t) for x, t in zip(o, (i32, i64, i64, i64, i64))])
    return _result(o)


CLOSEST, CLOSEST_SINGLE = 0, 1


def closest(a, b, mode=CLOSEST):
    """Closest.scala's SingleClosest (mode 0) / SingleClosestSingleOverlap
    (mode 1) over the sweep, restated (lo_closest): records carry a's own
    region; reference emission order."""
    L = lib()
    na, ac, as_, ae, ast = _in(*a)
    nb, bc, bs, be, bst = _in(*b)
    args = [na, _p(ac, i32), _p(as_, i64), _p(ae, i64), _p(ast, i8), nb, _p(bc, i32),
            _p(bs, i64), _p(be, i64), _p(bst, i8), int(mode)]
    n = L.lo_closest(*args, 0, None, None, None, None, None)
    o = _out(n)
    L.lo_closest(*args, n, *[_p(x, t) for x, t in zip(o, (i32, i64, i64, i64, i64))])
    return _result(o)


def subtract(a, b, threshold=0, mode=SUB_LIME):
    L = lib()
    na, ac, as_, ae, ast = _in(*a)
    nb, bc, bs, be, bst = _in(*b)
    args = [na, _p(ac, i32), _p(as_, i64), _p(ae, i64), _p(ast, i8), nb, _p(bc, i32),
            _p(bs, i64), _p(be, i64), _p(bst, i8), int(threshold), int(mode)]
    n = L.lo_subtract(*args, 0, None, None, None, None, None)
    o = _out(n)
    L.lo_subtract(*args, n, *[_p(x, t) for x, t in zip(o, (i32, i64, i64, i64, i64))])
    return _result(o)


def merge(a):
    L = lib()
    n, c, s, e, st = _in(*a)
    k = L.lo_merge(n, _p(c, i32), _p(s, i64), _p(e, i64), _p(st, i8), 0, None, None, None,
                   None, None)
    oc, os_, oe = np.zeros(k, np.int32), np.zeros(k, np.int64), np.zeros(k, np.int64)
    ost = np.zeros(k, np.int8)
    rid = np.zeros(n, np.int64)
    L.lo_merge(n, _p(c, i32), _p(s, i64), _p(e, i64), _p(st, i8), k, _p(oc, i32),
               _p(os_, i64), _p(oe, i64), _p(ost, i8), _p(rid, i64))
    return {"contig": oc, "start": os_, "end": oe, "strand": ost, "run_of_row": rid}


def complement(a, genome_lengths):
    L = lib()
    n, c, s, e, _ = _in(*a)
    g = np.ascontiguousarray(genome_lengths, dtype=np.int64)
    k = L.lo_complement(n, _p(c, i32), _p(s, i64), _p(e, i64), len(g), _p(g, i64), 0, None,
                        None, None)
    if k < 0:
        raise KeyError("contig not in genome")
    oc, os_, oe = np.zeros(k, np.int32), np.zeros(k, np.int64), np.zeros(k, np.int64)
    L.lo_complement(n, _p(c, i32), _p(s, i64), _p(e, i64), len(g), _p(g, i64), k, _p(oc, i32),
                    _p(os_, i64), _p(oe, i64))
    return {"contig": oc, "start": os_, "end": oe}


def pair_hash(start, end, a, b):
    return lib().lo_pair_hash(int(start), int(end), int(a), int(b))


def checksum_pairs(res):
    """Order-independent (sum, xor) of mix64 hashes of (start, end, a_row, b_row)."""
    from lime_amd.synth import mix64  # same finaliser as the C oracle
    s = np.asarray(res["start"], dtype=np.uint64)
    e = np.asarray(res["end"], dtype=np.uint64)
    a = np.asarray(res["a_row"], dtype=np.uint64)
    b = np.asarray(res["b_row"], dtype=np.uint64)
    x = (s << np.uint64(32)) | e
    y = (a << np.uint64(32)) | b
    h = mix64(x ^ mix64(y))
    with np.errstate(over="ignore"):
        tot = int(np.sum(h, dtype=np.uint64))
    xr = int(np.bitwise_xor.reduce(h)) if len(h) else 0
    return tot, xr


def threads():
    """Host threads for the contig-sharded drivers: OMP_NUM_THREADS (16 on the
    GPU box), at most os.cpu_count()."""
    return max(1, min(int(os.environ.get("OMP_NUM_THREADS", "16")), os.cpu_count() or 1, 64))


def _in32(contig, start, end):
    c = np.ascontiguousarray(contig, dtype=np.int32)
    s = np.ascontiguousarray(start, dtype=np.uint32)
    e = np.ascontiguousarray(end, dtype=np.uint32)
    return len(c), c, s, e


def intersect_mt(n_contigs, a, b, threshold=0, records=False, nthreads=None):
    """Contig-sharded intersect (lo_intersect_mt): the P = 1 result computed
    one contig per thread.  Returns {"n", "sum", "xor"} and, with
    records=True, the pair arrays in the reference's emission order."""
    L = lib()
    na, ac, as_, ae = _in32(*a)
    nb, bc, bs, be = _in32(*b)
    u32p = P(C.c_uint32)
    sm, xr = C.c_uint64(), C.c_uint64()
    args = [int(n_contigs), na, _p(ac, i32), as_.ctypes.data_as(u32p), ae.ctypes.data_as(u32p),
            nb, _p(bc, i32), bs.ctypes.data_as(u32p), be.ctypes.data_as(u32p), int(threshold),
            int(nthreads or threads())]
    n = L.lo_intersect_mt(*args, 0, None, None, None, None, None, C.byref(sm), C.byref(xr))
    if n < 0:
        raise KeyError("contig id outside [0, n_contigs)")
    out = {"n": int(n), "sum": sm.value, "xor": xr.value}
    if records:
        o = _out(n)
        L.lo_intersect_mt(*args, n, *[_p(x, t) for x, t in zip(o, (i32, i64, i64, i64, i64))],
                          C.byref(sm), C.byref(xr))
        out.update(_result(o))
    return out


def merge_mt(n_contigs, a, run_of_row=False, nthreads=None):
    """Contig-sharded merge (lo_merge_mt): runs in order plus the checksum of
    the run id of every input row ({"grp_sum", "grp_xor"})."""
    L = lib()
    n, c, s, e = _in32(*a)
    u32p = P(C.c_uint32)
    gs, gx = C.c_uint64(), C.c_uint64()
    rid = np.zeros(n, np.int64) if run_of_row else None
    args = [int(n_contigs), n, _p(c, i32), s.ctypes.data_as(u32p), e.ctypes.data_as(u32p),
            int(nthreads or threads())]
    # runs <= rows: size the buffers by the rows, one call
    oc, os_, oe = np.zeros(n, np.int32), np.zeros(n, np.int64), np.zeros(n, np.int64)
    k = L.lo_merge_mt(*args, n, _p(oc, i32), _p(os_, i64), _p(oe, i64), _p(rid, i64),
                      C.byref(gs), C.byref(gx))
    if k < 0:
        raise KeyError("contig id outside [0, n_contigs)")
    out = {"contig": oc[:k], "start": os_[:k], "end": oe[:k], "grp_sum": gs.value,
           "grp_xor": gx.value}
    if run_of_row:
        out["run_of_row"] = rid
    return out


def grouping_checksum(run_of_row):
    """sum / xor over rows r of mix64(r << 32 | run_of_row[r]) (lo_merge_mt's
    grouping checksum, restated in numpy for small cases)."""
    from lime_amd.synth import mix64
    r = np.arange(len(run_of_row), dtype=np.uint64)
    h = mix64((r << np.uint64(32)) | np.asarray(run_of_row, dtype=np.uint64))
    with np.errstate(over="ignore"):
        tot = int(np.sum(h, dtype=np.uint64))
    return tot, (int(np.bitwise_xor.reduce(h)) if len(h) else 0)


def subtract_mt(n_contigs, a, b, threshold=0, mode=SUB_LIME, nthreads=None):
    """Contig-sharded subtract (lo_subtract_mt): {"n", "sum", "xor"}, the
    checksum in lime_result_checksum's region form."""
    L = lib()
    na, ac, as_, ae = _in32(*a)
    nb, bc, bs, be = _in32(*b)
    u32p = P(C.c_uint32)
    sm, xr = C.c_uint64(), C.c_uint64()
    n = L.lo_subtract_mt(int(n_contigs), na, _p(ac, i32), as_.ctypes.data_as(u32p),
                         ae.ctypes.data_as(u32p), nb, _p(bc, i32), bs.ctypes.data_as(u32p),
                         be.ctypes.data_as(u32p), int(threshold), int(mode),
                         int(nthreads or threads()), C.byref(sm), C.byref(xr))
    if n < 0:
        raise KeyError("contig id outside [0, n_contigs)")
    return {"n": int(n), "sum": sm.value, "xor": xr.value}


def complement_mt(genome_lengths, a, nthreads=None):
    """Contig-sharded complement (lo_complement_mt): {"n", "sum", "xor"}, the
    checksum in lime_result_checksum's region form."""
    L = lib()
    g = np.ascontiguousarray(genome_lengths, dtype=np.int64)
    n, c, s, e = _in32(*a)
    u32p = P(C.c_uint32)
    sm, xr = C.c_uint64(), C.c_uint64()
    k = L.lo_complement_mt(len(g), _p(g, i64), n, _p(c, i32), s.ctypes.data_as(u32p),
                           e.ctypes.data_as(u32p), int(nthreads or threads()), C.byref(sm),
                           C.byref(xr))
    if k < 0:
        raise KeyError("contig not in genome")
    return {"n": int(k), "sum": sm.value, "xor": xr.value}


def result_checksum(res):
    """numpy restatement of lime_result_checksum's region part: sum / xor of
    mix64(pair_hash(start, end, a_row, b_row) + contig), absent rows
    (missing, or < 0) as 0xffffffff"""
    from lime_amd.synth import mix64
    n = len(res["start"])
    ff = np.full(n, 0xFFFFFFFF, np.uint64)

    def rows(k):
        r = res.get(k)
        if r is None:
            return ff
        r = np.asarray(r, np.int64)
        return np.where(r < 0, ff, r.astype(np.uint64))
    s = np.asarray(res["start"], np.uint64)
    e = np.asarray(res["end"], np.uint64)
    a, b = rows("a_row"), rows("b_row")
    with np.errstate(over="ignore"):
        h = mix64(mix64(((s << np.uint64(32)) | e) ^ mix64((a << np.uint64(32)) | b)) +
                  np.asarray(res["contig"], np.uint64))
        return int(np.sum(h, dtype=np.uint64)), (int(np.bitwise_xor.reduce(h)) if n else 0)

// intersect.hip -- DistributedIntersection as a two-stream merge-path join.
//
// Reference: SetTheory.scala:175-187 sweeps each sorted left row against a
// cache of right rows (advance/prune, OverlapBasedSetTheory.scala:21-38) and
// Intersection.scala:58-69 emits ([max s, min e), (L, R)) for every cached R
// with overlapsBy(L, R) >= threshold (strict half-open overlap).
//
// MI355X formulation.  A pair (a, b) overlaps strictly iff exactly one of
//   stream 0:  b.s in [a.s, a.e)        (b starts inside a, ties to a)
//   stream 1:  a.s in (b.s, b.e)        (a starts strictly inside b)
// holds, so every owner row's partners are a CONTIGUOUS range of the other
// sorted set, found by two lower_bounds:
//   lo = lb(P.gs, o.gs + lo_off)       lo_off = 0 (stream 0) / 1 (stream 1)
//   hi = lb(P.gs, o.ge - tp + 1)       tp = max(threshold, 1)
// With a threshold t >= 1 the range already encodes "overlap >= t" on the
// owner side; the partner must additionally have width >= t (a filter, only
// evaluated when the partner set actually holds rows narrower than t).  For
// t <= 0 the only false candidates are zero-width b at exactly a.s, which the
// canonical order puts first in the range, so lo just skips them.
//
// Work is decomposed by OUTPUT, not by input: per-owner counts are scanned
// into per-tile offsets and every fill workgroup writes exactly S consecutive
// output records, so pile-ups cannot unbalance the grid.  Output records are
// 16 B (start, end, a_row, b_row), written with 16-B non-temporal stores,
// fully coalesced (lane i writes record base + i).
//
// Kernels:
//   k_windows   one wave per owner tile (1024 owners): partner window
//   k_count     lo / count per owner (LDS-staged window), tile totals
//   scan (u64)  tile offsets
//   k_fill      S-record blocks: owner = load-balanced search, partner = lo + rank
//   k_fill_filtered  thread-per-owner fallback when a width filter applies
#include "common.hpp"

namespace lime {

struct PairsPlan {
    lime_ctx *ctx;
    const lime_set *A, *B;
    int64_t threshold;
    int64_t tp;
    bool filtered;
    int64_t a_own, b_own;  // owner rows (prefix) of A and B
    int64_t nt0, nt1;  // owner tiles of stream 0 (owners A) and 1 (owners B)
    uint32_t *olo = nullptr, *ocnt = nullptr;  // per owner, stream 0 then stream 1
    uint64_t *toff = nullptr;                  // per tile exclusive offsets
    uint32_t *win = nullptr;                   // per tile partner window [lo, hi)
    uint32_t *tseg = nullptr;                  // per tile contig offset (0xffffffff: mixed)
    int64_t total = 0;
    int tpf = 1;  // owner tiles per fill commit (k_fill<TPF>)
    // window plans (DistributedWindow): A is the widened set W, A_out the
    // caller's set whose own coordinates the pairs carry; reach = distance
    const lime_set *A_out = nullptr;
    lime_set *W = nullptr;  // owned: widened copy of A_out (row array borrowed)
    int64_t reach = -1;
};

void intersect_free(PairsPlan *pl);

namespace {

constexpr int IB = 256;
constexpr int OPT = 4;               // owners per thread
constexpr int OT = IB * OPT;         // owners per tile
constexpr int WCAP = 4096;           // LDS window capacity (partner starts)
constexpr int64_t SBLK = 131072;     // output records per fill workgroup

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

struct StreamArgs {
    const uint32_t *ogs, *oge, *orow;  // owner set (search keys)
    const uint32_t *pgs, *pge, *prow;  // partner set (search keys)
    // the coordinates the output records are made of: the same arrays for
    // intersect; the caller's unwidened rows for the window set's side
    const uint32_t *ogs_o, *oge_o, *pgs_o, *pge_o;
    int64_t no, np;
    uint32_t lo_off;  // 0 or 1
    int zw_skip;      // skip zero-width partners at exactly o.gs
    int64_t reach;    // window distance on the owner side (stream 0), else -1
    int64_t tile0;    // first global tile index of this stream
    int64_t owner0;   // first global owner slot of this stream (olo/ocnt)
};

__device__ __forceinline__ void owner_keys(uint32_t og, uint32_t oe, uint32_t lo_off, int64_t tp,
                                           int64_t &lo_key, int64_t &hi_key) {
    lo_key = (int64_t)og + lo_off;
    hi_key = (int64_t)oe - tp + 1;
}

using dev::wave_lower_bound;

__device__ __forceinline__ uint32_t contig_off(const uint32_t *__restrict__ off, int32_t nc,
                                               uint32_t g) {
    // largest c with off[c] <= g
    int64_t c = dev::upper_bound(off, 0, (int64_t)nc, g) - 1;
    return off[c < 0 ? 0 : c];
}

// Two independent lower_bounds by one wave, their probes interleaved so
// both searches share the same 5-6 memory round trips.
__device__ __forceinline__ void wave_lower_bound2(const uint32_t *__restrict__ a, int64_t n,
                                                  int64_t key0, int64_t key1, int64_t &r0,
                                                  int64_t &r1) {
    int64_t lo0 = 0, hi0 = n, lo1 = 0, hi1 = n;
    const int lane = dev::lane_id();
    while (hi0 - lo0 > 64 || hi1 - lo1 > 64) {
        const int64_t st0 = (hi0 - lo0 + 64) / 65, st1 = (hi1 - lo1 + 64) / 65;
        const int64_t i0 = lo0 + st0 * (lane + 1) - 1, i1 = lo1 + st1 * (lane + 1) - 1;
        const bool a0 = hi0 - lo0 > 64 && i0 < hi0;
        const bool a1 = hi1 - lo1 > 64 && i1 < hi1;
        const uint32_t v0 = a0 ? a[i0] : 0u, v1 = a1 ? a[i1] : 0u;
        if (hi0 - lo0 > 64) {
            const int c = __popcll(__ballot(a0 && (int64_t)v0 < key0));
            const int64_t nlo = c == 0 ? lo0 : lo0 + st0 * c;
            hi0 = c == 64 ? hi0 : min(hi0, lo0 + st0 * (c + 1) - 1);
            lo0 = nlo;
        }
        if (hi1 - lo1 > 64) {
            const int c = __popcll(__ballot(a1 && (int64_t)v1 < key1));
            const int64_t nlo = c == 0 ? lo1 : lo1 + st1 * c;
            hi1 = c == 64 ? hi1 : min(hi1, lo1 + st1 * (c + 1) - 1);
            lo1 = nlo;
        }
    }
    const int64_t j0 = lo0 + lane, j1 = lo1 + lane;
    const bool b0 = j0 < hi0, b1 = j1 < hi1;
    const uint32_t v0 = b0 ? a[j0] : 0u, v1 = b1 ? a[j1] : 0u;
    r0 = lo0 + __popcll(__ballot(b0 && (int64_t)v0 < key0));
    r1 = lo1 + __popcll(__ballot(b1 && (int64_t)v1 < key1));
}

// Per owner tile: partner window [lo, hi) and, when tseg is given, the
// tile's contig offset (0xffffffff when its owners span several contigs).
__global__ __launch_bounds__(IB) void k_windows(StreamArgs sa, int64_t tp, int64_t ntiles,
                                                uint32_t *__restrict__ win,
                                                const uint32_t *__restrict__ off, int32_t nc,
                                                uint32_t *__restrict__ tseg) {
    const int64_t t = (int64_t)blockIdx.x * (IB / 64) + threadIdx.x / 64;
    if (t >= ntiles) return;
    const int lane = dev::lane_id();
    const int64_t o0 = t * OT;
    const int64_t o1 = min(o0 + OT, sa.no);
    int64_t hmax = INT64_MIN;
    for (int64_t j = o0 + lane; j < o1; j += 64) hmax = max(hmax, (int64_t)sa.oge[j] - tp + 1);
    hmax = dev::wave_reduce_max(hmax);
    const int64_t lkey = (int64_t)sa.ogs[o0] + sa.lo_off;
    // every owner's lo = lb(P, o.gs + lo_off) must lie inside the window too
    // (subtract walks back from it even when the owner's range is empty)
    const int64_t lkey_last = (int64_t)sa.ogs[o1 - 1] + sa.lo_off;
    if (hmax < lkey_last) hmax = lkey_last;
    int64_t lo, hi;
    wave_lower_bound2(sa.pgs, sa.np, lkey, hmax, lo, hi);
    if (lane == 0) {
        win[2 * (sa.tile0 + t)] = (uint32_t)lo;
        win[2 * (sa.tile0 + t) + 1] = (uint32_t)hi;
    }
    if (tseg) {
        // contig offsets of the tile's first and last owner: one ballot over
        // off[] for up to 64 contigs, a binary search otherwise
        const uint32_t g0 = sa.ogs_o[o0], g1 = sa.ogs_o[o1 - 1];
        uint32_t a, b;
        if (nc <= 64) {
            const uint32_t v = lane < nc ? off[lane] : 0xffffffffu;
            const int c0 = __popcll(__ballot(lane < nc && v <= g0)) - 1;
            const int c1 = __popcll(__ballot(lane < nc && v <= g1)) - 1;
            a = off[c0 < 0 ? 0 : c0];
            b = off[c1 < 0 ? 0 : c1];
        } else {
            a = contig_off(off, nc, g0);
            b = contig_off(off, nc, g1);
        }
        if (lane == 0) tseg[sa.tile0 + t] = a == b ? a : 0xffffffffu;
    }
}

// k_windows with one LANE per owner tile, for owner sets whose widths are
// bounded by owmax (the common case): every owner's hi key o.ge - tp + 1 is at
// most last.gs + owmax - tp + 1, so the window needs the tile's first and last
// starts only, not a read of all its ends; its two lower bounds are
// branch-free binary searches (a fixed trip count, every lane in lockstep).
// A wave per tile searched 65-ary: 5-6 round trips, but 64 lanes' lines per
// level -- 0.86 GB fetched per 1e8 owners for 0.4 GB of owner ends.
__global__ __launch_bounds__(256) void k_windows_lane(StreamArgs sa, int64_t tp, int64_t ntiles,
                                                      int64_t owmax, uint32_t *__restrict__ win,
                                                      const uint32_t *__restrict__ off, int32_t nc,
                                                      uint32_t *__restrict__ tseg) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= ntiles) return;
    const int64_t o0 = t * OT;
    const int64_t o1 = min(o0 + OT, sa.no);
    const uint32_t g0 = sa.ogs[o0], g1 = sa.ogs[o1 - 1];
    const int64_t lkey = (int64_t)g0 + sa.lo_off;
    int64_t hkey = (int64_t)g1 + owmax - tp + 1;
    const int64_t lkey_last = (int64_t)g1 + sa.lo_off;  // (as k_windows)
    if (hkey < lkey_last) hkey = lkey_last;
    // the two searches interleaved: their loads overlap
    int64_t bl = 0, bh = 0;
    const int64_t n = sa.np;
    for (int64_t step = n > 0 ? (int64_t)1 << (63 - __builtin_clzll((uint64_t)n)) : 0; step > 0;
         step >>= 1) {
        const uint32_t vl = bl + step <= n ? sa.pgs[bl + step - 1] : 0xffffffffu;
        const uint32_t vh = bh + step <= n ? sa.pgs[bh + step - 1] : 0xffffffffu;
        if (bl + step <= n && (int64_t)vl < lkey) bl += step;
        if (bh + step <= n && (int64_t)vh < hkey) bh += step;
    }
    win[2 * (sa.tile0 + t)] = (uint32_t)bl;
    win[2 * (sa.tile0 + t) + 1] = (uint32_t)bh;
    if (tseg) {
        const uint32_t a = contig_off(off, nc, sa.ogs_o[o0]), b = contig_off(off, nc, sa.ogs_o[o1 - 1]);
        tseg[sa.tile0 + t] = a == b ? a : 0xffffffffu;
    }
}

// Per owner: lo and either its count (OFFS = false) or its exclusive output
// offset within the tile (OFFS = true, what the fill stages: no scan left in
// the fill's per-tile critical path).  Thread t handles the OPT consecutive
// owners 4t .. 4t+3 of the tile, so one block scan orders them.
template <bool FILTER, bool OFFS>
__global__ __launch_bounds__(IB) void k_count(StreamArgs sa, int64_t tp, int64_t threshold,
                                              const uint32_t *__restrict__ win,
                                              uint32_t *__restrict__ olo,
                                              uint32_t *__restrict__ ocnt,
                                              uint64_t *__restrict__ tcnt,
                                              uint32_t *__restrict__ oflow) {
    __shared__ uint32_t wgs[WCAP];
    __shared__ uint64_t red[IB / 64];
    __shared__ uint32_t scratch[IB / 64 + 1];
    const int64_t t = blockIdx.x;
    const int64_t o0 = t * OT;
    const int64_t o1 = min(o0 + OT, sa.no);
    // the window's partner starts first, every load unconditional (lanes
    // past the window re-read its last start, one line): issued together,
    // one round trip, where a bounds-tested loop waited per iteration
    const uint32_t wlo = win[2 * (sa.tile0 + t)], whi = win[2 * (sa.tile0 + t) + 1];
    const int64_t wlen = (int64_t)whi - wlo;
    const bool in_lds = wlen <= WCAP;
    constexpr int WPT = WCAP / IB;
    uint32_t wv[WPT];
    if (in_lds && wlen > 0) {  // (uniform)
#pragma unroll
        for (int k = 0; k < WPT; ++k)
            wv[k] = sa.pgs[wlo + min((int64_t)(k * IB + threadIdx.x), wlen - 1)];
    }
    // owner loads: independent of the window, in flight with it
    uint32_t ogv[OPT], oev[OPT];
    static_assert(OPT == 4, "owner loads are one 16-B vector per thread");
    if (o1 - o0 == OT) {  // full tile: lane-consecutive 16-B loads (sets are 16-B aligned)
        const uint4 g4 = reinterpret_cast<const uint4 *>(sa.ogs + o0)[threadIdx.x];
        const uint4 e4 = reinterpret_cast<const uint4 *>(sa.oge + o0)[threadIdx.x];
        ogv[0] = g4.x, ogv[1] = g4.y, ogv[2] = g4.z, ogv[3] = g4.w;
        oev[0] = e4.x, oev[1] = e4.y, oev[2] = e4.z, oev[3] = e4.w;
    } else {
#pragma unroll
        for (int k = 0; k < OPT; ++k) {
            const int64_t j = o0 + threadIdx.x * OPT + k;
            ogv[k] = j < o1 ? sa.ogs[j] : 0u;
            oev[k] = j < o1 ? sa.oge[j] : 0u;
        }
    }
    if (in_lds && wlen > 0) {
#pragma unroll
        for (int k = 0; k < WPT; ++k)
            if (k * IB + (int)threadIdx.x < wlen) wgs[k * IB + threadIdx.x] = wv[k];
    }
    __syncthreads();
    // lo = lb(P, o.gs + lo_off) always (subtract's spanning walk starts
    // below it); hi = lb(P, o.ge - tp + 1), the range [lo, hi) being empty
    // when hk <= lk.  In the LDS window all 2 * OPT searches of a thread run
    // in lockstep (branchless binary lifting, fixed trip count), so their
    // LDS reads overlap instead of forming one 2 * OPT * log2(wlen) chain.
    int64_t lkv[OPT], hkv[OPT], lov[OPT], hiv[OPT];
#pragma unroll
    for (int k = 0; k < OPT; ++k) owner_keys(ogv[k], oev[k], sa.lo_off, tp, lkv[k], hkv[k]);
    if (in_lds) {
        int64_t key[2 * OPT];
        int b[2 * OPT];
#pragma unroll
        for (int k = 0; k < OPT; ++k) {
            key[k] = lkv[k];
            key[OPT + k] = hkv[k];
        }
        dev::lds_lower_bounds(wgs, (int)wlen, key, b);
#pragma unroll
        for (int k = 0; k < OPT; ++k) {
            lov[k] = wlo + b[k];
            hiv[k] = hkv[k] > lkv[k] ? wlo + b[OPT + k] : lov[k];
        }
    } else {
#pragma unroll
        for (int k = 0; k < OPT; ++k) {
            lov[k] = dev::lower_bound(sa.pgs, (int64_t)wlo, (int64_t)whi, lkv[k]);
            hiv[k] = hkv[k] > lkv[k] ? dev::lower_bound(sa.pgs, lov[k], (int64_t)whi, hkv[k])
                                     : lov[k];
        }
    }
    uint32_t cv[OPT];
    uint64_t csum = 0;  // 4 owners can exceed 2^32 candidates (deep pile-ups)
#pragma unroll
    for (int k = 0; k < OPT; ++k) {
        const int64_t j = o0 + threadIdx.x * OPT + k;
        cv[k] = 0;
        if (j >= o1) continue;
        const uint32_t og = ogv[k];
        int64_t lo = lov[k], hi = hiv[k];
        // a window row clipped at global 0 (contig 0, a.s < reach) is
        // nearby a zero-width partner at 0 (distance a.s + 1 <= reach)
        const bool keep0 = sa.reach > 0 && og == 0 && (int64_t)sa.ogs_o[j] < sa.reach;
        if (sa.zw_skip && !keep0) {
            while (lo < whi && sa.pgs[lo] == og && sa.pge[lo] == og) ++lo;
            if (hi < lo) hi = lo;
        }
        if (FILTER) {
            uint32_t c = 0;
            for (int64_t p = lo; p < hi; ++p) c += (int64_t)(sa.pge[p] - sa.pgs[p]) >= threshold;
            cv[k] = c;
        } else {
            cv[k] = (uint32_t)(hi - lo);
        }
        lov[k] = lo;
        csum += cv[k];
    }
    // tile-local offsets are u32 (the fill stages them as such): a tile with
    // 2^32 or more pairs is flagged below and the plan fails with
    // LIME_ERR_OVERFLOW instead of wrapping
    uint32_t run = 0;
    if (OFFS) {
        uint32_t tot;
        run = dev::block_exclusive_sum<IB>((uint32_t)csum, scratch, &tot);
    }
    // blocked -> lane-consecutive through LDS (the window image is dead
    // now), so the olo / ocnt stores are coalesced whatever owner0's alignment
    __syncthreads();
    uint32_t *slo = wgs, *sct = wgs + OT;
#pragma unroll
    for (int k = 0; k < OPT; ++k) {
        slo[threadIdx.x * OPT + k] = (uint32_t)lov[k];
        sct[threadIdx.x * OPT + k] = OFFS ? run : cv[k];
        run += cv[k];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < OPT; ++k) {
        const int q = k * IB + threadIdx.x;
        if (o0 + q < o1) {
            olo[sa.owner0 + o0 + q] = slo[q];
            ocnt[sa.owner0 + o0 + q] = sct[q];
        }
    }
    uint64_t sum = csum;
    sum = dev::wave_reduce_sum(sum);
    if (dev::lane_id() == 0) red[threadIdx.x / 64] = sum;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t s = 0;
        for (int i = 0; i < IB / 64; ++i) s += red[i];
        tcnt[sa.tile0 + t] = s;
        // bit 0: a tile's u32 offsets would wrap; bit 1: two adjacent tiles'
        // might (the fill then keeps one tile per commit, see k_fill)
        if (s > 0xffffffffull && oflow)
            atomicOr(oflow, 1u);
        else if (s > 0x7fffffffull && oflow)
            atomicOr(oflow, 2u);
    }
}


struct FillArgs {
    StreamArgs s[2];
    const uint32_t *olo, *ocnt;
    const uint64_t *toff;
    const uint32_t *win;   // per tile partner window [lo, hi)
    const uint32_t *tseg;  // per tile contig offset, 0xffffffff if mixed
    int64_t ntiles;
    int64_t total;         // pairs of the plan
    const uint32_t *off;
    int32_t n_contigs;
    int64_t first, count;  // output window [first, first + count)
    u32x4 *out;            // out[0] is record `first`
    uint64_t *cksum;       // [sum, xor] when checksumming instead of writing
};

constexpr int FB = 512;           // fill workgroup: 8 waves
constexpr int FW = FB / 64;
#ifndef LIME_FILL_WGS
#define LIME_FILL_WGS 2  // fill workgroups per CU (LDS budget below)
#endif
// LDS partner window (16 B records): 1792 rows keep 3 workgroups per CU
constexpr int PCAP = LIME_FILL_WGS >= 3 ? 1792 : 2048;
// Two-tile commits (sparse plans) keep the window as three u32 arrays so
// that 2048 owners + 2496 partners still fit two workgroups per CU
constexpr int PCAP2 = 2496;
#ifndef LIME_FILL_SPARSE
// mean pairs per owner below which a plan fills two owner tiles per commit
#define LIME_FILL_SPARSE 16
#endif
constexpr int64_t GR = 1ll << 40;  // wave granule: default one equal chunk per wave

template <int TPF> struct FillShape {
    static constexpr int OTF = OT * TPF;                     // owners per commit
    static constexpr int FOPT = OTF / FB;                    // owners per thread when staging
    static constexpr int CAP = TPF == 1 ? PCAP : PCAP2;      // LDS partner window rows
    static constexpr int PPT = (CAP + FB - 1) / FB;          // partner rows per thread
};

// The LDS partner window: 16-B records (one b128 read per output) for
// one-tile commits, three u32 arrays for two-tile commits.
template <int TPF> struct ParWin {
    u32x4 v[PCAP];
    __device__ __forceinline__ void put(int i, uint32_t g, uint32_t e, uint32_t r) {
        v[i] = u32x4{g, e, r, 0u};
    }
    __device__ __forceinline__ u32x4 get(uint32_t i) const { return v[i]; }
};
template <> struct ParWin<2> {
    uint32_t g[PCAP2], e[PCAP2], r[PCAP2];
    __device__ __forceinline__ void put(int i, uint32_t pg, uint32_t pe, uint32_t pr) {
        g[i] = pg;
        e[i] = pe;
        r[i] = pr;
    }
    __device__ __forceinline__ u32x4 get(uint32_t i) const { return u32x4{g[i], e[i], r[i], 0u}; }
};

// 65-ary wave search on the u64 tile offsets: largest t with toff[t] <= key
__device__ __forceinline__ int64_t wave_tile_of(const uint64_t *__restrict__ a, int64_t n,
                                                uint64_t key) {
    int64_t lo = 0, hi = n;  // first index with a[i] > key lies in [lo, hi]
    const int lane = dev::lane_id();
    while (hi - lo > 64) {
        const int64_t step = (hi - lo + 64) / 65;
        const int64_t idx = lo + step * (lane + 1) - 1;
        const bool le = idx < hi && a[idx] <= key;
        const int c = __popcll(__ballot(le));
        const int64_t nlo = c == 0 ? lo : lo + step * c;
        const int64_t nhi = c == 64 ? hi : min(hi, lo + step * (c + 1) - 1);
        lo = nlo;
        hi = nhi;
    }
    const int64_t idx = lo + lane;
    const bool le = idx < hi && a[idx] <= key;
    return lo + __popcll(__ballot(le)) - 1;
}

// Everything a fill workgroup stages for one commit (TPF consecutive owner
// tiles of one stream), held in registers so that the NEXT commit's loads
// are in flight while the current one's records are being stored (the
// staging latency is hidden behind the store stream instead of stalling it
// once per tile).
template <int TPF> struct TileRegs {
    static constexpr int FO = FillShape<TPF>::FOPT, PP = FillShape<TPF>::PPT;
    uint32_t off[FO], lo[FO], og[FO], oe[FO], orw[FO];
    uint32_t pg[PP], pe[PP], pr[PP];
    uint32_t wlo, whi, seg;
    uint64_t tnext;  // toff[t1] (or the plan total): the commit's end
    int64_t t1;      // one past the commit's last owner tile
};

__device__ __forceinline__ int64_t stream0_tiles(const FillArgs &fa) {
    return fa.s[0].tile0 + (fa.s[0].no + OT - 1) / OT;
}

__device__ __forceinline__ int tile_stream(const FillArgs &fa, int64_t t) {
    return t < stream0_tiles(fa) ? 0 : 1;
}

template <int TPF>
__device__ __forceinline__ void tile_load(const FillArgs &fa, int64_t t, TileRegs<TPF> &r,
                                          const uint64_t *toff, const uint32_t *win,
                                          const uint32_t *tseg) {
    constexpr int FO = FillShape<TPF>::FOPT, PP = FillShape<TPF>::PPT;
    // (t is wave-uniform: the stream's arguments are selected, not indexed,
    // so they stay scalar kernel-argument loads -- an indexed fa.s[st] was
    // read by vector loads whose waits drained the store stream)
    const int st = tile_stream(fa, t);
    const StreamArgs sa = st ? fa.s[1] : fa.s[0];
    // a commit never spans the two streams
    const int64_t t1 = min(t + TPF, st == 0 ? stream0_tiles(fa) : fa.ntiles);
    const int64_t o0 = (t - sa.tile0) * OT;
    const int nown = (int)min((int64_t)FillShape<TPF>::OTF, sa.no - o0);
    // k_count's offsets are local to each owner tile: a thread's owners all
    // lie in tile t + u, whose offset within the commit is toff[t+u] - toff[t]
    uint32_t add = 0;
    if (TPF > 1) {
        const int u = __builtin_amdgcn_readfirstlane((int)(threadIdx.x / (FB / TPF)));
        if (u > 0 && t + u < t1) add = (uint32_t)(toff[t + u] - toff[t]);
    }
#pragma unroll
    for (int k = 0; k < FO; ++k) {
        const int q = threadIdx.x * FO + k;
        const bool v = q < nown;
        const int64_t j = o0 + q;
        r.off[k] = v ? fa.ocnt[sa.owner0 + j] + add : 0u;  // tile-local offsets (k_count<_, true>)
        r.lo[k] = v ? fa.olo[sa.owner0 + j] : 0u;
        r.og[k] = v ? sa.ogs_o[j] : 0u;
        r.oe[k] = v ? sa.oge_o[j] : 0u;
        r.orw[k] = v ? sa.orow[j] : 0u;
    }
    r.wlo = win[2 * t];
    r.whi = win[2 * t + 1];
    r.seg = tseg[t];
    if (TPF > 1 && t1 - 1 > t) {
        // the union of the tiles' windows (each window is an interval)
        r.wlo = min(r.wlo, win[2 * (t1 - 1)]);
        r.whi = max(r.whi, win[2 * (t1 - 1) + 1]);
        if (tseg[t1 - 1] != r.seg) r.seg = 0xffffffffu;
    }
    r.t1 = t1;
    r.tnext = t1 < fa.ntiles ? toff[t1] : (uint64_t)fa.total;
    const int wl = (int)min((int64_t)(r.whi - r.wlo), (int64_t)FillShape<TPF>::CAP);
#pragma unroll
    for (int k = 0; k < PP; ++k) {
        const int i = k * FB + threadIdx.x;
        const bool v = i < wl;
        r.pg[k] = v ? sa.pgs_o[r.wlo + i] : 0u;
        r.pe[k] = v ? sa.pge_o[r.wlo + i] : 0u;
        r.pr[k] = v ? sa.prow[r.wlo + i] : 0u;
    }
}

// Largest q in [lo, hi) with off[q].y <= key (off[lo].y <= key holds); the
// .y are non-decreasing.  One wave, wave-uniform result.
__device__ __forceinline__ int wave_owner_of(const uint2 *off, int lo, int hi, uint32_t key) {
    const int lane = dev::lane_id();
    while (hi - lo > 64) {
        const int step = (hi - lo + 64) / 65;
        const int idx = lo + step * (lane + 1) - 1;
        const bool le = idx < hi && off[idx].y <= key;
        const int c = __popcll(__ballot(le));
        const int nlo = c == 0 ? lo : lo + step * c;
        hi = c == 64 ? hi : min(hi, lo + step * (c + 1) - 1);
        lo = nlo;
    }
    const int idx = lo + lane;
    const bool le = idx < hi && off[idx].y <= key;
    return lo + __popcll(__ballot(le)) - 1;
}

// Emit outputs o, o + 64, ... < gend of one wave (lane-consecutive records).
// The LDS-window form has no global loads in its loop, so the compiler
// never makes an iteration wait (vmcnt) for the previous iteration's store:
// each wave keeps its stores in flight.  The owner walk carries the current
// (lo, off) pair and the next owner's pair in registers, leaving two
// dependent LDS steps per iteration (walk, then owner + partner reads).
template <bool LDSP, bool CKSUM, bool WIN, int TPF>
__device__ __forceinline__ void emit(const FillArgs &fa, const StreamArgs &sa, int st,
                                     const uint2 *s_lo_off, const u32x4 *s_own,
                                     const ParWin<TPF> &s_par, uint32_t wlo, int64_t tbase,
                                     int64_t o, int64_t gend, int &q, uint64_t &hsum,
                                     uint64_t &hxor) {
    uint2 lof = s_lo_off[q], nxt = s_lo_off[q + 1];
    u32x4 *out = fa.out + (tbase - fa.first);
    for (; o < gend; o += 64) {
        const uint32_t ou = (uint32_t)o;
        while (nxt.y <= ou) {
            ++q;
            lof = nxt;
            nxt = s_lo_off[q + 1];
        }
        const uint32_t p = lof.x + (ou - lof.y);
        const u32x4 ow = s_own[q];
        u32x4 pa;
        if (LDSP)
            pa = s_par.get(p - wlo);
        else
            pa = u32x4{sa.pgs_o[p], sa.pge_o[p], sa.prow[p], 0u};
        // intersect: the intersection; window: the left (a) row's own region
        const uint32_t rs =
            (WIN ? (st == 0 ? ow.x : pa.x) : (ow.x > pa.x ? ow.x : pa.x)) - ow.w;
        const uint32_t re =
            (WIN ? (st == 0 ? ow.y : pa.y) : (ow.y < pa.y ? ow.y : pa.y)) - ow.w;
        const uint32_t ar = st == 0 ? ow.z : pa.z;
        const uint32_t br = st == 0 ? pa.z : ow.z;
        if (CKSUM) {
            const uint64_t h = dev::pair_hash(rs, re, ar, br);
            hsum += h;
            hxor ^= h;
        } else {
            out[o] = u32x4{rs, re, ar, br};
        }
    }
}

// Sparse plans (a few pairs per owner): the 64 outputs of a wave iteration
// span ~16 owners, a walk of ~16 dependent LDS steps per lane.  Here the
// wave resolves them at once: each owner starting inside the window marks
// its output slot with an LDS max of its index (the last of owners with no
// pairs, sharing a slot, wins), and a DPP prefix max over the 64 slots gives
// every lane its owner: three LDS operations and no dependent search (a
// 7-step shuffle search over the owners' offsets took the 1e9-row fill 23.7
// ms, the slots 20.8: DESIGN.md section 9).  wslot: the wave's 64 LDS words.
template <bool LDSP, bool CKSUM, bool WIN, int TPF>
__device__ __forceinline__ void emit_sparse(const FillArgs &fa, const StreamArgs &sa, int st,
                                            const uint2 *s_lo_off, const u32x4 *s_own,
                                            const ParWin<TPF> &s_par, uint32_t wlo, int64_t tbase,
                                            int64_t gb, int64_t gend, int qa, int qmax,
                                            uint32_t *wslot, uint64_t &hsum, uint64_t &hxor) {
    const uint32_t lane = dev::lane_id();
    u32x4 *out = fa.out + (tbase - fa.first);
    for (int64_t ob = gb; ob < gend; ob += 64) {  // (uniform)
        const uint32_t o0 = (uint32_t)ob;
        int adv = 0;
        wslot[lane] = 0u;
        for (int qb = qa + 1;; qb += 64) {  // (uniform; one round unless > 64 owners)
            const int qj = qb + (int)lane;
            // > 0: owners past qa start after o0
            const uint32_t rel = qj <= qmax ? s_lo_off[qj].y - o0 : 0xffffffffu;
            if (rel < 64u) atomicMax(&wslot[rel], (uint32_t)qj + 1u);
            const uint64_t m = __ballot(rel <= 64u);
            adv += __popcll(m);  // owners starting by o0 + 64: the next iteration's qa
            if (m != ~0ull) break;
        }
        const uint32_t mx = dev::wave_inclusive_max(wslot[lane]);
        const int cnt = mx ? (int)mx - 1 - qa : 0;
        const int64_t o = ob + lane;
        if (o < gend) {
            const int q = qa + cnt;
            const uint2 lof = s_lo_off[q];
            const uint32_t ou = (uint32_t)o;
            const uint32_t p = lof.x + (ou - lof.y);
            const u32x4 ow = s_own[q];
            u32x4 pa;
            if (LDSP)
                pa = s_par.get(p - wlo);
            else
                pa = u32x4{sa.pgs_o[p], sa.pge_o[p], sa.prow[p], 0u};
            const uint32_t rs =
                (WIN ? (st == 0 ? ow.x : pa.x) : (ow.x > pa.x ? ow.x : pa.x)) - ow.w;
            const uint32_t re =
                (WIN ? (st == 0 ? ow.y : pa.y) : (ow.y < pa.y ? ow.y : pa.y)) - ow.w;
            const uint32_t ar = st == 0 ? ow.z : pa.z;
            const uint32_t br = st == 0 ? pa.z : ow.z;
            if (CKSUM) {
                const uint64_t h = dev::pair_hash(rs, re, ar, br);
                hsum += h;
                hxor ^= h;
            } else {
                out[o] = u32x4{rs, re, ar, br};
            }
        }
        qa += adv;
    }
}

// One workgroup writes the `per` consecutive output records of its slice of
// the output index space [first, first + count).  Per commit (TPF owner
// tiles of one stream) it stages, in LDS,
//   s_lo_off[q] = (lo_q, off_q)   partner range start, exclusive output offset
//   s_own[q]    = (gs, ge, row, contig offset) of the owner
//   s_par[i]    = (gs, ge, row) of partner wlo + i   (the commit's window)
// then deals its output range to the waves in GR-record granules; lane l of
// a wave handles outputs g + l + 64 k of a granule g, so an owner switch
// happens about once per 82/64 iterations (C2) and is a single LDS compare,
// and every iteration is 1 b64 + 2 b128 LDS reads and ONE 16-B store per
// lane, the wave's 64 stores forming one contiguous 1-KiB segment.  The next
// commit's staging data is prefetched into registers (TileRegs) before the
// store loop.  A commit costs a fixed stretch (two barriers, the staging
// stores, the wait for the prefetch behind the store stream): sparse plans
// (a few pairs per owner, ~4k records per tile) commit two tiles at a time
// (TPF = 2) to halve that cost per record.
template <int TPF, bool CKSUM, bool WIN>
// toff / win / tseg: fa's per-tile tables again, as restrict arguments: read
// at wave-uniform indices they are scalar loads (lgkmcnt), so the commit's
// table reads never wait on the vector memory counter -- which would drain
// the previous commit's stores first
__global__ __launch_bounds__(FB, 2 * LIME_FILL_WGS) void k_fill(FillArgs fa, int64_t per, int64_t gran,
                                                               const uint64_t *__restrict__ toff,
                                                               const uint32_t *__restrict__ win,
                                                               const uint32_t *__restrict__ tseg) {
    constexpr int OTF = FillShape<TPF>::OTF, FO = FillShape<TPF>::FOPT,
                  PP = FillShape<TPF>::PPT, CAP = FillShape<TPF>::CAP;
    __shared__ uint2 s_lo_off[OTF + 1];
    __shared__ u32x4 s_own[OTF];
    __shared__ ParWin<TPF> s_par;
    __shared__ uint32_t s_wslot[TPF > 1 ? FW : 1][64];  // emit_sparse's owner slots
    __shared__ int64_t s_tile;
    __shared__ uint64_t s_red[2][FW];
    // (every shared array above counts: one more pushes k_fill<2> below
    // LIME_FILL_WGS workgroups per CU)
    static_assert(sizeof(s_lo_off) + sizeof(s_own) + sizeof(s_par) + sizeof(s_wslot) +
                          sizeof(s_tile) + sizeof(s_red) <= 160 * 1024 / LIME_FILL_WGS,
                  "k_fill's LDS must keep LIME_FILL_WGS workgroups per CU");

    const int64_t ob = fa.first + (int64_t)blockIdx.x * per;
    const int64_t oend = min(fa.first + fa.count, ob + per);
    if (ob >= oend) return;
    const int w = threadIdx.x / 64, lane = dev::lane_id();
    if (w == 0) {
        int64_t t0 = wave_tile_of(fa.toff, fa.ntiles, (uint64_t)ob);
        // back to the first tile of its commit
        const int64_t base = t0 < stream0_tiles(fa) ? 0 : stream0_tiles(fa);
        t0 = base + (t0 - base) / TPF * TPF;
        if (lane == 0) s_tile = t0;
    }
    __syncthreads();
    int64_t t = dev::uni64(s_tile);
    uint64_t hsum = 0, hxor = 0;
    TileRegs<TPF> R;
    tile_load<TPF>(fa, t, R, toff, win, tseg);
    while (true) {
        const int st = tile_stream(fa, t);
        const StreamArgs sa = st ? fa.s[1] : fa.s[0];
        const int64_t o0 = (t - sa.tile0) * OT;
        const int nown = (int)min((int64_t)OTF, sa.no - o0);
        const int64_t tbase = (int64_t)toff[t];
        const int64_t tn = dev::uni64(R.t1);
        // ---- commit the staged registers to LDS (offsets come scanned
        // from k_count: no block scan here)
        const uint32_t ttot = (uint32_t)(R.tnext - (uint64_t)tbase);
#pragma unroll
        for (int k = 0; k < FO; ++k) {
            const int q = threadIdx.x * FO + k;
            if (q < nown) {
                const uint32_t sg =
                    R.seg != 0xffffffffu ? R.seg : contig_off(fa.off, fa.n_contigs, R.og[k]);
                s_own[q] = u32x4{R.og[k], R.oe[k], R.orw[k], sg};
            }
            s_lo_off[q] = make_uint2(R.lo[k], q < nown ? R.off[k] : ttot);
        }
        if (threadIdx.x == 0) s_lo_off[OTF] = make_uint2(0u, ttot);
        const uint32_t wlo = R.wlo, whi = R.whi;
        const bool par_lds = (int64_t)whi - wlo <= CAP;
        if (par_lds) {
#pragma unroll
            for (int k = 0; k < PP; ++k) {
                const int i = k * FB + threadIdx.x;
                if (i < (int)(whi - wlo)) s_par.put(i, R.pg[k], R.pe[k], R.pr[k]);
            }
        }
        __syncthreads();
        // ---- prefetch the next commit (its loads overlap this one's stores)
        // (R.tnext = toff[tn]: no table read)
        const bool more = tn < fa.ntiles && (int64_t)R.tnext < oend;
        if (more) tile_load<TPF>(fa, tn, R, toff, win, tseg);
        // ---- this commit's slice of the output window, in granules dealt
        // round-robin to the waves (wave w: granules w, w + FW, ...).  The
        // default granule is one equal chunk per wave: 2048-record granules
        // (the fastest shape of the plain store probe, profiles/
        // r05_bw_probe.jsonl) measured 2% slower inside the fill
        // (profiles/r05_fill_sweep.txt)
        const int64_t lb = max(ob - tbase, (int64_t)0);
        const int64_t le = min(oend - tbase, (int64_t)ttot);
        // equal shares: `rounds` granules per wave of ~GR records each, so no
        // wave idles at the commit's closing barrier
        const int64_t rounds = max((int64_t)1, (le - lb + FW * gran - 1) / (FW * gran));
        const int64_t gsz = (((le - lb + FW * rounds - 1) / (FW * rounds)) + 63) & ~(int64_t)63;
        int qw = 0;  // wave-uniform: owner of the wave's previous granule start
        for (int64_t gb = lb + (int64_t)w * gsz; gb < le; gb += (int64_t)FW * gsz) {
            const int64_t gend = min(le, gb + gsz);
            int64_t o = gb + lane;
            // owner of the wave's first output (largest q with off_q <= gb),
            // by a 65-ary wave search over the LDS offsets (2-3 steps); each
            // lane then walks to its own owner
            qw = wave_owner_of(s_lo_off, qw, nown, (uint32_t)gb);
            int q = qw;
            if (TPF > 1) {
                uint32_t *wslot = s_wslot[TPF > 1 ? w : 0];
                if (par_lds)
                    emit_sparse<true, CKSUM, WIN, TPF>(fa, sa, st, s_lo_off, s_own, s_par, wlo,
                                                       tbase, gb, gend, qw, OTF, wslot, hsum,
                                                       hxor);
                else
                    emit_sparse<false, CKSUM, WIN, TPF>(fa, sa, st, s_lo_off, s_own, s_par, wlo,
                                                        tbase, gb, gend, qw, OTF, wslot, hsum,
                                                        hxor);
            } else if (par_lds)
                emit<true, CKSUM, WIN, TPF>(fa, sa, st, s_lo_off, s_own, s_par, wlo, tbase, o,
                                            gend, q, hsum, hxor);
            else
                emit<false, CKSUM, WIN, TPF>(fa, sa, st, s_lo_off, s_own, s_par, wlo, tbase, o,
                                             gend, q, hsum, hxor);
        }
        __syncthreads();
        if (!more) break;
        t = tn;
    }
    if (CKSUM) {
        hsum = dev::wave_reduce_sum(hsum);
        uint64_t x = hxor;
        x = dev::wave_reduce_xor(x);
        if (lane == 0) {
            s_red[0][w] = hsum;
            s_red[1][w] = x;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            uint64_t a = 0, b = 0;
            for (int i = 0; i < FW; ++i) {
                a += s_red[0][i];
                b ^= s_red[1][i];
            }
            atomicAdd((unsigned long long *)&fa.cksum[0], (unsigned long long)a);
            atomicXor((unsigned long long *)&fa.cksum[1], (unsigned long long)b);
        }
    }
}

// Filtered fallback (threshold >= 1 with partners narrower than it): thread per
// owner walks its candidate range and emits the qualifying ones in order.
template <bool CKSUM>
__global__ __launch_bounds__(IB) void k_fill_filtered(FillArgs fa, int64_t threshold) {
    __shared__ uint32_t scratch[IB / 64 + 1];
    __shared__ uint64_t s_red[2][IB / 64];
    const int64_t t = blockIdx.x;
    const int st = t < fa.s[0].tile0 + (fa.s[0].no + OT - 1) / OT ? 0 : 1;
    const StreamArgs sa = st ? fa.s[1] : fa.s[0];
    const int64_t lt = t - sa.tile0;
    const int64_t o0 = lt * OT;
    const int nown = (int)min((int64_t)OT, sa.no - o0);
    const int64_t tbase = (int64_t)fa.toff[t];
    uint32_t c[OPT];
    uint32_t csum = 0;
#pragma unroll
    for (int k = 0; k < OPT; ++k) {
        const int q = threadIdx.x * OPT + k;
        c[k] = q < nown ? fa.ocnt[sa.owner0 + o0 + q] : 0u;
        csum += c[k];
    }
    uint32_t ttot;
    int64_t pos = tbase + dev::block_exclusive_sum<IB>(csum, scratch, &ttot);
    uint64_t hsum = 0, hxor = 0;
    const int64_t wend = fa.first + fa.count;
    for (int k = 0; k < OPT; ++k) {
        const int q = threadIdx.x * OPT + k;
        if (q >= nown || c[k] == 0) continue;
        if (pos + c[k] <= fa.first || pos >= wend) {
            pos += c[k];
            continue;
        }
        const int64_t j = o0 + q;
        const uint32_t og = sa.ogs[j], oe = sa.oge[j], orow = sa.orow[j];
        const uint32_t sg = contig_off(fa.off, fa.n_contigs, og);
        uint32_t p = fa.olo[sa.owner0 + j];
        uint32_t left = c[k];
        for (; left > 0; ++p) {
            const uint32_t pg = sa.pgs[p], pe = sa.pge[p];
            if ((int64_t)(pe - pg) < threshold) continue;
            --left;
            if (pos >= fa.first && pos < wend) {
                const uint32_t pr = sa.prow[p];
                const uint32_t rs = (og > pg ? og : pg) - sg;
                const uint32_t re = (oe < pe ? oe : pe) - sg;
                const uint32_t ar = st == 0 ? orow : pr;
                const uint32_t br = st == 0 ? pr : orow;
                if (CKSUM) {
                    uint64_t h = dev::pair_hash(rs, re, ar, br);
                    hsum += h;
                    hxor ^= h;
                } else {
                    u32x4 v = {rs, re, ar, br};
                    fa.out[pos - fa.first] = v;
                }
            }
            ++pos;
        }
    }
    if (CKSUM) {
        hsum = dev::wave_reduce_sum(hsum);
        uint64_t x = hxor;
        x = dev::wave_reduce_xor(x);
        if (dev::lane_id() == 0) {
            s_red[0][threadIdx.x / 64] = hsum;
            s_red[1][threadIdx.x / 64] = x;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            uint64_t a = 0, b = 0;
            for (int i = 0; i < IB / 64; ++i) {
                a += s_red[0][i];
                b ^= s_red[1][i];
            }
            atomicAdd((unsigned long long *)&fa.cksum[0], (unsigned long long)a);
            atomicXor((unsigned long long *)&fa.cksum[1], (unsigned long long)b);
        }
    }
}

// The partner windows of stream `sa`'s owner tiles: one lane per tile when
// the owners' widths are bounded by owmax <= WLANE_MAX (the window then
// needs no read of the owners' ends), else one wave per tile (exact max end).
constexpr int64_t WLANE_MAX = 65536;
void launch_windows(lime_ctx *ctx, const StreamArgs &sa, int64_t tp, int64_t ntl, int64_t owmax,
                    uint32_t *win, const uint32_t *off, int32_t nc, uint32_t *tseg) {
    if (owmax <= WLANE_MAX)
        hipLaunchKernelGGL(k_windows_lane, dim3(blocks_for(ntl, 256)), dim3(256), 0, S(ctx), sa, tp,
                           ntl, owmax, win, off, nc, tseg);
    else
        hipLaunchKernelGGL(k_windows, dim3(blocks_for(ntl, IB / 64)), dim3(IB), 0, S(ctx), sa, tp,
                           ntl, win, off, nc, tseg);
}

// O_out / P_out: the sets whose coordinates the output records carry (the
// caller's set behind a window plan's widened set), default O / P.
StreamArgs stream_args(const lime_set *O, const lime_set *P, int st, int64_t threshold,
                       int64_t tile0, int64_t owner0, int64_t n_own = -1,
                       const lime_set *O_out = nullptr, const lime_set *P_out = nullptr,
                       int64_t reach = -1) {
    StreamArgs s;
    if (!O_out) O_out = O;
    if (!P_out) P_out = P;
    s.ogs = O->gs;
    s.oge = O->ge;
    s.orow = O->row;
    s.pgs = P->gs;
    s.pge = P->ge;
    s.prow = P->row;
    s.ogs_o = O_out->gs;
    s.oge_o = O_out->ge;
    s.pgs_o = P_out->gs;
    s.pge_o = P_out->ge;
    s.no = n_own >= 0 ? n_own : O->n;  // owners: the first n_own rows (halo rows own nothing)
    s.np = P->n;
    s.lo_off = st == 0 ? 0u : 1u;
    s.zw_skip = (st == 0 && threshold <= 0 && P->has_zero_width) ? 1 : 0;
    s.reach = st == 0 ? reach : -1;
    s.tile0 = tile0;
    s.owner0 = owner0;
    return s;
}

FillArgs fill_args(PairsPlan *pl) {
    FillArgs fa;
    fa.s[0] = stream_args(pl->A, pl->B, 0, pl->threshold, 0, 0, pl->a_own, pl->A_out, nullptr,
                          pl->reach);
    fa.s[1] = stream_args(pl->B, pl->A, 1, pl->threshold, pl->nt0, pl->a_own, pl->b_own, nullptr,
                          pl->A_out);
    fa.olo = pl->olo;
    fa.ocnt = pl->ocnt;
    fa.toff = pl->toff;
    fa.win = pl->win;
    fa.tseg = pl->tseg;
    fa.total = pl->total;
    fa.ntiles = pl->nt0 + pl->nt1;
    fa.off = pl->A->d_off;
    fa.n_contigs = pl->A->n_contigs;
    fa.first = 0;
    fa.count = 0;
    fa.out = nullptr;
    fa.cksum = nullptr;
    return fa;
}

// Output records per fill workgroup: one wave of resident workgroups covers
// the window, each prefetching its next tile behind its stores (1-3% faster
// than 131072-record workgroups, profiles/r05_fill_sweep.txt).  The device's
// slot count is queried once per process.
int64_t fill_span(int64_t count) {
    static const int64_t slots = [] {
        int dev = 0, cus = 256, occ = 2;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_fill<1, false, false>, FB, 0);
        return (int64_t)cus * (occ > 0 ? occ : 1);
    }();
    int64_t per = (count + slots - 1) / slots;
    per = (per + 63) & ~(int64_t)63;
    return per < 4096 ? 4096 : per;
}

template <int TPF>
void launch_k_fill(lime_ctx *ctx, dim3 g, const FillArgs &fa, int64_t per, bool cksum, bool win) {
    if (cksum && win)
        hipLaunchKernelGGL((k_fill<TPF, true, true>), g, dim3(FB), 0, S(ctx), fa, per, (int64_t)GR,
                           fa.toff, fa.win, fa.tseg);
    else if (cksum)
        hipLaunchKernelGGL((k_fill<TPF, true, false>), g, dim3(FB), 0, S(ctx), fa, per, (int64_t)GR,
                           fa.toff, fa.win, fa.tseg);
    else if (win)
        hipLaunchKernelGGL((k_fill<TPF, false, true>), g, dim3(FB), 0, S(ctx), fa, per, (int64_t)GR,
                           fa.toff, fa.win, fa.tseg);
    else
        hipLaunchKernelGGL((k_fill<TPF, false, false>), g, dim3(FB), 0, S(ctx), fa, per,
                           (int64_t)GR, fa.toff, fa.win, fa.tseg);
}

int launch_fill(PairsPlan *pl, int64_t first, int64_t count, u32x4 *out, uint64_t *cksum) {
    lime_ctx *ctx = pl->ctx;
    if (count <= 0) return LIME_OK;
    FillArgs fa = fill_args(pl);
    fa.first = first;
    fa.count = count;
    fa.out = out;
    fa.cksum = cksum;
    if (pl->filtered) {
        const unsigned grid = (unsigned)(pl->nt0 + pl->nt1);
        if (cksum)
            hipLaunchKernelGGL(k_fill_filtered<true>, dim3(grid), dim3(IB), 0, S(ctx), fa,
                               pl->threshold);
        else
            hipLaunchKernelGGL(k_fill_filtered<false>, dim3(grid), dim3(IB), 0, S(ctx), fa,
                               pl->threshold);
    } else {
        const int64_t per = fill_span(count);
        const int64_t grid = (count + per - 1) / per;
        if (grid > 0x7fffffff) return fail(LIME_ERR_OVERFLOW, "fill window too large");
        const dim3 g((unsigned)grid);
        const bool win = pl->reach >= 0;
        if (pl->tpf == 2)
            launch_k_fill<2>(ctx, g, fa, per, cksum != nullptr, win);
        else
            launch_k_fill<1>(ctx, g, fa, per, cksum != nullptr, win);
    }
    LIME_HIP(hipGetLastError());
    return LIME_OK;
}

// DistributedWindow's widened set (Window.scala:34-39 condition isNearby):
// with ADAM's distance (0 if overlapping, gap + 1 otherwise, SURVEY.md
// Appendix A), a and b are within d >= 1 iff b strictly overlaps
// W(a) = [a.s - d, a.e + d), so a window is the intersection join of W(A)
// with B.  W is clipped to the contig's pad positions (off[c] - 1 and
// off[c + 1]), so no row of a neighbouring contig can fall inside it; the
// map is monotone in a.s, so W keeps A's sorted order.
__global__ __launch_bounds__(256) void k_widen(const uint32_t *__restrict__ gs,
                                               const uint32_t *__restrict__ ge, int64_t n,
                                               int64_t d, const uint32_t *__restrict__ off,
                                               int32_t nc, uint32_t *__restrict__ ws,
                                               uint32_t *__restrict__ we) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const uint32_t g = gs[i];
    int64_t c = dev::upper_bound(off, 0, (int64_t)nc, g) - 1;
    if (c < 0) c = 0;
    const int64_t lo = c == 0 ? 0 : (int64_t)off[c] - 1;
    const int64_t hi = (int64_t)off[c + 1];
    const int64_t s = (int64_t)g - d, e = (int64_t)ge[i] + d;
    ws[i] = (uint32_t)(s > lo ? s : lo);
    we[i] = (uint32_t)(e < hi ? e : hi);
}

}  // namespace

// Owners are the first a_own rows of A (stream 0) and b_own rows of B
// (stream 1); the remaining rows are a halo (partners only), used when a
// coordinate shard carries its right neighbours' boundary rows.
// A_out / reach: window plans (see window_plan); nullptr / -1 for intersect.
int intersect_plan(lime_ctx *ctx, const lime_set *A, const lime_set *B, int64_t threshold,
                   int64_t a_own, int64_t b_own, PairsPlan **out, const lime_set *A_out,
                   int64_t reach) {
    if (a_own < 0 || a_own > A->n) a_own = A->n;
    if (b_own < 0 || b_own > B->n) b_own = B->n;
    PairsPlan *pl = new PairsPlan();
    pl->ctx = ctx;
    pl->A = A;
    pl->B = B;
    pl->A_out = A_out;
    pl->reach = reach;
    pl->a_own = a_own;
    pl->b_own = b_own;
    pl->threshold = threshold;
    pl->tp = threshold > 1 ? threshold : 1;
    pl->filtered = threshold >= 1 && (int64_t)std::min(A->min_width, B->min_width) < threshold &&
                   A->n > 0 && B->n > 0;
    pl->nt0 = (a_own + OT - 1) / OT;
    pl->nt1 = (b_own + OT - 1) / OT;
    const int64_t nt = pl->nt0 + pl->nt1;
    int rc = LIME_OK;
    uint64_t *tcnt = nullptr, *total = nullptr;
    if ((rc = alloc(ctx, &pl->olo, (size_t)(a_own + b_own))) ||
        (rc = alloc(ctx, &pl->ocnt, (size_t)(a_own + b_own))) ||
        (rc = alloc(ctx, &pl->toff, (size_t)nt)) || (rc = alloc(ctx, &pl->win, (size_t)2 * nt)) ||
        (rc = alloc(ctx, &pl->tseg, (size_t)nt)) ||
        (rc = alloc(ctx, &tcnt, (size_t)nt)) || (rc = alloc(ctx, &total, 2))) {
        delete pl;
        return rc;
    }
    // total[1]: overflow flag of the u32 tile-local offsets
    uint32_t *oflow = reinterpret_cast<uint32_t *>(total + 1);
    LIME_HIP(hipMemsetAsync(total + 1, 0, sizeof(uint64_t), S(ctx)));
    if (A->n > 0 && B->n > 0) {
        for (int st = 0; st < 2; ++st) {
            const lime_set *O = st == 0 ? A : B;
            const lime_set *P = st == 0 ? B : A;
            const int64_t ntl = st == 0 ? pl->nt0 : pl->nt1;
            StreamArgs sa = stream_args(O, P, st, threshold, st == 0 ? 0 : pl->nt0,
                                        st == 0 ? 0 : a_own, st == 0 ? a_own : b_own,
                                        st == 0 ? A_out : nullptr, st == 0 ? nullptr : A_out,
                                        reach);
            if (ntl == 0) continue;
            // owner widths: a window plan's widened rows are up to 2 d wider
            const int64_t owmax = (int64_t)O->max_width + (st == 0 && reach > 0 ? 2 * reach : 0);
            launch_windows(ctx, sa, pl->tp, ntl, owmax, pl->win, (const uint32_t *)O->d_off,
                           O->n_contigs, pl->tseg);
            if (pl->filtered)
                hipLaunchKernelGGL((k_count<true, false>), dim3((unsigned)ntl), dim3(IB), 0, S(ctx), sa,
                                   pl->tp, threshold, (const uint32_t *)pl->win, pl->olo, pl->ocnt,
                                   tcnt, oflow);
            else
                hipLaunchKernelGGL((k_count<false, true>), dim3((unsigned)ntl), dim3(IB), 0, S(ctx), sa,
                                   pl->tp, threshold, (const uint32_t *)pl->win, pl->olo, pl->ocnt,
                                   tcnt, oflow);
            LIME_HIP(hipGetLastError());
        }
    } else {
        LIME_HIP(hipMemsetAsync(tcnt, 0, sizeof(uint64_t) * (size_t)(nt > 0 ? nt : 1), S(ctx)));
        LIME_HIP(hipMemsetAsync(pl->ocnt, 0,
                                sizeof(uint32_t) * (size_t)(a_own + b_own > 0 ? a_own + b_own : 1),
                                S(ctx)));
    }
    LIME_TRY(scan_exclusive_u64(ctx, tcnt, pl->toff, nt, total));
    uint64_t tot[2] = {0, 0};
    LIME_TRY(read_back(ctx, tot, total, sizeof(tot)));
    release(ctx, tcnt);
    release(ctx, total);
    if (tot[1] & 1) {
        intersect_free(pl);
        return fail(LIME_ERR_OVERFLOW,
                    "a tile of 1024 owner rows has 2^32 or more candidate pairs (pile-up)");
    }
    pl->total = (int64_t)tot[0];
    // sparse plans commit two owner tiles per fill step (k_fill<2>) unless
    // a tile holds 2^31 or more pairs (two tiles' u32 offsets could wrap)
    pl->tpf = !(tot[1] & 2) && pl->total < (int64_t)LIME_FILL_SPARSE * (a_own + b_own) ? 2 : 1;
    *out = pl;
    return LIME_OK;
}

// Candidate range [olo, olo + ocnt) of every owner row of O in P for stream
// `st` (unfiltered), used by subtract (stream 0: b.s in [a.s, a.e - tp]).
int owner_ranges(lime_ctx *ctx, const lime_set *O, const lime_set *P, int st, int64_t threshold,
                 uint32_t *olo, uint32_t *ocnt) {
    if (O->n == 0) return LIME_OK;
    if (P->n == 0) {
        LIME_HIP(hipMemsetAsync(olo, 0, sizeof(uint32_t) * (size_t)O->n, S(ctx)));
        LIME_HIP(hipMemsetAsync(ocnt, 0, sizeof(uint32_t) * (size_t)O->n, S(ctx)));
        return LIME_OK;
    }
    const int64_t tp = threshold > 1 ? threshold : 1;
    const int64_t ntl = (O->n + OT - 1) / OT;
    uint32_t *win;
    uint64_t *tcnt;
    LIME_TRY(alloc(ctx, &win, (size_t)2 * ntl));
    LIME_TRY(alloc(ctx, &tcnt, (size_t)ntl));
    StreamArgs sa = stream_args(O, P, st, threshold, 0, 0);
    launch_windows(ctx, sa, tp, ntl, (int64_t)O->max_width, win, nullptr, 0, nullptr);
    hipLaunchKernelGGL((k_count<false, false>), dim3((unsigned)ntl), dim3(IB), 0, S(ctx), sa, tp,
                       threshold,
                       (const uint32_t *)win, olo, ocnt, tcnt, (uint32_t *)nullptr);
    LIME_HIP(hipGetLastError());
    release(ctx, win);
    release(ctx, tcnt);
    return LIME_OK;
}

int intersect_fill(PairsPlan *pl, int64_t first, int64_t count, lime_pair *d_out) {
    if (first < 0 || count < 0 || first + count > pl->total)
        return fail(LIME_ERR_ARG, "fill window outside [0, n_pairs)");
    return launch_fill(pl, first, count, reinterpret_cast<u32x4 *>(d_out), nullptr);
}

int intersect_checksum(PairsPlan *pl, uint64_t *sum, uint64_t *xr) {
    lime_ctx *ctx = pl->ctx;
    uint64_t *ck;
    LIME_TRY(alloc(ctx, &ck, 2));
    LIME_HIP(hipMemsetAsync(ck, 0, 16, S(ctx)));
    // bound each launch to keep the grid size in range
    const int64_t step = (int64_t)SBLK * 1048576;
    for (int64_t f = 0; f < pl->total; f += step)
        LIME_TRY(launch_fill(pl, f, std::min(step, pl->total - f), nullptr, ck));
    uint64_t h[2];
    LIME_TRY(read_back(ctx, h, ck, 16));
    release(ctx, ck);
    *sum = h[0];
    *xr = h[1];
    return LIME_OK;
}

int64_t plan_total(const PairsPlan *pl) { return pl->total; }

// Pairs (a, b) with ADAM a.isNearby(b, d) (DistributedWindow,
// Window.scala:71-95); the records carry a's own region (primitive returns
// the first region, :17-22).
int window_plan(lime_ctx *ctx, const lime_set *A, const lime_set *B, int64_t d,
                PairsPlan **out) {
    if (d < 1) return intersect_plan(ctx, A, B, 0, -1, -1, out, A, 0);
    lime_set *W = new lime_set();
    W->ctx = ctx;
    W->n = A->n;
    W->row = A->row;  // borrowed: W's row i is A's row i
    W->d_off = A->d_off;
    W->space_keep = A->space_keep;
    W->n_contigs = A->n_contigs;
    W->off = A->off;
    W->len = A->len;
    W->min_width = A->min_width;
    W->max_width = A->max_width;
    W->has_zero_width = false;  // every W row is >= 2d wide or clipped to > 0
    int rc = LIME_OK;
    if ((rc = alloc(ctx, &W->gs, (size_t)std::max<int64_t>(A->n, 1))) ||
        (rc = alloc(ctx, &W->ge, (size_t)std::max<int64_t>(A->n, 1)))) {
        release(ctx, W->gs);
        delete W;
        return rc;
    }
    if (A->n > 0) {
        hipLaunchKernelGGL(k_widen, dim3(blocks_for(A->n, 256)), dim3(256), 0, S(ctx), A->gs,
                           A->ge, A->n, d, (const uint32_t *)A->d_off, A->n_contigs, W->gs,
                           W->ge);
        LIME_HIP(hipGetLastError());
    }
    PairsPlan *pl = nullptr;
    rc = intersect_plan(ctx, W, B, 0, -1, -1, &pl, A, d);
    if (rc != LIME_OK) {
        release(ctx, W->gs);
        release(ctx, W->ge);
        delete W;
        return rc;
    }
    pl->W = W;
    *out = pl;
    return LIME_OK;
}

void intersect_free(PairsPlan *pl) {
    lime_ctx *ctx = pl->ctx;
    if (pl->W) {
        release(ctx, pl->W->gs);
        release(ctx, pl->W->ge);
        delete pl->W;
    }
    release(ctx, pl->olo);
    release(ctx, pl->ocnt);
    release(ctx, pl->toff);
    release(ctx, pl->win);
    release(ctx, pl->tseg);
    delete pl;
}

}  // namespace lime

// merge.hip -- DistributedMerge / localCompute as a segmented max-end scan.
//
// Reference: SetTheory.scala:208-225 folds the sorted partition, keeping the
// running hull at the list head and merging the next region iff
// head.overlaps(next) (Merge.scala:15-20, threshold not passed: quirk Q6).
// With the canonical order (start, zero-width first) that fold starts a new
// run at row i exactly when
//       M_i = max(ge[0..i-1])  <=  gs[i]
// (strict overlap: book-ended rows do not merge).  Contigs need no segment
// flags: in global coordinates every earlier contig ends below the next
// contig's offset (off[c+1] = off[c] + len[c] + 1), so the flag fires at a
// contig change by itself.  Run r = [gs[first_r], M at first_{r+1}), the last
// run ends at max(ge).
//
// k_merge_scan: ONE pass over the set (8 B read + 4 B run id written per
// row, 8 B per run).  Tiles of 16384 rows are taken in ticket order; a tile
// publishes its max(ge) and learns M at its first row by a decoupled
// look-back over its predecessors' (flag | value) status words, flags its
// rows, then publishes its run count and learns its first run index by a
// second look-back.  Plain sets run k_merge_scan2 (no LDS transposes, two
// workgroups per CU); stranded sets k_merge_scan<true> (a segmented scan).
// The multi-pass kernels (k_tile_max, k_scan_max, k_prefix_max) remain for
// subtract's inclusive prefix max.
#include "common.hpp"

namespace lime {
namespace {

constexpr int MB = 256;
constexpr int MITEMS = 16;
constexpr int MTILE = MB * MITEMS;

__global__ __launch_bounds__(MB) void k_tile_max(const uint32_t *__restrict__ ge, int64_t n,
                                                 uint32_t *__restrict__ tmax) {
    const int64_t base = (int64_t)blockIdx.x * MTILE;
    uint32_t m = 0;
#pragma unroll
    for (int k = 0; k < MITEMS; ++k) {
        int64_t i = base + k * MB + threadIdx.x;
        if (i < n) m = max(m, ge[i]);
    }
    m = dev::wave_reduce_max(m);
    __shared__ uint32_t ws[MB / 64];
    if (dev::lane_id() == 0) ws[threadIdx.x / 64] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
        for (int i = 0; i < MB / 64; ++i) t = max(t, ws[i]);
        tmax[blockIdx.x] = t;
    }
}

// exclusive max-scan of v[0..m) in place (identity 0), single block
__global__ __launch_bounds__(MB) void k_scan_max(uint32_t *v, int64_t m) {
    __shared__ uint32_t scratch[MB / 64 + 1];
    uint32_t carry = 0;
    for (int64_t base = 0; base < m; base += MB) {
        int64_t i = base + threadIdx.x;
        uint32_t x = i < m ? v[i] : 0u;
        uint32_t tot;
        uint32_t ex = dev::block_exclusive_max<MB>(x, 0u, scratch, &tot);
        if (i < m) v[i] = max(carry, ex);
        carry = max(carry, tot);
    }
}

// Load a tile in blocked arrangement (thread t owns rows t*16..t*16+15) via
// coalesced loads staged through LDS.
template <typename T>
__device__ __forceinline__ void load_blocked(const T *__restrict__ src, int64_t base, int64_t n,
                                             T fill, T *lds, T (&v)[MITEMS]) {
#pragma unroll
    for (int k = 0; k < MITEMS; ++k) {
        int64_t i = base + k * MB + threadIdx.x;
        lds[k * MB + threadIdx.x] = i < n ? src[i] : fill;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < MITEMS; ++k) v[k] = lds[threadIdx.x * MITEMS + k];
    __syncthreads();
}

// ---------------------------------------------------------- single pass
// (decoupled look-back: dev::lookback and the status words, common.hpp)
using dev::ST_AGG;
using dev::ST_INC;
using dev::ST_VAL;
using dev::st_publish;
using dev::st_poll;
using dev::lookback;

struct MergeScanArgs {
    const uint32_t *gs, *ge;
    int64_t n;
    uint64_t *st_max, *st_cnt;  // per-tile status words (zeroed before launch)
    uint32_t *ticket;
    uint32_t *run_gs, *run_ge;  // capacity n
    uint32_t *run_of_sorted;    // may be null
    uint32_t *pmax;             // may be null: inclusive prefix max of ge (plain sets)
    uint64_t *total;            // runs
    const int8_t *strand;       // stranded sets: strand per input row
    const uint32_t *row;        // sorted row ids (strand lookups; null: by position)
    int8_t *run_strand;         // stranded sets: the strand of every run (may be null)
    uint32_t *tie;              // k_merge_scan2, may be null: set to 1 when some start
                                // is shared by more than TIE_G consecutive rows
};
// subtract's same-start group bound (subtract.hip TIE_G): k_merge_scan2 tests
// gs[i] == gs[i + 16], row i + 16 being held by lane + 4 (4 rows per lane)
constexpr int MERGE_TIE_G = 16;

// Full tile <-> blocked registers (thread t: rows 16t .. 16t+15) through
// LDS: global traffic is lane-consecutive 16-B accesses (whole lines per
// wave instruction); the LDS image pads 4 words after every 16 rows so the
// blocked b128 reads (stride 80 B per lane) are conflict-free.
// 1024 threads x 16 rows = 16384-row tiles, one workgroup per CU: half the
// tiles (and look-backs) of 8192-row tiles, C3's merge 1.89 -> 1.67 ms;
// 4096-row tiles at 5 workgroups per CU were slower (2.2-2.3 ms)
#ifndef LIME_MERGE_SB
#define LIME_MERGE_SB 1024
#endif
#ifndef LIME_MERGE_WPE
#define LIME_MERGE_WPE 1
#endif
constexpr int SB = LIME_MERGE_SB;    // scan workgroup
constexpr int STILE = SB * MITEMS;   // rows per scan tile
constexpr int MPADW = STILE + STILE / 4;
__device__ __forceinline__ int pad_word(int u4) { return 4 * u4 + 4 * (u4 >> 2); }

__device__ __forceinline__ void tile_to_blocked(const uint32_t *__restrict__ src, uint32_t *lds,
                                                uint32_t (&v)[MITEMS]) {
    const uint4 *s4 = reinterpret_cast<const uint4 *>(src);
#pragma unroll
    for (int k = 0; k < MITEMS / 4; ++k) {
        const int u = k * SB + threadIdx.x;
        *reinterpret_cast<uint4 *>(lds + pad_word(u)) = s4[u];
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < MITEMS / 4; ++j) {
        const uint4 x = *reinterpret_cast<const uint4 *>(lds + 20 * threadIdx.x + 4 * j);
        v[4 * j] = x.x, v[4 * j + 1] = x.y, v[4 * j + 2] = x.z, v[4 * j + 3] = x.w;
    }
    __syncthreads();
}

__device__ __forceinline__ void blocked_to_tile(const uint32_t (&v)[MITEMS], uint32_t *lds,
                                                uint32_t *__restrict__ dst) {
#pragma unroll
    for (int j = 0; j < MITEMS / 4; ++j)
        *reinterpret_cast<uint4 *>(lds + 20 * threadIdx.x + 4 * j) =
            make_uint4(v[4 * j], v[4 * j + 1], v[4 * j + 2], v[4 * j + 3]);
    __syncthreads();
    uint4 *d4 = reinterpret_cast<uint4 *>(dst);
#pragma unroll
    for (int k = 0; k < MITEMS / 4; ++k) {
        const int u = k * SB + threadIdx.x;
        d4[u] = *reinterpret_cast<const uint4 *>(lds + pad_word(u));
    }
}

// Segmented max (stranded merge): a segment starts at every strand change;
// (b, v) = (segment start seen, max since the last start).
struct SegMax {
    uint32_t b, v;
};
__device__ __forceinline__ SegMax seg_combine(SegMax x, SegMax y) {  // x before y
    return SegMax{x.b | y.b, y.b ? y.v : (x.v > y.v ? x.v : y.v)};
}
// block-wide exclusive segmented-max scan (identity {0, 0}); *total = all
template <int BLOCK>
__device__ SegMax block_exclusive_segmax(SegMax x, SegMax *scratch, SegMax *total) {
    constexpr int NW = BLOCK / 64;
    const int w = threadIdx.x / 64, lane = dev::lane_id();
    // the pair packed as b << 32 | v: the DPP scan with seg_combine
    auto pk = [](SegMax m) { return ((uint64_t)m.b << 32) | m.v; };
    auto up = [](uint64_t u) { return SegMax{(uint32_t)(u >> 32), (uint32_t)u}; };
    const uint64_t incp = dev::wave_scan_dpp(
        pk(x), (uint64_t)0, [&](uint64_t a, uint64_t b) { return pk(seg_combine(up(b), up(a))); });
    const SegMax inc = up(incp);
    const SegMax exc = up(dev::wave_shr1(incp, (uint64_t)0));
    if (lane == 63) scratch[w] = inc;
    __syncthreads();
    if (threadIdx.x == 0) {
        SegMax run{0u, 0u};
        for (int i = 0; i < NW; ++i) {
            const SegMax t = scratch[i];
            scratch[i] = run;
            run = seg_combine(run, t);
        }
        scratch[NW] = run;
    }
    __syncthreads();
    const SegMax res = seg_combine(scratch[w], exc);
    *total = scratch[NW];
    __syncthreads();
    return res;
}

// STR: stranded set -- a run also breaks where the strand changes (the
// reference fold's Merge.condition is overlaps, which needs equal strands);
// the max-end carry restarts there, so a tile holding a strand change
// publishes its inclusive carry without looking back.
template <bool STR>
__global__ __launch_bounds__(SB) __attribute__((amdgpu_waves_per_eu(LIME_MERGE_WPE, 8)))
void k_merge_scan(MergeScanArgs a) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[MPADW];
    __shared__ uint32_t scratch[SB / 64 + 1];
    __shared__ SegMax sscratch[SB / 64 + 1];
    __shared__ uint64_t s_carry;
    __shared__ uint32_t s_tile;
    if (threadIdx.x == 0) s_tile = atomicAdd(a.ticket, 1u);
    __syncthreads();
    const int64_t tile = s_tile;
    const int64_t n = a.n;
    const int64_t r0 = tile * STILE + (int64_t)threadIdx.x * MITEMS;  // blocked rows
    uint32_t s[MITEMS], e[MITEMS];
    const int64_t t0 = tile * STILE;
    const bool full = t0 + STILE <= n;
    if (full) {
        tile_to_blocked(a.gs + t0, lds, s);
        tile_to_blocked(a.ge + t0, lds, e);
    } else {
#pragma unroll
        for (int k = 0; k < MITEMS; ++k) {
            const bool v = r0 + k < n;
            s[k] = v ? a.gs[r0 + k] : 0xffffffffu;
            e[k] = v ? a.ge[r0 + k] : 0u;
        }
    }
    uint32_t brk = 0;  // bit k: row r0 + k starts a strand segment
    if (STR) {
        int prev = r0 > 0 && r0 - 1 < n ? a.strand[a.row ? a.row[r0 - 1] : r0 - 1] : -1;
#pragma unroll
        for (int k = 0; k < MITEMS; ++k) {
            if (r0 + k < n) {
                const int c = a.strand[a.row ? a.row[r0 + k] : r0 + k];
                if (c != prev) brk |= 1u << k;
                prev = c;
            }
        }
    }
    // thread aggregate and the tile's exclusive carry
    SegMax agg{0u, 0u};
#pragma unroll
    for (int k = 0; k < MITEMS; ++k) {
        if (brk & (1u << k)) agg = SegMax{1u, 0u};
        agg.v = max(agg.v, e[k]);
    }
    SegMax tot;
    SegMax pre;
    if (STR) {
        pre = block_exclusive_segmax<SB>(agg, sscratch, &tot);
    } else {
        uint32_t tmax;
        pre = SegMax{0u, dev::block_exclusive_max<SB>(agg.v, 0u, scratch, &tmax)};
        tot = SegMax{0u, tmax};
    }
    // ---- chain 1: max end (since the last strand change) before the tile
    if (threadIdx.x < 64) {
        uint64_t ex = 0;
        if (tile == 0 || tot.b) {  // nothing before matters past a segment start
            if (threadIdx.x == 0) st_publish(a.st_max + tile, ST_INC | tot.v);
            if (!tot.b || tile == 0) ex = 0;
            if (tile > 0 && tot.b) ex = lookback<true>(a.st_max, tile);
        } else {
            if (threadIdx.x == 0) st_publish(a.st_max + tile, ST_AGG | tot.v);
            ex = lookback<true>(a.st_max, tile);
            if (threadIdx.x == 0)
                st_publish(a.st_max + tile, ST_INC | (ex > tot.v ? ex : (uint64_t)tot.v));
        }
        if (threadIdx.x == 0) s_carry = ex;
    }
    __syncthreads();
    const uint32_t M0 = pre.b ? pre.v : max(pre.v, (uint32_t)s_carry);
    uint32_t M = M0;
    uint32_t flags = 0;
#pragma unroll
    for (int k = 0; k < MITEMS; ++k) {
        const bool b = (brk >> k) & 1u;
        if (r0 + k < n && (b || M <= s[k])) flags |= 1u << k;
        M = b ? e[k] : max(M, e[k]);
    }
    uint32_t ctot;
    const uint32_t rpre = dev::block_exclusive_sum<SB>((uint32_t)__popc(flags), scratch, &ctot);
    // ---- chain 2: index of the tile's first run
    if (threadIdx.x < 64) {
        uint64_t ex = 0;
        if (tile == 0) {
            if (threadIdx.x == 0) st_publish(a.st_cnt, ST_INC | ctot);
        } else {
            if (threadIdx.x == 0) st_publish(a.st_cnt + tile, ST_AGG | ctot);
            ex = lookback<false>(a.st_cnt, tile);
            if (threadIdx.x == 0) st_publish(a.st_cnt + tile, ST_INC | (ex + ctot));
        }
        if (threadIdx.x == 0) s_carry = ex;
    }
    __syncthreads();
    uint32_t r = (uint32_t)s_carry + rpre;  // runs started before this thread's rows
    uint32_t rid[MITEMS];
    M = M0;  // the run so far: its end where row k starts a new run
#pragma unroll
    for (int k = 0; k < MITEMS; ++k) {
        const int64_t i = r0 + k;
        const bool b = (brk >> k) & 1u;
        if (i < n) {
            if (flags & (1u << k)) {
                a.run_gs[r] = s[k];
                if (STR && a.run_strand) a.run_strand[r] = a.strand[a.row ? a.row[i] : i];
                if (r > 0) a.run_ge[r - 1] = M;
                ++r;
            }
            if (i == n - 1) {
                a.run_ge[r - 1] = b ? e[k] : max(M, e[k]);
                *a.total = r;
            }
        }
        M = b ? e[k] : max(M, e[k]);
        rid[k] = r - 1;
    }
    if (a.run_of_sorted) {
        if (full) {
            blocked_to_tile(rid, lds, a.run_of_sorted + t0);
        } else {
#pragma unroll
            for (int k = 0; k < MITEMS; ++k)
                if (r0 + k < n) a.run_of_sorted[r0 + k] = rid[k];
        }
    }
    // the inclusive prefix max of ge per row (subtract's spanning search),
    // recomputed from the tile's carry: saves the set a k_tile_max +
    // k_prefix_max pass over ge
    if (!STR && a.pmax) {
        uint32_t pm[MITEMS];
        M = M0;
#pragma unroll
        for (int k = 0; k < MITEMS; ++k) {
            M = max(M, e[k]);
            pm[k] = M;
        }
        if (full) {
            __syncthreads();  // the LDS image is reused
            blocked_to_tile(pm, lds, a.pmax + t0);
        } else {
#pragma unroll
            for (int k = 0; k < MITEMS; ++k)
                if (r0 + k < n) a.pmax[r0 + k] = pm[k];
        }
    }
}

// Plain sets: the same single pass without the LDS transposes, so two
// workgroups share a CU and one's look-backs overlap the other's loads (the
// 80 KiB transpose image held k_merge_scan to one workgroup per CU, its loads
// idle through both look-backs).  Wave w of the tile owns rows
// [RW w, RW (w + 1)) in rounds of 256 (lane l: rows 256 q + 4 l .. + 3, 16-B
// loads and stores), scanned round by round with DPP wave scans; one barrier
// per chain combines the waves.
template <int NT, int Q>
struct ScanGeom {
    static constexpr int NW = NT / 64;
    static constexpr int RQ = Q;               // rounds of 256 rows per wave
    static constexpr int RW = RQ * 256;        // rows per wave
    static constexpr int TILE = NW * RW;       // rows per tile
};
// 1024 threads x 32 rows: 32768-row tiles, one workgroup per CU (<= 128
// VGPRs): half the look-backs of 16384-row tiles at two per CU, C3's merge
// 1.355 -> 1.313 ms; 8192-row tiles at four per CU: 1.55 ms
// (profiles/round5/merge_scan2_tiles_ab.txt)
#ifndef LIME_MS2_NT
#define LIME_MS2_NT 1024
#endif
#ifndef LIME_MS2_Q
#define LIME_MS2_Q 8
#endif
#ifndef LIME_MS2_WPE
#define LIME_MS2_WPE 4
#endif
constexpr int MS2 = LIME_MS2_NT;
using G2 = ScanGeom<MS2, LIME_MS2_Q>;

// TIE: also test for subtract's long same-start groups (a.tie)
template <bool TIE>
__global__ __launch_bounds__(MS2) __attribute__((amdgpu_waves_per_eu(LIME_MS2_WPE, 8)))
void k_merge_scan2(MergeScanArgs a) {
    constexpr int NW = G2::NW, RQ = G2::RQ;
    __shared__ uint32_t s_wmax[NW], s_wcnt[NW];
    __shared__ uint32_t s_c1, s_c2, s_tile;
    if (threadIdx.x == 0) s_tile = atomicAdd(a.ticket, 1u);
    __syncthreads();
    const int64_t tile = s_tile;
    const int64_t n = a.n;
    const int w = threadIdx.x / 64, lane = dev::lane_id();
    const int64_t wb = tile * G2::TILE + (int64_t)w * G2::RW;  // the wave's first row
    uint32_t s[4 * RQ], e[4 * RQ];
    // lane maxima per round; the wave's and the tile's maximum
    uint32_t rmax[RQ], lmax = 0;
    auto round_max = [&]() {
#pragma unroll
        for (int q = 0; q < RQ; ++q) {
            rmax[q] = max(max(e[4 * q], e[4 * q + 1]), max(e[4 * q + 2], e[4 * q + 3]));
            lmax = max(lmax, rmax[q]);
        }
    };
    // every end first, then every start: loads return in order, so the
    // tile's aggregate (its max end) is published while the starts are still
    // in flight (successors' look-backs wait on it).  A full tile takes the
    // branch-free path, where the wait before the maximum counts only the
    // ends (per-lane bounds checks made it wait for every load)
    if ((tile + 1) * G2::TILE <= n) {  // (uniform)
        const uint4 *e4 = reinterpret_cast<const uint4 *>(a.ge + wb) + lane;
        const uint4 *s4 = reinterpret_cast<const uint4 *>(a.gs + wb) + lane;
#pragma unroll
        for (int q = 0; q < RQ; ++q) {
            const uint4 y = e4[64 * q];
            e[4 * q] = y.x, e[4 * q + 1] = y.y, e[4 * q + 2] = y.z, e[4 * q + 3] = y.w;
        }
#pragma unroll
        for (int q = 0; q < RQ; ++q) {
            const uint4 x = s4[64 * q];
            s[4 * q] = x.x, s[4 * q + 1] = x.y, s[4 * q + 2] = x.z, s[4 * q + 3] = x.w;
        }
        round_max();  // (inside the branch: its wait counts the ends only)
    } else {
#pragma unroll
        for (int k = 0; k < 4 * RQ; ++k) {
            const int64_t i = wb + 256 * (k / 4) + 4 * lane + (k % 4);
            e[k] = i < n ? a.ge[i] : 0u;
        }
#pragma unroll
        for (int k = 0; k < 4 * RQ; ++k) {
            const int64_t i = wb + 256 * (k / 4) + 4 * lane + (k % 4);
            s[k] = i < n ? a.gs[i] : 0xffffffffu;
        }
        round_max();
    }
    const uint32_t wmax = dev::wave_reduce_max(lmax);
    if (lane == 0) s_wmax[w] = wmax;
    __syncthreads();
    // ---- chain 1: max end before the tile
    if (w == 0) {
        const uint32_t tmax = dev::wave_reduce_max(lane < NW ? s_wmax[lane] : 0u);
        uint64_t ex = 0;
        if (tile == 0) {
            if (lane == 0) st_publish(a.st_max, ST_INC | tmax);
        } else {
            if (lane == 0) st_publish(a.st_max + tile, ST_AGG | tmax);
            ex = lookback<true>(a.st_max, tile);
            if (lane == 0) st_publish(a.st_max + tile, ST_INC | (ex > tmax ? ex : (uint64_t)tmax));
        }
        if (lane == 0) s_c1 = (uint32_t)ex;
    }
    __syncthreads();
    uint32_t M0 = s_c1;  // max end before the wave's rows
    for (int i = 0; i < w; ++i) M0 = max(M0, s_wmax[i]);
    // run flags: row i starts a run iff max(ge before it) <= gs[i]; the max
    // before each round is kept (Mq) for the write-out below
    uint32_t flags = 0, Mq[RQ];
    {
        uint32_t M = M0;
#pragma unroll
        for (int q = 0; q < RQ; ++q) {
            Mq[q] = M;
            const uint32_t inc = dev::wave_inclusive_max(rmax[q]);
            uint32_t m = max(M, dev::wave_shr1(inc, 0u));
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int k = 4 * q + j;
                if (wb + 256 * q + 4 * lane + j < n && m <= s[k]) flags |= 1u << k;
                m = max(m, e[k]);
            }
            M = max(M, dev::lane63(inc));
        }
    }
    const uint32_t wcnt = dev::wave_reduce_sum((uint32_t)__popc(flags));
    if (lane == 0) s_wcnt[w] = wcnt;
    __syncthreads();
    // ---- chain 2: index of the tile's first run
    if (w == 0) {
        const uint32_t ctot = dev::wave_reduce_sum(lane < NW ? s_wcnt[lane] : 0u);
        uint64_t ex = 0;
        if (tile == 0) {
            if (lane == 0) st_publish(a.st_cnt, ST_INC | ctot);
        } else {
            if (lane == 0) st_publish(a.st_cnt + tile, ST_AGG | ctot);
            ex = lookback<false>(a.st_cnt, tile);
            if (lane == 0) st_publish(a.st_cnt + tile, ST_INC | (ex + ctot));
        }
        if (lane == 0) s_c2 = (uint32_t)ex;
    }
    __syncthreads();
    uint32_t r = s_c2;  // runs started before the wave's rows
    for (int i = 0; i < w; ++i) r += s_wcnt[i];
#pragma unroll
    for (int q = 0; q < RQ; ++q) {
        const uint32_t c = (uint32_t)__popc((flags >> (4 * q)) & 0xfu);
        const uint32_t ci = dev::wave_inclusive_sum(c);
        uint32_t rr = r + ci - c;  // runs started before this lane's rows
        const uint32_t inc = dev::wave_inclusive_max(rmax[q]);
        uint32_t m = max(Mq[q], dev::wave_shr1(inc, 0u));
        const int64_t i0 = wb + 256 * q + 4 * lane;
        uint32_t rid[4], pm[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int k = 4 * q + j;
            const int64_t i = i0 + j;
            if (i < n) {
                if (flags & (1u << k)) {
                    a.run_gs[rr] = s[k];
                    if (rr > 0) a.run_ge[rr - 1] = m;
                    ++rr;
                }
                if (i == n - 1) {
                    a.run_ge[rr - 1] = max(m, e[k]);
                    *a.total = rr;
                }
            }
            m = max(m, e[k]);
            rid[j] = rr - 1;
            pm[j] = m;
        }
        if (i0 + 4 <= n) {
            if (a.run_of_sorted)
                *reinterpret_cast<uint4 *>(a.run_of_sorted + i0) = make_uint4(rid[0], rid[1], rid[2], rid[3]);
            if (a.pmax) *reinterpret_cast<uint4 *>(a.pmax + i0) = make_uint4(pm[0], pm[1], pm[2], pm[3]);
        } else {
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if (i0 + j < n) {
                    if (a.run_of_sorted) a.run_of_sorted[i0 + j] = rid[j];
                    if (a.pmax) a.pmax[i0 + j] = pm[j];
                }
        }
        r += dev::lane63(ci);
    }
    if (TIE) {
        // a start shared by rows i and i + 16 (a same-start group past
        // subtract's TIE_G): row i + 16 is lane + 4's, the next round's for
        // lanes 60-63, whose sources (lanes 0-3) offer that round's rows
        // instead (past the wave's last round: the next rows, loaded here).
        // Tested last, once the ends are dead (before chain 1 it spilled)
        static_assert(MERGE_TIE_G == 16, "lane + 4 holds row i + 16");
        uint32_t nx[4] = {0u, 0u, 0u, 0u};
        if (lane < 4) {
            const int64_t i0 = wb + G2::RW + 4 * lane;
#pragma unroll
            for (int j = 0; j < 4; ++j) nx[j] = i0 + j < n ? a.gs[i0 + j] : 0u;
        }
        bool hit = false;
        const int src = (lane + 4) & 63;
#pragma unroll
        for (int q = 0; q < RQ; ++q)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint32_t v =
                    lane < 4 ? (q + 1 < RQ ? s[4 * (q + 1) + j] : nx[j]) : s[4 * q + j];
                const uint32_t p = __shfl(v, src);
                hit |= wb + 256 * q + 4 * lane + j + MERGE_TIE_G < n && p == s[4 * q + j];
            }
        if (__ballot(hit) != 0 && lane == 0) atomicOr(a.tie, 1u);
    }
}

// inclusive prefix max of ge (subtract's spanning-hit search)
__global__ __launch_bounds__(MB) void k_prefix_max(const uint32_t *__restrict__ ge, int64_t n,
                                                   const uint32_t *__restrict__ tpre,
                                                   uint32_t *__restrict__ pmax) {
    __shared__ uint32_t lds[MTILE];
    __shared__ uint32_t scratch[MB / 64 + 1];
    const int64_t base = (int64_t)blockIdx.x * MTILE;
    uint32_t e[MITEMS];
    load_blocked(ge, base, n, 0u, lds, e);
    uint32_t agg = 0;
#pragma unroll
    for (int k = 0; k < MITEMS; ++k) agg = max(agg, e[k]);
    uint32_t tot;
    uint32_t run = max(tpre[blockIdx.x], dev::block_exclusive_max<MB>(agg, 0u, scratch, &tot));
#pragma unroll
    for (int k = 0; k < MITEMS; ++k) {
        run = max(run, e[k]);
        lds[threadIdx.x * MITEMS + k] = run;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < MITEMS; ++k) {
        int64_t i = base + k * MB + threadIdx.x;
        if (i < n) pmax[i] = lds[k * MB + threadIdx.x];
    }
}

int tile_prefix(lime_ctx *ctx, const uint32_t *ge, int64_t n, uint32_t **tpre_out) {
    const int64_t nt = (n + MTILE - 1) / MTILE;
    uint32_t *tpre;
    LIME_TRY(alloc(ctx, &tpre, (size_t)nt));
    hipLaunchKernelGGL(k_tile_max, dim3((unsigned)nt), dim3(MB), 0, S(ctx), ge, n, tpre);
    hipLaunchKernelGGL(k_scan_max, dim3(1), dim3(MB), 0, S(ctx), tpre, nt);
    LIME_HIP(hipGetLastError());
    *tpre_out = tpre;
    return LIME_OK;
}

}  // namespace

int prefix_max_u32(lime_ctx *ctx, const uint32_t *in, uint32_t *out, int64_t n) {
    if (n <= 0) return LIME_OK;
    uint32_t *tpre;
    LIME_TRY(tile_prefix(ctx, in, n, &tpre));
    const int64_t nt = (n + MTILE - 1) / MTILE;
    hipLaunchKernelGGL(k_prefix_max, dim3((unsigned)nt), dim3(MB), 0, S(ctx), in, n,
                       (const uint32_t *)tpre, out);
    LIME_HIP(hipGetLastError());
    release(ctx, tpre);
    return LIME_OK;
}

// Lazily built state of a const set: built from and owned by the SET's
// context (operators already reject sets of another context), under that
// context's lock so two calls cannot both build it.
int build_prefix_max(lime_ctx *ctx, const lime_set *set) {
    if (set->ctx != ctx) return fail(LIME_ERR_ARG, "set belongs to another context");
    std::lock_guard<std::mutex> lock(set->ctx->mu);
    if (set->pmax) return LIME_OK;
    uint32_t *pm;
    LIME_TRY(alloc(set->ctx, &pm, (size_t)set->n));
    LIME_TRY(prefix_max_u32(set->ctx, set->ge, pm, set->n));
    set->pmax = pm;
    return LIME_OK;
}

// merge runs of a sorted set; result owns run_gs / run_ge / run_of_sorted
static int merge_runs_impl(lime_ctx *ctx, const lime_set *set, lime_result *res,
                           bool want_run_ids, uint32_t *pmax, int *tie_big = nullptr) {
    if (tie_big) *tie_big = -1;  // unknown unless k_merge_scan2 tests it
    const int64_t n = set->n;
    res->n = 0;
    if (n == 0) {
        LIME_TRY(alloc(ctx, &res->gs, 1));
        LIME_TRY(alloc(ctx, &res->ge, 1));
        return LIME_OK;
    }
    // plain sets: k_merge_scan2 (C3's merge 1.62 -> 1.41 ms); stranded sets
    // keep the transposing kernel's segmented scan
    const bool plain = set->strand_in == nullptr;
    const int64_t nt = (n + (plain ? G2::TILE : STILE) - 1) / (plain ? G2::TILE : STILE);
    // status words of both chains + ticket + total + tie flag in one zeroed
    // block
    uint64_t *st;
    LIME_TRY(alloc(ctx, &st, (size_t)(2 * nt + 3)));
    LIME_HIP(hipMemsetAsync(st, 0, sizeof(uint64_t) * (size_t)(2 * nt + 3), S(ctx)));
    uint32_t *run_gs, *run_ge;
    LIME_TRY(alloc(ctx, &run_gs, (size_t)n));
    LIME_TRY(alloc(ctx, &run_ge, (size_t)n));
    if (want_run_ids) LIME_TRY(alloc(ctx, &res->run_of_sorted, (size_t)n));
    int8_t *run_st = nullptr;  // stranded sets: the strand of every run
    if (set->strand_in) LIME_TRY(alloc(ctx, &run_st, (size_t)n));
    MergeScanArgs a;
    a.gs = set->gs;
    a.ge = set->ge;
    a.n = n;
    a.st_max = st;
    a.st_cnt = st + nt;
    a.ticket = reinterpret_cast<uint32_t *>(st + 2 * nt);
    a.total = st + 2 * nt + 1;
    a.run_gs = run_gs;
    a.run_ge = run_ge;
    a.run_of_sorted = res->run_of_sorted;
    a.pmax = pmax;
    a.strand = set->strand_in;
    a.row = set->strand_sorted ? nullptr : set->row;
    a.run_strand = run_st;
    a.tie = plain && tie_big ? reinterpret_cast<uint32_t *>(st + 2 * nt + 2) : nullptr;
    if (set->strand_in)
        hipLaunchKernelGGL(k_merge_scan<true>, dim3((unsigned)nt), dim3(SB), 0, S(ctx), a);
    else if (a.tie)
        hipLaunchKernelGGL(k_merge_scan2<true>, dim3((unsigned)nt), dim3(MS2), 0, S(ctx), a);
    else
        hipLaunchKernelGGL(k_merge_scan2<false>, dim3((unsigned)nt), dim3(MS2), 0, S(ctx), a);
    LIME_HIP(hipGetLastError());
    uint64_t nr = 0;
    if (a.tie) {
        uint64_t h[2] = {0, 0};  // total, tie flag: one read-back
        LIME_TRY(read_back(ctx, h, a.total, sizeof(h)));
        nr = h[0];
        *tie_big = h[1] != 0;
    } else {
        LIME_TRY(read_back(ctx, &nr, a.total, sizeof(nr)));
    }
    release(ctx, st);
    if (nr * 2 > (uint64_t)n) {
        // most rows start a run: keep the capacity-n arrays
        res->gs = run_gs;
        res->ge = run_ge;
        res->run_strand = run_st;
    } else {
        LIME_TRY(alloc(ctx, &res->gs, (size_t)nr));
        LIME_TRY(alloc(ctx, &res->ge, (size_t)nr));
        LIME_HIP(hipMemcpyAsync(res->gs, run_gs, sizeof(uint32_t) * nr, hipMemcpyDeviceToDevice,
                                S(ctx)));
        LIME_HIP(hipMemcpyAsync(res->ge, run_ge, sizeof(uint32_t) * nr, hipMemcpyDeviceToDevice,
                                S(ctx)));
        release(ctx, run_gs);
        release(ctx, run_ge);
        if (run_st) {
            LIME_TRY(alloc(ctx, &res->run_strand, (size_t)std::max<uint64_t>(nr, 1)));
            LIME_HIP(hipMemcpyAsync(res->run_strand, run_st, (size_t)nr, hipMemcpyDeviceToDevice,
                                    S(ctx)));
            release(ctx, run_st);
        }
    }
    res->n = (int64_t)nr;
    return LIME_OK;
}

int merge_runs(lime_ctx *ctx, const lime_set *set, lime_result *res, bool want_run_ids) {
    return merge_runs_impl(ctx, set, res, want_run_ids, nullptr);
}

// merge runs with run ids of a plain set, building the set's prefix max in
// the same pass when it is not built yet (under the set's context lock, as
// build_prefix_max).  *tie_big (may be null): 1 / 0 whether some start is
// shared by more than MERGE_TIE_G rows, -1 when not tested
int merge_runs_with_pmax(lime_ctx *ctx, const lime_set *set, lime_result *res, int *tie_big) {
    if (tie_big) *tie_big = -1;
    if (set->ctx != ctx) return fail(LIME_ERR_ARG, "set belongs to another context");
    if (set->strand_in || set->n == 0) {
        LIME_TRY(build_prefix_max(ctx, set));
        return merge_runs_impl(ctx, set, res, true, nullptr);
    }
    std::lock_guard<std::mutex> lock(set->ctx->mu);
    if (set->pmax) return merge_runs_impl(ctx, set, res, true, nullptr, tie_big);
    uint32_t *pm;
    LIME_TRY(alloc(set->ctx, &pm, (size_t)set->n));
    const int rc = merge_runs_impl(ctx, set, res, true, pm, tie_big);
    if (rc != LIME_OK) {
        release(set->ctx, pm);
        return rc;
    }
    set->pmax = pm;
    return LIME_OK;
}

}  // namespace lime

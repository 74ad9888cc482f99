// sort.hip -- the partition-and-sort stage: device LSD radix sort of an
// interval set into the canonical order (global start, zero-width first).
//
// Replaces ADAM repartitionAndSort() (cli/Intersection.scala:42-43,
// cli/Merge.scala:37, cli/Complement.scala:42) and the right-side
// repartitionAndSortWithinPartitions of OverlapBasedSetTheory.scala:81-82.
//
// Layout in HBM (SoA, 12 B per interval):
//   gs[i]  = off[contig] + start   (u32 global start, the sort key)
//   ge[i]  = off[contig] + end     (u32 global end)
//   row[i] = input row             (payload handle for T / U)
// Order: gs ascending; among equal gs, zero-width intervals first (the only
// tie order that changes a fold result, see DESIGN.md "canonical order");
// remaining ties keep input order (every pass is stable).
//
// Passes: an optional 1-bit pass on (ge > gs) when the set holds zero-width
// intervals (LSD: least-significant digit first), then ceil(bits(max gs)/8)
// 8-bit digit passes.  A pass = per-tile digit histogram, one exclusive scan
// over the digit-major count matrix, and a stable scatter that ranks items
// with wave ballots, stages the 8192-row tile in LDS in digit order and
// writes each digit's run contiguously (32 rows = 128 B per array and digit
// on average: whole L2 lines).  The first histogram is fused into the prep
// kernel that builds gs / ge / row from the caller's (contig, start, end).
#include "common.hpp"

#include <type_traits>

namespace lime {
namespace {

constexpr int RB = 512;
constexpr int RITEMS = 16;
constexpr int RTILE = RB * RITEMS;  // 8192 items per tile
constexpr int RBINS = 256;
constexpr int RWAVES = RB / 64;     // 8
constexpr int WITEMS = RTILE / RWAVES;  // 1024 consecutive rows per wave

struct SetStats {
    uint32_t err;        // bit0 contig out of range, bit1 end < start, bit2 end > contig length
    uint32_t max_gs;
    uint32_t min_width;
    uint32_t max_width;
    uint32_t has_zero;
    uint32_t unsorted;
    uint32_t pad[2];
};

// Pass kinds: an 8-bit digit of gs (M_GS); the zero-width bit (M_NZ, 0 =
// zero width); an 8-bit digit of the width ge - gs (M_GE: among equal gs,
// width order is end order); the strand code of the row (M_ST).  Stranded
// sets sort by (gs, ge, strand) -- RegionOrdering -- with passes ST (skipped
// when every row has one strand), GE x ceil(bits(max width) / 8), GS; plain
// sets by (gs, zero-width first) with NZ?, GS.
// M_RW: an 8-bit digit of the row id (the full (gs, ge, row) order of
// subtract's tie index, tie.hip)
enum { M_GS = 0, M_NZ = 1, M_GE = 2, M_ST = 3, M_RW = 4 };
// where a pass's row ids come from: none kept (binned sets), loaded, or the
// identity (the first pass of a set built from caller rows: row = position)
enum { ROWS_NONE = 0, ROWS_LOAD = 1, ROWS_IDENT = 2 };

// DB: digit bits of a GS pass (8; 9 for the bucketed sort's wider passes)
template <int M, int DB = 8>
__device__ __forceinline__ uint32_t digit_of(uint32_t k, uint32_t e, uint32_t r, int shift,
                                             const int8_t *st) {
    if (M == M_NZ) return e > k ? 1u : 0u;
    if (M == M_GE) return ((e - k) >> shift) & (RBINS - 1);
    // strand codes 0 independent, 1 forward, 2 reverse, 3 unknown sort by
    // bdg-formats' enum ordinal: FORWARD, REVERSE, INDEPENDENT, UNKNOWN
    if (M == M_ST) return (0xd2u >> (2 * ((uint32_t)(uint8_t)st[r] & 3u))) & 3u;
    if (M == M_RW) return (r >> shift) & (RBINS - 1);
    return (k >> shift) & ((1u << DB) - 1u);
}

// lanes of the wave holding the same digit (among `valid` lanes)
template <int M, int DB = 8>
__device__ __forceinline__ uint64_t match_digit(uint32_t d, bool valid) {
    uint64_t m = __ballot(valid);
    if (M == M_ST) {
#pragma unroll
        for (int b = 0; b < 2; ++b) {
            uint32_t bit = (d >> b) & 1u;
            uint64_t bb = __ballot(bit);
            m &= bit ? bb : ~bb;
        }
        return m;
    }
    if (M == M_NZ) {
        uint64_t b = __ballot(d & 1u);
        return m & ((d & 1u) ? b : ~b);
    }
#pragma unroll
    for (int b = 0; b < DB; ++b) {
        uint32_t bit = (d >> b) & 1u;
        uint64_t bb = __ballot(bit);
        m &= bit ? bb : ~bb;
    }
    return m;
}

__global__ __launch_bounds__(256) void k_rows_iota(uint32_t *__restrict__ r, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) r[i] = (uint32_t)i;
}

// bijective blockIdx -> tile map giving each XCD (blockIdx % 8) a contiguous
// range of tiles (MI355X_MICROARCH.md: workgroups are dealt round-robin)
__device__ __forceinline__ uint32_t xcd_swizzle(uint32_t bid, uint32_t ntiles) {
    const uint32_t q = ntiles / 8, r = ntiles % 8, x = bid % 8, i = bid / 8;
    return x * q + (x < r ? x : r) + i;
}

// (tile = the block's tile: consecutive tiles on one XCD, so the digit-major
// column stores of neighbouring tiles complete each other's lines in its L2)
template <int BINS>
__device__ __forceinline__ void flush_hist(uint32_t (*hist)[BINS], uint32_t *counts,
                                           uint32_t ntiles, uint32_t tile) {
    for (int d = threadIdx.x; d < BINS; d += RB) {
        uint32_t t = 0;
#pragma unroll
        for (int ww = 0; ww < RWAVES; ++ww) t += hist[ww][d];
        counts[(int64_t)d * ntiles + tile] = t;
    }
}

// Build gs / ge / row from (contig, start, end), validate, gather statistics
// (per-tile partials, reduced by k_stats) and the digit-0 histogram.
// GLOBAL: the input is already (gs, ge, row) in global coordinates (rows of
// sets of this space, e.g. a shard's own rows + its halo); `contig` / `start`
// / `end` then carry gs / ge / row and only order and span are validated.
// WRITE = false: only validate, gather statistics and histogram -- the first
// radix pass then reads the caller's rows itself (k_scatter RAW for plain
// rows, the caller's (gs, ge, row) for global ones), so nothing is written
// and read back in between (the bucketed sort).
// LC: the contig table (<= PCMAX contigs) is staged in LDS, so the per-row
// off / len gathers are LDS reads rather than dependent cache round trips
constexpr int PCMAX = 1024;
// W16 (caller rows, WRITE): ge receives the u16 width ge - gs, not the end
// (the bucketed sort's first pass then reads 6 B per row; a set with a width
// past 2^16 discards it and reads the caller's rows instead)
template <bool GLOBAL, bool WRITE = true, bool LC = false, int DB = 8, bool W16 = false>
__global__ __launch_bounds__(RB) void k_prep(const int32_t *__restrict__ contig,
                                             const uint32_t *__restrict__ start,
                                             const uint32_t *__restrict__ end,
                                             const uint32_t *__restrict__ goff,
                                             const uint32_t *__restrict__ glen, int32_t n_contigs,
                                             int64_t n, uint32_t *__restrict__ gs,
                                             uint32_t *__restrict__ ge, uint32_t *__restrict__ row,
                                             SetStats *__restrict__ part,
                                             uint32_t *__restrict__ counts, uint32_t ntiles,
                                             int hshift) {
    constexpr int BINS = 1 << DB;
    static_assert(!(GLOBAL && W16), "u16 widths from caller rows only");
    __shared__ uint32_t hist[RWAVES][BINS];
    __shared__ SetStats ws[RWAVES];
    __shared__ uint32_t s_off[LC ? PCMAX : 1], s_len[LC ? PCMAX : 1];
    for (int i = threadIdx.x; i < RWAVES * BINS; i += RB) (&hist[0][0])[i] = 0;
    if (LC) {
        for (int i = threadIdx.x; i < n_contigs; i += RB) {
            s_off[i] = goff[i];
            s_len[i] = glen[i];
        }
        __syncthreads();
    }
    const uint32_t *off = LC ? s_off : goff, *len = LC ? s_len : glen;
    const int w = threadIdx.x / 64, lane = dev::lane_id();
    const uint32_t tile = xcd_swizzle(blockIdx.x, ntiles);
    const int64_t base = (int64_t)tile * RTILE + w * WITEMS;
    uint32_t err = 0, mx = 0, mnw = 0xffffffffu, mxw = 0, zero = 0, uns = 0;
    uint32_t vk[RITEMS], ve[RITEMS];
    bool valid[RITEMS];
    if (GLOBAL) {
        const uint32_t *igs = reinterpret_cast<const uint32_t *>(contig);
        const uint32_t span = off[n_contigs];
#pragma unroll
        for (int k = 0; k < RITEMS; ++k) {
            const int64_t i = base + k * 64 + lane;
            valid[k] = i < n;
            uint32_t g0 = 0, g1 = 0;
            if (valid[k]) {
                g0 = igs[i];
                g1 = start[i];
                if (g1 < g0) err |= 2u;
                if (g1 >= span) err |= 4u;
                if (WRITE) {
                    gs[i] = g0;
                    ge[i] = g1;
                    if (row) row[i] = end[i];
                }
                mx = g0 > mx ? g0 : mx;
                const uint32_t wd = g1 - g0;
                mnw = wd < mnw ? wd : mnw;
                mxw = wd > mxw ? wd : mxw;
                zero |= (wd == 0);
                if (i > 0) {
                    const uint32_t p0 = igs[i - 1], p1 = start[i - 1];
                    if (p0 > g0 || (p0 == g0 && p1 > p0 && g1 == g0)) uns = 1;
                }
            }
            vk[k] = g0;
            ve[k] = g1;
        }
    } else if (base + WITEMS <= n) {
        // full wave chunk: 16-B loads and stores, 4 consecutive rows per lane
        // (the histogram below ignores order, so vk / ve may be held in any order)
        const int4 *c4 = reinterpret_cast<const int4 *>(contig + base);
        const uint4 *s4 = reinterpret_cast<const uint4 *>(start + base);
        const uint4 *e4 = reinterpret_cast<const uint4 *>(end + base);
        uint4 *g4 = reinterpret_cast<uint4 *>(gs + base);
        uint4 *h4 = reinterpret_cast<uint4 *>(ge + base);
        uint4 *r4 = reinterpret_cast<uint4 *>(row + base);
        // every load issued before any is used (12 x 16 B per lane in flight:
        // one iteration's loads at a time held the prep at 4.1 TB/s), and the
        // row before the wave's chunk (lane 0's predecessor in iteration 0;
        // in later iterations it is lane 63's last row of the one before)
        int4 cv[RITEMS / 4];
        uint4 sv[RITEMS / 4], ev[RITEMS / 4];
#pragma unroll
        for (int k = 0; k < RITEMS / 4; ++k) {
            const int q = k * 64 + lane;
            cv[k] = c4[q];
            sv[k] = s4[q];
            ev[k] = e4[q];
        }
        int32_t bc = -1;
        uint32_t bs = 0, be = 0;
        if (lane == 0 && base > 0) {
            bc = contig[base - 1];
            bs = start[base - 1];
            be = end[base - 1];
        }
        uint32_t l0 = 0, l1 = 0, lok = 0;  // lane 63's last row of the previous iteration
#pragma unroll
        for (int k = 0; k < RITEMS / 4; ++k) {
            const int q = k * 64 + lane;
            const int32_t cc[4] = {cv[k].x, cv[k].y, cv[k].z, cv[k].w};
            const uint32_t ss[4] = {sv[k].x, sv[k].y, sv[k].z, sv[k].w},
                           ee[4] = {ev[k].x, ev[k].y, ev[k].z, ev[k].w};
            uint32_t a0[4], a1[4], ok[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int32_t c = cc[j];
                ok[j] = c >= 0 && c < n_contigs;
                a0[j] = a1[j] = 0;
                if (!ok[j]) {
                    err |= 1u;
                } else {
                    if (ee[j] < ss[j]) err |= 2u;
                    if (ee[j] > len[c]) err |= 4u;
                    a0[j] = off[c] + ss[j];
                    a1[j] = off[c] + ee[j];
                }
                mx = a0[j] > mx ? a0[j] : mx;
                const uint32_t wd = a1[j] - a0[j];
                mnw = wd < mnw ? wd : mnw;
                mxw = wd > mxw ? wd : mxw;
                zero |= (wd == 0);
                vk[4 * k + j] = a0[j];
                ve[4 * k + j] = a1[j];
            }
            // canonical-order check: the row before this lane's first row is
            // the previous lane's last one
            uint32_t p0 = dev::wave_shr1(a0[3], 0u), p1 = dev::wave_shr1(a1[3], 0u),
                     pok = dev::wave_shr1(ok[3], 0u);
            const int64_t i0 = base + 4 * (int64_t)q;
            if (lane == 0) {
                if (k > 0) {
                    p0 = l0, p1 = l1, pok = lok;
                } else {
                    pok = bc >= 0 && bc < n_contigs;
                    if (pok) {
                        p0 = off[bc] + bs;
                        p1 = off[bc] + be;
                    }
                }
            }
            l0 = (uint32_t)__builtin_amdgcn_readlane((int)a0[3], 63);
            l1 = (uint32_t)__builtin_amdgcn_readlane((int)a1[3], 63);
            lok = (uint32_t)__builtin_amdgcn_readlane((int)ok[3], 63);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                if (pok && ok[j] && (p0 > a0[j] || (p0 == a0[j] && p1 > p0 && a1[j] == a0[j])))
                    uns = 1;
                p0 = a0[j], p1 = a1[j], pok = ok[j];
            }
            if (WRITE && W16) {
                g4[q] = make_uint4(a0[0], a0[1], a0[2], a0[3]);
                reinterpret_cast<uint2 *>(reinterpret_cast<uint16_t *>(ge) + base)[q] =
                    make_uint2(((a1[0] - a0[0]) & 0xffffu) | (a1[1] - a0[1]) << 16,
                               ((a1[2] - a0[2]) & 0xffffu) | (a1[3] - a0[3]) << 16);
            } else if (WRITE) {
                g4[q] = make_uint4(a0[0], a0[1], a0[2], a0[3]);
                h4[q] = make_uint4(a1[0], a1[1], a1[2], a1[3]);
            }
            if (row)
                r4[q] = make_uint4((uint32_t)i0, (uint32_t)i0 + 1, (uint32_t)i0 + 2,
                                   (uint32_t)i0 + 3);
        }
#pragma unroll
        for (int k = 0; k < RITEMS; ++k) valid[k] = true;
    } else {
#pragma unroll
    for (int k = 0; k < RITEMS; ++k) {
        const int64_t i = base + k * 64 + lane;
        valid[k] = i < n;
        uint32_t g0 = 0, g1 = 0;
        if (valid[k]) {
            const int32_t c = contig[i];
            const uint32_t s = start[i], e = end[i];
            if (c < 0 || c >= n_contigs) {
                err |= 1u;
            } else {
                if (e < s) err |= 2u;
                if (e > len[c]) err |= 4u;
                g0 = off[c] + s;
                g1 = off[c] + e;
            }
            if (WRITE) {
                gs[i] = g0;
                if (W16)
                    reinterpret_cast<uint16_t *>(ge)[i] = (uint16_t)(g1 - g0);
                else
                    ge[i] = g1;
            }
            if (row) row[i] = (uint32_t)i;
            mx = g0 > mx ? g0 : mx;
            const uint32_t wd = g1 - g0;
            mnw = wd < mnw ? wd : mnw;
            mxw = wd > mxw ? wd : mxw;
            zero |= (wd == 0);
            if (i > 0) {  // canonical-order check against the previous row
                const int32_t pc = contig[i - 1];
                if (pc >= 0 && pc < n_contigs && c >= 0 && c < n_contigs) {
                    const uint32_t p0 = off[pc] + start[i - 1], p1 = off[pc] + end[i - 1];
                    if (p0 > g0 || (p0 == g0 && p1 > p0 && g1 == g0)) uns = 1;
                }
            }
        }
        vk[k] = g0;
        ve[k] = g1;
    }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < RITEMS; ++k)
        if (valid[k]) atomicAdd(&hist[w][(vk[k] >> hshift) & (BINS - 1)], 1u);
    err = dev::wave_reduce_or(err);
    mx = dev::wave_reduce_max(mx);
    mnw = dev::wave_reduce_min(mnw);
    mxw = dev::wave_reduce_max(mxw);
    zero = dev::wave_reduce_or(zero);
    uns = dev::wave_reduce_or(uns);
    if (lane == 0) ws[w] = SetStats{err, mx, mnw, mxw, zero, uns, {0, 0}};
    __syncthreads();
    flush_hist(hist, counts, ntiles, tile);
    if (threadIdx.x == 0) {
        SetStats s = ws[0];
        for (int i = 1; i < RWAVES; ++i) {
            s.err |= ws[i].err;
            s.max_gs = max(s.max_gs, ws[i].max_gs);
            s.min_width = min(s.min_width, ws[i].min_width);
            s.max_width = max(s.max_width, ws[i].max_width);
            s.has_zero |= ws[i].has_zero;
            s.unsorted |= ws[i].unsorted;
        }
        part[blockIdx.x] = s;
    }
}

__global__ __launch_bounds__(256) void k_stats(const SetStats *__restrict__ part, int64_t m,
                                               SetStats *out) {
    uint32_t err = 0, mx = 0, mnw = 0xffffffffu, mxw = 0, zero = 0, uns = 0;
    for (int64_t i = threadIdx.x; i < m; i += 256) {
        const SetStats s = part[i];
        err |= s.err;
        mx = max(mx, s.max_gs);
        mnw = min(mnw, s.min_width);
        mxw = max(mxw, s.max_width);
        zero |= s.has_zero;
        uns |= s.unsorted;
    }
    __shared__ SetStats ws[4];
    err = dev::wave_reduce_or(err);
    mx = dev::wave_reduce_max(mx);
    mnw = dev::wave_reduce_min(mnw);
    mxw = dev::wave_reduce_max(mxw);
    zero = dev::wave_reduce_or(zero);
    uns = dev::wave_reduce_or(uns);
    if (dev::lane_id() == 0) ws[threadIdx.x / 64] = SetStats{err, mx, mnw, mxw, zero, uns, {0, 0}};
    __syncthreads();
    if (threadIdx.x == 0) {
        SetStats s = ws[0];
        for (int i = 1; i < 4; ++i) {
            s.err |= ws[i].err;
            s.max_gs = max(s.max_gs, ws[i].max_gs);
            s.min_width = min(s.min_width, ws[i].min_width);
            s.max_width = max(s.max_width, ws[i].max_width);
            s.has_zero |= ws[i].has_zero;
            s.unsorted |= ws[i].unsorted;
        }
        *out = s;
    }
}

template <int M, int DB = 8>
__global__ __launch_bounds__(RB) void k_hist(const uint32_t *__restrict__ key,
                                             const uint32_t *__restrict__ ge,
                                             const uint32_t *__restrict__ row, int64_t n, int shift,
                                             const int8_t *__restrict__ st,
                                             uint32_t *__restrict__ counts, uint32_t ntiles,
                                             int rows) {
    constexpr int BINS = M == M_GS ? 1 << DB : RBINS;
    __shared__ uint32_t hist[RWAVES][BINS];
    for (int i = threadIdx.x; i < RWAVES * BINS; i += RB) (&hist[0][0])[i] = 0;
    const int w = threadIdx.x / 64, lane = dev::lane_id();
    const uint32_t tile = xcd_swizzle(blockIdx.x, ntiles);
    const int64_t base = (int64_t)tile * RTILE + w * WITEMS;
    constexpr bool NEED_E = M == M_NZ || M == M_GE;
    uint32_t vk[RITEMS], ve[RITEMS], vr[RITEMS];
    bool valid[RITEMS];
    if (base + WITEMS <= n) {
        // a histogram ignores order: 16-B loads, 4 consecutive rows per lane
        const uint4 *k4 = reinterpret_cast<const uint4 *>(key + base);
        const uint4 *e4 = reinterpret_cast<const uint4 *>(ge + base);
        const uint4 *r4 = reinterpret_cast<const uint4 *>(row + base);
#pragma unroll
        for (int k = 0; k < RITEMS / 4; ++k) {
            const uint4 v = k4[k * 64 + lane];
            vk[4 * k] = v.x, vk[4 * k + 1] = v.y, vk[4 * k + 2] = v.z, vk[4 * k + 3] = v.w;
            if (NEED_E) {
                const uint4 u = e4[k * 64 + lane];
                ve[4 * k] = u.x, ve[4 * k + 1] = u.y, ve[4 * k + 2] = u.z, ve[4 * k + 3] = u.w;
            } else {
                ve[4 * k] = ve[4 * k + 1] = ve[4 * k + 2] = ve[4 * k + 3] = 0u;
            }
            if ((M == M_ST || M == M_RW) && rows == ROWS_IDENT) {
                const uint32_t r = (uint32_t)(base + 4 * (k * 64 + lane));
                vr[4 * k] = r, vr[4 * k + 1] = r + 1, vr[4 * k + 2] = r + 2, vr[4 * k + 3] = r + 3;
            } else if (M == M_ST || M == M_RW) {
                const uint4 u = r4[k * 64 + lane];
                vr[4 * k] = u.x, vr[4 * k + 1] = u.y, vr[4 * k + 2] = u.z, vr[4 * k + 3] = u.w;
            } else {
                vr[4 * k] = vr[4 * k + 1] = vr[4 * k + 2] = vr[4 * k + 3] = 0u;
            }
        }
#pragma unroll
        for (int k = 0; k < RITEMS; ++k) valid[k] = true;
    } else {
#pragma unroll
        for (int k = 0; k < RITEMS; ++k) {
            const int64_t i = base + k * 64 + lane;
            valid[k] = i < n;
            vk[k] = valid[k] ? key[i] : 0u;
            ve[k] = (NEED_E && valid[k]) ? ge[i] : 0u;
            vr[k] = ((M == M_ST || M == M_RW) && valid[k]) ? (rows == ROWS_IDENT ? (uint32_t)i : row[i]) : 0u;
        }
    }
    __syncthreads();
    // LDS atomics, not the scatter's 8 ballots per row: a histogram needs no
    // ranks (190 -> 104 us per 1e8-row pass)
#pragma unroll
    for (int k = 0; k < RITEMS; ++k)
        if (valid[k]) atomicAdd(&hist[w][digit_of<M, DB>(vk[k], ve[k], vr[k], shift, st)], 1u);
    __syncthreads();
    flush_hist(hist, counts, ntiles, tile);
}

// The bucketed sort's second histogram (DB2 bits at L + DB1, over pass 1's
// output, whose rows are ordered by the first digit d1 = bits [L, L + DB1))
// and the partials that place every bucket without reading its keys again:
// the rows of first digit D form one region of pass 1's output; for every D
// whose region starts inside this tile (D in (d1 of the row before the
// tile, d1 of the tile's last row]), part[D][d2] = the tile's rows with
// second digit d2 and d1 < D.  Bucket (d2, D) then starts at the scanned
// count of (d2, the tile) + part[D][d2] (k_bucket_starts_part).  Most tiles
// lie inside one region and only histogram.
template <int DB1, int DB2>
__global__ __launch_bounds__(RB) void k_hist_part(const uint32_t *__restrict__ key, int64_t n,
                                                  int L, uint32_t *__restrict__ counts,
                                                  uint32_t ntiles, uint32_t *__restrict__ part) {
    constexpr int B1 = 1 << DB1, B2 = 1 << DB2, PC = 16;  // first digits per partial round
    __shared__ uint32_t hist[RWAVES][B2];
    __shared__ uint32_t ph[PC + 1][B2];  // [0]: rows below the round's first D
    for (int i = threadIdx.x; i < RWAVES * B2; i += RB) (&hist[0][0])[i] = 0;
    const int w = threadIdx.x / 64, lane = dev::lane_id();
    const uint32_t tile = xcd_swizzle(blockIdx.x, ntiles);
    const int64_t tile0 = (int64_t)tile * RTILE, base = tile0 + w * WITEMS;
    const int s2 = L + DB1;
    uint32_t vk[RITEMS];
    bool valid[RITEMS];
    if (base + WITEMS <= n) {
        const uint4 *k4 = reinterpret_cast<const uint4 *>(key + base);
#pragma unroll
        for (int k = 0; k < RITEMS / 4; ++k) {
            const uint4 v = k4[k * 64 + lane];
            vk[4 * k] = v.x, vk[4 * k + 1] = v.y, vk[4 * k + 2] = v.z, vk[4 * k + 3] = v.w;
        }
#pragma unroll
        for (int k = 0; k < RITEMS; ++k) valid[k] = true;
    } else {
#pragma unroll
        for (int k = 0; k < RITEMS; ++k) {
            const int64_t i = base + k * 64 + lane;
            valid[k] = i < n;
            vk[k] = valid[k] ? key[i] : 0u;
        }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < RITEMS; ++k)
        if (valid[k]) atomicAdd(&hist[w][(vk[k] >> s2) & (B2 - 1)], 1u);
    __syncthreads();
    flush_hist(hist, counts, ntiles, tile);
    // (uniform: every thread reads the same two keys)
    const int64_t tend = tile0 + RTILE < n ? tile0 + RTILE : n;
    const int prev = tile0 > 0 ? (int)((key[tile0 - 1] >> L) & (B1 - 1)) : -1;
    const int last = (int)((key[tend - 1] >> L) & (B1 - 1));
    for (int c0 = prev + 1; c0 <= last; c0 += PC) {
        __syncthreads();  // (ph reused by the previous round)
        for (int i = threadIdx.x; i < (PC + 1) * B2; i += RB) (&ph[0][0])[i] = 0;
        __syncthreads();
#pragma unroll
        for (int k = 0; k < RITEMS; ++k) {
            const int d1 = (int)((vk[k] >> L) & (B1 - 1));
            if (valid[k] && d1 < c0 + PC)
                atomicAdd(&ph[d1 < c0 ? 0 : 1 + d1 - c0][(vk[k] >> s2) & (B2 - 1)], 1u);
        }
        __syncthreads();
        for (int d2 = threadIdx.x; d2 < B2; d2 += RB) {
            uint32_t run = ph[0][d2];
            for (int j = 0; j < PC && c0 + j <= last; ++j) {
                part[(int64_t)(c0 + j) * B2 + d2] = run;
                run += ph[1 + j][d2];
            }
        }
    }
}

// bucket b = (d2 << DB1) | D (= gs >> L) starts at pass 2's scanned count of
// (d2, the tile where D's region starts) + part[D][d2]; a D without rows
// (its region starts at n) puts every (d2, D) at the end of d2's rows.
// start[nb] = n.  dstart1[D]: pass 1's scanned count of (D, tile 0).
__global__ __launch_bounds__(256) void k_bucket_starts_part(
    const uint32_t *__restrict__ dstart1, const uint32_t *__restrict__ mat2,
    const uint32_t *__restrict__ part, int64_t n, uint32_t ntiles, uint32_t nb, int DB1, int DB2,
    uint32_t *__restrict__ start) {
    const int64_t b = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (b > nb) return;
    if (b == nb) {
        start[b] = (uint32_t)n;
        return;
    }
    const uint32_t D = (uint32_t)b & ((1u << DB1) - 1u), d2 = (uint32_t)(b >> DB1);
    const uint32_t ds = dstart1[D];
    if ((int64_t)ds >= n)
        start[b] = d2 + 1 < (1u << DB2) ? mat2[(int64_t)(d2 + 1) * ntiles] : (uint32_t)n;
    else
        start[b] = mat2[(int64_t)d2 * ntiles + ds / RTILE] + part[((int64_t)D << DB2) + d2];
}

// column 0 of a digit-major count matrix: the scanned start of every digit
__global__ __launch_bounds__(256) void k_take_col0(const uint32_t *__restrict__ mat,
                                                   uint32_t ntiles, int nd,
                                                   uint32_t *__restrict__ out) {
    const int d = blockIdx.x * 256 + threadIdx.x;
    if (d < nd) out[d] = mat[(int64_t)d * ntiles];
}

// RAW (first pass over caller rows only): key_in / ge_in / row_in are the
// caller's contig / start / end, and (gs, ge) = off[contig] + (start, end)
// EW (GS passes of sets narrower than 2^16 bases): how the ends travel.
// Between the first and the last pass only the width ge - gs is carried, as
// u16 (10 B per row and pass instead of 12): the first pass turns ends into
// widths (EW_TO16), the middle ones move widths (EW_16), the last turns them
// back into ends (EW_FROM16, ge = gs + width, gs staged beside it)
// (RAW passes may start the u16 widths: EW_TO16 from the caller's ends.)
// DB: digit bits of a GS pass.  9-bit passes (the bucketed sort of dense
// sets: 512 digits, runs of ~16 rows per digit and tile) keep their per-wave
// digit counters as u16 and the RAW contig table aliased onto the staging
// array, so two workgroups still fit a CU (~76 KiB LDS each)
// EW_PACK (the bucketed sort's last digit pass): reads u16 widths like
// EW_FROM16 and writes ONE word per row, (gs mod 2^L) << 16 | width (the
// bucket id gs >> L is implied by the position: k_bucket_starts_part), so the
// pass writes 8 B per row and the local sort reads 8 instead of 12
enum { EW_32 = 0, EW_TO16 = 1, EW_16 = 2, EW_FROM16 = 3, EW_PACK = 4 };
template <int M, int ROWS, bool RAW = false, int EW = EW_32, int DB = 8>
// 2 workgroups per CU (4 waves per SIMD): <= 128 VGPRs, ~70 KiB LDS each
__global__ __launch_bounds__(RB, 4) void k_scatter(const uint32_t *__restrict__ key_in,
                                                const uint32_t *__restrict__ ge_in,
                                                const uint32_t *__restrict__ row_in, int64_t n,
                                                int shift, const int8_t *__restrict__ st,
                                                const uint32_t *__restrict__ base_mat,
                                                uint32_t ntiles, uint32_t *__restrict__ key_out,
                                                uint32_t *__restrict__ ge_out,
                                                uint32_t *__restrict__ row_out,
                                                const uint32_t *__restrict__ off = nullptr,
                                                int32_t nc = 0, int lbits = 0) {
    constexpr int BINS = M == M_GS ? 1 << DB : RBINS;
    static_assert(M == M_GS || DB == 8, "wider digits: GS passes only");
    using CT = typename std::conditional<(DB > 8), uint16_t, uint32_t>::type;
    __shared__ CT cnt[RWAVES][BINS];
    __shared__ uint32_t dstart[BINS];
    __shared__ uint32_t gbase[BINS];
    __shared__ uint32_t scratch[RWAVES + 1];
    constexpr bool ALL3 = M != M_GS;  // digit not recomputable from the key alone
    static_assert(EW == EW_32 || M == M_GS, "u16 widths: GS passes only");
    static_assert(!RAW || EW == EW_32 || EW == EW_TO16, "a RAW pass reads the caller's ends");
    static_assert(EW != EW_PACK || ROWS == ROWS_LOAD, "the packed pass keeps loaded rows");
    __shared__ uint32_t sk[RTILE], se[RTILE], sr[ALL3 ? RTILE : 1];
    // RAW: the contig table staged in LDS (<= PCMAX contigs), so the per-row
    // off[contig] gather is an LDS read, not a dependent cache round trip.
    // It lives in se: its lookups all precede the barrier after the loads,
    // and se is written only after two more
    static_assert(PCMAX <= RTILE, "contig table within the staging array");
    uint32_t *s_off = se;
    if (RAW && nc <= PCMAX)  // (its barrier follows the tile's loads)
        for (int i = threadIdx.x; i < nc; i += RB) s_off[i] = off[i];
    const uint32_t *offp = RAW && nc <= PCMAX ? s_off : off;

    for (int i = threadIdx.x; i < RWAVES * BINS; i += RB) (&cnt[0][0])[i] = 0;

    const int w = threadIdx.x / 64, lane = dev::lane_id();
    // XCD-aware tile order: consecutive tiles run on one XCD, so the partial
    // 128-B lines where a digit's run of tile t meets the same digit's run
    // of tile t+1 are completed in one L2 instead of being written back
    // half-filled by two XCDs (blocks are dealt round-robin over 8 XCDs;
    // speed only -- any placement gives the same result)
    const uint32_t tile = xcd_swizzle(blockIdx.x, ntiles);
    const int64_t tile0 = (int64_t)tile * RTILE;
    const int64_t base = tile0 + w * WITEMS;
    // pd[k] = (position among the wave's rows of its digit) << 8 | digit;
    // packed to keep the kernel within 128 VGPRs (2 workgroups per CU)
    uint32_t vk[RITEMS], ve[RITEMS], vr[RITEMS], pd[RITEMS];
    // 32-bit offsets from per-wave base pointers keep address math scalar
    const int lim = (int)min((int64_t)WITEMS, n - base);  // valid rows of this wave
    // ROWS_NONE (GS passes of binned sets): no row ids are kept;
    // ROWS_IDENT (first pass over caller rows): row id = position
    const uint32_t *kin = key_in + base, *ein = ge_in + base, *rin = row_in + base;
#pragma unroll
    for (int k = 0; k < RITEMS; ++k) {
        const int o = k * 64 + lane;
        const bool valid = o < lim;
        if (RAW) {  // the contig ids (in vr), starts and ends: all loads first
            vr[k] = valid ? kin[o] : 0u;
            vk[k] = valid ? ein[o] : 0u;
            ve[k] = valid ? rin[o] : 0u;
        } else if (EW == EW_16 || EW == EW_FROM16 || EW == EW_PACK) {
            vk[k] = valid ? kin[o] : 0u;
            ve[k] = valid ? (uint32_t)reinterpret_cast<const uint16_t *>(ge_in)[base + o] : 0u;
        } else {
            vk[k] = valid ? kin[o] : 0u;
            ve[k] = valid ? ein[o] : 0u;
            if (EW == EW_TO16) ve[k] -= vk[k];  // (< 2^16: checked by the caller)
        }
        // (GS passes write identity rows straight from the position below,
        // keeping vr out of the registers of that path)
        if (!RAW)
            vr[k] = ROWS == ROWS_IDENT && M != M_GS ? (uint32_t)(base + o)
                    : ROWS == ROWS_LOAD             ? (valid ? rin[o] : 0u)
                                                    : 0u;
    }
    if (RAW) {
        // (gs, ge) = off[contig] + (start, end), the table in LDS; the
        // lookups follow every load of the tile (one dependent round trip
        // per item serialised the loads: 1.14 ms per 1e8 rows)
        if (nc <= PCMAX) __syncthreads();  // s_off staged
#pragma unroll
        for (int k = 0; k < RITEMS; ++k) {
            const uint32_t o = offp[vr[k]];  // (vr = 0 for invalid rows: in range)
            vk[k] += o;
            ve[k] += o;
            if (EW == EW_TO16) ve[k] -= vk[k];  // (< 2^16: checked by the caller)
            vr[k] = 0u;
        }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < RITEMS; ++k) {
        const bool valid = k * 64 + lane < lim;
        const uint32_t d = valid ? digit_of<M, DB>(vk[k], ve[k], vr[k], shift, st) : 0u;
        const uint64_t m = match_digit<M, DB>(d, valid);
        const uint32_t rank = (uint32_t)__popcll(m & dev::lanemask_lt());
        const uint32_t old = valid ? (uint32_t)cnt[w][d] : 0u;
        pd[k] = ((old + rank) << DB) | d;
        if (valid && rank == 0) cnt[w][d] = (CT)(old + (uint32_t)__popcll(m));
    }
    __syncthreads();
    // per digit: block offset of the digit, then per-wave offsets
    static_assert(BINS <= RB, "one digit per thread in the offset scan");
    {
        const int d = threadIdx.x;
        uint32_t tot = 0;
        if (d < BINS)
            for (int ww = 0; ww < RWAVES; ++ww) tot += cnt[ww][d];
        uint32_t all;
        const uint32_t ds = dev::block_exclusive_sum<RB>(tot, scratch, &all);
        if (d < BINS) {
            dstart[d] = ds;
            uint32_t run = ds;
            for (int ww = 0; ww < RWAVES; ++ww) {
                const uint32_t c = cnt[ww][d];
                cnt[ww][d] = (CT)run;
                run += c;
            }
            gbase[d] = base_mat[(int64_t)d * ntiles + tile];
        }
    }
    __syncthreads();
    const int64_t rem = n - tile0;
    const int count = rem < RTILE ? (int)rem : RTILE;
    uint32_t *lp = pd;  // local position within the tile, in place
#pragma unroll
    for (int k = 0; k < RITEMS; ++k)
        lp[k] = k * 64 + lane < lim ? (uint32_t)cnt[w][pd[k] & (BINS - 1)] + (pd[k] >> DB)
                                    : 0xffffffffu;
    if (ALL3) {  // digit needs (key, end, row): stage all three arrays at once
#pragma unroll
        for (int k = 0; k < RITEMS; ++k)
            if (lp[k] != 0xffffffffu) {
                sk[lp[k]] = vk[k];
                se[lp[k]] = ve[k];
                sr[lp[k]] = vr[k];
            }
        __syncthreads();
        for (int j = threadIdx.x; j < count; j += RB) {
            const uint32_t k = sk[j], e = se[j];
            const uint32_t d = digit_of<M>(k, e, sr[j], shift, st);
            const uint32_t g = gbase[d] + (uint32_t)j - dstart[d];
            key_out[g] = k;
            ge_out[g] = e;
            row_out[g] = sr[j];
        }
        return;
    }
    // keys and ends staged together (sk, se) and stored by one loop, then
    // the rows through se: 64 KiB of staging, two workgroups per CU, two
    // store rounds (keys, ends, rows in three rounds: C3's first pass
    // 2.21 ms against 2.05 for the packed second pass's two)
#pragma unroll
    for (int k = 0; k < RITEMS; ++k)
        if (lp[k] != 0xffffffffu) {
            sk[lp[k]] = vk[k];
            se[lp[k]] = ve[k];
        }
    __syncthreads();
    {
        const uint32_t lmask = (1u << lbits) - 1u;
        for (int j = threadIdx.x; j < count; j += RB) {
            const uint32_t k = sk[j], e = se[j];
            const uint32_t d = digit_of<M, DB>(k, 0u, 0u, shift, st);
            const uint32_t g = gbase[d] + (uint32_t)j - dstart[d];
            if (EW == EW_PACK) {
                key_out[g] = (k & lmask) << 16 | e;  // (gs mod 2^L, width)
            } else {
                key_out[g] = k;
                if (EW == EW_TO16 || EW == EW_16)
                    reinterpret_cast<uint16_t *>(ge_out)[g] = (uint16_t)e;
                else
                    ge_out[g] = EW == EW_FROM16 ? k + e : e;
            }
        }
    }
    if (ROWS == ROWS_NONE) return;
    __syncthreads();
#pragma unroll
    for (int k = 0; k < RITEMS; ++k)
        if (lp[k] != 0xffffffffu)
            se[lp[k]] = ROWS == ROWS_IDENT ? (uint32_t)(base + k * 64 + lane) : vr[k];
    __syncthreads();
    for (int j = threadIdx.x; j < count; j += RB) {
        const uint32_t d = digit_of<M, DB>(sk[j], 0u, 0u, shift, st);
        row_out[gbase[d] + (uint32_t)j - dstart[d]] = se[j];
    }
}

template <int M>
void launch_pass(lime_ctx *ctx, int shift, bool have_hist, int64_t n, const uint32_t *k0,
                 const uint32_t *e0, const uint32_t *r0, const int8_t *st, uint32_t *k1,
                 uint32_t *e1, uint32_t *r1, uint32_t *mat, uint32_t ntiles, int rows, int &rc,
                 const uint32_t *raw_off = nullptr, int32_t raw_nc = 0, int ew = EW_32) {
    if (raw_off) {  // first gs pass straight from the caller's rows (k_prep's histogram)
        if ((rc = scan_exclusive_u32(ctx, mat, mat, (int64_t)RBINS * ntiles, nullptr)) != LIME_OK)
            return;
        if (M == M_GS && rows == ROWS_IDENT)
            hipLaunchKernelGGL((k_scatter<M_GS, ROWS_IDENT, true>), dim3(ntiles), dim3(RB), 0,
                               S(ctx), k0, e0, r0, n, shift, st, (const uint32_t *)mat, ntiles, k1,
                               e1, r1, raw_off, raw_nc);
        return;
    }
    if (!have_hist)
        hipLaunchKernelGGL(k_hist<M>, dim3(ntiles), dim3(RB), 0, S(ctx), k0, e0, r0, n, shift, st,
                           mat, ntiles, rows);
    if ((rc = scan_exclusive_u32(ctx, mat, mat, (int64_t)RBINS * ntiles, nullptr)) != LIME_OK)
        return;
    if (M == M_GS && ew != EW_32) {
        // (u16 widths: rows kept, GS passes only)
#define LIME_EW_LAUNCH(R, E)                                                                     \
    hipLaunchKernelGGL((k_scatter<M_GS, R, false, E>), dim3(ntiles), dim3(RB), 0, S(ctx), k0, e0, \
                       r0, n, shift, st, (const uint32_t *)mat, ntiles, k1, e1, r1)
        if (rows == ROWS_IDENT && ew == EW_TO16) LIME_EW_LAUNCH(ROWS_IDENT, EW_TO16);
        else if (rows == ROWS_LOAD && ew == EW_TO16) LIME_EW_LAUNCH(ROWS_LOAD, EW_TO16);
        else if (rows == ROWS_LOAD && ew == EW_16) LIME_EW_LAUNCH(ROWS_LOAD, EW_16);
        else if (rows == ROWS_LOAD && ew == EW_FROM16) LIME_EW_LAUNCH(ROWS_LOAD, EW_FROM16);
        else rc = LIME_ERR_ARG;  // (no such combination is planned)
#undef LIME_EW_LAUNCH
        return;
    }
    if (rows == ROWS_IDENT)
        hipLaunchKernelGGL((k_scatter<M, ROWS_IDENT>), dim3(ntiles), dim3(RB), 0, S(ctx), k0, e0,
                           r0, n, shift, st, (const uint32_t *)mat, ntiles, k1, e1, r1);
    else if (rows == ROWS_LOAD)
        hipLaunchKernelGGL((k_scatter<M, ROWS_LOAD>), dim3(ntiles), dim3(RB), 0, S(ctx), k0, e0,
                           r0, n, shift, st, (const uint32_t *)mat, ntiles, k1, e1, r1);
    else if (M == M_GS)  // binned sets: GS passes only
        hipLaunchKernelGGL((k_scatter<M_GS, ROWS_NONE>), dim3(ntiles), dim3(RB), 0, S(ctx), k0,
                           e0, r0, n, shift, st, (const uint32_t *)mat, ntiles, k1, e1, r1);
}

int radix_pass(lime_ctx *ctx, int mode, int shift, bool have_hist, int64_t n, const uint32_t *k0,
               const uint32_t *e0, const uint32_t *r0, const int8_t *st, uint32_t *k1,
               uint32_t *e1, uint32_t *r1, uint32_t *mat, uint32_t ntiles, int rows,
               const uint32_t *raw_off = nullptr, int32_t raw_nc = 0, int ew = EW_32) {
    int rc = LIME_OK;
    if (raw_off) {
        launch_pass<M_GS>(ctx, shift, true, n, k0, e0, r0, st, k1, e1, r1, mat, ntiles, rows, rc,
                          raw_off, raw_nc);
        if (rc != LIME_OK) return rc;
        LIME_HIP(hipGetLastError());
        return LIME_OK;
    }
    switch (mode) {
        case M_NZ:
            launch_pass<M_NZ>(ctx, shift, have_hist, n, k0, e0, r0, st, k1, e1, r1, mat, ntiles, rows, rc);
            break;
        case M_GE:
            launch_pass<M_GE>(ctx, shift, have_hist, n, k0, e0, r0, st, k1, e1, r1, mat, ntiles, rows, rc);
            break;
        case M_ST:
            launch_pass<M_ST>(ctx, shift, have_hist, n, k0, e0, r0, st, k1, e1, r1, mat, ntiles, rows, rc);
            break;
        case M_RW:
            launch_pass<M_RW>(ctx, shift, have_hist, n, k0, e0, r0, st, k1, e1, r1, mat, ntiles, rows, rc);
            break;
        default:
            launch_pass<M_GS>(ctx, shift, have_hist, n, k0, e0, r0, st, k1, e1, r1, mat, ntiles, rows, rc,
                              nullptr, 0, ew);
    }
    if (rc != LIME_OK) return rc;
    LIME_HIP(hipGetLastError());
    return LIME_OK;
}


// ------------------------------------------------------------ bucketed sort
// Plain sets past 2^16 rows (the default for C2 / C3-sized inputs): two 8-bit
// LSD digit passes on bits [L, L + 16) of gs group the rows into buckets of
// 2^L bases (input order kept inside each: the passes are stable), then ONE
// pass sorts every bucket in LDS by (gs mod 2^L, non-zero width) -- the
// zero-width rule rides in the local key, so no NZ pass.  The first digit
// pass reads the caller's rows itself (k_scatter RAW: k_prep only validates
// and histograms), so per row: 12 B (prep) + 24 B (pass 1) + 4 B (hist) +
// 24 B (pass 2) + 24 B (local) = 88 B, against 12 + 8 + 20 + 3 x 28 = 124 B
// (+28 with zero-width rows) of five digit passes.
//
// The local key packs (gs mod 2^L) << 1 | (width > 0) above the row's
// position in its bucket, so a stable pair of LDS digit passes over the key
// bits gives (gs, zero-width first, input order) -- the canonical order.
// Buckets of <= LCAP_S rows: one 512-thread workgroup each, their ge / row
// staged in LDS; larger ones are listed and taken by a persistent 1024-thread
// kernel (<= LCAP_B rows in LDS, gathering ge / row from L2; past that a
// chunked workgroup-wide radix over the bucket's rows in global memory).
constexpr int LNT_B = 1024, LPOS_B = 14, LCAP_B = 1 << LPOS_B;  // 16 items / thread
constexpr int LDMAX = 9;  // local digit bits (key L + 1 <= 18 bits in two passes)

struct LocalArgs {
    // rows grouped by gs >> L; packed (PK) sets: k0 holds (gs mod 2^L) << 16 |
    // width (EW_PACK) and e0 is unused scratch of n words
    const uint32_t *k0, *e0, *r0;
    const uint32_t *start;         // nb + 1 bucket starts
    int L;
    int zb;                        // k_local_mid: 1 if the set has zero-width rows
    uint32_t *k1, *e1, *r1;        // the sorted set
    unsigned int *nover;           // [0] listed buckets, [1] the big kernel's ticket
    uint32_t *over;                // listed bucket ids
    uint32_t *sink;                // LSINK words: stores past a bucket's rows
};
constexpr int LSINK = 1024;

__global__ __launch_bounds__(256) void k_bucket_starts(const uint32_t *__restrict__ k, int64_t n,
                                                       uint32_t nb, int L,
                                                       uint32_t *__restrict__ start) {
    const int64_t b = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (b > nb) return;
    start[b] = b == nb ? (uint32_t)n : (uint32_t)dev::lower_bound(k, 0, n, (uint64_t)b << L);
}

// One stable LDS digit pass of D (<= LDMAX) bits at `shift` over the packed
// items v (wave w holds items [w c, (w + 1) c) in (it, lane) order, c =
// nit * 64): ranks by wave ballots with per-wave digit counters, offsets by a
// digit-major scan, items written to dst.
template <int NT, int ITEMS, typename CT>
__device__ __forceinline__ void lds_digit_pass(const uint32_t (&v)[ITEMS], int nit, int shift,
                                               int D, CT (*cnt)[1 << LDMAX], uint32_t *scratch,
                                               uint32_t *dst) {
    constexpr int NW = NT / 64;
    const int w = threadIdx.x / 64, lane = dev::lane_id();
    const uint32_t ND = 1u << D, dm = ND - 1;
    for (int i = threadIdx.x; i < NW * (1 << LDMAX); i += NT) (&cnt[0][0])[i] = 0;
    __syncthreads();
    uint32_t pd[ITEMS];
#pragma unroll
    for (int it = 0; it < ITEMS; ++it) {
        if (it < nit) {
            const uint32_t d = (v[it] >> shift) & dm;
            uint64_t m = ~0ull;
    #pragma unroll
            for (int b = 0; b < LDMAX; ++b) {
                const uint32_t bit = (d >> b) & 1u;
                const uint64_t bb = __ballot(bit);
                m &= bit ? bb : ~bb;
            }
            const uint32_t rank = (uint32_t)__popcll(m & dev::lanemask_lt());
            const uint32_t old = cnt[w][d];
            pd[it] = old + rank;
            if (rank == 0) cnt[w][d] = (CT)(old + (uint32_t)__popcll(m));
        }
    }
    __syncthreads();
    {  // digit d's start, then each wave's start within it
        const int d = threadIdx.x;
        uint32_t tot = 0;
        if (d < (int)ND)
            for (int ww = 0; ww < NW; ++ww) tot += cnt[ww][d];
        uint32_t all;
        const uint32_t ds = dev::block_exclusive_sum<NT>(tot, scratch, &all);
        if (d < (int)ND) {
            uint32_t run = ds;
            for (int ww = 0; ww < NW; ++ww) {
                const uint32_t c = cnt[ww][d];
                cnt[ww][d] = (CT)run;
                run += c;
            }
        }
    }
    __syncthreads();
#pragma unroll
    for (int it = 0; it < ITEMS; ++it) {
        if (it < nit) {
            dst[(uint32_t)cnt[w][(v[it] >> shift) & dm] + pd[it]] = v[it];
        }
    }
    __syncthreads();
}

// a row's local key parts from its loaded words: (gs mod 2^L, non-zero
// width); PK: g is the packed word, e unused
template <bool PK>
__device__ __forceinline__ uint32_t lk_low(uint32_t g, uint32_t lmask) {
    return PK ? g >> 16 : g & lmask;
}
template <bool PK>
__device__ __forceinline__ bool lk_nz(uint32_t g, uint32_t e) {
    return PK ? (g & 0xffffu) != 0u : e > g;
}
// what a row stages for its end: the end, or (PK) the width
template <bool PK>
__device__ __forceinline__ uint32_t lk_endw(uint32_t g, uint32_t e) {
    return PK ? g & 0xffffu : e;
}

// bucket b = rows [s0, s0 + m), m <= NT * ITEMS, sorted in LDS from its
// rows in registers (g, e, r: item it * 64 + lane of wave w at position
// w c + it 64 + lane, c = nit 64; past m: padding).  STAGE: ge and row are
// staged in LDS (else gathered from global memory, where the bucket's lines
// are L2-resident after the load).
template <int NT, int ITEMS, int POSB, bool STAGE, typename CT, bool PK = false>
__device__ __forceinline__ void bucket_sort_regs(const LocalArgs &a, uint32_t b, uint32_t s0,
                                                 uint32_t m, const uint32_t (&g)[ITEMS],
                                                 const uint32_t (&e)[ITEMS],
                                                 const uint32_t (&r)[ITEMS], uint32_t *A,
                                                 uint32_t *B, CT (*cnt)[1 << LDMAX],
                                                 uint32_t *scratch, uint32_t *s_e, uint32_t *s_r) {
    constexpr int NW = NT / 64;
    const int w = threadIdx.x / 64, lane = dev::lane_id();
    const int nit = (int)((m + NW * 64 - 1) / (NW * 64));
    const int c = nit * 64;
    const uint32_t lmask = (1u << a.L) - 1u;
    uint32_t v[ITEMS];
#pragma unroll
    for (int it = 0; it < ITEMS; ++it) {
        const uint32_t pos = (uint32_t)(w * c + it * 64 + lane);
        // padding sorts last (after every row: it follows them)
        v[it] = pos < m ? (((lk_low<PK>(g[it], lmask) << 1) | (lk_nz<PK>(g[it], e[it]) ? 1u : 0u))
                           << POSB) | pos
                        : 0xffffffffu;
        if (STAGE && it < nit && pos < m) {
            s_e[pos] = lk_endw<PK>(g[it], e[it]);
            s_r[pos] = r[it];
        }
    }
    const int kb = a.L + 1, d1 = kb - kb / 2, d2 = kb / 2;
    lds_digit_pass<NT, ITEMS, CT>(v, nit, POSB, d1, cnt, scratch, B);
#pragma unroll
    for (int it = 0; it < ITEMS; ++it) {
        if (it < nit) {
            v[it] = B[w * c + it * 64 + lane];
        }
    }
    lds_digit_pass<NT, ITEMS, CT>(v, nit, POSB + d1, d2, cnt, scratch, A);
    const uint32_t base = b << a.L, pm = (1u << POSB) - 1u;
    for (uint32_t q = threadIdx.x; q < m; q += NT) {
        const uint32_t x = A[q], j = x & pm;
        const uint32_t gq = base | ((x >> (POSB + 1)) & lmask);
        const uint32_t ew = STAGE ? s_e[j] : PK ? a.k0[s0 + j] & 0xffffu : a.e0[s0 + j];
        a.k1[s0 + q] = gq;
        a.e1[s0 + q] = PK ? gq + ew : ew;
        a.r1[s0 + q] = STAGE ? s_r[j] : a.r0[s0 + j];
    }
}

// The common case of bucket_sort_regs without its two ranked digit passes
// (17 wave ballots per row: k_local_small was issue-bound, 34 % of its wave
// cycles issuing, 26 % waiting on dependencies): every row gets the unique
// composite key u = local key << POSB | position (local key = (gs mod 2^L)
// << 1 | non-zero width), and
//   1. an LDS histogram of the key's top SBB bits (sub-bins of a few rows),
//   2. one block scan of the sub-bin counts (and their max),
//   3. each row claims a slot of its sub-bin (one returning LDS atomic; the
//      order inside a sub-bin is arbitrary),
//   4. each row's rank in its sub-bin = the number of its keys below u
//      (unique keys: no tie, so the result is the stable order),
// and the rows are written in rank order.  A sub-bin past SMAX rows (piled-up
// starts) sends the bucket to k_local_big's ranked digit passes: returns false
// (nothing written).
constexpr int SMAX = 48;
// NSB = 2^SBB sub-bins (NSB / NT per thread in the scan); CT: the sub-bin
// counter type (u32: LDS atomics); STAGE: e / r staged in LDS by
// position (else gathered from global memory at the end, where the
// bucket's lines are L2-resident after its load)
template <int NT, int ITEMS, int POSB, int SBB, bool STAGE, typename CT, bool PK = false>
__device__ __forceinline__ bool bucket_sort_claim(const LocalArgs &a, uint32_t b, uint32_t s0,
                                                  uint32_t m, const uint32_t (&g)[ITEMS],
                                                  const uint32_t (&e)[ITEMS],
                                                  const uint32_t (&r)[ITEMS], uint32_t *T,
                                                  uint32_t *O, CT *sstart, CT *scur,
                                                  uint32_t *scratch, uint32_t *s_e, uint32_t *s_r) {
    constexpr int NSB = 1 << SBB, SPT = NSB / NT;
    static_assert(NSB % NT == 0 && SPT >= 1, "whole sub-bins per thread in the scan");
    constexpr int NW = NT / 64;
    const int w = threadIdx.x / 64, lane = dev::lane_id();
    const int nit = (int)((m + NW * 64 - 1) / (NW * 64));
    const int c = nit * 64;
    const uint32_t lmask = (1u << a.L) - 1u;
    const int kb = a.L + 1;                      // local key bits
    const int sh = kb > SBB ? kb - SBB : 0;      // sub-bin = key >> sh
#pragma unroll
    for (int q = 0; q < SPT; ++q) scur[SPT * threadIdx.x + q] = 0;
    __syncthreads();
    uint32_t u[ITEMS];
#pragma unroll
    for (int it = 0; it < ITEMS; ++it) {
        const uint32_t pos = (uint32_t)(w * c + it * 64 + lane);
        u[it] = 0xffffffffu;
        if (it < nit && pos < m) {
            const uint32_t k = (lk_low<PK>(g[it], lmask) << 1) | (lk_nz<PK>(g[it], e[it]) ? 1u : 0u);
            u[it] = (k << POSB) | pos;
            atomicAdd(&scur[k >> sh], 1u);
            if (STAGE) {
                s_e[pos] = lk_endw<PK>(g[it], e[it]);
                s_r[pos] = r[it];
            }
        }
    }
    __syncthreads();
    uint32_t cv[SPT], csum = 0, cmax = 0;
#pragma unroll
    for (int q = 0; q < SPT; ++q) {
        cv[q] = scur[SPT * threadIdx.x + q];
        csum += cv[q];
        cmax = max(cmax, cv[q]);
    }
    uint32_t tot;
    uint32_t st = dev::block_exclusive_sum<NT>(csum, scratch, &tot);
    const uint32_t mx = dev::wave_reduce_max(cmax);
    if (lane == 0) scratch[NW + 1 + w] = mx;  // (past the scan's NW + 1 words)
#pragma unroll
    for (int q = 0; q < SPT; ++q) {
        sstart[SPT * threadIdx.x + q] = (CT)st;
        scur[SPT * threadIdx.x + q] = (CT)st;
        st += cv[q];
    }
    __syncthreads();
    uint32_t big = 0;
#pragma unroll
    for (int i = 0; i < NW; ++i) big = max(big, scratch[NW + 1 + i]);
    if (big > (uint32_t)SMAX) {  // (uniform: every thread read the same words)
        __syncthreads();  // (sstart / scur are reset by the next bucket)
        return false;
    }
#pragma unroll
    for (int it = 0; it < ITEMS; ++it)
        if (u[it] != 0xffffffffu) T[atomicAdd(&scur[(u[it] >> POSB) >> sh], 1u)] = u[it];
    __syncthreads();
#pragma unroll
    for (int it = 0; it < ITEMS; ++it) {
        if (u[it] == 0xffffffffu) continue;
        const uint32_t sb = (u[it] >> POSB) >> sh;
        const uint32_t lo = sstart[sb], hi = scur[sb];
        uint32_t rk = lo;
        for (uint32_t j = lo; j < hi; ++j) rk += T[j] < u[it] ? 1u : 0u;
        O[rk] = u[it];
    }
    __syncthreads();
    const uint32_t base = b << a.L, pm = (1u << POSB) - 1u;
    for (uint32_t q = threadIdx.x; q < m; q += NT) {
        const uint32_t x = O[q], j = x & pm;
        const uint32_t gq = base | ((x >> (POSB + 1)) & lmask);
        const uint32_t ew = STAGE ? s_e[j] : PK ? a.k0[s0 + j] & 0xffffu : a.e0[s0 + j];
        a.k1[s0 + q] = gq;
        a.e1[s0 + q] = PK ? gq + ew : ew;
        a.r1[s0 + q] = STAGE ? s_r[j] : a.r0[s0 + j];
    }
    return true;
}

// a bucket's rows into registers, branch-free (positions past the bucket
// clamped to its last row; a bucket too large for the shape, or empty, loads
// row 0): every load issued before any is used
// SKIP: items past the wave's share of the bucket are not loaded (a
// wave-uniform branch per item; else they reload the bucket's last row)
template <int NT, int ITEMS, int CAP, bool LR = true, bool PK = false, bool SKIP = false>
struct BucketRegs {
    uint32_t g[ITEMS], e[PK ? 1 : ITEMS], r[LR ? ITEMS : 1];
    // the ends to pass on: PK rows carry their widths in g (the sorts then
    // never read e), so g stands in and no e registers are held
    __device__ __forceinline__ const uint32_t (&ends() const)[ITEMS] {
        if constexpr (PK)
            return g;
        else
            return e;
    }
    uint32_t s0, m;
    // start: the bucket starts (a.start; the persistent kernel passes them as
    // a restrict argument, read at its wave-uniform bucket index by scalar
    // loads -- a vector load's wait there drained the previous bucket's
    // stores before this bucket's rows were requested)
    __device__ __forceinline__ void load(const LocalArgs &a, uint32_t b, uint32_t nb,
                                         const uint32_t *start) {
        constexpr int NW = NT / 64;
        const int w = threadIdx.x / 64, lane = dev::lane_id();
        s0 = 0;
        m = 0;
        if (b < nb) {
            s0 = start[b];
            m = start[b + 1] - s0;
        }
        const bool ok = m >= 1 && m <= (uint32_t)CAP;
        const uint32_t base = ok ? s0 : 0u;
        const int c = ok ? (int)((m + NW * 64 - 1) / (NW * 64)) * 64 : 0;
#pragma unroll
        for (int it = 0; it < ITEMS; ++it) {
            if (SKIP && it * 64 >= c) continue;
            const uint32_t pos = (uint32_t)(w * c + it * 64 + lane);
            const uint32_t q = base + (ok ? min(pos, m - 1) : 0u);
            g[it] = a.k0[q];
            if (!PK) e[it] = a.e0[q];  // (PK: the width rides in g)
            if (LR) r[it] = a.r0[q];  // (LR = false: gathered at the end)
        }
    }
};

// Persistent (three workgroups per CU, <= 80 VGPRs, ~50 KiB LDS): each
// workgroup takes buckets b, b + grid, ... and loads the next one's rows into
// registers before sorting the current one, so the load latency hides behind
// the LDS work (one bucket per workgroup, loads then sort, left the memory
// pipe idle half the time).  Buckets past LCAP_S rows, or with a sub-bin past
// SMAX rows, are listed for k_local_big.  (Two workgroups per CU with 4096-row
// buckets and the ranked digit passes inline took 78 KiB of LDS each: the
// loads in flight per CU, not the bytes, bounded it at 3.75 TB/s.)
constexpr int LNT_S = 512, LPOS_S = 12, LCAP_S = 3072;  // 6 items / thread
template <bool PK>
__global__ __launch_bounds__(LNT_S) __attribute__((amdgpu_waves_per_eu(6, 8)))
void k_local_small(LocalArgs a, uint32_t nb, const uint32_t *__restrict__ start) {
    __shared__ uint32_t A[LCAP_S], B[LCAP_S], s_e[LCAP_S], s_r[LCAP_S];
    __shared__ uint32_t sstart[LNT_S], scur[LNT_S];
    __shared__ uint32_t scratch[2 * (LNT_S / 64) + 1];
    BucketRegs<LNT_S, LCAP_S / LNT_S, LCAP_S, true, PK> cur, nxt;
    cur.load(a, blockIdx.x, nb, start);
    for (uint32_t b = blockIdx.x; b < nb; b += gridDim.x) {
        nxt.load(a, b + gridDim.x, nb, start);
        bool listed = cur.m > (uint32_t)LCAP_S;
        if (!listed && cur.m > 0)
            listed = !bucket_sort_claim<LNT_S, LCAP_S / LNT_S, LPOS_S, 9, true, uint32_t, PK>(
                a, b, cur.s0, cur.m, cur.g, cur.ends(), cur.r, A, B, sstart, scur, scratch, s_e,
                s_r);
        if (listed && threadIdx.x == 0) a.over[atomicAdd(&a.nover[0], 1u)] = b;  // for the big kernel
        __syncthreads();  // (the next bucket overwrites the staging)
        cur = nxt;
    }
}

// Buckets of a few thousand rows (the bucketed sort of dense sets: 9-bit
// digit passes, 2^14-base buckets of ~2.6k rows at C3's density): a claim
// sort over sub-bins of ONE local key each (u16 cursors, two per LDS word:
// 2^SBB of them in 2^(SBB - 1) words).
//   1. every row's key k = (gs mod 2^L) << zb | (non-zero width), zb = 1
//      when the set has zero-width rows (else the bit is constant and left
//      out, so 2^14-base buckets need only 2^14 sub-bins);
//   2. a histogram of the sub-bins k >> sh (sh = 0 whenever the key fits);
//   3. one block scan of the counts: each cursor at its sub-bin's start;
//   4. each row claims a slot of its sub-bin (one returning LDS atomic): a
//      row alone in its sub-bin (most rows) has its rank -- the slot;
//   5. rows sharing a sub-bin (equal starts, or sh > 0) count the entries
//      below their unique u = k << POSB | position (the stable order);
//   6. the outputs leave in three rounds through T (gs, ge, row written at
//      their ranks, stored coalesced); PK: two (the packed word gives gs
//      and ge, then the row).
// Every row's rank stays in a register: no per-slot pass, no rank table.
// A sub-bin past SMAX rows (a pile of identical starts) sends the bucket to
// k_local_big.
// prefetch(): called once the ranks are known, before the output stores --
// the persistent kernel loads its next bucket there.  Every thread then
// issues exactly ITEMS stores per output array (slots past the bucket's rows
// go to the sink): loads and stores share vmcnt, so with a static store
// count the next bucket's first use of its rows waits for those loads only,
// not for this bucket's stores (a loop bounded by the bucket's size made the
// compiler wait for every store: the prefetch then bought nothing)
template <int NT, int ITEMS, int POSB, int SBB, bool PK = false, class PF>
__device__ __forceinline__ bool bucket_sort_keys(const LocalArgs &a, uint32_t b, uint32_t s0,
                                                 uint32_t m,
                                                 const uint32_t (&g)[ITEMS],
                                                 const uint32_t (&e)[ITEMS],
                                                 const uint32_t (&rw)[ITEMS], uint32_t *T,
                                                 uint32_t *cw, uint32_t *scratch, PF &&prefetch) {
    constexpr int NWD = 1 << (SBB - 1), SPW = NWD / NT;  // cursor words, per thread
    static_assert(NWD % NT == 0 && SPW >= 2 && (SPW & (SPW - 1)) == 0, "cursor words per thread");
    static_assert(NT * ITEMS <= (1 << POSB) && NT * ITEMS < 65536, "positions / ranks");
    constexpr int NW = NT / 64;
    const int w = threadIdx.x / 64, lane = dev::lane_id();
    const int nit = (int)((m + NW * 64 - 1) / (NW * 64));
    const int c = nit * 64;
    const uint32_t lmask = (1u << a.L) - 1u;
    const int zb = a.zb;
    const int kb = a.L + zb;                 // local key bits
    const int sh = kb > SBB ? kb - SBB : 0;  // sub-bin = key >> sh
    // cursor word i lives at i + i / SPW: a thread's SPW words (its share of
    // the scan) then start SPW + 1 words after its neighbour's -- every lane
    // in its own bank (at 16 words apart, 16 lanes shared each bank)
    auto pw = [](uint32_t i) { return i + i / SPW; };
    uint32_t *mine = cw + (SPW + 1) * threadIdx.x;
#pragma unroll
    for (int q = 0; q < SPW; ++q) mine[q] = 0u;
    __syncthreads();
    uint32_t u[ITEMS];
#pragma unroll
    for (int it = 0; it < ITEMS; ++it) {
        const uint32_t pos = (uint32_t)(w * c + it * 64 + lane);
        u[it] = 0xffffffffu;
        if (it < nit && pos < m) {
            const uint32_t k = (lk_low<PK>(g[it], lmask) << zb) |
                               (lk_nz<PK>(g[it], e[it]) ? (uint32_t)zb : 0u);
            u[it] = (k << POSB) | pos;
            const uint32_t sb = k >> sh;
            atomicAdd(&cw[pw(sb >> 1)], 1u << ((sb & 1u) << 4));
        }
    }
    __syncthreads();
    // (the thread's words are read twice, sum then starts, rather than held:
    // 16 more registers spilled the wide shape)
    uint32_t csum = 0, cmax = 0;
#pragma unroll
    for (int q = 0; q < SPW; ++q) {
        const uint32_t v = mine[q], lo = v & 0xffffu, hi = v >> 16;
        csum += lo + hi;
        cmax = max(cmax, max(lo, hi));
    }
    uint32_t tot;
    uint32_t st = dev::block_exclusive_sum<NT>(csum, scratch, &tot);
    const uint32_t mx = dev::wave_reduce_max(cmax);
    if (lane == 0) scratch[NW + 1 + w] = mx;  // (past the scan's NW + 1 words)
#pragma unroll
    for (int q = 0; q < SPW; ++q) {
        const uint32_t v = mine[q], lo = v & 0xffffu, hi = v >> 16;
        mine[q] = st | (st + lo) << 16;
        st += lo + hi;
    }
    __syncthreads();
    uint32_t big = 0;
#pragma unroll
    for (int i = 0; i < NW; ++i) big = max(big, scratch[NW + 1 + i]);
    if (big > (uint32_t)SMAX) {  // (uniform: every thread read the same words)
        __syncthreads();
        return false;
    }
    uint32_t rk[ITEMS];
#pragma unroll
    for (int it = 0; it < ITEMS; ++it) {
        rk[it] = 0xffffffffu;
        if (u[it] != 0xffffffffu) {
            const uint32_t sb = (u[it] >> POSB) >> sh, sft = (sb & 1u) << 4;
            rk[it] = (atomicAdd(&cw[pw(sb >> 1)], 1u << sft) >> sft) & 0xffffu;
            T[rk[it]] = u[it];
        }
    }
    __syncthreads();
    // rows sharing a sub-bin (equal starts): their rank among its entries,
    // one item at a time (few rows share one; every item scanning to the
    // wave's largest shared sub-bin in one loop took C3's local sort 3.8 ->
    // 4.9 ms).  After the claims each cursor is its sub-bin's end.
#pragma unroll
    for (int it = 0; it < ITEMS; ++it) {
        if (u[it] == 0xffffffffu) continue;
        const uint32_t sb = (u[it] >> POSB) >> sh;
        const uint32_t hi = (cw[pw(sb >> 1)] >> ((sb & 1u) << 4)) & 0xffffu;
        const uint32_t lo = sb ? (cw[pw((sb - 1) >> 1)] >> (((sb - 1) & 1u) << 4)) & 0xffffu : 0u;
        if (hi - lo > 1) {
            uint32_t r = lo;
            for (uint32_t j = lo; j < hi; ++j) r += T[j] < u[it] ? 1u : 0u;
            rk[it] = r;
        }
    }
    prefetch();
    uint32_t *const sink = a.sink + threadIdx.x % LSINK;
    if (PK) {  // packed word -> (gs, ge), then rows
        const uint32_t base = b << a.L;
#pragma unroll
        for (int round = 0; round < 2; ++round) {
            __syncthreads();  // (T free: ranks taken / the previous round stored)
#pragma unroll
            for (int it = 0; it < ITEMS; ++it)
                if (rk[it] != 0xffffffffu) T[rk[it]] = round == 0 ? g[it] : rw[it];
            __syncthreads();
#pragma unroll
            for (int it = 0; it < ITEMS; ++it) {
                const uint32_t q = threadIdx.x + (uint32_t)it * NT;
                const bool in = q < m;
                const uint32_t x = T[q];  // (q < NT ITEMS: inside T)
                if (round == 0) {
                    const uint32_t gq = base | (x >> 16);
                    *(in ? a.k1 + s0 + q : sink) = gq;
                    *(in ? a.e1 + s0 + q : sink) = gq + (x & 0xffffu);
                } else {
                    *(in ? a.r1 + s0 + q : sink) = x;
                }
            }
        }
        return true;
    }
#pragma unroll
    for (int round = 0; round < 3; ++round) {
        __syncthreads();  // (T free: ranks taken / the previous round stored)
#pragma unroll
        for (int it = 0; it < ITEMS; ++it)
            if (rk[it] != 0xffffffffu) T[rk[it]] = round == 0 ? g[it] : round == 1 ? e[it] : rw[it];
        __syncthreads();
        uint32_t *dst = round == 0 ? a.k1 : round == 1 ? a.e1 : a.r1;
#pragma unroll
        for (int it = 0; it < ITEMS; ++it) {
            const uint32_t q = threadIdx.x + (uint32_t)it * NT;
            *(q < m ? dst + s0 + q : sink) = T[q];
        }
    }
    return true;
}

// Persistent, WGS workgroups of NT threads per CU (the others overlap one
// bucket's loads with another's sort), buckets of up to NT * ITEMS rows;
// larger ones, or with a sub-bin past SMAX rows, are listed for
// k_local_big.  Two shapes:
//   mid: 512 threads x 12 rows, two per CU (~59 KiB LDS): buckets averaging
//        up to LAVG_M rows;
//   wide: 1024 threads x 16 rows, one per CU (~132 KiB LDS: 2^15 sub-bins
//        for 2^16-base buckets): buckets averaging up to LAVG_W rows (C3's
//        5e8 pile-up rows, ~10.6k per 2^16-base bucket, under two 8-bit
//        passes -- the 9-bit passes run at ~3 ms per 5e8 rows against ~2.4).
template <int NT, int ITEMS, int POSB, int SBB, int WGS, bool PK>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(WGS * NT / 256, 8)))
void k_local_keys(LocalArgs a, uint32_t nb, const uint32_t *__restrict__ start) {
    constexpr int CAP = NT * ITEMS;
    __shared__ uint32_t T[CAP];
    // (padded: one word per thread's share of the scan)
    __shared__ uint32_t cw[(1 << (SBB - 1)) + NT];
    __shared__ uint32_t scratch[2 * (NT / 64) + 1];
    // (the next bucket's keys prefetched into a second register set during
    // this one's sort, rows loaded at its start: no faster, same box --
    // the kernel waits on LDS and barriers, not loads; not kept)
    if constexpr (!PK) {  // (u32 ends: no registers to spare for a second bucket)
        for (uint32_t b = blockIdx.x; b < nb; b += gridDim.x) {
            BucketRegs<NT, ITEMS, CAP, true, PK, true> cur;
            cur.load(a, b, nb, start);
            bool listed = cur.m > (uint32_t)CAP;
            if (!listed && cur.m > 0)
                listed = !bucket_sort_keys<NT, ITEMS, POSB, SBB, PK>(
                    a, b, cur.s0, cur.m, cur.g, cur.ends(), cur.r, T, cw, scratch, [] {});
            if (listed && threadIdx.x == 0) a.over[atomicAdd(&a.nover[0], 1u)] = b;
            __syncthreads();  // (the next bucket overwrites the staging)
        }
        return;
    }
    // PK: the next bucket's rows are loaded behind this one's sort, before
    // its output stores (bucket_sort_keys' prefetch)
    BucketRegs<NT, ITEMS, CAP, true, PK, true> cur, nxt;
    cur.load(a, blockIdx.x, nb, start);
    for (uint32_t b = blockIdx.x; b < nb; b += gridDim.x) {
        bool listed = cur.m > (uint32_t)CAP, fetched = false;
        auto prefetch = [&]() {
            nxt.load(a, b + gridDim.x, nb, start);
            fetched = true;
        };
        if (!listed && cur.m > 0)
            listed = !bucket_sort_keys<NT, ITEMS, POSB, SBB, PK>(
                a, b, cur.s0, cur.m, cur.g, cur.ends(), cur.r, T, cw, scratch, prefetch);
        if (!fetched) nxt.load(a, b + gridDim.x, nb, start);  // (listed or empty)
        if (listed && threadIdx.x == 0) a.over[atomicAdd(&a.nover[0], 1u)] = b;  // for the big kernel
        __syncthreads();  // (the next bucket overwrites the staging)
        cur = nxt;
    }
}
constexpr int LCAP_M = 6144, LCAP_W = 16384;
#define LIME_LOCAL_MID(PK) k_local_keys<512, 12, 13, 14, 2, PK>
#ifndef LIME_WIDE_SBB
#define LIME_WIDE_SBB 15
#endif
#define LIME_LOCAL_WIDE(PK) k_local_keys<1024, 16, 14, LIME_WIDE_SBB, 1, PK>

// A bucket past LCAP_B rows: LSD over its key (gs mod 2^L, non-zero width) in
// 6-bit digits by the whole workgroup, NT rows per step in order (wave ballot
// ranks, per-wave digit counts, running digit offsets): stable.  Passes
// alternate (k0, e0, r0) -> (k1, e1, r1) -> ...; the result is copied into
// (k1, e1, r1) when it ends on the other side.  PK: the packed rows are
// first unpacked into (k1, e1, r1), and the passes start from there.
template <int NT, bool PK = false>
__device__ void bucket_sort_global(const LocalArgs &a, uint32_t b, uint32_t s0, uint32_t m,
                                   uint32_t *lds) {
    constexpr int NW = NT / 64, GD = 6, GB = 1 << GD;
    uint32_t *hist = lds, *run = lds + GB, *wc = lds + 2 * GB;  // wc[NW][GB]
    const int w = threadIdx.x / 64, lane = dev::lane_id();
    const uint32_t lmask = (1u << a.L) - 1u;
    const int kb = a.L + 1, np = (kb + GD - 1) / GD;
    uint32_t *const fin[3] = {a.k1 + s0, a.e1 + s0, a.r1 + s0};
    uint32_t *const inp[3] = {const_cast<uint32_t *>(a.k0) + s0, const_cast<uint32_t *>(a.e0) + s0,
                              const_cast<uint32_t *>(a.r0) + s0};
    const uint32_t *src[3] = {inp[0], inp[1], inp[2]};
    uint32_t *dst[3] = {fin[0], fin[1], fin[2]};
    if (PK) {  // (each thread rereads only the rows it wrote, in pass 0)
        const uint32_t base = b << a.L;
        for (uint32_t i = threadIdx.x; i < m; i += NT) {
            const uint32_t x = inp[0][i], g = base | (x >> 16);
            fin[0][i] = g;
            fin[1][i] = g + (x & 0xffffu);
            fin[2][i] = inp[2][i];
        }
        for (int q = 0; q < 3; ++q) {
            src[q] = fin[q];
            dst[q] = inp[q];
        }
    }
    for (int p = 0; p < np; ++p) {
        const int shift = p * GD;
        auto digit = [&](uint32_t g, uint32_t e) {
            return ((((g & lmask) << 1) | (e > g ? 1u : 0u)) >> shift) & (GB - 1);
        };
        for (int i = threadIdx.x; i < GB; i += NT) hist[i] = 0;
        __syncthreads();
        for (uint32_t i = threadIdx.x; i < m; i += NT) atomicAdd(&hist[digit(src[0][i], src[1][i])], 1u);
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t r = 0;
            for (int d = 0; d < GB; ++d) {
                run[d] = r;
                r += hist[d];
            }
        }
        __syncthreads();
        for (uint32_t c0 = 0; c0 < m; c0 += NT) {
            const uint32_t i = c0 + threadIdx.x;
            const bool ok = i < m;
            uint32_t g = 0, e = 0, r = 0;
            if (ok) g = src[0][i], e = src[1][i], r = src[2][i];
            const uint32_t d = ok ? digit(g, e) : 0u;
            uint64_t mm = __ballot(ok);
#pragma unroll
            for (int bt = 0; bt < GD; ++bt) {
                const uint32_t bit = (d >> bt) & 1u;
                const uint64_t bb = __ballot(bit);
                mm &= bit ? bb : ~bb;
            }
            const uint32_t rank = (uint32_t)__popcll(mm & dev::lanemask_lt());
            for (int q = threadIdx.x; q < NW * GB; q += NT) wc[q] = 0;
            __syncthreads();
            if (ok && rank == 0) wc[w * GB + d] = (uint32_t)__popcll(mm);
            __syncthreads();
            if (threadIdx.x < GB) {  // per digit: the waves' starts, then the run
                uint32_t t = run[threadIdx.x];
                for (int ww = 0; ww < NW; ++ww) {
                    const uint32_t x = wc[ww * GB + threadIdx.x];
                    wc[ww * GB + threadIdx.x] = t;
                    t += x;
                }
                run[threadIdx.x] = t;
            }
            __syncthreads();
            if (ok) {
                const uint32_t o = wc[w * GB + d] + rank;
                dst[0][o] = g;
                dst[1][o] = e;
                dst[2][o] = r;
            }
            __syncthreads();
        }
        for (int q = 0; q < 3; ++q) {
            const uint32_t *t = src[q];
            src[q] = dst[q];
            dst[q] = const_cast<uint32_t *>(t);
        }
    }
    if (src[0] != fin[0])  // the result ended on the input side: copy it over
        for (uint32_t i = threadIdx.x; i < m; i += NT) {
            fin[0][i] = src[0][i];
            fin[1][i] = src[1][i];
            fin[2][i] = src[2][i];
        }
}

// the listed buckets (> LCAP_S rows), taken in ticket order by one resident
// workgroup per CU until the list is done
// (the claim sort with 2048 sub-bins first, the ranked digit passes when a
// pile-up puts more than SMAX rows in one of them)
template <bool PK>
__global__ __launch_bounds__(LNT_B) void k_local_big(LocalArgs a) {
    __shared__ uint32_t A[LCAP_B], B[LCAP_B];
    // the ranked passes' digit counters and the claim sort's sub-bin starts /
    // cursors share one 16 KiB block (the two paths never overlap in time)
    __shared__ uint32_t aux[4096];
    static_assert(sizeof(uint16_t) * (LNT_B / 64) * (1 << LDMAX) <= sizeof(aux), "aux");
    uint16_t(*cnt)[1 << LDMAX] = reinterpret_cast<uint16_t(*)[1 << LDMAX]>(aux);
    uint32_t *sstart = aux, *scur = aux + 2048;
    __shared__ uint32_t scratch[2 * (LNT_B / 64) + 1];
    __shared__ uint32_t s_i;
    for (;;) {
        if (threadIdx.x == 0) s_i = atomicAdd(&a.nover[1], 1u);
        __syncthreads();
        const uint32_t i = s_i;
        __syncthreads();
        if (i >= a.nover[0]) break;
        const uint32_t b = a.over[i];
        const uint32_t s0 = a.start[b], m = a.start[b + 1] - s0;
        if (m <= (uint32_t)LCAP_B) {
            BucketRegs<LNT_B, LCAP_B / LNT_B, LCAP_B, true, PK> R;
            R.load(a, b, b + 1, a.start);
            if (!bucket_sort_claim<LNT_B, LCAP_B / LNT_B, LPOS_B, 11, false, uint32_t, PK>(
                    a, b, s0, m, R.g, R.ends(), R.r, A, B, sstart, scur, scratch, nullptr,
                    nullptr))
                bucket_sort_regs<LNT_B, LCAP_B / LNT_B, LPOS_B, false, uint16_t, PK>(
                    a, b, s0, m, R.g, R.ends(), R.r, A, B, cnt, scratch, nullptr, nullptr);
        } else
            bucket_sort_global<LNT_B, PK>(a, b, s0, m, A);
        __syncthreads();
    }
}

}  // namespace

int sort_set_impl(lime_ctx *ctx, lime_set *set, bool global, const int32_t *d_contig,
                  const uint32_t *d_start, const uint32_t *d_end, const uint32_t *d_len);

int sort_set(lime_ctx *ctx, lime_set *set, const int32_t *d_contig, const uint32_t *d_start,
             const uint32_t *d_end, const uint32_t *d_len) {
    return sort_set_impl(ctx, set, false, d_contig, d_start, d_end, d_len);
}

int sort_set_global(lime_ctx *ctx, lime_set *set, const uint32_t *d_gs, const uint32_t *d_ge,
                    const uint32_t *d_row, const uint32_t *d_len) {
    return sort_set_impl(ctx, set, true, reinterpret_cast<const int32_t *>(d_gs), d_ge, d_row,
                         d_len);
}

// the bucketed sort's choice: 2^L-base buckets under two digit passes of TB
// bits in all (L = bits - TB): 8 + 8 with buckets averaging LMIN to LAVG rows
// (k_local_small), else 9 + 8 or 9 + 9 with buckets averaging at most LAVG_M
// rows (k_local_mid: C3's 5e8 pile-up rows, ~2.65k per 2^14-base bucket);
// denser sets take the digit passes.  (8 + 8 with C3's ~10.6k rows per
// bucket through k_local_big, one workgroup per CU, took 7.0 ms there.)
#ifndef LIME_SORT_W16
#define LIME_SORT_W16 1
#endif
#ifndef LIME_SORT_TBMAX
#define LIME_SORT_TBMAX 18
#endif
#ifndef LIME_SORT_PACK
#define LIME_SORT_PACK 1
#endif
constexpr int64_t LMIN = 32, LAVG = 3 * LCAP_S / 4, LAVG_M = LCAP_M / 2, LAVG_W = 11500;
// the local kernel of a bucket geometry: 0 small, 1 mid, 2 wide
static int local_shape(int tb, int64_t avg) {
    return tb == 16 && avg <= LAVG ? 0 : avg <= LAVG_M ? 1 : 2;
}

// the (validate-only) prep of the bucketed sort, histogramming a DB-bit digit
template <int DB>
void launch_prep_nowrite(lime_ctx *ctx, lime_set *set, bool global, const int32_t *d_contig,
                         const uint32_t *d_start, const uint32_t *d_end, const uint32_t *d_len,
                         int64_t n, SetStats *part, uint32_t *mat, uint32_t ntiles, int hshift) {
    if (global)
        hipLaunchKernelGGL((k_prep<true, false, false, DB>), dim3(ntiles), dim3(RB), 0, S(ctx),
                           d_contig, d_start, d_end, (const uint32_t *)set->d_off, d_len,
                           set->n_contigs, n, nullptr, nullptr, nullptr, part, mat, ntiles, hshift);
    else if (set->n_contigs <= PCMAX)
        hipLaunchKernelGGL((k_prep<false, false, true, DB>), dim3(ntiles), dim3(RB), 0, S(ctx),
                           d_contig, d_start, d_end, (const uint32_t *)set->d_off, d_len,
                           set->n_contigs, n, nullptr, nullptr, nullptr, part, mat, ntiles, hshift);
    else
        hipLaunchKernelGGL((k_prep<false, false, false, DB>), dim3(ntiles), dim3(RB), 0, S(ctx),
                           d_contig, d_start, d_end, (const uint32_t *)set->d_off, d_len,
                           set->n_contigs, n, nullptr, nullptr, nullptr, part, mat, ntiles, hshift);
}

// the prep of the bucketed sort over caller rows when their widths may fit
// u16: validation, statistics, the DB-bit histogram, and (gs, u16 width)
// written for the first pass (6 B per row: it then reads those instead of
// the caller's 12, with half the registers of the RAW pass, whose 48 loads
// in flight spilled and waited mid-stream)
template <int DB>
void launch_prep_w16(lime_ctx *ctx, lime_set *set, const int32_t *d_contig,
                     const uint32_t *d_start, const uint32_t *d_end, const uint32_t *d_len,
                     int64_t n, uint32_t *gs, uint32_t *w16, SetStats *part, uint32_t *mat,
                     uint32_t ntiles, int hshift) {
    if (set->n_contigs <= PCMAX)
        hipLaunchKernelGGL((k_prep<false, true, true, DB, true>), dim3(ntiles), dim3(RB), 0, S(ctx),
                           d_contig, d_start, d_end, (const uint32_t *)set->d_off, d_len,
                           set->n_contigs, n, gs, w16, nullptr, part, mat, ntiles, hshift);
    else
        hipLaunchKernelGGL((k_prep<false, true, false, DB, true>), dim3(ntiles), dim3(RB), 0,
                           S(ctx), d_contig, d_start, d_end, (const uint32_t *)set->d_off, d_len,
                           set->n_contigs, n, gs, w16, nullptr, part, mat, ntiles, hshift);
}

// the bucketed sort's two digit passes: pass 1 (DB1 bits at L) from the
// caller's rows (histogrammed by the prep), pass 2 (DB2 bits at L + DB1);
// with u16 widths (every width < 2^16) pass 1 writes widths, pass 2 ends.
// pk / pw (caller rows with u16 widths): the prep's (gs, width), read by
// pass 1 instead of the caller's rows.  pack (u16 widths, L <= 16): pass 2
// writes the packed word (EW_PACK) and its histogram leaves the bucket-start
// partials (k_hist_part: part, with pass 1's digit starts in dstart1)
template <int DB1, int DB2>
int bucket_passes(lime_ctx *ctx, lime_set *set, bool global, const int32_t *d_contig,
                  const uint32_t *d_start, const uint32_t *d_end, int64_t n, int L, bool w16,
                  uint32_t *mat, int mat_bits, uint32_t ntiles, uint32_t *const (&a)[3],
                  uint32_t *const (&o)[3], const uint32_t *pk = nullptr,
                  const uint32_t *pw = nullptr, bool pack = false, uint32_t *dstart1 = nullptr,
                  uint32_t *part = nullptr) {
    if (pack && (!w16 || L > 16 || !dstart1 || !part))
        return fail(LIME_ERR_ARG, "sort: packed pass without u16 widths");
    // (mat: 2^mat_bits counts per tile, the histograms of both passes)
    if (DB1 > mat_bits || DB2 > mat_bits) return fail(LIME_ERR_ARG, "sort: digit matrix too small");
    LIME_TRY(scan_exclusive_u32(ctx, mat, mat, ((int64_t)1 << DB1) * ntiles, nullptr));
    const uint32_t *kc = reinterpret_cast<const uint32_t *>(d_contig);
    const int8_t *nost = nullptr;
    const uint32_t *cm = mat;
    if (pk && w16)
        hipLaunchKernelGGL((k_scatter<M_GS, ROWS_IDENT, false, EW_16, DB1>), dim3(ntiles),
                           dim3(RB), 0, S(ctx), pk, pw, (const uint32_t *)nullptr, n, L, nost, cm,
                           ntiles, a[0], a[1], a[2]);
    else if (global && w16)
        hipLaunchKernelGGL((k_scatter<M_GS, ROWS_LOAD, false, EW_TO16, DB1>), dim3(ntiles), dim3(RB),
                           0, S(ctx), kc, d_start, d_end, n, L, nost, cm, ntiles, a[0], a[1], a[2]);
    else if (global)
        hipLaunchKernelGGL((k_scatter<M_GS, ROWS_LOAD, false, EW_32, DB1>), dim3(ntiles), dim3(RB),
                           0, S(ctx), kc, d_start, d_end, n, L, nost, cm, ntiles, a[0], a[1], a[2]);
    else if (w16)
        hipLaunchKernelGGL((k_scatter<M_GS, ROWS_IDENT, true, EW_TO16, DB1>), dim3(ntiles),
                           dim3(RB), 0, S(ctx), kc, d_start, d_end, n, L, nost, cm, ntiles, a[0],
                           a[1], a[2], (const uint32_t *)set->d_off, set->n_contigs);
    else
        hipLaunchKernelGGL((k_scatter<M_GS, ROWS_IDENT, true, EW_32, DB1>), dim3(ntiles),
                           dim3(RB), 0, S(ctx), kc, d_start, d_end, n, L, nost, cm, ntiles, a[0],
                           a[1], a[2], (const uint32_t *)set->d_off, set->n_contigs);
    LIME_HIP(hipGetLastError());
    if (pack) {
        // (pass 1's digit starts, before the second histogram reuses mat)
        hipLaunchKernelGGL(k_take_col0, dim3(blocks_for((int64_t)1 << DB1, 256)), dim3(256), 0,
                           S(ctx), (const uint32_t *)mat, ntiles, 1 << DB1, dstart1);
        hipLaunchKernelGGL((k_hist_part<DB1, DB2>), dim3(ntiles), dim3(RB), 0, S(ctx),
                           (const uint32_t *)a[0], n, L, mat, ntiles, part);
    } else {
        hipLaunchKernelGGL((k_hist<M_GS, DB2>), dim3(ntiles), dim3(RB), 0, S(ctx), a[0], a[1],
                           a[2], n, L + DB1, nost, mat, ntiles, (int)ROWS_LOAD);
    }
    LIME_TRY(scan_exclusive_u32(ctx, mat, mat, ((int64_t)1 << DB2) * ntiles, nullptr));
    if (pack)
        hipLaunchKernelGGL((k_scatter<M_GS, ROWS_LOAD, false, EW_PACK, DB2>), dim3(ntiles),
                           dim3(RB), 0, S(ctx), a[0], a[1], a[2], n, L + DB1, nost, cm, ntiles,
                           o[0], o[1], o[2], (const uint32_t *)nullptr, 0, L);
    else if (w16)
        hipLaunchKernelGGL((k_scatter<M_GS, ROWS_LOAD, false, EW_FROM16, DB2>), dim3(ntiles),
                           dim3(RB), 0, S(ctx), a[0], a[1], a[2], n, L + DB1, nost, cm, ntiles,
                           o[0], o[1], o[2]);
    else
        hipLaunchKernelGGL((k_scatter<M_GS, ROWS_LOAD, false, EW_32, DB2>), dim3(ntiles), dim3(RB),
                           0, S(ctx), a[0], a[1], a[2], n, L + DB1, nost, cm, ntiles, o[0], o[1],
                           o[2]);
    LIME_HIP(hipGetLastError());
    return LIME_OK;
}

int sort_set_impl(lime_ctx *ctx, lime_set *set, bool global, const int32_t *d_contig,
                  const uint32_t *d_start, const uint32_t *d_end, const uint32_t *d_len) {
    const int64_t n = set->n;
    const uint32_t ntiles = (uint32_t)((n + RTILE - 1) / RTILE);
    uint32_t *k0 = nullptr, *e0 = nullptr, *r0 = nullptr, *mat = nullptr;
    SetStats *part, *st;
    // binned sets (bitset painting) keep no row ids: 8 B per row per pass
    const bool keep_rows = set->min_shift == 0;
    const bool stranded = set->strand_in != nullptr;
    const bool row_ties = set->row_ties;  // (gs, ge, row): subtract's tie index
    // the bucketed sort is a candidate for plain sets whose span needs more
    // than TB key bits: its prep then only validates and histograms the
    // first digit (bits [L, L + DB1)), L = bits(span) - TB
    // (and rows enough that the buckets average LMIN rows: a workgroup per
    // bucket costs more than the digit passes below that)
    const int64_t span = set->off.empty() ? 0 : (int64_t)set->off.back();
    const int sbits = span > 1 ? 64 - __builtin_clzll((uint64_t)(span - 1)) : 1;
    // (and few enough that they average at most LAVG / LAVG_M over the span:
    // denser sets take the digit passes, decided before the prep so it runs
    // once -- a validate-only prep then a writing one cost C3 1.4 ms)
    int TB = 0;
    if (keep_rows && !stranded && !row_ties)
        for (int tb = 16; tb <= LIME_SORT_TBMAX && sbits - tb >= 1; ++tb) {
            const int64_t nbs = (span >> (sbits - tb)) + 1;
            if (n < LMIN * nbs) break;  // (sparser still at more digit bits)
            if (n <= LAVG_W * nbs) {
                TB = tb;
                break;
            }
        }
    const bool bucket_cand = TB != 0;
    // 8 + 8, 8 + 9, 9 + 9 bits: at TB = 17 the 9-bit digit goes second,
    // where its runs of ~16 rows per digit and tile carry u32 ends (64-B
    // pieces) instead of u16 widths (32 B), and the first pass reads the
    // prep's rows with 256 digits: 1e9-row sort 22.34 -> 22.03 ms, same box
    const int DB1 = TB / 2, DB2 = TB - DB1;
    // (the digit-count matrix serves both bucket passes: sized for the wider)
    const int mat_bits = bucket_cand ? std::max(DB1, DB2) : 8;
    LIME_TRY(alloc(ctx, &mat, ((size_t)1 << mat_bits) * (ntiles ? ntiles : 1)));
    LIME_TRY(alloc(ctx, &part, (size_t)(ntiles ? ntiles : 1)));
    LIME_TRY(alloc(ctx, &st, 1));
    const int hshift = bucket_cand ? sbits - TB : set->min_shift;
    SetStats h = {0u, 0u, 0xffffffffu, 0u, 0u, 0u, {0, 0}};
    if (n > 0) {
        if (bucket_cand && !global && LIME_SORT_W16) {
            // validate + statistics + histogram, and (gs, u16 width) for the
            // first pass (unused if a width reaches 2^16)
            LIME_TRY(alloc(ctx, &k0, (size_t)n));
            LIME_TRY(alloc(ctx, &e0, (size_t)(n + 1) / 2));
            if (DB1 == 9)
                launch_prep_w16<9>(ctx, set, d_contig, d_start, d_end, d_len, n, k0, e0, part, mat,
                                   ntiles, hshift);
            else
                launch_prep_w16<8>(ctx, set, d_contig, d_start, d_end, d_len, n, k0, e0, part, mat,
                                   ntiles, hshift);
        } else if (bucket_cand) {  // validate + statistics + histogram only
            if (DB1 == 9)
                launch_prep_nowrite<9>(ctx, set, global, d_contig, d_start, d_end, d_len, n, part,
                                       mat, ntiles, hshift);
            else
                launch_prep_nowrite<8>(ctx, set, global, d_contig, d_start, d_end, d_len, n, part,
                                       mat, ntiles, hshift);
        } else {
            LIME_TRY(alloc(ctx, &k0, (size_t)n));
            LIME_TRY(alloc(ctx, &e0, (size_t)n));
            if (keep_rows) LIME_TRY(alloc(ctx, &r0, (size_t)n));
            if (global)
                hipLaunchKernelGGL(k_prep<true>, dim3(ntiles), dim3(RB), 0, S(ctx), d_contig,
                                   d_start, d_end, (const uint32_t *)set->d_off, d_len,
                                   set->n_contigs, n, k0, e0, r0, part, mat, ntiles, hshift);
            else if (set->n_contigs <= PCMAX)
                hipLaunchKernelGGL((k_prep<false, true, true>), dim3(ntiles), dim3(RB), 0, S(ctx),
                                   d_contig, d_start, d_end, (const uint32_t *)set->d_off, d_len,
                                   set->n_contigs, n, k0, e0, nullptr, part, mat, ntiles,
                                   hshift);  // rows = positions: made by the first pass
            else
                hipLaunchKernelGGL(k_prep<false>, dim3(ntiles), dim3(RB), 0, S(ctx), d_contig,
                                   d_start, d_end, (const uint32_t *)set->d_off, d_len,
                                   set->n_contigs, n, k0, e0, nullptr, part, mat, ntiles, hshift);
        }
        hipLaunchKernelGGL(k_stats, dim3(1), dim3(256), 0, S(ctx), (const SetStats *)part,
                           (int64_t)ntiles, st);
        LIME_HIP(hipGetLastError());
        LIME_TRY(read_back(ctx, &h, st, sizeof(h)));
    }
    release(ctx, part);
    release(ctx, st);
    if (h.err) {
        release(ctx, k0);
        release(ctx, e0);
        release(ctx, r0);
        release(ctx, mat);
        if (h.err & 1u) return fail(LIME_ERR_CONTIG, "interval contig id outside the space");
        if (h.err & 2u) return fail(LIME_ERR_RANGE, "interval end < start");
        return fail(LIME_ERR_RANGE, "interval end beyond its contig length");
    }
    set->min_width = n > 0 ? h.min_width : 0;
    set->max_width = h.max_width;
    set->has_zero_width = h.has_zero != 0;
    const int bits = h.max_gs ? 32 - __builtin_clz(h.max_gs) : 1;
    const bool need = n > 1 && (h.unsorted || stranded || row_ties) &&
                      !(set->min_shift > 0 && (h.max_gs >> set->min_shift) == 0);

    if (bucket_cand) {
        // the bucketed sort when the rows are not in order yet and the
        // buckets stay small on average; else materialise (gs, ge, row) the
        // way the digit passes start from
        const int L = sbits - TB;
        const uint32_t nb = (h.max_gs >> L) + 1;
        const int shape = local_shape(TB, n / (int64_t)nb);
        if (need && n / (int64_t)nb <= LAVG_W) {
            uint32_t *a[3], *o[3];
            for (int q = 0; q < 3; ++q) {
                LIME_TRY(alloc(ctx, &a[q], (size_t)n));
                LIME_TRY(alloc(ctx, &o[q], (size_t)n));
            }
            const bool w16 = LIME_SORT_W16 && h.max_width < 65536u;
            // the packed second pass: (gs mod 2^L, width) in one word, the
            // buckets placed from the histogram partials (no key search)
            const bool pack = LIME_SORT_PACK && w16 && L <= 16;
            uint32_t *dstart1 = nullptr, *part = nullptr;
            if (pack) {
                LIME_TRY(alloc(ctx, &dstart1, (size_t)1 << DB1));
                LIME_TRY(alloc(ctx, &part, (size_t)1 << TB));
            }
            PoolGuard<uint32_t> gd{ctx, dstart1}, gpart{ctx, part};
            if (TB == 16)
                LIME_TRY((bucket_passes<8, 8>(ctx, set, global, d_contig, d_start, d_end, n, L, w16,
                                              mat, mat_bits, ntiles, a, o, k0, e0, pack, dstart1,
                                              part)));
            else if (TB == 17)
                LIME_TRY((bucket_passes<8, 9>(ctx, set, global, d_contig, d_start, d_end, n, L, w16,
                                              mat, mat_bits, ntiles, a, o, k0, e0, pack, dstart1,
                                              part)));
            else
                LIME_TRY((bucket_passes<9, 9>(ctx, set, global, d_contig, d_start, d_end, n, L, w16,
                                              mat, mat_bits, ntiles, a, o, k0, e0, pack, dstart1,
                                              part)));
            release(ctx, k0);
            release(ctx, e0);
            // every bucket sorted locally: (o) -> (a)
            uint32_t *start, *over;
            unsigned int *nover;
            LIME_TRY(alloc(ctx, &start, (size_t)nb + 1));
            PoolGuard<uint32_t> g0{ctx, start};
            LIME_TRY(alloc(ctx, &over, (size_t)nb));
            PoolGuard<uint32_t> g1{ctx, over};
            LIME_TRY(alloc(ctx, &nover, 2));
            PoolGuard<unsigned int> g2{ctx, nover};
            LIME_HIP(hipMemsetAsync(nover, 0, 8, S(ctx)));
            if (pack)
                hipLaunchKernelGGL(k_bucket_starts_part, dim3(blocks_for((int64_t)nb + 1, 256)),
                                   dim3(256), 0, S(ctx), (const uint32_t *)dstart1,
                                   (const uint32_t *)mat, (const uint32_t *)part, n, ntiles, nb,
                                   DB1, DB2, start);
            else
                hipLaunchKernelGGL(k_bucket_starts, dim3(blocks_for((int64_t)nb + 1, 256)),
                                   dim3(256), 0, S(ctx), (const uint32_t *)o[0], n, nb, L, start);
            release(ctx, mat);
            LocalArgs la;
            la.k0 = o[0], la.e0 = o[1], la.r0 = o[2];
            la.start = start;
            la.L = L;
            la.zb = h.has_zero ? 1 : 0;
            la.k1 = a[0], la.e1 = a[1], la.r1 = a[2];
            la.nover = nover;
            la.over = over;
            uint32_t *sink;
            LIME_TRY(alloc(ctx, &sink, (size_t)LSINK));
            PoolGuard<uint32_t> g3{ctx, sink};
            la.sink = sink;
            int dev = 0, cus = 256;
            (void)hipGetDevice(&dev);
            (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
            if (cus <= 0) cus = 256;
#define LIME_LOCAL_LAUNCH(PK)                                                                     \
    do {                                                                                          \
        if (shape == 0)                                                                           \
            hipLaunchKernelGGL(k_local_small<PK>,                                                 \
                               dim3(std::min<uint32_t>(nb, 3u * (uint32_t)cus)), dim3(LNT_S), 0,  \
                               S(ctx), la, nb, (const uint32_t *)start);                          \
        else if (shape == 1)                                                                      \
            hipLaunchKernelGGL(LIME_LOCAL_MID(PK), dim3(std::min<uint32_t>(nb, 2u * (uint32_t)cus)), \
                               dim3(512), 0, S(ctx), la, nb, (const uint32_t *)start);            \
        else                                                                                      \
            hipLaunchKernelGGL(LIME_LOCAL_WIDE(PK), dim3(std::min<uint32_t>(nb, (uint32_t)cus)),  \
                               dim3(1024), 0, S(ctx), la, nb, (const uint32_t *)start);           \
        hipLaunchKernelGGL(k_local_big<PK>, dim3((unsigned)(cus > 0 ? cus : 256)), dim3(LNT_B),  \
                           0, S(ctx), la);                                                        \
    } while (0)
            if (pack)
                LIME_LOCAL_LAUNCH(true);
            else
                LIME_LOCAL_LAUNCH(false);
#undef LIME_LOCAL_LAUNCH
            LIME_HIP(hipGetLastError());
            for (int q = 0; q < 3; ++q) release(ctx, o[q]);
            set->gs = a[0];
            set->ge = a[1];
            set->row = a[2];
            // the first pass read the caller's arrays after the statistics
            // read-back: on the context's own stream the call returns only once
            // they are consumed (a caller stream orders their reuse itself)
            if (ctx->stream == ctx->own_stream) LIME_HIP(hipStreamSynchronize(S(ctx)));
            return LIME_OK;
        }
        // (in order, or dense buckets) the digit-pass layout from the caller's rows
        release(ctx, k0);  // (the speculative (gs, u16 width) of the prep)
        release(ctx, e0);
        LIME_TRY(alloc(ctx, &k0, (size_t)n));
        LIME_TRY(alloc(ctx, &e0, (size_t)n));
        LIME_TRY(alloc(ctx, &r0, (size_t)n));
        if (global) {
            LIME_HIP(hipMemcpyAsync(k0, d_contig, 4 * (size_t)n, hipMemcpyDeviceToDevice, S(ctx)));
            LIME_HIP(hipMemcpyAsync(e0, d_start, 4 * (size_t)n, hipMemcpyDeviceToDevice, S(ctx)));
            LIME_HIP(hipMemcpyAsync(r0, d_end, 4 * (size_t)n, hipMemcpyDeviceToDevice, S(ctx)));
        } else {
            // gs / ge, and the digit-0 histogram the passes below start from
            PoolGuard<SetStats> gp{ctx, part};
            PoolGuard<SetStats> gq{ctx, st};
            LIME_TRY(alloc(ctx, &part, (size_t)ntiles));
            LIME_TRY(alloc(ctx, &st, 1));
            if (set->n_contigs <= PCMAX)
                hipLaunchKernelGGL((k_prep<false, true, true>), dim3(ntiles), dim3(RB), 0, S(ctx),
                                   d_contig, d_start, d_end, (const uint32_t *)set->d_off, d_len,
                                   set->n_contigs, n, k0, e0, nullptr, part, mat, ntiles, 0);
            else
                hipLaunchKernelGGL(k_prep<false>, dim3(ntiles), dim3(RB), 0, S(ctx), d_contig,
                                   d_start, d_end, (const uint32_t *)set->d_off, d_len,
                                   set->n_contigs, n, k0, e0, nullptr, part, mat, ntiles, 0);
            LIME_HIP(hipGetLastError());
        }
    }

    if (need) {
        uint32_t *k1, *e1, *r1 = nullptr;
        LIME_TRY(alloc(ctx, &k1, (size_t)n));
        LIME_TRY(alloc(ctx, &e1, (size_t)n));
        if (keep_rows) LIME_TRY(alloc(ctx, &r1, (size_t)n));
        std::vector<std::pair<int, int>> passes;  // (mode, shift), least significant first
        if (row_ties) {
            // (gs, ge, row): row digits, then width digits, then gs
            for (int sh = 0; sh < 32; sh += 8) passes.push_back({M_RW, sh});
            const int wbits = h.max_width ? 32 - __builtin_clz(h.max_width) : 0;
            for (int sh = 0; sh < wbits; sh += 8) passes.push_back({M_GE, sh});
        } else if (stranded) {
            // RegionOrdering (start, end, strand): strand, then ge, then gs.
            // The strand pass runs first, while row i is still input row i.
            const int wbits = h.max_width ? 32 - __builtin_clz(h.max_width) : 0;
            if (!set->strand_uniform) passes.push_back({M_ST, 0});
            for (int sh = 0; sh < wbits; sh += 8) passes.push_back({M_GE, sh});
        } else if (set->has_zero_width && set->max_width > 0 && set->min_shift == 0) {
            // (all rows zero-width: the bit is constant, no pass)
            passes.push_back({M_NZ, 0});
        }
        for (int sh = 0; sh < bits; sh += 8)
            if (sh >= set->min_shift) passes.push_back({M_GS, sh});
        // caller rows: the first pass writes row = position (k_prep did not)
        int rows = !keep_rows ? ROWS_NONE : global ? ROWS_LOAD : ROWS_IDENT;
        // k_prep already histogrammed the gs digit at its shift (the bucketed
        // candidate's fallback re-ran it at 0)
        const int prep_shift = bucket_cand ? 0 : hshift;
        bool have = passes.front().first == M_GS && passes.front().second == prep_shift &&
                    !(bucket_cand && global);
        // GS passes only, rows kept, every width < 2^16: u16 widths between
        // the first and the last pass (EW_TO16 .. EW_FROM16)
        bool w16 = LIME_SORT_W16 && keep_rows && passes.size() >= 2 && h.max_width < 65536u;
        for (auto &p : passes) w16 = w16 && p.first == M_GS;
        for (size_t q = 0; q < passes.size(); ++q) {
            const auto &p = passes[q];
            const int ew = !w16 ? EW_32 : q == 0 ? EW_TO16 : q + 1 == passes.size() ? EW_FROM16 : EW_16;
            LIME_TRY(radix_pass(ctx, p.first, p.second, have, n, k0, e0, r0, set->strand_in, k1,
                                e1, r1, mat, ntiles, rows, nullptr, 0, ew));
            have = false;
            if (rows == ROWS_IDENT) rows = ROWS_LOAD;
            std::swap(k0, k1);
            std::swap(e0, e1);
            std::swap(r0, r1);
        }
        release(ctx, k1);
        release(ctx, e1);
        release(ctx, r1);
    } else if (keep_rows && !global && n > 0) {
        // already in order: the row ids are the positions
        hipLaunchKernelGGL(k_rows_iota, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, S(ctx),
                           r0, n);
        LIME_HIP(hipGetLastError());
    }
    release(ctx, mat);
    set->gs = k0;
    set->ge = e0;
    set->row = r0;
    return LIME_OK;
}

}  // namespace lime

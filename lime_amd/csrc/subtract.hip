// subtract.hip -- DistributedSubtract (difference) per left row.
//
// Reference: Subtract.scala:91-116.  For each sorted left row L the hits are
// the cached right rows with overlapsBy(L, R) >= threshold, in sorted order;
// they are folded into blocks (foldLeft(List(head)) over the WHOLE hit list,
// so the head is visited twice -- a no-op for a non-empty head, a duplicated
// block for a zero-width one), and each block independently contributes
// [L.s, B.s) if B.s > L.s and [B.e, L.e) if L.e > B.e (quirk Q5), blocks in
// REVERSE order (the fold prepends).  No hit: (L, None).
// Mode LIME_SUBTRACT_SET emits L minus the union of the blocks instead.
//
// Hits of a left row a in sorted order are
//   spanning:  b.s < a.s, B.ge > thr   (thr = a.s, or a.s + t - 1)
//   inside:    j in [lo1, hi1) (width(b) >= t when t >= 1)
// where [lo1, hi1) is the intersect stream-0 candidate range.  Every
// spanning hit contains the point a.s, so they all overlap each other and the
// fold merges them into ONE block: [start of the first spanning hit, max end
// of the rows before lo1) -- the first spanning hit by a galloping search of
// B's inclusive prefix max of ends (monotone), the max end is that prefix
// max at lo1 - 1.  No walk over the spanning rows: a long B row (a gene body,
// a segmental duplication) costs every later left row O(log n), not a walk
// back to it (the O(n_A * n_B) cliff of a per-row backward scan).  The block
// head is the spanning hit with the smallest (start, end, row): the rows
// sharing the first hit's start are scanned for it.  The inside hits then
// continue the fold one by one (work proportional to the hits).
// One thread per left row, two passes (count, write); the write pass stages
// a block's records in LDS and stores them lane-consecutively.
#include <type_traits>

#include "common.hpp"

namespace lime {

int owner_ranges(lime_ctx *ctx, const lime_set *O, const lime_set *P, int st, int64_t threshold,
                 uint32_t *olo, uint32_t *ocnt);

namespace {

constexpr int SUB_B = 256;

struct SubArgs {
    // per block (inline ranges: per 4 blocks): first B row a spanning hit can be
    const uint32_t *wstart;
    // k_sub_fused: per tile, the first B row past every inside hit of its
    // rows (a start >= the last row's start + A's max width); null otherwise
    const uint32_t *wend;
    // runs: every block's own window start, found by the count pass in its
    // staged window and read by the write pass (no search there)
    uint32_t *bwlo;
    uint32_t maxw;  // max width of B
    const uint32_t *ags, *age, *arow;
    const uint32_t *bgs, *bge, *brow, *bpmax;
    const uint32_t *olo, *ocnt;
    // RUNS (threshold <= 0): B's merge runs -- run id of every sorted row
    const uint32_t *brun;
    int64_t na, nb;
    int64_t t;
    int mode;
    // zw = B holds zero-width rows
    int zw;
    uint64_t *count;        // pass 1
    // RUNS: every left row's record count from the count pass (255: the write
    // pass folds the row twice, counting first), so the write pass folds once
    uint8_t *rcnt;
    const uint64_t *off;    // pass 2
    unsigned int *err;      // pass 2 (RUNS): a block's recount differs from pass 1
    uint32_t *ogs, *oge, *oar, *obr;
    // the tie index of B (rows of its multi-row same-start groups by (gs,
    // ge, row)); tn = 0: B has no same-start group past TIE_G rows
    const uint32_t *tgs, *tge, *trow;
    int64_t tn;
};

// A block's head is the min (end, row) among its same-start hits.  Past
// TIE_G of them (identical PCR duplicates, repeated annotations) the head
// comes from the tie index by one search instead of a walk over the group:
// the first row with start bs and end > thr.  (A walk per left row was
// O(n_A x D) for D rows sharing a start.)
constexpr int TIE_G = 16;
__device__ __forceinline__ void tie_head(const SubArgs &sa, uint32_t bs, uint32_t thr,
                                         uint32_t &bh, uint32_t &bhe) {
    int64_t lo = 0, hi = sa.tn;  // first p with (tgs, tge) > (bs, thr)
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        const uint32_t g = sa.tgs[mid];
        if (g < bs || (g == bs && sa.tge[mid] <= thr))
            lo = mid + 1;
        else
            hi = mid;
    }
    if (lo < sa.tn && sa.tgs[lo] == bs) {
        bh = sa.trow[lo];
        bhe = sa.tge[lo];
    }
}

__device__ __forceinline__ int64_t first_spanning(const uint32_t *__restrict__ pm, int64_t lo1,
                                                  uint32_t thr) {
    if (lo1 == 0 || pm[lo1 - 1] <= thr) return lo1;
    int64_t r = lo1 - 1, step = 1;
    while (r - step >= 0 && pm[r - step] > thr) {
        r -= step;
        step <<= 1;
    }
    int64_t lo = r - step + 1;
    if (lo < 0) lo = 0;
    // first j in [lo, r] with pm[j] > thr
    int64_t hi = r;
    while (lo < hi) {
        int64_t mid = lo + ((hi - lo) >> 1);
        if (pm[mid] > thr)
            hi = mid;
        else
            lo = mid + 1;
    }
    return lo;
}

// the runs count pass (k_sub_count_runs): blocks per workgroup, rows, B window
#ifndef LIME_SUB_CNT_WAVES
#define LIME_SUB_CNT_WAVES 4
#endif
#ifndef LIME_SUB_CNT_WIN
#define LIME_SUB_CNT_WIN 1536
#endif
constexpr int CNT_WAVES = LIME_SUB_CNT_WAVES;
constexpr int CNT_ROWS = CNT_WAVES * SUB_B;  // left rows per workgroup
constexpr int CNT_WIN = LIME_SUB_CNT_WIN;    // B rows staged (C2: ~1200 needed at 4 waves)
constexpr int SCAP = 512;   // records staged per block in the write pass
constexpr int BWIN = 1024;  // B rows of a block's hit window staged in LDS
// (24 KiB of LDS in all: the walk is latency-bound, occupancy is its speed)

// A left row's inside-hit range [lo1, hi1) at threshold <= 0: stream 0 of
// owner_ranges (intersect.hip k_count, tp = 1): lo = lb(B.gs, a.s) past the
// zero-width rows at a.s, hi = lb(B.gs, a.e) if a.e > a.s, else lo.  Searched
// in the staged starts w_gs of B rows [wlo, wlo + nst) (wlo <= lb(B.gs, a.s):
// the window start of a block is the bound of its first row minus B's max
// width), then in global memory past them.
__device__ __forceinline__ void sub_range(const SubArgs &sa, const uint32_t *w_gs, int64_t wlo,
                                          int nst, uint32_t a_s, uint32_t a_e, int64_t &lo1,
                                          int64_t &hi1) {
    auto lb = [&](int64_t from, uint32_t key) -> int64_t {
        if (from - wlo < nst) {
            int l = (int)(from - wlo), r = nst;
            while (l < r) {
                const int m = (l + r) >> 1;
                if (w_gs[m] < key)
                    l = m + 1;
                else
                    r = m;
            }
            if (l < nst) return wlo + l;
            from = wlo + nst;
        }
        return dev::lower_bound(sa.bgs, from, sa.nb, (int64_t)key);
    };
    int64_t lo = lb(wlo, a_s);
    int64_t hi = a_e > a_s ? lb(lo, a_e) : lo;
    if (sa.zw) {
        while (lo < sa.nb && (lo - wlo < nst ? w_gs[lo - wlo] : sa.bgs[lo]) == a_s &&
               sa.bge[lo] == a_s)
            ++lo;
        if (hi < lo) hi = lo;
    }
    lo1 = lo;
    hi1 = hi;
}

// per block: first B row that can span any of the block's left rows: a
// spanning b starts after a.s - max width(B).  One LANE per block, a
// branch-free binary search (as k_windows_lane): a 65-ary wave search
// fetched 64 lanes' lines per level, 4 GB per 1e9-row subtract (0.65 ms)
// (wend, when given: the first B row starting at or past the block's last
// row's start + maxwa, A's max width -- the two searches interleaved)
__global__ __launch_bounds__(256) void k_sub_window(const uint32_t *__restrict__ ags, int64_t na,
                                                    const uint32_t *__restrict__ bgs, int64_t nb,
                                                    uint32_t maxw, int64_t nblk, int stride,
                                                    uint32_t *__restrict__ wstart, uint32_t maxwa,
                                                    uint32_t *__restrict__ wend,
                                                    unsigned int *__restrict__ wmax) {
    const int64_t b0 = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const bool ok = b0 < nblk;  // (no early exit: the wave reduces wmax below)
    const int64_t b = ok ? b0 : nblk - 1;
    const int64_t key = (int64_t)ags[b * SUB_B * stride] - maxw;
    const int64_t hkey =
        wend ? (int64_t)ags[min((b + 1) * SUB_B * stride, na) - 1] + maxwa : (int64_t)0;
    int64_t r = 0, h = 0;  // first j with bgs[j] >= key, >= hkey
    for (int64_t step = nb > 0 ? (int64_t)1 << (63 - __builtin_clzll((uint64_t)nb)) : 0; step > 0;
         step >>= 1) {
        if (r + step <= nb && (int64_t)bgs[r + step - 1] < key) r += step;
        if (wend && h + step <= nb && (int64_t)bgs[h + step - 1] < hkey) h += step;
    }
    if (ok) {
        wstart[b] = (uint32_t)r;
        if (wend) wend[b] = (uint32_t)h;
    }
    if (wmax) {  // the longest window (wend + 1 - wstart), one atomic per wave
        const uint32_t len = dev::wave_reduce_max((uint32_t)min(h + 1 - r, (int64_t)0xffffffff));
        if (dev::lane_id() == 0) atomicMax(wmax, len);
    }
}

// RUNS (threshold <= 0): the inside hits are not walked one by one.  A new
// block starts at an inside hit exactly when its start reaches the prefix
// max end of every earlier B row -- B's merge run boundaries (earlier blocks
// end at or before the current one's start; non-hit rows before a.s end at or
// before a.s).  So each block is a run of B cut at hi1: seeded by the run's
// first row (head re-picked among its same-start rows as below), ended by
// the prefix max at its last row before hi1.  O(runs overlapping a) per left
// row instead of O(hits): at C2's depth (~160 hits per row) one or two runs.
template <bool WRITE, bool RUNS>
__device__ __forceinline__ void sub_block(const SubArgs &sa, const int64_t blk) {
    __shared__ uint32_t st_gs[WRITE ? SCAP : 1], st_ge[WRITE ? SCAP : 1];
    __shared__ uint32_t st_ar[WRITE ? SCAP : 1], st_br[WRITE ? SCAP : 1];
    __shared__ uint32_t w_pm[BWIN];
    // (RUNS reads ends and row ids at block heads only: global memory.
    // Staging them too cost the sparse 1e9-row subtract 12.4 -> 14.3 ms)
    __shared__ uint32_t w_gs[BWIN], w_ge[RUNS ? 1 : BWIN], w_row[RUNS ? 1 : BWIN];
    __shared__ uint32_t w_run[RUNS ? BWIN : 1];
    __shared__ uint32_t s_whi[SUB_B / 64];
    const int64_t i = (int64_t)blk * SUB_B + threadIdx.x;
    // RUNS write pass: a block without records has nothing to do (at C2's
    // depth nearly every block)
    if (RUNS && WRITE && sa.off[blk + 1] == sa.off[blk]) return;
    // the block's hit window [wlo, whi) of B (spanning and inside hits):
    // consecutive left rows share most of it, so it is loaded once,
    // coalesced, into LDS
    // RUNS: each row's inside-hit range is found in the staged window (no
    // owner_ranges pass)
    constexpr bool inl = RUNS;
    // inline ranges: wstart holds one start per 4 blocks (the count pass's
    // workgroups); the block's own is searched from there (every wave alike)
    int64_t wlo;
    if (inl && WRITE) {
        wlo = sa.bwlo[blk];  // (the count pass's)
    } else if (inl) {
        const int64_t c = sa.wstart[blk / CNT_WAVES];
        const int64_t key = max((int64_t)sa.ags[(int64_t)blk * SUB_B] - sa.maxw, (int64_t)0);
        wlo = c + dev::wave_lower_bound(sa.bgs + c, sa.nb - c, key);
    } else {
        wlo = sa.wstart[blk];
    }
    // inline ranges (RUNS): B rows from wlo staged with their starts, 256 at
    // a time up to BWIN, until the staged starts pass every end of the
    // block's left rows (no row's hit lies past that: sparse sets need a
    // fraction of BWIN rows, 12 B each, per block)
    int nst = 0;
    if (inl) {
        uint32_t amax = 0;
        for (int64_t q = (int64_t)blk * SUB_B + threadIdx.x; q < sa.na &&
             q < (int64_t)(blk + 1) * SUB_B; q += SUB_B)
            amax = sa.age[q];
        amax = dev::wave_reduce_max(amax);
        if (dev::lane_id() == 0) s_whi[threadIdx.x / 64] = amax;
        __syncthreads();
        for (int w = 0; w < SUB_B / 64; ++w) amax = max(amax, s_whi[w]);
        const int cap = (int)min((int64_t)BWIN, sa.nb - wlo);
        for (int k0 = 0; k0 < cap; k0 += SUB_B) {  // (uniform over the block)
            const int k = k0 + threadIdx.x;
            if (k < cap) {
                w_pm[k] = sa.bpmax[wlo + k];
                w_gs[k] = sa.bgs[wlo + k];
                w_run[k] = sa.brun[wlo + k];
            }
            nst = min(k0 + SUB_B, cap);
            __syncthreads();
            if (w_gs[nst - 1] >= amax) break;
        }
    }
    if (!inl) {
        uint32_t h = 0;
        if (i < sa.na) h = sa.olo[i] + sa.ocnt[i];
        h = dev::wave_reduce_max(h);
        if (dev::lane_id() == 0) s_whi[threadIdx.x / 64] = h;
    }
    __syncthreads();
    int64_t whi = inl ? wlo + nst : wlo;
    if (!inl)
        for (int w = 0; w < SUB_B / 64; ++w) whi = max(whi, (int64_t)s_whi[w]);
    const bool win = whi - wlo <= BWIN;
    if (win && !inl)
        for (int64_t k = threadIdx.x; k < whi - wlo; k += SUB_B) {
            w_pm[k] = sa.bpmax[wlo + k];
            if (RUNS) {
                w_run[k] = sa.brun[wlo + k];
            } else {
                w_gs[k] = sa.bgs[wlo + k];
                w_ge[k] = sa.bge[wlo + k];
                w_row[k] = sa.brow[wlo + k];
            }
        }
    __syncthreads();
    // B's arrays at row j, from the window when staged
    // (inl: rows [wlo, whi) are staged whatever the rows' ranges)
    auto inw = [&](int64_t j) { return win && j >= wlo && (!inl || j < whi); };
    auto Bgs = [&](int64_t j) {
        return (win && !RUNS) || (inl && inw(j)) ? w_gs[j - wlo] : sa.bgs[j];
    };
    auto Bge = [&](int64_t j) { return win && !RUNS ? w_ge[j - wlo] : sa.bge[j]; };
    auto Brow = [&](int64_t j) { return win && !RUNS ? w_row[j - wlo] : sa.brow[j]; };
    auto Bpm = [&](int64_t j) { return inw(j) ? w_pm[j - wlo] : sa.bpmax[j]; };
    auto Brun = [&](int64_t j) { return RUNS ? (inw(j) ? w_run[j - wlo] : sa.brun[j]) : 0u; };
    // end of j's run cut at hi1 (j < hi1): a search over the run ids
    // (monotone)
    auto run_end = [&](int64_t j, int64_t hi1) -> int64_t {
        const uint32_t r = Brun(j);
        if (Brun(hi1 - 1) == r) return hi1;
        int64_t l = j + 1, h = hi1 - 1;
        while (l < h) {
            const int64_t m = (l + h) >> 1;
            if (Brun(m) > r)
                h = m;
            else
                l = m + 1;
        }
        return l;
    };
    // the block's output window (write pass): staged in LDS when it fits
    int64_t bbase = 0, bend = 0;
    bool staged = false;
    if (WRITE && !RUNS) {
        const int64_t first = (int64_t)blk * SUB_B;
        const int64_t last = min(first + SUB_B, sa.na);
        bbase = (int64_t)sa.off[first];
        bend = (int64_t)sa.off[last];
        staged = bend - bbase <= SCAP;
    }
    uint32_t as = 0, ae = 0, ar = 0;
    if (i < sa.na) as = sa.ags[i], ae = sa.age[i], ar = sa.arow[i];
    int64_t rlo = 0, rhi = 0;  // inline: the row's inside-hit range
    if (inl && i < sa.na) sub_range(sa, w_gs, wlo, nst, as, ae, rlo, rhi);
    const int64_t t = sa.t;
    int64_t pos = 0, end = 0;
    if (WRITE && !RUNS && i < sa.na) {
        pos = (int64_t)sa.off[i];
        end = (int64_t)sa.off[i + 1];
    }
    auto emit = [&](uint32_t s, uint32_t e, uint32_t br, int64_t at) {
        if (WRITE && RUNS && (at < bbase || at >= bend)) {  // (a count mismatch: flagged)
            atomicOr(sa.err, 1u);
            return;
        }
        if (WRITE) {
            if (staged) {
                const int k = (int)(at - bbase);
                st_gs[k] = s;
                st_ge[k] = e;
                st_ar[k] = ar;
                st_br[k] = br;
            } else {
                sa.ogs[at] = s;
                sa.oge[at] = e;
                sa.oar[at] = ar;
                sa.obr[at] = br;
            }
        }
    };
    // the fold of one left row; do_emit = false only counts its records
    auto fold = [&](bool do_emit) -> uint64_t {
    const bool wr = WRITE && do_emit;
    uint64_t n_out = 0;
    bool any = false;
    if (i < sa.na && !(t >= 1 && (int64_t)(ae - as) < t)) {
        const int64_t lo1 = inl ? rlo : (int64_t)sa.olo[i];
        const int64_t hi1 = inl ? rhi : lo1 + (int64_t)sa.ocnt[i];
        const uint32_t thr = t <= 0 ? as : (uint32_t)((int64_t)as + t - 1);
        // fold state.  The block's value is its head = first hit in the
        // reference's (start, end, row) order; the device order only ties
        // starts by (zero-width first, row), so among same-start non-empty
        // hits the head is re-picked as the min (end, row).
        uint32_t bs = 0, be = 0, bh = 0, bhe = 0;  // block, head row, head end
        uint64_t cum = 0;  // remnants of finished blocks (lime mode, write order)
        uint32_t setpos = as;
        // the spanning block (all spanning hits overlap at a.s): the first
        // spanning row lies in [wlo, lo1) (rows before wlo end before a.s)
        const uint32_t pm_last = lo1 > 0 ? Bpm(lo1 - 1) : 0u;
        if (lo1 > 0 && pm_last > thr) {
            int64_t j0;
            if (win && (!inl || lo1 - 1 < whi)) {  // first j in [wlo, lo1) with pmax > thr, in LDS
                int64_t lo = wlo, hi = lo1 - 1;
                while (lo < hi) {
                    const int64_t mid = (lo + hi) >> 1;
                    if (w_pm[mid - wlo] > thr)
                        hi = mid;
                    else
                        lo = mid + 1;
                }
                j0 = lo;
            } else {
                j0 = first_spanning(sa.bpmax, lo1, thr);
            }
            any = true;
            bs = Bgs(j0);
            be = pm_last;
            bh = Brow(j0);
            bhe = Bge(j0);
            int64_t j = j0 + 1;
            for (; j < lo1 && j <= j0 + TIE_G && Bgs(j) == bs; ++j) {
                const uint32_t ge = Bge(j), row = Brow(j);
                if (ge > thr && (ge < bhe || (ge == bhe && row < bh))) {
                    bh = row;
                    bhe = ge;
                }
            }
            if (j < lo1 && Bgs(j) == bs) tie_head(sa, bs, thr, bh, bhe);  // a long group
        }
        // close the current block (bs, be, bh): its records
        auto close_block = [&]() {
            if (sa.mode == LIME_SUBTRACT_LIME) {
                uint32_t r = (bs > as) + (ae > be);
                if (wr) {
                    int64_t at = end - (int64_t)cum - r;
                    if (bs > as) emit(as, bs, bh, at++);
                    if (ae > be) emit(be, ae, bh, at++);
                }
                cum += r;
            } else {
                if (bs > setpos) {
                    if (wr) emit(setpos, bs, bh, pos + (int64_t)cum);
                    ++cum;
                }
                if (be > setpos) setpos = be;
            }
        };
        if (RUNS) {
            int64_t j = lo1;
            // the spanning block goes on through the inside rows of its run
            if (any && j < hi1 && Brun(j) == Brun(lo1 - 1)) {
                const int64_t nx = run_end(j, hi1);
                be = max(be, Bpm(nx - 1));
                j = nx;
            }
            while (j < hi1) {
                const uint32_t r = Brun(j);
                const int64_t nx = run_end(j, hi1);
                const uint32_t gs = Bgs(j), ge = Bge(j), row = Brow(j);
                if (!any) {  // foldLeft(List(head)): the head is folded against itself
                    any = true;
                    if (ge == gs) {  // a zero-width head closes a duplicate of itself
                        bs = be = gs;
                        bh = row;
                        bhe = ge;
                        close_block();
                    }
                } else {
                    close_block();
                }
                bs = gs;
                be = ge;
                bh = row;
                bhe = ge;
                // the head among the run's same-start non-empty hits: min (end, row)
                if (bhe > bs) {
                    int64_t k = j + 1;
                    for (; k < nx && k <= j + TIE_G && Bgs(k) == bs; ++k) {
                        const uint32_t e2 = Bge(k), r2 = Brow(k);
                        if (e2 < bhe || (e2 == bhe && r2 < bh)) {
                            bh = r2;
                            bhe = e2;
                        }
                    }
                    if (k < nx && Bgs(k) == bs) tie_head(sa, bs, bs, bh, bhe);  // a long group
                }
                be = max(be, Bpm(nx - 1));
                j = nx;
            }
        }
        // four hits per step: their loads are independent of the fold state
        for (int64_t j4 = lo1; !RUNS && j4 < hi1; j4 += 4) {
            uint32_t vg[4], ve[4], vr[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int64_t j = j4 + q;
                const bool ok = j < hi1;
                vg[q] = ok ? Bgs(j) : 0u;
                ve[q] = ok ? Bge(j) : 0u;
                vr[q] = ok ? Brow(j) : 0u;
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) {
            if (j4 + q >= hi1) break;
            const uint32_t gs = vg[q], ge = ve[q];
            if (t >= 1 && (int64_t)(ge - gs) < t) continue;
            const uint32_t row = vr[q];
            if (!any) {  // foldLeft(List(filteredCache.head)): the head seeds the
                any = true;  // list and is then folded against itself once
                bs = gs;
                be = ge;
                bh = row;
                bhe = ge;
            }
            if (be > gs && bs < ge) {  // block.overlaps(b): hull
                if (gs == bs && bhe > bs && (ge < bhe || (ge == bhe && row < bh))) {
                    bh = row;
                    bhe = ge;
                }
                bs = gs < bs ? gs : bs;
                be = ge > be ? ge : be;
            } else {
                // close block (bs, be, bh)
                if (sa.mode == LIME_SUBTRACT_LIME) {
                    uint32_t r = (bs > as) + (ae > be);
                    if (wr) {
                        int64_t at = end - (int64_t)cum - r;
                        if (bs > as) emit(as, bs, bh, at++);
                        if (ae > be) emit(be, ae, bh, at++);
                    }
                    cum += r;
                } else {
                    if (bs > setpos) {
                        if (wr) emit(setpos, bs, bh, pos + (int64_t)cum);
                        ++cum;
                    }
                    if (be > setpos) setpos = be;
                }
                bs = gs;
                be = ge;
                bh = row;
                bhe = ge;
            }
            }
        }
        if (any) {  // close the last block
            if (sa.mode == LIME_SUBTRACT_LIME) {
                uint32_t r = (bs > as) + (ae > be);
                if (wr) {
                    int64_t at = end - (int64_t)cum - r;
                    if (bs > as) emit(as, bs, bh, at++);
                    if (ae > be) emit(be, ae, bh, at++);
                }
                cum += r;
            } else {
                if (bs > setpos) {
                    if (wr) emit(setpos, bs, bh, pos + (int64_t)cum);
                    ++cum;
                }
                if (be > setpos) setpos = be;
                if (ae > setpos) {
                    if (wr) emit(setpos, ae, bh, pos + (int64_t)cum);
                    ++cum;
                }
            }
            n_out = cum;
        }
    }
    if (i < sa.na && !any) {
        if (wr) emit(as, ae, 0xffffffffu, pos);
        n_out = 1;
    }
    return n_out;
    };
    if (!RUNS) {
        const uint64_t n_out = fold(WRITE);
        if (!WRITE) {
            if (i < sa.na) sa.count[i] = n_out;
            return;
        }
    } else {
        // RUNS: per-block totals (count pass); the write pass counts again
        // (O(runs) per row) and places its rows by a block scan
        __shared__ uint64_t s_part[SUB_B / 64];
        // (write pass: the count pass's per-row count; the sparse 1e9-row
        // subtract's write pass folded every row twice)
        uint64_t n_out;
        if (WRITE) {
            const uint32_t rc = i < sa.na ? sa.rcnt[i] : 0u;
            n_out = rc < 255u ? rc : fold(false);
        } else {
            n_out = fold(false);
        }
        const uint64_t inc = dev::wave_inclusive_sum(n_out);
        if (dev::lane_id() == 63) s_part[threadIdx.x / 64] = inc;
        __syncthreads();
        uint64_t before = 0, total = 0;
        for (int w = 0; w < SUB_B / 64; ++w) {
            if (w < (int)(threadIdx.x / 64)) before += s_part[w];
            total += s_part[w];
        }
        if (!WRITE) {
            if (threadIdx.x == 0) sa.count[blk] = total;
            return;
        }
        bbase = (int64_t)sa.off[blk];
        // the recount must equal the count pass's block total (k_sub_count_runs
        // folds the same runs): a mismatch would write outside the block
        if ((int64_t)total != (int64_t)sa.off[blk + 1] - bbase) {
            if (threadIdx.x == 0) atomicOr(sa.err, 1u);
            return;
        }
        bend = bbase + (int64_t)total;
        staged = total <= (uint64_t)SCAP;
        pos = bbase + (int64_t)(before + inc - n_out);
        end = pos + (int64_t)n_out;
        // (a row without records -- covered by B in lime mode: 85 % of the
        // sparse 1e9-row subtract's rows -- has nothing to fold for)
        if (n_out > 0 && fold(true) != n_out) atomicOr(sa.err, 1u);
    }
    if (staged) {  // the block's records, lane-consecutive
        __syncthreads();
        const int cnt = (int)(bend - bbase);
        for (int k = threadIdx.x; k < cnt; k += SUB_B) {
            sa.ogs[bbase + k] = st_gs[k];
            sa.oge[bbase + k] = st_ge[k];
            sa.oar[bbase + k] = st_ar[k];
            sa.obr[bbase + k] = st_br[k];
        }
    }
}

// One block of left rows per workgroup, or (RUNS write pass with records
// rare, SWEEP) a sweep: each workgroup tests SUB_B blocks' record counts at
// once and folds only the blocks that have records (C2's inputs: 16 records
// in 390k blocks, whose one-workgroup-per-block launch cost 90 us)
template <bool WRITE, bool RUNS, bool SWEEP = false>
__global__ __launch_bounds__(SUB_B) void k_subtract(SubArgs sa) {
    if (SWEEP) {
        __shared__ uint64_t s_mask[SUB_B / 64];
        const int64_t nblk = (sa.na + SUB_B - 1) / SUB_B;
        for (int64_t b0 = (int64_t)blockIdx.x * SUB_B; b0 < nblk;
             b0 += (int64_t)gridDim.x * SUB_B) {
            const int64_t b = b0 + threadIdx.x;
            const uint64_t m = __ballot(b < nblk && sa.off[b + 1] != sa.off[b]);
            if (dev::lane_id() == 0) s_mask[threadIdx.x / 64] = m;
            __syncthreads();
            for (int w = 0; w < SUB_B / 64; ++w) {
                for (uint64_t mm = s_mask[w]; mm; mm &= mm - 1) {  // (uniform)
                    sub_block<WRITE, RUNS>(sa, b0 + 64 * w + __builtin_ctzll(mm));
                    __syncthreads();
                }
            }
            __syncthreads();
        }
    } else {
        sub_block<WRITE, RUNS>(sa, blockIdx.x);
    }
}

// RUNS count pass: the fold of k_subtract<false, true>, counting only, four
// 256-row blocks per workgroup (one per wave: its block total is a wave sum).
// The per-row work of that fold is a chain of dependent loads (window start,
// candidate range, spanning start, run ids): here CNT_WIN B rows from the
// workgroup's window start are staged in LDS at once, and every row finds its
// inside-hit range in them (sub_range: no owner_ranges pass), so 1024 rows
// cost two load round trips and one barrier, then fold from LDS and
// registers.  A run's end inside the row's range is found by a search over
// the (monotone) run ids, so no first-row-of-run table is built.  Rows
// outside the window (a B row wider than it holds) read global memory, as in
// k_subtract.

// (wstart: sa.wstart again, restrict: the workgroup's window start is a
// scalar load, so the window's loads issue beside the rows' -- as
// k_sub_fused, whose loads are batched the same way)
__global__ __launch_bounds__(CNT_WAVES * 64) void k_sub_count_runs(SubArgs sa, int64_t nblk,
                                                                  const uint32_t *__restrict__ wstart) {
    __shared__ uint32_t w_pm[CNT_WIN], w_gs[CNT_WIN], w_run[CNT_WIN];
    const int wv = threadIdx.x / 64, lane = dev::lane_id();
    const int64_t base = (int64_t)blockIdx.x * CNT_ROWS + (int64_t)wv * SUB_B;
    constexpr int RPL = SUB_B / 64;  // rows per lane
    uint32_t as[RPL], ae[RPL];
    // every load unconditional (clamped, zeroed past the set)
#pragma unroll
    for (int k = 0; k < RPL; ++k) {
        const int64_t i = base + k * 64 + lane;
        const int64_t ic = min(i, sa.na - 1);
        const uint32_t s_ = sa.ags[ic], e_ = sa.age[ic];
        as[k] = i < sa.na ? s_ : 0u;
        ae[k] = i < sa.na ? e_ : 0u;
    }
    // the workgroup's window start (its first block's); the window staged by
    // one batch of unconditional loads (lanes past it re-read its last row)
    const int64_t wlo = wstart[blockIdx.x];
    const int nst = (int)min((int64_t)CNT_WIN, sa.nb - wlo);
    constexpr int WPT = (CNT_WIN + CNT_WAVES * 64 - 1) / (CNT_WAVES * 64);
    if (nst > 0) {  // (uniform)
        uint32_t vp[WPT], vg[WPT], vr[WPT];
#pragma unroll
        for (int q = 0; q < WPT; ++q) {
            const int64_t j = wlo + min(q * CNT_WAVES * 64 + (int)threadIdx.x, nst - 1);
            vp[q] = sa.bpmax[j];
            vg[q] = sa.bgs[j];
            vr[q] = sa.brun[j];
        }
#pragma unroll
        for (int q = 0; q < WPT; ++q) {
            const int k = q * CNT_WAVES * 64 + threadIdx.x;
            if (k < nst) {
                w_pm[k] = vp[q];
                w_gs[k] = vg[q];
                w_run[k] = vr[q];
            }
        }
    }
    __syncthreads();
    const int64_t whi = wlo + nst;
    auto in = [&](int64_t j) { return j >= wlo && j < whi; };
    auto PM = [&](int64_t j) { return in(j) ? w_pm[j - wlo] : sa.bpmax[j]; };
    auto GS = [&](int64_t j) { return in(j) ? w_gs[j - wlo] : sa.bgs[j]; };
    auto RUN = [&](int64_t j) { return in(j) ? w_run[j - wlo] : sa.brun[j]; };
    // end of j's run, cut at hi1 (j < hi1): the first row of a later run,
    // by a search over the run ids (monotone)
    auto NX = [&](int64_t j, int64_t hi1) -> int64_t {
        const uint32_t r = RUN(j);
        if (RUN(hi1 - 1) == r) return hi1;
        int64_t l = j + 1, h = hi1 - 1;
        while (l < h) {
            const int64_t m = (l + h) >> 1;
            if (RUN(m) > r)
                h = m;
            else
                l = m + 1;
        }
        return l;
    };
    const bool lime_mode = sa.mode == LIME_SUBTRACT_LIME;
    // the rows' bounds in the staged window, a lane's 2 * RPL searches in
    // lockstep (branchless binary lifting: their LDS reads overlap): lower
    // bounds of a.s and a.e among the starts.  (The first spanning row is
    // not searched: a spanning block starts before a.s, so its start never
    // yields a record and the count needs only its existence and end.)
    int bl[RPL], bh[RPL];
    {
        uint32_t key[2 * RPL];
        int b[2 * RPL];
#pragma unroll
        for (int k = 0; k < RPL; ++k) {
            key[k] = as[k];
            key[RPL + k] = ae[k];
        }
        dev::lds_lower_bounds(w_gs, nst, key, b);
#pragma unroll
        for (int k = 0; k < RPL; ++k) {
            bl[k] = b[k];
            bh[k] = b[RPL + k];
        }
    }
    uint64_t tot = 0;
#pragma unroll
    for (int k = 0; k < RPL; ++k) {
        if (base + k * 64 + lane >= sa.na) break;
        const uint32_t a_s = as[k], a_e = ae[k];
        // the inside-hit range, as sub_range: past the window by global search
        int64_t lo1 = bl[k] < nst ? wlo + bl[k] : dev::lower_bound(sa.bgs, whi, sa.nb, (int64_t)a_s);
        int64_t hi1 = lo1;
        if (a_e > a_s)
            hi1 = bh[k] < nst ? wlo + bh[k] : dev::lower_bound(sa.bgs, max(lo1, whi), sa.nb, (int64_t)a_e);
        if (sa.zw) {
            while (lo1 < sa.nb && GS(lo1) == a_s && sa.bge[lo1] == a_s) ++lo1;
            if (hi1 < lo1) hi1 = lo1;
        }
        const uint32_t thr = a_s;  // RUNS: threshold <= 0
        bool any = false;
        uint32_t bs = 0, be = 0, setpos = a_s;
        uint64_t cum = 0;
        auto close_block = [&]() {
            if (lime_mode) {
                cum += (uint64_t)(bs > a_s) + (uint64_t)(a_e > be);
            } else {
                if (bs > setpos) ++cum;
                if (be > setpos) setpos = be;
            }
        };
        // the spanning block (rows before lo1 reaching past thr): it starts
        // before a.s (bs = 0 stands for that start), ends at the prefix max
        const uint32_t pm_last = lo1 > 0 ? PM(lo1 - 1) : 0u;
        if (lo1 > 0 && pm_last > thr) {
            any = true;
            bs = 0;
            be = pm_last;
        }
        int64_t j = lo1;
        // the spanning block goes on through the inside rows of its run
        if (any && j < hi1 && RUN(j) == RUN(lo1 - 1)) {
            const int64_t nx = NX(j, hi1);
            be = max(be, PM(nx - 1));
            j = nx;
        }
        while (j < hi1) {
            const int64_t nx = NX(j, hi1);
            const uint32_t gs = GS(j);
            if (!any) {
                any = true;
                if (sa.bge[j] == gs) {  // a zero-width head closes a duplicate of itself
                    bs = be = gs;
                    close_block();
                }
            } else {
                close_block();
            }
            bs = gs;
            be = PM(nx - 1);  // the inclusive prefix max: >= the head's end
            j = nx;
        }
        uint64_t n_out = 1;  // no hit: (L, None)
        if (any) {
            close_block();
            if (!lime_mode && a_e > setpos) ++cum;
            n_out = cum;
        }
        sa.rcnt[base + k * 64 + lane] = (uint8_t)(n_out < 255 ? n_out : 255);
        tot += n_out;
    }
    tot = dev::wave_reduce_sum(tot);
    const int64_t sb = (int64_t)blockIdx.x * CNT_WAVES + wv;
    if (lane == 0 && sb < nblk) sa.count[sb] = tot;
    // the block's own window start (its first row's start - max width of B,
    // lower bound among B's starts) for the write pass, from the staged
    // window when it reaches that far
    if (lane == 0 && sb < nblk && base < sa.na) {
        const int64_t key = max((int64_t)as[0] - (int64_t)sa.maxw, (int64_t)0);
        int64_t r;
        if (nst > 0 && (int64_t)w_gs[nst - 1] >= key) {
            int l = 0, h = nst - 1;
            while (l < h) {
                const int m = (l + h) >> 1;
                if ((int64_t)w_gs[m] < key)
                    l = m + 1;
                else
                    h = m;
            }
            r = wlo + l;
        } else {
            r = dev::lower_bound(sa.bgs, whi, sa.nb, key);
        }
        sa.bwlo[sb] = (uint32_t)r;
    }
}

// RUNS (threshold <= 0), count and write in ONE pass: the workgroup of
// k_sub_count_runs (CNT_ROWS left rows, their B window staged once, each
// lane's bounds by lockstep searches) counts every row's records, places its
// rows by a workgroup scan and its tile by a decoupled look-back over the
// per-tile totals (tiles in ticket order), then folds again, writing, only
// the rows that have records.  (The two-kernel form re-staged a window per
// 256 rows and folded every row again: on the sparse 1e9-row subtract, 0.15
// records per left row, its write pass took twice its count pass.)  Records
// are staged in LDS and stored coalesced when the tile's fit in FCAP, else
// stored where they fall.  The output arrays are sized before the launch
// (cap records): nothing is stored past cap, the exact total comes back
// through `total`, and the caller runs the pass again at that size.
// (26 KiB of LDS in all: six workgroups per CU; at 64 records and eight per
// CU the sparse 1e9-row subtract took the same time)
// (20 KiB of LDS -- a 1152-row window, 384 staged records -- for 8 waves per
// SIMD cost 12 VGPR spills and the sparse 1e9-row subtract 11.8 -> 13.3 ms)
#ifndef LIME_SUB_FW
#define LIME_SUB_FW 8
#endif
#ifndef LIME_SUB_FCAP
#define LIME_SUB_FCAP (112 * LIME_SUB_FW)
#endif
#ifndef LIME_SUB_FWIN
#define LIME_SUB_FWIN (384 * LIME_SUB_FW)
#endif
constexpr int FCAP = LIME_SUB_FCAP;
// 1024 left rows per tile, the count pass's window (2048-row tiles with a
// 3072-row window: the sparse 1e9-row subtract's pass 9.6 -> 10.2 ms)
constexpr int FW = LIME_SUB_FW, FROWS = FW * SUB_B, FWIN = LIME_SUB_FWIN;
struct FusedArgs {
    uint64_t *st;          // per-tile status words (zeroed)
    unsigned int *ticket;  // tile ticket (zeroed)
    uint64_t *total;       // every tile's records (stored by the last tile)
    uint64_t cap;          // output capacity (records)
    int64_t ntiles;
};

#ifndef LIME_SUB_PHASES
#define LIME_SUB_PHASES 0
#endif
#if LIME_SUB_PHASES
// (measurement build only) wave-cycles per phase of k_sub_fused, summed over
// the waves of every 32nd workgroup and printed by k_sub_phases after each
// launch (wall clock, 100 MHz)
__device__ unsigned long long g_sub_phase[8];
__global__ void k_sub_phases() {
    printf("sub phases:");
    for (int i = 0; i < 8; ++i) {
        printf(" %llu", g_sub_phase[i]);
        g_sub_phase[i] = 0;
    }
    printf("\n");
}
#define SUB_PH(i)                 \
    do {                          \
        const uint64_t t_ = wall_clock64(); \
        ph_d[i] = t_ - ph_t;      \
        ph_t = t_;                \
    } while (0)
#else
#define SUB_PH(i) \
    do {          \
    } while (0)
#endif

// wstart / wend: sa's per-tile window bounds again, as restrict arguments,
// read at the wave-uniform tile index by scalar loads: the window's staging
// loads issue right behind the rows' loads instead of after them
// LS (local scan): B has no zero-width rows and every tile's window fits in
// FWIN (k_sub_window's wmax): the window's prefix max and run ids come from
// its own starts and ends by two block scans instead of from B's merge scan
// (4 B per row of run ids and 4 B of prefix max written and read again per
// call: 1.6 ms of a 1e9-row subtract).  Rows before the window end before
// the tile's first start, so the window-local prefix max equals B's wherever
// the fold compares it (> a row's start) and a local run start (prefix max
// before it <= its start, merge.hip) equals B's from any row's lo1 on; every
// row's fold is the window-local one.
template <bool LS>
__global__ __launch_bounds__(FW * 64) void k_sub_fused(SubArgs sa, FusedArgs fa,
                                                      const uint32_t *__restrict__ wstart,
                                                      const uint32_t *__restrict__ wend) {
    __shared__ uint32_t w_pm[FWIN], w_gs[FWIN], w_run[FWIN];
    __shared__ uint32_t f_gs[FCAP], f_ge[FCAP], f_ar[FCAP], f_br[FCAP];
    __shared__ uint64_t s_wtot[FW];
    __shared__ uint64_t s_base;
    __shared__ uint32_t s_tile;
    __shared__ uint32_t s_scan[2 * FW];
#if LIME_SUB_PHASES
    uint64_t ph_t = wall_clock64(), ph_d[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#endif
    if (threadIdx.x == 0) s_tile = atomicAdd(fa.ticket, 1u);
    __syncthreads();
    SUB_PH(0);
    // (uniform values held in scalar registers: every VGPR here costs
    // occupancy, 78 -> 84 VGPRs was 6 -> 5 waves per SIMD and +13 %)
    const int64_t tile = (uint32_t)__builtin_amdgcn_readfirstlane((int)s_tile);
    const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x / 64)), lane = dev::lane_id();
    const int64_t base = tile * FROWS + (int64_t)wv * SUB_B;
    constexpr int RPL = SUB_B / 64;  // rows per lane: row base + k 64 + lane
    uint32_t as[RPL], ae[RPL];
    // every load unconditional (rows past the set read its last row and are
    // zeroed after): behind a per-lane bounds branch they were issued and
    // waited for pair by pair
#pragma unroll
    for (int k = 0; k < RPL; ++k) {
        const int64_t i = base + k * 64 + lane;
        const int64_t ic = min(i, sa.na - 1);
        const uint32_t s_ = sa.ags[ic], e_ = sa.age[ic];
        as[k] = i < sa.na ? s_ : 0u;
        ae[k] = i < sa.na ? e_ : 0u;
    }
    const int64_t wlo = (uint32_t)__builtin_amdgcn_readfirstlane((int)wstart[tile]);
    // the rows' hits end before wend: staged up to one row past it, so every
    // row's bound lies inside the window (the sparse 1e9-row subtract: ~1030
    // of the 1536 rows a fixed window staged)
    const int nst = __builtin_amdgcn_readfirstlane(
        (int)min(min((int64_t)FWIN, sa.nb - wlo),
                 (int64_t)wend[tile] + 1 - wlo));
    {
        // every staging load issued before any is stored: SPT rows per
        // thread, the index clamped into B (a loop bounded by nst waited for
        // its loads every one or two rows: 3-4 serial round trips per tile)
        constexpr int SPT = (FWIN + FW * 64 - 1) / (FW * 64);
        uint32_t v0[SPT], v1[SPT], v2[SPT];
#pragma unroll
        for (int i = 0; i < SPT; ++i) {
            const int64_t j = min(wlo + threadIdx.x + i * FW * 64, sa.nb - 1);
            if constexpr (LS) {
                v0[i] = sa.bge[j];  // (ends: scanned below)
                v1[i] = sa.bgs[j];
            } else {
                v0[i] = sa.bpmax[j];
                v1[i] = sa.bgs[j];
                v2[i] = sa.brun[j];
            }
        }
#pragma unroll
        for (int i = 0; i < SPT; ++i) {
            const int k = threadIdx.x + i * FW * 64;
            if (k < nst) {
                w_pm[k] = v0[i];
                w_gs[k] = v1[i];
                if constexpr (!LS) w_run[k] = v2[i];
            }
        }
    }
    __syncthreads();
    if constexpr (LS) {  // thread t scans window rows [PER t, PER t + PER)
        constexpr int PER = FWIN / (FW * 64);
        static_assert(FWIN % (FW * 64) == 0, "whole rows per thread");
        const int r0 = threadIdx.x * PER;
        uint32_t pv[PER], m = 0;
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            m = max(m, r0 + i < nst ? w_pm[r0 + i] : 0u);
            pv[i] = m;
        }
        const uint32_t inc = dev::wave_inclusive_max(m);
        if (lane == 63) s_scan[wv] = inc;
        __syncthreads();
        uint32_t c = dev::wave_shr1(inc, 0u);  // the prefix max before row r0
        for (int w = 0; w < wv; ++w) c = max(c, s_scan[w]);
        uint32_t cnt = 0;
#pragma unroll
        for (int i = 0; i < PER; ++i) {  // run starts: prefix max before the row <= its start
            const uint32_t pm = max(c, pv[i]);
            if (r0 + i < nst) {
                cnt += (r0 + i > 0 && c <= w_gs[r0 + i]) ? 1u : 0u;
                w_pm[r0 + i] = pm;
            }
            pv[i] = cnt;
            c = pm;
        }
        const uint32_t sinc = dev::wave_inclusive_sum(cnt);
        if (lane == 63) s_scan[FW + wv] = sinc;
        __syncthreads();
        uint32_t sb = sinc - cnt;
        for (int w = 0; w < wv; ++w) sb += s_scan[FW + w];
#pragma unroll
        for (int i = 0; i < PER; ++i)
            if (r0 + i < nst) w_run[r0 + i] = sb + pv[i];
        __syncthreads();
    }
    SUB_PH(1);
    const int64_t whi = wlo + nst;
    auto in = [&](int64_t j) { return j >= wlo && j < whi; };
    auto PM = [&](int64_t j) { return in(j) ? w_pm[j - wlo] : sa.bpmax[j]; };
    auto GS = [&](int64_t j) { return in(j) ? w_gs[j - wlo] : sa.bgs[j]; };
    auto RUN = [&](int64_t j) { return in(j) ? w_run[j - wlo] : sa.brun[j]; };
    const bool lime_mode = sa.mode == LIME_SUBTRACT_LIME;
    // lockstep bounds of a.s and a.e (the first spanning row, needed by the
    // writing fold only, is searched there: fewer registers, more waves)
    int bl[RPL], bh[RPL];
    {
        uint32_t key[2 * RPL];
        int b[2 * RPL];
#pragma unroll
        for (int k = 0; k < RPL; ++k) {
            key[k] = as[k];
            key[RPL + k] = ae[k];
        }
        dev::lds_lower_bounds(w_gs, nst, key, b);
#pragma unroll
        for (int k = 0; k < RPL; ++k) {
            bl[k] = b[k];
            bh[k] = b[RPL + k];
        }
    }
    SUB_PH(2);
    // a row's fold (k_subtract<_, true>'s, over this window): counts its
    // records, or with `wr` emits them into [pos, end) -- tile-local
    // positions in the LDS stage when `staged`, else global ones.  Two forms
    // of one body: window-local (LOC: u32 indices relative to wlo, every
    // read but the heads' from LDS, no bounds checks) for a row whose bounds
    // both fall inside the window -- rows before it end before the tile's
    // first start (k_sub_window), so its fold reads nothing else -- and B
    // without zero-width rows; the general form (global indices, each read
    // from the window or else global memory) for the rest.  (The kernel is
    // VALU-issue bound: ~2000 VALU instructions per wave at 1e9 rows, the
    // general form's 64-bit index arithmetic and window checks a large part)
    // a long same-start group's head from the tie index; tn < 0: the index
    // is not built (LS defers it to the first call that meets such a group):
    // flagged, and the caller builds it and runs the pass again
    auto tie = [&](uint32_t bs, uint32_t thr, uint32_t &hr, uint32_t &he) {
        if (sa.tn < 0)
            atomicOr(sa.err, 4u);
        else
            tie_head(sa, bs, thr, hr, he);
    };
    auto fold = [&](auto L, uint32_t a_s, uint32_t a_e, int blk, int bhk, bool wr, uint64_t pos,
                    uint64_t end, uint32_t ar, bool staged) -> uint32_t {
        constexpr bool LOC = decltype(L)::value;
        using I = std::conditional_t<LOC, int, int64_t>;
        auto pmf = [&](I j) -> uint32_t {
            if constexpr (LOC) return w_pm[j];
            else return PM(j);
        };
        auto gsf = [&](I j) -> uint32_t {
            if constexpr (LOC) return w_gs[j];
            else return GS(j);
        };
        auto runf = [&](I j) -> uint32_t {
            if constexpr (LOC) return w_run[j];
            else return RUN(j);
        };
        auto gef = [&](I j) -> uint32_t {
            if constexpr (LOC) return sa.bge[wlo + j];
            else return sa.bge[j];
        };
        auto rowf = [&](I j) -> uint32_t {
            if constexpr (LOC) return sa.brow[wlo + j];
            else return sa.brow[j];
        };
        auto nxf = [&](I j, I hi1) -> I {  // end of j's run, cut at hi1
            const uint32_t r = runf(j);
            if (runf(hi1 - 1) == r) return hi1;
            I l = j + 1, h = hi1 - 1;
            while (l < h) {
                const I m = (l + h) >> 1;
                if (runf(m) > r)
                    h = m;
                else
                    l = m + 1;
            }
            return l;
        };
        I lo1, hi1;
        if constexpr (LOC) {
            lo1 = blk;
            hi1 = a_e > a_s ? bhk : blk;
        } else {
            lo1 = blk < nst ? wlo + blk : dev::lower_bound(sa.bgs, whi, sa.nb, (int64_t)a_s);
            hi1 = lo1;
            if (a_e > a_s)
                hi1 = bhk < nst ? wlo + bhk
                                : dev::lower_bound(sa.bgs, max(lo1, whi), sa.nb, (int64_t)a_e);
            if (sa.zw) {
                while (lo1 < sa.nb && GS(lo1) == a_s && sa.bge[lo1] == a_s) ++lo1;
                if (hi1 < lo1) hi1 = lo1;
            }
        }
        const uint32_t thr = a_s;  // threshold <= 0
        auto emit = [&](uint32_t s, uint32_t e, uint32_t br, uint64_t at) {
            if (staged) {
                const uint32_t li = (uint32_t)at;
                f_gs[li] = s;
                f_ge[li] = e;
                f_ar[li] = ar;
                f_br[li] = br;
            } else if (at < fa.cap) {
                sa.ogs[at] = s;
                sa.oge[at] = e;
                sa.oar[at] = ar;
                sa.obr[at] = br;
            }
        };
        bool any = false;
        uint32_t bs = 0, be = 0, hr = 0, he = 0, setpos = a_s;  // block, head row and end
        uint32_t cum = 0;  // (a row's records: at most 2 per B run, < 2^32)
        auto close_block = [&]() {
            if (lime_mode) {
                const uint32_t r = (bs > a_s) + (a_e > be);
                if (wr) {
                    uint64_t at = end - cum - r;
                    if (bs > a_s) emit(a_s, bs, hr, at++);
                    if (a_e > be) emit(be, a_e, hr, at++);
                }
                cum += r;
            } else {
                if (bs > setpos) {
                    if (wr) emit(setpos, bs, hr, pos + cum);
                    ++cum;
                }
                if (be > setpos) setpos = be;
            }
        };
        // the spanning block: first j in [wlo, lo1) with pmax > thr; its head
        // the min (end, row) among its same-start rows.  (Rows before the
        // window end before the tile's first start: pmax[wlo - 1] <= thr, so
        // lo1 == wlo has no spanning block and j0 >= wlo.)
        const uint32_t pm_last = lo1 > 0 ? pmf(lo1 - 1) : 0u;
        if (lo1 > 0 && pm_last > thr) {
            any = true;
            bs = 0;  // (counting: the spanning block starts before a.s)
            be = pm_last;
            if (wr) {
                // first j with pmax > thr: in the window when some staged
                // pmax exceeds thr (pmax ascends)
                I j0;
                if constexpr (LOC) {
                    int l = 0, h = lo1 - 1;
                    while (l < h) {
                        const int m = (l + h) >> 1;
                        if (w_pm[m] > thr)
                            h = m;
                        else
                            l = m + 1;
                    }
                    j0 = l;
                } else if (nst > 0 && w_pm[nst - 1] > thr) {
                    int l = 0, h = nst - 1;
                    while (l < h) {
                        const int m = (l + h) >> 1;
                        if (w_pm[m] > thr)
                            h = m;
                        else
                            l = m + 1;
                    }
                    j0 = wlo + l;
                } else {
                    j0 = first_spanning(sa.bpmax, lo1, thr);
                }
                bs = gsf(j0);
                hr = rowf(j0);
                he = gef(j0);
                I j = j0 + 1;
                for (; j < lo1 && j <= j0 + TIE_G && gsf(j) == bs; ++j) {
                    const uint32_t g2 = gef(j), r2 = rowf(j);
                    if (g2 > thr && (g2 < he || (g2 == he && r2 < hr))) {
                        hr = r2;
                        he = g2;
                    }
                }
                if (j < lo1 && gsf(j) == bs) tie(bs, thr, hr, he);  // a long group
            }
        }
        I j = lo1;
        // the spanning block goes on through the inside rows of its run
        if (any && j < hi1 && runf(j) == runf(lo1 - 1)) {
            const I nx = nxf(j, hi1);
            be = max(be, pmf(nx - 1));
            j = nx;
        }
        while (j < hi1) {
            const I nx = nxf(j, hi1);
            const uint32_t gs = gsf(j);
            if (!any) {  // foldLeft(List(head)): the head is folded against itself
                any = true;
                // a zero-width head closes a duplicate of itself (B without
                // zero-width rows has none: no head load in the counting fold)
                if (!LOC && sa.zw && gef(j) == gs) {
                    bs = be = gs;
                    if (wr) {
                        hr = rowf(j);
                        he = gs;
                    }
                    close_block();
                }
            } else {
                close_block();
            }
            bs = gs;
            be = pmf(nx - 1);  // (the inclusive prefix max: >= the head's end)
            if (wr) {  // the head among the run's same-start non-empty hits: min (end, row)
                hr = rowf(j);
                he = gef(j);
                if (he > bs) {
                    I q = j + 1;
                    for (; q < nx && q <= j + TIE_G && gsf(q) == bs; ++q) {
                        const uint32_t e2 = gef(q), r2 = rowf(q);
                        if (e2 < he || (e2 == he && r2 < hr)) {
                            hr = r2;
                            he = e2;
                        }
                    }
                    if (q < nx && gsf(q) == bs) tie(bs, bs, hr, he);  // a long group
                }
            }
            j = nx;
        }
        if (any) {
            close_block();
            if (!lime_mode && a_e > setpos) {
                if (wr) emit(setpos, a_e, hr, pos + cum);
                ++cum;
            }
            return cum;
        }
        if (wr) emit(a_s, a_e, 0xffffffffu, pos);  // no hit: (L, None)
        return 1;
    };
    // whether a row's fold may take the window-local form
    const bool tail = whi == sa.nb;  // (bounds at nst are exact: the window reaches B's end)
    auto local = [&](uint32_t a_s, uint32_t a_e, int blk, int bhk) {
        return !sa.zw && (blk < nst || tail) && (a_e <= a_s || bhk < nst || tail);
    };
    auto fold_sel = [&](uint32_t a_s, uint32_t a_e, int blk, int bhk, bool wr, uint64_t pos,
                        uint64_t end, uint32_t ar, bool staged) -> uint32_t {
        if constexpr (LS)  // (every row's bounds inside the window)
            return fold(std::true_type{}, a_s, a_e, blk, bhk, wr, pos, end, ar, staged);
        else
            return local(a_s, a_e, blk, bhk)
                       ? fold(std::true_type{}, a_s, a_e, blk, bhk, wr, pos, end, ar, staged)
                       : fold(std::false_type{}, a_s, a_e, blk, bhk, wr, pos, end, ar, staged);
    };
    // counts, then each row's place: rows in order (k, lane) within a wave,
    // waves in order within the tile
    // (u32: a tile's records past 2^32 would need 4M records per row)
    uint32_t cnt[RPL], ex[RPL], run = 0;
#pragma unroll
    for (int k = 0; k < RPL; ++k) {
        cnt[k] = base + k * 64 + lane < sa.na
                     ? fold_sel(as[k], ae[k], bl[k], bh[k], false, 0, 0, 0, false)
                     : 0u;
        const uint32_t inc = dev::wave_inclusive_sum(cnt[k]);
        ex[k] = run + inc - cnt[k];
        run += dev::lane63(inc);
    }
    SUB_PH(3);
    if (lane == 0) s_wtot[wv] = run;
    __syncthreads();
    uint64_t wpre = 0, T = 0;
#pragma unroll
    for (int w = 0; w < FW; ++w) {
        if (w < wv) wpre += s_wtot[w];
        T += s_wtot[w];
    }
    // the tile's place: its total published at once; the look-back (wave 0)
    // runs before the writing folds only when they store to global memory
    // directly, else after them (the folds stage tile-local records in LDS
    // meanwhile, and the predecessors have published by then)
    const bool staged = T <= (uint64_t)FCAP;
    auto place = [&]() {
        if (wv == 0) {
            const uint64_t excl = tile > 0 ? dev::lookback<false>(fa.st, tile) : 0;
            if (lane == 0) {
                if (tile > 0) dev::st_publish(fa.st + tile, dev::ST_INC | (excl + T));
                if (tile == fa.ntiles - 1) *fa.total = excl + T;
                s_base = excl;
            }
        }
        __syncthreads();
    };
    if (wv == 0 && lane == 0)
        dev::st_publish(fa.st + tile, (tile == 0 ? dev::ST_INC : dev::ST_AGG) | T);
    SUB_PH(4);
    if (!staged) place();
    const uint64_t tb = staged ? 0 : s_base;
    // the writing folds over the wave's rows WITH records only, compacted
    // onto the lanes: in the sparse 1e9-row subtract 15 % of the rows have
    // records, but one in each lane-row k nearly always does, so folding by
    // k ran all 4 writing folds (their head loads dependent global reads) in
    // every wave.  Entry e (in (k, lane) order) is row k of lane src: its
    // count and place come over by shuffles (every lane takes part), its
    // start and end are read again (L2) and its bounds searched again in the
    // window (holding every row's bounds through this loop cost occupancy)
    uint64_t msk[RPL];
    int cum[RPL + 1];
    cum[0] = 0;
#pragma unroll
    for (int k = 0; k < RPL; ++k) {
        msk[k] = __ballot(cnt[k] > 0);
        cum[k + 1] = cum[k] + __popcll(msk[k]);
    }
    for (int e0 = 0; e0 < cum[RPL]; e0 += 64) {  // (uniform)
        const int e = e0 + lane;
        int kk = 0;
#pragma unroll
        for (int k = 1; k < RPL; ++k)
            if (e >= cum[k]) kk = k;
        uint64_t m = msk[0];
#pragma unroll
        for (int k = 1; k < RPL; ++k)
            if (kk == k) m = msk[k];
        // the lane holding entry e: the (e - cum[kk])-th set bit of m
        int nth = e - cum[kk], src = 0;
#pragma unroll
        for (int w = 32; w >= 1; w >>= 1) {
            const int c = __popcll(m & ((1ull << w) - 1));
            if (nth >= c) {
                nth -= c;
                m >>= w;
                src += w;
            }
        }
        src &= 63;
        uint32_t r_cnt = 0, r_ex = 0, r_s = 0, r_e = 0, r_b = 0;
        // (LS: the row's start, end and bounds from the counting lane's
        // registers, no reload and no second search; the merge-scan form
        // has no registers to spare: 78 -> 89 VGPRs, 6 -> 5 waves)
        constexpr bool KEEP = LS;
#pragma unroll
        for (int k = 0; k < RPL; ++k) {
            const uint32_t v_cnt = __shfl(cnt[k], src), v_ex = __shfl(ex[k], src);
            uint32_t v_s = 0, v_e = 0, v_b = 0;
            if constexpr (KEEP) {
                v_s = __shfl(as[k], src);
                v_e = __shfl(ae[k], src);
                v_b = __shfl((uint32_t)bl[k] | (uint32_t)bh[k] << 16, src);
            }
            if (kk == k) {
                r_cnt = v_cnt;
                r_ex = v_ex;
                r_s = v_s;
                r_e = v_e;
                r_b = v_b;
            }
        }
        if (e < cum[RPL]) {
            const int64_t i = base + kk * 64 + src;
            uint32_t a_s, a_e;
            int lb, hb;
            if constexpr (KEEP) {
                static_assert(FWIN < (1 << 16), "bounds packed in 16 bits");
                a_s = r_s;
                a_e = r_e;
                lb = r_b & 0xffff;
                hb = r_b >> 16;
            } else {
                a_s = sa.ags[i];
                a_e = sa.age[i];
                const uint32_t key[2] = {a_s, a_e};
                int b[2];  // the lockstep bounds, again
                dev::lds_lower_bounds(w_gs, nst, key, b);
                lb = b[0];
                hb = b[1];
            }
            const uint64_t pos = tb + wpre + r_ex;
            if (fold_sel(a_s, a_e, lb, hb, true, pos, pos + r_cnt, sa.arow[i], staged) != r_cnt)
                atomicOr(sa.err, 1u);  // (the two folds disagree: flagged, not written past)
        }
    }
    SUB_PH(5);
    if (staged) {  // the tile's records, lane-consecutive
        place();  // (its barrier also orders the staged records)
        SUB_PH(6);
        const uint64_t gb = s_base;
        for (int q = threadIdx.x; q < (int)T; q += FW * 64) {
            const uint64_t at = gb + q;
            if (at >= fa.cap) break;
            sa.ogs[at] = f_gs[q];
            sa.oge[at] = f_ge[q];
            sa.oar[at] = f_ar[q];
            sa.obr[at] = f_br[q];
        }
    }
    SUB_PH(7);
#if LIME_SUB_PHASES  // (the sums' atomics after the last phase: none waits on them)
    if ((threadIdx.x & 63) == 0 && (blockIdx.x & 31) == 0)
        for (int i = 0; i < 8; ++i) atomicAdd(&g_sub_phase[i], (unsigned long long)ph_d[i]);
#endif
}

// whether any same-start group has more than TIE_G rows: gs[j] == gs[j +
// TIE_G] for some j (4 rows per thread, 16-B loads; reads gs once: the tie
// index's flag + scan passes run only when it does)
__global__ __launch_bounds__(256) void k_tie_detect(const uint32_t *__restrict__ gs, int64_t n,
                                                    unsigned int *__restrict__ big) {
    static_assert(TIE_G % 4 == 0, "aligned 16-B loads at j and j + TIE_G");
    const int64_t j = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
    if (j + TIE_G >= n) return;
    bool hit = false;
    if (j + TIE_G + 4 <= n) {
        const uint4 x = *reinterpret_cast<const uint4 *>(gs + j);
        const uint4 y = *reinterpret_cast<const uint4 *>(gs + j + TIE_G);
        hit = x.x == y.x || x.y == y.y || x.z == y.z || x.w == y.w;
    } else {
        for (int64_t q = j; q + TIE_G < n && q < j + 4; ++q) hit |= gs[q] == gs[q + TIE_G];
    }
    if (__ballot(hit) != 0 && dev::lane_id() == 0) atomicOr(big, 1u);
}

// any same-start group past TIE_G rows (*big), and every row of a
// multi-row same-start group flagged for the tie index
__global__ __launch_bounds__(256) void k_tie_flags(const uint32_t *__restrict__ gs, int64_t n,
                                                   uint32_t *__restrict__ flag,
                                                   unsigned int *__restrict__ big) {
    const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (j >= n) return;
    const uint32_t g = gs[j];
    flag[j] = (j + 1 < n && gs[j + 1] == g) || (j > 0 && gs[j - 1] == g);
    if (j + TIE_G < n && gs[j + TIE_G] == g) atomicOr(big, 1u);
}

__global__ __launch_bounds__(256) void k_tie_compact(const uint32_t *__restrict__ gs,
                                                     const uint32_t *__restrict__ ge,
                                                     const uint32_t *__restrict__ row, int64_t n,
                                                     const uint32_t *__restrict__ flag,
                                                     const uint32_t *__restrict__ pos,
                                                     uint32_t *__restrict__ tg,
                                                     uint32_t *__restrict__ te,
                                                     uint32_t *__restrict__ tr) {
    const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (j >= n || !flag[j]) return;
    const uint32_t p = pos[j];
    tg[p] = gs[j];
    te[p] = ge[j];
    tr[p] = row[j];
}

}  // namespace

int sort_set_global(lime_ctx *ctx, lime_set *set, const uint32_t *d_gs, const uint32_t *d_ge,
                    const uint32_t *d_row, const uint32_t *d_len);

// B's tie index, built once per set (under its context's lock) when some
// same-start group has more than TIE_G rows; else tie_n = 0.  known: whether
// one has (the merge scan tests it on the runs path), -1 unknown
static int build_tie_index(lime_ctx *ctx, const lime_set *B, int known) {
    std::lock_guard<std::mutex> lock(B->ctx->mu);
    if (B->tie_n >= 0) return LIME_OK;
    const int64_t n = B->n;
    if (n <= TIE_G || known == 0) {
        B->tie_n = 0;
        return LIME_OK;
    }
    uint32_t *flag, *pos, *tot;
    unsigned int *big;
    LIME_TRY(alloc(ctx, &tot, 2));
    PoolGuard<uint32_t> g2{ctx, tot};
    big = reinterpret_cast<unsigned int *>(tot + 1);
    LIME_HIP(hipMemsetAsync(tot, 0, 8, S(ctx)));
    // (most sets have no long same-start group: one read of gs decides)
    if (known < 0) {
        hipLaunchKernelGGL(k_tie_detect, dim3(blocks_for((n + 3) / 4, 256)), dim3(256), 0,
                           S(ctx), B->gs, n, big);
        LIME_HIP(hipGetLastError());
        uint32_t hb[2] = {0, 0};
        LIME_TRY(read_back(ctx, hb, tot, sizeof(hb)));
        if (!hb[1]) {
            B->tie_n = 0;
            return LIME_OK;
        }
    }
    LIME_TRY(alloc(ctx, &flag, (size_t)n));
    PoolGuard<uint32_t> g0{ctx, flag};
    LIME_TRY(alloc(ctx, &pos, (size_t)n));
    PoolGuard<uint32_t> g1{ctx, pos};
    hipLaunchKernelGGL(k_tie_flags, dim3(blocks_for(n, 256)), dim3(256), 0, S(ctx), B->gs, n, flag,
                       big);
    LIME_TRY(scan_exclusive_u32(ctx, flag, pos, n, tot));
    uint32_t h[2] = {0, 0};
    LIME_TRY(read_back(ctx, h, tot, sizeof(h)));
    if (!h[1]) {  // no long group: the bounded walks suffice
        B->tie_n = 0;
        return LIME_OK;
    }
    const int64_t T = h[0];
    uint32_t *tg, *te, *tr;
    LIME_TRY(alloc(ctx, &tg, (size_t)T));
    PoolGuard<uint32_t> g3{ctx, tg};
    LIME_TRY(alloc(ctx, &te, (size_t)T));
    PoolGuard<uint32_t> g4{ctx, te};
    LIME_TRY(alloc(ctx, &tr, (size_t)T));
    PoolGuard<uint32_t> g5{ctx, tr};
    hipLaunchKernelGGL(k_tie_compact, dim3(blocks_for(n, 256)), dim3(256), 0, S(ctx), B->gs, B->ge,
                       B->row, n, (const uint32_t *)flag, (const uint32_t *)pos, tg, te, tr);
    LIME_HIP(hipGetLastError());
    lime_set t;  // (gs, ge, row) order
    t.ctx = ctx;
    t.n = T;
    t.d_off = B->d_off;
    t.n_contigs = B->n_contigs;
    t.off = B->off;
    t.len = B->len;
    t.row_ties = true;
    LIME_TRY(sort_set_global(ctx, &t, tg, te, tr, nullptr));
    B->tie_gs = t.gs;
    B->tie_ge = t.ge;
    B->tie_row = t.row;
    B->tie_n = T;
    return LIME_OK;
}

int merge_runs(lime_ctx *ctx, const lime_set *set, lime_result *res, bool want_run_ids);
int merge_runs_with_pmax(lime_ctx *ctx, const lime_set *set, lime_result *res, int *tie_big);

int subtract_run(lime_ctx *ctx, const lime_set *A, const lime_set *B, int64_t threshold, int mode,
                 lime_result *res) {
    const int64_t na = A->n;
    res->n = 0;
    if (na == 0) {
        LIME_TRY(alloc(ctx, &res->gs, 1));
        LIME_TRY(alloc(ctx, &res->ge, 1));
        LIME_TRY(alloc(ctx, &res->a_row, 1));
        LIME_TRY(alloc(ctx, &res->b_row, 1));
        return LIME_OK;
    }
    // threshold <= 0: blocks are B's merge runs (k_subtract<_, true>); the
    // runs of a stranded set also break at strand changes, so those walk
    const bool runs = threshold <= 0 && B->n > 0 && B->strand_in == nullptr;
    // B's prefix max: with the runs, out of the same merge scan (below)
    if (!runs) LIME_TRY(build_prefix_max(ctx, B));
    // runs: the count (k_sub_count_runs) and write passes find each row's
    // inside-hit range in their staged windows, no owner_ranges pass
    const bool inl = runs;
    uint32_t *olo = nullptr, *ocnt = nullptr;
    uint64_t *cnt, *off;
    if (!inl) {
        LIME_TRY(alloc(ctx, &olo, (size_t)na));
        LIME_TRY(alloc(ctx, &ocnt, (size_t)na));
    }
    PoolGuard<uint32_t> go1{ctx, olo}, go2{ctx, ocnt};
    LIME_TRY(alloc(ctx, &cnt, (size_t)na + 1));
    PoolGuard<uint64_t> gc{ctx, cnt};
    LIME_TRY(alloc(ctx, &off, (size_t)na + 1));
    PoolGuard<uint64_t> go{ctx, off};
    unsigned int *err;
    LIME_TRY(alloc(ctx, &err, 1));
    PoolGuard<unsigned int> ge{ctx, err};
    LIME_HIP(hipMemsetAsync(err, 0, 4, S(ctx)));
    if (!inl) LIME_TRY(owner_ranges(ctx, A, B, 0, threshold, olo, ocnt));
    const int64_t nblk = (na + SUB_B - 1) / SUB_B;
    // runs: B's merge runs with their run ids and B's prefix max (one scan)
    lime_result mb;
    mb.ctx = ctx;
    PoolGuard<uint32_t> g1{ctx, mb.run_of_sorted};
    PoolGuard<uint32_t> g2{ctx, mb.gs};
    PoolGuard<uint32_t> g3{ctx, mb.ge};
    // LS (k_sub_fused<true>): B without zero-width rows and every fused
    // tile's window within FWIN (one read-back) -- no merge scan of B
    uint32_t *wstart = nullptr, *wend = nullptr;
    PoolGuard<uint32_t> gw{ctx, wstart};
    PoolGuard<uint32_t> gwe{ctx, wend};
    bool ls = false;
    // (LIME_SUB_NO_LS set: the merge-scan paths, as tests force them)
    if (runs && !B->has_zero_width && !getenv("LIME_SUB_NO_LS")) {
        const int64_t nt = blocks_for(na, FROWS);
        unsigned int *wm;
        LIME_TRY(alloc(ctx, &wm, 1));
        PoolGuard<unsigned int> gm{ctx, wm};
        LIME_TRY(alloc(ctx, &wstart, (size_t)nt));
        LIME_TRY(alloc(ctx, &wend, (size_t)nt));
        LIME_HIP(hipMemsetAsync(wm, 0, 4, S(ctx)));
        hipLaunchKernelGGL(k_sub_window, dim3(blocks_for(nt, 256)), dim3(256), 0, S(ctx), A->gs,
                           na, B->gs, B->n, B->max_width, nt, FW, wstart, A->max_width, wend, wm);
        LIME_HIP(hipGetLastError());
        unsigned int h_wm = 0;
        LIME_TRY(read_back(ctx, &h_wm, wm, sizeof(h_wm)));
        ls = h_wm <= (unsigned)FWIN;
        if (!ls) {
            release(ctx, wstart);
            release(ctx, wend);
            wstart = wend = nullptr;
        }
    }
    // (the same scan tells whether B has a same-start group past TIE_G)
    int tie_big = -1;
    if (runs && !ls) LIME_TRY(merge_runs_with_pmax(ctx, B, &mb, &tie_big));
    // runs, one pass (k_sub_fused) when records are plentiful (they come
    // from A rows crossing the ends of B's runs: the sparse 1e9-row subtract,
    // 9.2e6 runs of B, 7.4e7 records for 5e8 rows); B merging into fewer runs
    // than A's rows / 64 (B covers A deeply: C2's inputs, 16 records for 1e8
    // rows) leaves most tiles without a record, and there the count pass + a
    // write pass that skips them wins (1.0 vs 1.4 ms on C2's inputs: no
    // tickets, no look-back)
    // (LS: fused always -- without the merge scan the two-pass path's one
    // advantage, no look-back, does not pay for the scan it needs)
    const bool fused = ls || (runs && mb.n * 64 >= na);
    // window starts: per block; per count workgroup (CNT_WAVES blocks) or
    // fused tile (FW blocks) with inline ranges
    const int stride = fused ? FW : inl ? CNT_WAVES : 1;
    const int64_t nws = (nblk + stride - 1) / stride;
    if (!ls) {
        LIME_TRY(alloc(ctx, &wstart, (size_t)nws));
        if (fused) LIME_TRY(alloc(ctx, &wend, (size_t)nws));
        if (B->n > 0)
            hipLaunchKernelGGL(k_sub_window, dim3(blocks_for(nws, 256)), dim3(256), 0, S(ctx),
                               A->gs, na, B->gs, B->n, B->max_width, nws, stride, wstart,
                               A->max_width, wend, (unsigned int *)nullptr);
        else
            LIME_HIP(hipMemsetAsync(wstart, 0, 4 * (size_t)nws, S(ctx)));
    }
    uint32_t *bwlo = nullptr;  // runs: per-block window starts (count -> write pass)
    if (inl) LIME_TRY(alloc(ctx, &bwlo, (size_t)nblk));
    PoolGuard<uint32_t> gb{ctx, bwlo};
    uint8_t *rcnt = nullptr;  // runs: per-row record counts (count -> write pass)
    if (inl) LIME_TRY(alloc(ctx, &rcnt, (size_t)na));
    PoolGuard<uint8_t> gr{ctx, rcnt};
    SubArgs sa;
    sa.wstart = wstart;
    sa.wend = wend;
    sa.bwlo = bwlo;
    sa.maxw = B->max_width;
    sa.ags = A->gs;
    sa.age = A->ge;
    sa.arow = A->row;
    sa.bgs = B->gs;
    sa.bge = B->ge;
    sa.brow = B->row;
    sa.bpmax = B->pmax;
    sa.olo = olo;
    sa.ocnt = ocnt;
    sa.na = na;
    sa.nb = B->n;
    sa.t = threshold;
    sa.mode = mode;
    sa.count = cnt;
    sa.rcnt = rcnt;
    sa.off = off;
    sa.err = err;
    // the tie index of B (long same-start groups), built once per set; LS
    // (no merge scan to test for such groups) builds it only when its pass
    // meets one (err bit 4) and then runs again
    int64_t tn_now;
    {
        std::lock_guard<std::mutex> lock(B->ctx->mu);
        tn_now = B->tie_n;
    }
    auto tie_args = [&]() {
        sa.tgs = B->tie_gs;
        sa.tge = B->tie_ge;
        sa.trow = B->tie_row;
        sa.tn = B->tie_n > 0 ? B->tie_n : 0;
    };
    if (ls && tn_now < 0) {
        sa.tgs = sa.tge = sa.trow = nullptr;
        sa.tn = -1;
    } else {
        if (B->n > 0) LIME_TRY(build_tie_index(ctx, B, tie_big));
        tie_args();
    }
    sa.ogs = sa.oge = sa.oar = sa.obr = nullptr;
    sa.brun = nullptr;
    sa.zw = B->has_zero_width ? 1 : 0;
    if (runs) {
        sa.bpmax = B->pmax;  // built by the merge scan when it was not yet
        sa.brun = mb.run_of_sorted;
    }
    if (fused) {  // one pass: counts, places (look-back) and records
        const int64_t ntiles = blocks_for(na, FROWS);
        uint64_t *st;
        LIME_TRY(alloc(ctx, &st, (size_t)ntiles + 3));  // + ticket, total, error flags
        PoolGuard<uint64_t> gs_{ctx, st};
        FusedArgs fa;
        fa.st = st;
        fa.ticket = reinterpret_cast<unsigned int *>(st + ntiles);
        fa.total = st + ntiles + 1;
        fa.ntiles = ntiles;
        // (the error flags beside the total: one read-back brings both)
        sa.err = reinterpret_cast<unsigned int *>(st + ntiles + 2);
        // records rarely pass one per left row; past the guess the pass runs
        // again at the exact total
        uint64_t cap = (uint64_t)na + 4096, total = 0;
        unsigned int fe = 0;
        auto drop = [&]() {  // (nulled: a failed call's result is deleted)
            for (uint32_t **p : {&res->gs, &res->ge, &res->a_row, &res->b_row}) {
                release(ctx, *p);
                *p = nullptr;
            }
        };
        // test hook: LIME_TEST_SUB_SKEW=1 reports one record more on the second
        // pass than its capacity, so the disagreement guard below is exercised
        const char *skew_env = getenv("LIME_TEST_SUB_SKEW");
        const uint64_t skew = (skew_env && skew_env[0] == '1') ? 1 : 0;
        for (int attempt = 0, tie_runs = 0; attempt < 2; ++attempt) {
            LIME_TRY(alloc(ctx, &res->gs, (size_t)cap));
            LIME_TRY(alloc(ctx, &res->ge, (size_t)cap));
            LIME_TRY(alloc(ctx, &res->a_row, (size_t)cap));
            LIME_TRY(alloc(ctx, &res->b_row, (size_t)cap));
            sa.ogs = res->gs;
            sa.oge = res->ge;
            sa.oar = res->a_row;
            sa.obr = res->b_row;
            fa.cap = cap;
            LIME_HIP(hipMemsetAsync(st, 0, 8 * ((size_t)ntiles + 3), S(ctx)));
            if (ls)
                hipLaunchKernelGGL(k_sub_fused<true>, dim3((unsigned)ntiles), dim3(FW * 64), 0,
                                   S(ctx), sa, fa, (const uint32_t *)wstart,
                                   (const uint32_t *)wend);
            else
                hipLaunchKernelGGL(k_sub_fused<false>, dim3((unsigned)ntiles), dim3(FW * 64), 0,
                                   S(ctx), sa, fa, (const uint32_t *)wstart,
                                   (const uint32_t *)wend);
            LIME_HIP(hipGetLastError());
#if LIME_SUB_PHASES
            hipLaunchKernelGGL(k_sub_phases, dim3(1), dim3(1), 0, S(ctx));
#endif
            uint64_t te[2];  // total, error flags
            LIME_TRY(read_back(ctx, te, fa.total, sizeof(te)));
            total = (skew && te[0] <= cap) ? cap + 1 : te[0];
            fe = (unsigned int)te[1];
            if (sa.tn < 0) {  // (LS, B's tie index not yet built)
                if (fe & 4u) {  // a long same-start group: build the index, run again
                    if (tie_runs++) return fail(LIME_ERR_DEVICE, "subtract: tie index missing");
                    LIME_TRY(build_tie_index(ctx, B, 1));
                    tie_args();
                    drop();
                    --attempt;
                    continue;
                }
            }
            if (total <= cap) break;
            drop();
            // the second attempt ran at the first one's exact total: a larger
            // total means the passes disagree (the arrays held only cap)
            if (attempt == 1)
                return fail(LIME_ERR_DEVICE, "subtract: record total changed between passes");
            cap = total;
        }
        if (fe) return fail(LIME_ERR_DEVICE, "subtract: the writing fold differs from the count");
        res->n = (int64_t)total;
        return LIME_OK;
    }
    // runs write pass with records rare (under one per 16 blocks): the
    // sweeping form of k_subtract, SUB_B blocks tested per workgroup
    int sparse = 0;
    auto launch = [&](bool write) {
        const dim3 g(sparse ? blocks_for(nblk, SUB_B) : blocks_for(na, SUB_B)), b(SUB_B);
        if (write && runs && sparse)
            hipLaunchKernelGGL((k_subtract<true, true, true>), g, b, 0, S(ctx), sa);
        else if (write && runs) hipLaunchKernelGGL((k_subtract<true, true>), g, b, 0, S(ctx), sa);
        else if (write) hipLaunchKernelGGL((k_subtract<true, false>), g, b, 0, S(ctx), sa);
        else if (runs) hipLaunchKernelGGL((k_subtract<false, true>), g, b, 0, S(ctx), sa);
        else hipLaunchKernelGGL((k_subtract<false, false>), g, b, 0, S(ctx), sa);
    };
    if (runs)
        hipLaunchKernelGGL(k_sub_count_runs, dim3(blocks_for(na, CNT_ROWS)), dim3(CNT_WAVES * 64),
                           0, S(ctx), sa, nblk, (const uint32_t *)sa.wstart);
    else
        launch(false);
    LIME_HIP(hipGetLastError());
    // counts per left row (walk), per 256-row block (runs)
    const int64_t nc = runs ? nblk : na;
    LIME_TRY(scan_exclusive_u64(ctx, cnt, off, nc, off + nc));
    uint64_t total = 0;
    LIME_TRY(read_back(ctx, &total, off + nc, sizeof(total)));
    LIME_TRY(alloc(ctx, &res->gs, (size_t)total));
    LIME_TRY(alloc(ctx, &res->ge, (size_t)total));
    LIME_TRY(alloc(ctx, &res->a_row, (size_t)total));
    LIME_TRY(alloc(ctx, &res->b_row, (size_t)total));
    sa.ogs = res->gs;
    sa.oge = res->ge;
    sa.oar = res->a_row;
    sa.obr = res->b_row;
    sparse = runs && (int64_t)total * 16 < nblk;
    launch(true);
    LIME_HIP(hipGetLastError());
    if (runs) {
        unsigned int e = 0;
        LIME_TRY(read_back(ctx, &e, err, sizeof(e)));
        if (e) return fail(LIME_ERR_DEVICE, "subtract: write pass recount differs from the count pass");
    }
    res->n = (int64_t)total;
    return LIME_OK;
}

}  // namespace lime

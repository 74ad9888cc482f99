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
//   spanning:  j < lo1 with B.ge[j] > thr   (b.s < a.s; thr = a.s, or a.s+t-1)
//   inside:    j in [lo1, hi1) (width(b) >= t when t >= 1)
// where [lo1, hi1) is the intersect stream-0 candidate range, and the first
// spanning candidate is found by galloping backwards on the inclusive prefix
// max of B.ge (monotone).  One thread per left row walks its hits twice
// (count pass, write pass); remnants are written at owner offsets from a scan.
#include "common.hpp"

namespace lime {

int owner_ranges(lime_ctx *ctx, const lime_set *O, const lime_set *P, int st, int64_t threshold,
                 uint32_t *olo, uint32_t *ocnt);

namespace {

constexpr int SUB_B = 256;

struct SubArgs {
    const uint32_t *ags, *age, *arow;
    const uint32_t *bgs, *bge, *brow, *bpmax;
    const uint32_t *olo, *ocnt;
    int64_t na;
    int64_t t;
    int mode;
    uint64_t *count;        // pass 1
    const uint64_t *off;    // pass 2
    uint32_t *ogs, *oge, *oar, *obr;
};

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

template <bool WRITE>
__global__ __launch_bounds__(SUB_B) void k_subtract(SubArgs sa) {
    const int64_t i = (int64_t)blockIdx.x * SUB_B + threadIdx.x;
    if (i >= sa.na) return;
    const uint32_t as = sa.ags[i], ae = sa.age[i], ar = sa.arow[i];
    const int64_t t = sa.t;
    int64_t pos = 0, end = 0;
    if (WRITE) {
        pos = (int64_t)sa.off[i];
        end = (int64_t)sa.off[i + 1];
    }
    uint64_t n_out = 0;
    auto emit = [&](uint32_t s, uint32_t e, uint32_t br, int64_t at) {
        if (WRITE) {
            sa.ogs[at] = s;
            sa.oge[at] = e;
            sa.oar[at] = ar;
            sa.obr[at] = br;
        }
    };
    bool any = false;
    if (!(t >= 1 && (int64_t)(ae - as) < t)) {
        const int64_t lo1 = sa.olo[i];
        const int64_t hi1 = lo1 + sa.ocnt[i];
        const uint32_t thr = t <= 0 ? as : (uint32_t)((int64_t)as + t - 1);
        const int64_t j0 = first_spanning(sa.bpmax, lo1, thr);
        // fold state.  The block's value is its head = first hit in the
        // reference's (start, end, row) order; the device order only ties
        // starts by (zero-width first, row), so among same-start non-empty
        // hits the head is re-picked as the min (end, row).
        uint32_t bs = 0, be = 0, bh = 0, bhe = 0;  // block, head row, head end
        uint64_t cum = 0;  // remnants of finished blocks (lime mode, write order)
        uint32_t setpos = as;
        for (int64_t j = j0; j < hi1; ++j) {
            const uint32_t gs = sa.bgs[j], ge = sa.bge[j];
            bool hit;
            if (j < lo1)
                hit = ge > thr;
            else
                hit = t >= 1 ? (int64_t)(ge - gs) >= t : true;
            if (!hit) continue;
            const uint32_t row = sa.brow[j];
            if (!any) {  // foldLeft(List(filteredCache.head)): the head seeds the
                any = true;  // list and is then folded against itself once
                bs = gs;
                be = ge;
                bh = row;
                bhe = ge;
            }
            {
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
                        if (WRITE) {
                            int64_t at = end - (int64_t)cum - r;
                            if (bs > as) emit(as, bs, bh, at++);
                            if (ae > be) emit(be, ae, bh, at++);
                        }
                        cum += r;
                    } else {
                        if (bs > setpos) {
                            if (WRITE) emit(setpos, bs, bh, pos + (int64_t)cum);
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
                if (WRITE) {
                    int64_t at = end - (int64_t)cum - r;
                    if (bs > as) emit(as, bs, bh, at++);
                    if (ae > be) emit(be, ae, bh, at++);
                }
                cum += r;
            } else {
                if (bs > setpos) {
                    if (WRITE) emit(setpos, bs, bh, pos + (int64_t)cum);
                    ++cum;
                }
                if (be > setpos) setpos = be;
                if (ae > setpos) {
                    if (WRITE) emit(setpos, ae, bh, pos + (int64_t)cum);
                    ++cum;
                }
            }
            n_out = cum;
        }
    }
    if (!any) {
        if (WRITE) emit(as, ae, 0xffffffffu, pos);
        n_out = 1;
    }
    if (!WRITE) sa.count[i] = n_out;
}

}  // namespace

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
    LIME_TRY(build_prefix_max(ctx, B));
    uint32_t *olo, *ocnt;
    uint64_t *cnt, *off;
    LIME_TRY(alloc(ctx, &olo, (size_t)na));
    LIME_TRY(alloc(ctx, &ocnt, (size_t)na));
    LIME_TRY(alloc(ctx, &cnt, (size_t)na + 1));
    LIME_TRY(alloc(ctx, &off, (size_t)na + 1));
    LIME_TRY(owner_ranges(ctx, A, B, 0, threshold, olo, ocnt));
    SubArgs sa;
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
    sa.t = threshold;
    sa.mode = mode;
    sa.count = cnt;
    sa.off = off;
    sa.ogs = sa.oge = sa.oar = sa.obr = nullptr;
    if (B->n == 0) {
        // every left row survives whole; the walk sees no candidates
        sa.bpmax = B->pmax;
    }
    hipLaunchKernelGGL(k_subtract<false>, dim3(blocks_for(na, SUB_B)), dim3(SUB_B), 0, S(ctx), sa);
    LIME_HIP(hipGetLastError());
    LIME_TRY(scan_exclusive_u64(ctx, cnt, off, na, off + na));
    uint64_t total = 0;
    LIME_TRY(read_back(ctx, &total, off + na, sizeof(total)));
    LIME_TRY(alloc(ctx, &res->gs, (size_t)total));
    LIME_TRY(alloc(ctx, &res->ge, (size_t)total));
    LIME_TRY(alloc(ctx, &res->a_row, (size_t)total));
    LIME_TRY(alloc(ctx, &res->b_row, (size_t)total));
    sa.ogs = res->gs;
    sa.oge = res->ge;
    sa.oar = res->a_row;
    sa.obr = res->b_row;
    hipLaunchKernelGGL(k_subtract<true>, dim3(blocks_for(na, SUB_B)), dim3(SUB_B), 0, S(ctx), sa);
    LIME_HIP(hipGetLastError());
    release(ctx, olo);
    release(ctx, ocnt);
    release(ctx, cnt);
    release(ctx, off);
    res->n = (int64_t)total;
    return LIME_OK;
}

}  // namespace lime

// complement.hip -- DistributedComplement: gap emission over merged runs.
//
// Reference: Complement.scala:59-128 (getComplement) emits, per partition,
// [prev.end, cur.start) between merged runs of one contig, the contig tail /
// head at a contig change, and Complement.scala:33-50 appends whole contigs
// without data.  The canonical, partition-count-independent form pinned by
// ComplementSuite.scala:19-114: for every genome
// contig in String order, [0, r0.s), [r_i.e, r_{i+1}.s), [r_k.e, len), a contig
// without runs emits [0, len), zero-width gaps (quirk Q4) are dropped.
//
// Input: merged runs (global coordinates, sorted).  Kernels:
//   k_gap_count   per run: gap before it (if non-empty) + contig tail if last
//   scan          exclusive sum over runs
//   k_contig_off  one block: per contig run range, gap count, offsets
//   k_gap_write   per run + per empty contig: write gaps
#include "common.hpp"

namespace lime {
namespace {

constexpr int CB = 256;

__device__ __forceinline__ int32_t seg_of(const uint32_t *off, int32_t nc, uint32_t g) {
    return (int32_t)dev::upper_bound(off, 0, (int64_t)nc, g) - 1;
}

struct GapArgs {
    const uint32_t *rgs, *rge;
    int64_t nr;
    const uint32_t *off;  // nc + 1
    const uint32_t *len;  // nc
    int32_t nc;
    // only gaps whose start lies in [wlo, whi) (a coordinate shard's window;
    // [0, 2^32) unsharded)
    uint32_t wlo, whi;
};

__device__ __forceinline__ bool in_win(const GapArgs &a, uint32_t lo, uint32_t hi) {
    return hi > lo && lo >= a.wlo && lo < a.whi;
}

// gap before run r (lo, hi) and tail after r if last in its contig
__device__ __forceinline__ void run_gaps(const GapArgs &a, int64_t r, uint32_t &b_lo, uint32_t &b_hi,
                                         uint32_t &t_lo, uint32_t &t_hi) {
    const uint32_t s = a.rgs[r];
    const int32_t c = seg_of(a.off, a.nc, s);
    const bool first = r == 0 || seg_of(a.off, a.nc, a.rgs[r - 1]) != c;
    const bool last = r == a.nr - 1 || seg_of(a.off, a.nc, a.rgs[r + 1]) != c;
    b_lo = first ? a.off[c] : a.rge[r - 1];
    b_hi = s;
    if (last) {
        t_lo = a.rge[r];
        t_hi = a.off[c] + a.len[c];
    } else {
        t_lo = t_hi = 0;
    }
}

__global__ __launch_bounds__(CB) void k_gap_count(GapArgs a, uint32_t *__restrict__ cnt) {
    const int64_t r = (int64_t)blockIdx.x * CB + threadIdx.x;
    if (r >= a.nr) return;
    uint32_t bl, bh, tl, th;
    run_gaps(a, r, bl, bh, tl, th);
    cnt[r] = in_win(a, bl, bh) + in_win(a, tl, th);
}

// single block: per contig gap counts -> exclusive offsets coff[c], first run crb[c]
__global__ __launch_bounds__(CB) void k_contig_off(GapArgs a, const uint32_t *__restrict__ pre,
                                                   uint32_t *__restrict__ coff,
                                                   uint32_t *__restrict__ crb,
                                                   uint32_t *__restrict__ total) {
    __shared__ uint32_t scratch[CB / 64 + 1];
    uint32_t carry = 0;
    for (int32_t base = 0; base < a.nc; base += CB) {
        const int32_t c = base + threadIdx.x;
        uint32_t n = 0;
        if (c < a.nc) {
            const int64_t rb = dev::lower_bound(a.rgs, 0, a.nr, a.off[c]);
            const int64_t re = dev::lower_bound(a.rgs, rb, a.nr, a.off[c + 1]);
            crb[c] = (uint32_t)rb;
            n = rb == re ? (in_win(a, a.off[c], a.off[c] + a.len[c]) ? 1u : 0u) : pre[re] - pre[rb];
        }
        uint32_t tot;
        uint32_t ex = dev::block_exclusive_sum<CB>(n, scratch, &tot);
        if (c < a.nc) coff[c] = carry + ex;
        carry += tot;
    }
    if (threadIdx.x == 0) *total = carry;
}

__global__ __launch_bounds__(CB) void k_gap_write(GapArgs a, const uint32_t *__restrict__ pre,
                                                  const uint32_t *__restrict__ coff,
                                                  const uint32_t *__restrict__ crb,
                                                  uint32_t *__restrict__ ogs,
                                                  uint32_t *__restrict__ oge) {
    const int64_t r = (int64_t)blockIdx.x * CB + threadIdx.x;
    if (r < a.nr) {
        uint32_t bl, bh, tl, th;
        run_gaps(a, r, bl, bh, tl, th);
        const int32_t c = seg_of(a.off, a.nc, a.rgs[r]);
        uint32_t at = coff[c] + pre[r] - pre[crb[c]];
        if (in_win(a, bl, bh)) {
            ogs[at] = bl;
            oge[at] = bh;
            ++at;
        }
        if (in_win(a, tl, th)) {
            ogs[at] = tl;
            oge[at] = th;
        }
    }
    // contigs without runs (the first a.nc threads of the grid)
    const int64_t c = r;
    if (c < a.nc) {
        const int64_t rb = crb[c];
        const bool empty = rb >= a.nr || a.rgs[rb] >= a.off[c + 1];
        if (empty && in_win(a, a.off[c], a.off[c] + a.len[c])) {
            ogs[coff[c]] = a.off[c];
            oge[coff[c]] = a.off[c] + a.len[c];
        }
    }
}

}  // namespace

// gaps of the sorted, disjoint runs (rgs, rge) over the genome, those
// starting in [wlo, whi) only
int complement_run(lime_ctx *ctx, const lime_result *runs, const uint32_t *d_off,
                   const uint32_t *d_len, int32_t nc, lime_result *res, uint32_t wlo,
                   uint32_t whi) {
    const int64_t nr = runs->n;
    GapArgs a;
    a.wlo = wlo;
    a.whi = whi;
    a.rgs = runs->gs;
    a.rge = runs->ge;
    a.nr = nr;
    a.off = d_off;
    a.len = d_len;
    a.nc = nc;
    uint32_t *cnt, *pre, *coff, *crb, *total;
    LIME_TRY(alloc(ctx, &cnt, (size_t)nr + 1));
    LIME_TRY(alloc(ctx, &pre, (size_t)nr + 1));
    LIME_TRY(alloc(ctx, &coff, (size_t)nc + 1));
    LIME_TRY(alloc(ctx, &crb, (size_t)nc + 1));
    LIME_TRY(alloc(ctx, &total, 1));
    if (nr > 0)
        hipLaunchKernelGGL(k_gap_count, dim3(blocks_for(nr, CB)), dim3(CB), 0, S(ctx), a, cnt);
    LIME_TRY(scan_exclusive_u32(ctx, cnt, pre, nr, pre + nr));
    hipLaunchKernelGGL(k_contig_off, dim3(1), dim3(CB), 0, S(ctx), a, (const uint32_t *)pre, coff,
                       crb, total);
    LIME_HIP(hipGetLastError());
    uint32_t n = 0;
    LIME_TRY(read_back(ctx, &n, total, sizeof(n)));
    LIME_TRY(alloc(ctx, &res->gs, n));
    LIME_TRY(alloc(ctx, &res->ge, n));
    const int64_t items = nr > nc ? nr : nc;
    if (items > 0)
        hipLaunchKernelGGL(k_gap_write, dim3(blocks_for(items, CB)), dim3(CB), 0, S(ctx), a,
                           (const uint32_t *)pre, (const uint32_t *)coff, (const uint32_t *)crb,
                           res->gs, res->ge);
    LIME_HIP(hipGetLastError());
    release(ctx, cnt);
    release(ctx, pre);
    release(ctx, coff);
    release(ctx, crb);
    release(ctx, total);
    res->n = n;
    return LIME_OK;
}

}  // namespace lime

// route.hip -- range sharding of unsorted rows over coordinate shards
// (SURVEY.md 8(e)): the device half of the Spark shuffles that move every
// record to the partition owning it (ADAM repartitionAndSort at
// cli/Intersection.scala:42-43; OverlapBasedSetTheory.scala:75-84 with the
// explicit-destination ReferenceRegionRangePartitioner of
// util/Partitioners.scala:10-20).
//
// Shard r owns global coordinates [split[r], split[r + 1]).  A row goes to
// the shard owning its start (pairwise ops and merge: the owner of a row is
// the shard of its start) or, clipped, to every shard it overlaps (bit-per-
// base algebra, where clipping at shard bounds is exact).  The rows leave
// grouped by destination, each destination's rows in input order, as
// global-coordinate (gs, ge, row) arrays ready for one all_to_all per array.
//
//   k_route_count  per 1024-row block: pieces per destination -> column b of
//                  the destination-major count matrix mat[d][b]
//   scan           every (destination, block) segment's start
//   k_route_write  pieces at their slots: per destination a block scan over
//                  the threads keeps input order (deterministic output)
#include "common.hpp"

namespace lime {
namespace {

constexpr int RT = 256;
constexpr int RPT = 4;           // rows per thread
constexpr int RBLK = RT * RPT;   // rows per block
constexpr int MAXSH = 64;

struct RouteArgs {
    const int32_t *contig;  // contig-local rows; null: start / end are global
    const uint32_t *start, *end;
    const uint32_t *off, *len;
    int32_t nc;
    int64_t n;
    uint32_t span;
    const uint32_t *split;  // nsh + 1 global bounds
    int nsh;
    int clip;
    uint32_t row_base;
    uint32_t *mat;  // nsh * nblk + 1
    uint32_t nblk;
    uint32_t *gs, *ge, *row;
    // interleaved output (iv != null): piece p at iv[p * ik ...] = gs, ge
    // (, row when ik = 3) -- the send buffer of one all_to_all, no repacking
    uint32_t *iv;
    int ik;
    const int8_t *strand_in;  // may be null
    int8_t *strand_out;
    unsigned int *err;  // bit0 contig, bit1 end < start, bit2 end > length / span
};

// global [g0, g1) of a row from its loaded (contig, start, end) (validated;
// invalid rows become [0, 0) and raise err)
__device__ __forceinline__ void route_vals(const RouteArgs &a, int32_t c, uint32_t s, uint32_t e,
                                           uint32_t &g0, uint32_t &g1, uint32_t &err,
                                           const uint32_t *off, const uint32_t *len) {
    g0 = g1 = 0;
    if (!a.contig) {
        if (e < s) err |= 2u;
        else if (e > a.span) err |= 4u;
        else g0 = s, g1 = e;
        return;
    }
    if (c < 0 || c >= a.nc) err |= 1u;
    else if (e < s) err |= 2u;
    else if (e > len[c]) err |= 4u;
    else g0 = off[c] + s, g1 = off[c] + e;
}
// the same for row i
__device__ __forceinline__ void route_row(const RouteArgs &a, int64_t i, uint32_t &g0, uint32_t &g1,
                                          uint32_t &err, const uint32_t *off, const uint32_t *len) {
    route_vals(a, a.contig ? a.contig[i] : 0, a.start[i], a.end[i], g0, g1, err, off, len);
}
// the contig table in LDS when it fits (the per-row off / len gathers are
// then LDS reads, not dependent cache round trips behind the contig load)
constexpr int RCMAX = 1024;
__device__ __forceinline__ void route_tables(const RouteArgs &a, uint32_t *s_off, uint32_t *s_len,
                                             const uint32_t *&off, const uint32_t *&len) {
    off = a.off;
    len = a.len;
    if (a.contig && a.nc <= RCMAX) {
        for (int i = threadIdx.x; i < a.nc; i += blockDim.x) {
            s_off[i] = a.off[i];
            s_len[i] = a.len[i];
        }
        off = s_off;
        len = s_len;
    }
}

// largest r with split[r] <= g (split in LDS, nsh <= 64)
__device__ __forceinline__ int owner_of(const uint32_t *sp, int nsh, uint32_t g) {
    int lo = 0, hi = nsh;  // answer in [lo, hi)
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (sp[mid] <= g)
            lo = mid;
        else
            hi = mid;
    }
    return lo;
}

// destinations [d0, d1] of a row
__device__ __forceinline__ void dests(const RouteArgs &a, const uint32_t *sp, uint32_t g0,
                                      uint32_t g1, int &d0, int &d1) {
    d0 = owner_of(sp, a.nsh, g0);
    d1 = (a.clip && g1 > g0) ? owner_of(sp, a.nsh, g1 - 1) : d0;
}

__global__ __launch_bounds__(RT) void k_route_count(RouteArgs a) {
    __shared__ uint32_t sp[MAXSH + 1];
    __shared__ uint32_t cnt[MAXSH];
    __shared__ uint32_t s_off[RCMAX], s_len[RCMAX];
    const uint32_t *off, *len;
    route_tables(a, s_off, s_len, off, len);
    for (int i = threadIdx.x; i <= a.nsh; i += RT) sp[i] = a.split[i];
    for (int i = threadIdx.x; i < a.nsh; i += RT) cnt[i] = 0;
    __syncthreads();
    uint32_t err = 0;
    // the wave's pieces per destination: one LDS add per (wave, destination)
    // over the wave's destination range (a per-row atomic sent all 64 lanes
    // of a wave to ONE counter at one shard)
    int d0[RPT], d1[RPT], dmin = MAXSH, dmax = -1;
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
        const int64_t i = (int64_t)blockIdx.x * RBLK + k * RT + threadIdx.x;
        d0[k] = 0, d1[k] = -1;
        if (i >= a.n) continue;
        uint32_t g0, g1;
        route_row(a, i, g0, g1, err, off, len);
        dests(a, sp, g0, g1, d0[k], d1[k]);
        dmin = min(dmin, d0[k]);
        dmax = max(dmax, d1[k]);
    }
    const int wlo = -dev::wave_reduce_max(-dmin), whi = dev::wave_reduce_max(dmax);
    for (int d = wlo; d <= whi; ++d) {  // (wave-uniform bounds)
        uint32_t c = 0;
#pragma unroll
        for (int k = 0; k < RPT; ++k) c += (d >= d0[k] && d <= d1[k]);
        c = dev::wave_reduce_sum(c);
        if (c && dev::lane_id() == 0) atomicAdd(&cnt[d], c);
    }
    err = dev::wave_reduce_or(err);
    if (err && dev::lane_id() == 0) atomicOr(a.err, err);
    __syncthreads();
    for (int d = threadIdx.x; d < a.nsh; d += RT) a.mat[(int64_t)d * a.nblk + blockIdx.x] = cnt[d];
}

// vec: every input pointer 16-B aligned, so a whole block's thread loads its
// RPT = 4 consecutive rows by one 16-B load per array (four 4-B loads at a
// 16-B lane stride had each touched four times the lines)
__global__ __launch_bounds__(RT) void k_route_write(RouteArgs a, int vec) {
    __shared__ uint32_t sp[MAXSH + 1];
    __shared__ uint64_t scratch[RT / 64 + 1];
    __shared__ uint32_t s_off[RCMAX], s_len[RCMAX];
    const uint32_t *off, *len;
    route_tables(a, s_off, s_len, off, len);
    for (int i = threadIdx.x; i <= a.nsh; i += RT) sp[i] = a.split[i];
    __syncthreads();
    // rows of this thread: blocked (k * RT + t keeps loads coalesced; the
    // order within a destination is the thread-major order below)
    static_assert(RPT == 4, "one 16-B load per array and thread");
    uint32_t g0[RPT], g1[RPT];
    int d0[RPT], d1[RPT];
    uint32_t err = 0;
    int dmin = MAXSH, dmax = -1;
    const int64_t i0 = (int64_t)blockIdx.x * RBLK + threadIdx.x * RPT;
    if (vec && i0 + RPT <= a.n) {
        const int4 cv = a.contig ? *reinterpret_cast<const int4 *>(a.contig + i0) : int4{0, 0, 0, 0};
        const uint4 sv = *reinterpret_cast<const uint4 *>(a.start + i0);
        const uint4 ev = *reinterpret_cast<const uint4 *>(a.end + i0);
        const int32_t cc[4] = {cv.x, cv.y, cv.z, cv.w};
        const uint32_t ss[4] = {sv.x, sv.y, sv.z, sv.w}, ee[4] = {ev.x, ev.y, ev.z, ev.w};
#pragma unroll
        for (int k = 0; k < RPT; ++k) {
            route_vals(a, cc[k], ss[k], ee[k], g0[k], g1[k], err, off, len);
            dests(a, sp, g0[k], g1[k], d0[k], d1[k]);
            dmin = min(dmin, d0[k]);
            dmax = max(dmax, d1[k]);
        }
    } else {
#pragma unroll
        for (int k = 0; k < RPT; ++k) {
            const int64_t i = i0 + k;
            d0[k] = 0, d1[k] = -1;
            if (i >= a.n) continue;
            route_row(a, i, g0[k], g1[k], err, off, len);
            dests(a, sp, g0[k], g1[k], d0[k], d1[k]);
            dmin = min(dmin, d0[k]);
            dmax = max(dmax, d1[k]);
        }
    }
    // per destination: offset of this thread's pieces = block scan, four
    // destinations per scan (16-bit fields of a u64: a block holds at most
    // RBLK pieces per destination)
    static_assert(RBLK < 65536, "16-bit piece counts per destination");
    for (int db = 0; db < a.nsh; db += 4) {
        uint64_t c4 = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int d = db + j;
            uint32_t c = 0;
            if (d >= dmin && d <= dmax)
#pragma unroll
                for (int k = 0; k < RPT; ++k) c += (d >= d0[k] && d <= d1[k]);
            c4 |= (uint64_t)c << (16 * j);
        }
        uint64_t tot;
        const uint64_t ex = dev::block_exclusive_sum<RT>(c4, scratch, &tot);
        if (c4 == 0) continue;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int d = db + j;
            if (((c4 >> (16 * j)) & 0xffffu) == 0) continue;
            uint32_t pos = a.mat[(int64_t)d * a.nblk + blockIdx.x] + (uint32_t)((ex >> (16 * j)) & 0xffffu);
#pragma unroll
            for (int k = 0; k < RPT; ++k) {
                if (d < d0[k] || d > d1[k]) continue;
                const uint32_t lo = sp[d], hi = sp[d + 1];
                const uint32_t gs = a.clip ? max(g0[k], lo) : g0[k];
                const uint32_t ge = a.clip && g1[k] > g0[k] ? min(g1[k], hi) : g1[k];
                const int64_t i = i0 + k;
                if (a.iv) {  // one store per piece: 12 B (gs, ge, row) or 8 B
                    if (a.ik == 3)
                        *reinterpret_cast<uint3 *>(a.iv + (int64_t)pos * 3) =
                            make_uint3(gs, ge, a.row_base + (uint32_t)i);
                    else
                        *reinterpret_cast<uint2 *>(a.iv + (int64_t)pos * 2) = make_uint2(gs, ge);
                    ++pos;
                    continue;
                }
                a.gs[pos] = gs;
                a.ge[pos] = ge;
                if (a.row) a.row[pos] = a.row_base + (uint32_t)i;
                if (a.strand_out) a.strand_out[pos] = a.strand_in ? a.strand_in[i] : (int8_t)0;
                ++pos;
            }
        }
    }
}

// the destination starts (and the total) + the error flags in out[nsh + 1]:
// one read-back
__global__ void k_route_totals(const uint32_t *__restrict__ mat, uint32_t nblk, int nsh,
                               const unsigned int *__restrict__ err, int64_t *__restrict__ out) {
    const int d = threadIdx.x;
    if (d <= nsh) out[d] = mat[(int64_t)d * nblk];
    if (d == nsh + 1) out[d] = *err;
}

// interleaved rows (k words per row) -> k column arrays; 4 rows per thread,
// 16-B loads and stores when every pointer is 16-B aligned
template <int K, bool VEC>
__global__ __launch_bounds__(256) void k_deinterleave(const uint32_t *__restrict__ src, int64_t n,
                                                      uint32_t *__restrict__ d0,
                                                      uint32_t *__restrict__ d1,
                                                      uint32_t *__restrict__ d2) {
    const int64_t r0 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
    if (r0 >= n) return;
    uint32_t *dst[3] = {d0, d1, d2};
    if (VEC && r0 + 4 <= n) {
        uint32_t w[4 * K];
        const uint4 *s4 = reinterpret_cast<const uint4 *>(src + r0 * K);
#pragma unroll
        for (int q = 0; q < K; ++q) {
            const uint4 v = s4[q];
            w[4 * q] = v.x, w[4 * q + 1] = v.y, w[4 * q + 2] = v.z, w[4 * q + 3] = v.w;
        }
#pragma unroll
        for (int c = 0; c < K; ++c)
            *reinterpret_cast<uint4 *>(dst[c] + r0) =
                make_uint4(w[c], w[K + c], w[2 * K + c], w[3 * K + c]);
        return;
    }
    for (int64_t r = r0; r < n && r < r0 + 4; ++r)
#pragma unroll
        for (int c = 0; c < K; ++c) dst[c][r] = src[r * K + c];
}

// k evenly spaced rows' global starts (row i * n / k), for count-balanced
// splitters (dist.sample_splits): d_contig == NULL: d_start is global
__global__ void k_sample_starts(const int32_t *__restrict__ contig,
                                const uint32_t *__restrict__ start,
                                const uint32_t *__restrict__ off, int32_t nc, int64_t n, int32_t k,
                                uint32_t *__restrict__ out) {
    const int32_t j = (int32_t)(blockIdx.x * 256 + threadIdx.x);
    if (j >= k) return;
    const int64_t i = (int64_t)j * n / k;
    uint32_t g = start[i];
    if (contig) {
        const int32_t c = contig[i];
        g += (c >= 0 && c < nc) ? off[c] : 0u;  // (routing validates the row itself)
    }
    out[j] = g;
}

}  // namespace

int sample_starts(lime_ctx *ctx, const lime_space *sp, int64_t n, const int32_t *d_contig,
                  const uint32_t *d_start, int32_t k, uint32_t *d_out) {
    if (k <= 0 || n <= 0) return LIME_OK;
    const uint32_t *d_off = nullptr, *d_len = nullptr;
    if (d_contig) LIME_TRY(space_device(ctx, sp->off, &d_off, &d_len));
    hipLaunchKernelGGL(k_sample_starts, dim3(blocks_for(k, 256)), dim3(256), 0, S(ctx), d_contig,
                       d_start, d_off, (int32_t)sp->n, n, k, d_out);
    LIME_HIP(hipGetLastError());
    return LIME_OK;
}

int deinterleave_u32(lime_ctx *ctx, int64_t n, int32_t k, const uint32_t *src, uint32_t *d0,
                     uint32_t *d1, uint32_t *d2) {
    if (n < 0 || (k != 2 && k != 3) || !src || !d0 || !d1 || (k == 3 && !d2))
        return fail(LIME_ERR_ARG, "deinterleave: k = 2 or 3 columns, every pointer set");
    if (n == 0) return LIME_OK;
    const bool vec = ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(d0) |
                       reinterpret_cast<uintptr_t>(d1) | reinterpret_cast<uintptr_t>(d2)) & 15u) == 0;
    const dim3 g(blocks_for((n + 3) / 4, 256)), b(256);
    if (k == 3 && vec) hipLaunchKernelGGL((k_deinterleave<3, true>), g, b, 0, S(ctx), src, n, d0, d1, d2);
    else if (k == 3) hipLaunchKernelGGL((k_deinterleave<3, false>), g, b, 0, S(ctx), src, n, d0, d1, d2);
    else if (vec) hipLaunchKernelGGL((k_deinterleave<2, true>), g, b, 0, S(ctx), src, n, d0, d1, d2);
    else hipLaunchKernelGGL((k_deinterleave<2, false>), g, b, 0, S(ctx), src, n, d0, d1, d2);
    LIME_HIP(hipGetLastError());
    return LIME_OK;
}

int route_rows(lime_ctx *ctx, const lime_space *sp, int64_t n, const int32_t *d_contig,
               const uint32_t *d_start, const uint32_t *d_end, uint32_t row_base, int32_t nsh,
               const uint32_t *splits, int clip, int64_t cap, uint32_t *d_gs, uint32_t *d_ge,
               uint32_t *d_row, int64_t *counts, const int8_t *d_strand_in,
               int8_t *d_strand_out, uint32_t *d_iv, int32_t ik) {
    if (nsh < 1 || nsh > MAXSH) return fail(LIME_ERR_ARG, "1 to 64 shards");
    if (splits[0] != 0 || (int64_t)splits[nsh] != sp->span)
        return fail(LIME_ERR_ARG, "splits must start at 0 and end at the span");
    for (int r = 0; r < nsh; ++r)
        if (splits[r + 1] < splits[r]) return fail(LIME_ERR_ARG, "splits must be non-decreasing");
    const uint32_t nblk = (uint32_t)std::max<int64_t>((n + RBLK - 1) / RBLK, 1);
    const int64_t mlen = (int64_t)nsh * nblk + 1;
    uint32_t *mat = nullptr, *d_split = nullptr;
    const uint32_t *d_off = nullptr, *d_len = nullptr;  // the context's cached space arrays
    unsigned int *err = nullptr;
    int64_t *tot = nullptr;
    LIME_TRY(alloc(ctx, &mat, (size_t)mlen));
    PoolGuard<uint32_t> g0{ctx, mat};
    LIME_TRY(alloc(ctx, &d_split, (size_t)nsh + 1));
    PoolGuard<uint32_t> g1{ctx, d_split};
    LIME_TRY(space_device(ctx, sp->off, &d_off, &d_len));
    LIME_TRY(alloc(ctx, &err, 1));
    PoolGuard<unsigned int> g4{ctx, err};
    LIME_TRY(alloc(ctx, &tot, (size_t)nsh + 2));
    PoolGuard<int64_t> g5{ctx, tot};
    LIME_HIP(hipMemcpyAsync(d_split, splits, 4 * ((size_t)nsh + 1), hipMemcpyHostToDevice, S(ctx)));
    LIME_HIP(hipMemsetAsync(err, 0, 4, S(ctx)));
    LIME_HIP(hipMemsetAsync(mat, 0, 4 * (size_t)mlen, S(ctx)));
    RouteArgs a;
    a.contig = d_contig;
    a.start = d_start;
    a.end = d_end;
    a.off = d_off;
    a.len = d_len;
    a.nc = sp->n;
    a.n = n;
    a.span = (uint32_t)sp->span;
    a.split = d_split;
    a.nsh = nsh;
    a.clip = clip;
    a.row_base = row_base;
    a.mat = mat;
    a.nblk = nblk;
    a.gs = d_gs;
    a.ge = d_ge;
    a.row = d_row;
    a.iv = d_iv;
    a.ik = ik;
    a.strand_in = d_strand_in;
    a.strand_out = d_strand_out;
    a.err = err;
    if (n > 0) hipLaunchKernelGGL(k_route_count, dim3(nblk), dim3(RT), 0, S(ctx), a);
    LIME_TRY(scan_exclusive_u32(ctx, mat, mat, mlen, nullptr));
    hipLaunchKernelGGL(k_route_totals, dim3(1), dim3(MAXSH + 2), 0, S(ctx), (const uint32_t *)mat,
                       nblk, nsh, (const unsigned int *)err, tot);
    LIME_HIP(hipGetLastError());
    // the destination starts (and the total) + the error flags: one read-back
    std::vector<int64_t> h((size_t)nsh + 2);
    LIME_TRY(read_back(ctx, h.data(), tot, 8 * ((size_t)nsh + 2)));
    const unsigned int herr = (unsigned int)h[nsh + 1];
    if (herr & 1u) return fail(LIME_ERR_CONTIG, "interval contig id outside the space");
    if (herr & 2u) return fail(LIME_ERR_RANGE, "interval end < start");
    if (herr & 4u) return fail(LIME_ERR_RANGE, "interval end beyond its contig / the span");
    // (h[nsh] is mat's last entry: the total, the scan's exclusive sum)
    for (int d = 0; d < nsh; ++d) counts[d] = h[d + 1] - h[d];
    if (h[nsh] > cap || n == 0) return LIME_OK;  // counts only
    const int vec = ((reinterpret_cast<uintptr_t>(d_contig) | reinterpret_cast<uintptr_t>(d_start) |
                      reinterpret_cast<uintptr_t>(d_end)) & 15u) == 0;
    hipLaunchKernelGGL(k_route_write, dim3(nblk), dim3(RT), 0, S(ctx), a, vec);
    LIME_HIP(hipGetLastError());
    // (the caller's rows are consumed before the return on the context's own
    // stream, as lime_amd.h states for device inputs)
    if (ctx->stream == ctx->own_stream) LIME_HIP(hipStreamSynchronize(S(ctx)));
    return LIME_OK;
}

}  // namespace lime

// bitset.hip -- bit-per-base set algebra over a coordinate space.
//
// North-star path for dense multi-way algebra (BASELINE configs C4/C5): one
// bit per base of the global coordinate space (span = sum(len + 1) bits,
// ~386 MB for hg38).  The pad base after every contig is never set, so runs
// never cross a contig boundary.
//   k_paint     merged runs -> bits, one 4096-word (32 KiB) tile per
//               workgroup: the tile's runs (two binary searches) are OR-ed
//               into an LDS image, which is then stored once, coalesced --
//               every word written exactly once, no memset, no global atomics
//   k_ev_count  per 4096-word tile: events (run starts + run ends) of
//               op(words) where op = A | ~A | A&B | A&~B | AND of k sets;
//               operands are combined while loading (coalesced) into LDS
//   k_ev_write  the same, writing events at scanned offsets: event 2r is the
//               start and event 2r+1 the end of output run r
// Semantics: base-level algebra; book-ended runs of
// the operands coalesce in the output.
#include "common.hpp"

namespace lime {
namespace {

constexpr int BB = 256;
constexpr int BW = 16;            // words per thread
constexpr int BT = BB * BW;       // words per tile
constexpr int MAXK = 16;
constexpr int MAXPAD = 64;        // contig pads per tile handled in LDS

__global__ __launch_bounds__(BB) void k_paint(const uint32_t *__restrict__ rgs,
                                              const uint32_t *__restrict__ rge, int64_t nr,
                                              uint64_t *__restrict__ words, int64_t n_words) {
    __shared__ unsigned long long img[BT];
    __shared__ int64_t s_r[2];
    const int64_t w0 = (int64_t)blockIdx.x * BT;
    const uint64_t blo = (uint64_t)w0 * 64, bhi = blo + (uint64_t)BT * 64;
    for (int i = threadIdx.x; i < BT; i += BB) img[i] = 0ull;
    if (threadIdx.x == 0) s_r[0] = dev::upper_bound(rge, 0, nr, blo);   // first end > blo
    if (threadIdx.x == 64) s_r[1] = dev::lower_bound(rgs, 0, nr, bhi);  // first start >= bhi
    __syncthreads();
    for (int64_t r = s_r[0] + threadIdx.x; r < s_r[1]; r += BB) {
        const uint64_t s = max((uint64_t)rgs[r], blo) - blo;
        const uint64_t e = min((uint64_t)rge[r], bhi) - blo;
        if (e <= s) continue;
        const uint64_t a = s >> 6, b = (e - 1) >> 6;
        for (uint64_t w = a; w <= b; ++w) {
            const uint64_t lo = w == a ? (s & 63) : 0;
            const uint64_t hi = w == b ? ((e - 1) & 63) : 63;
            const uint64_t m = (hi == 63 ? ~0ull : ((1ull << (hi + 1)) - 1)) & (~0ull << lo);
            if (m == ~0ull)
                img[w] = m;  // interior word: only this run covers it
            else
                atomicOr(&img[w], (unsigned long long)m);
        }
    }
    __syncthreads();
    const int cnt = (int)min((int64_t)BT, n_words - w0);
    for (int i = threadIdx.x; i < cnt; i += BB) words[w0 + i] = img[i];
}

// Binned rows -> bits: rows grouped by gs >> 16 (two radix passes instead of
// a full sort + merge).  A tile (4096 words = 2^18 bases = 4 bins) paints
// the rows that START in it into its LDS image (clipped at the tile end) and
// stores it once; the remainders of rows reaching past the tile are queued
// and OR-ed into global words by k_paint_cross after every tile is stored.
constexpr int BINSH = 16;
__device__ __forceinline__ int64_t lb_bin(const uint32_t *gs, int64_t n, uint32_t bin) {
    int64_t lo = 0, hi = n;  // first row with (gs >> BINSH) >= bin
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if ((gs[mid] >> BINSH) < bin)
            lo = mid + 1;
        else
            hi = mid;
    }
    return lo;
}

__device__ __forceinline__ void paint_lds(unsigned long long *img, uint64_t s, uint64_t e) {
    const uint64_t a = s >> 6, b = (e - 1) >> 6;
    for (uint64_t w = a; w <= b; ++w) {
        const uint64_t lo = w == a ? (s & 63) : 0;
        const uint64_t hi = w == b ? ((e - 1) & 63) : 63;
        const uint64_t m = (hi == 63 ? ~0ull : ((1ull << (hi + 1)) - 1)) & (~0ull << lo);
        atomicOr(&img[w], (unsigned long long)m);
    }
}

// first row of every paint tile (4 bins), searched once per tile up front
// instead of by each painting block (27 dependent loads on its critical path)
__global__ __launch_bounds__(BB) void k_tile_starts(const uint32_t *__restrict__ gs, int64_t n,
                                                    int64_t nt, uint32_t *__restrict__ tstart) {
    const int64_t t = (int64_t)blockIdx.x * BB + threadIdx.x;
    if (t > nt) return;
    const uint64_t bin = ((uint64_t)t * BT * 64) >> BINSH;
    tstart[t] = (uint32_t)(bin > 0xffffffffull ? n : lb_bin(gs, n, (uint32_t)bin));
}

__global__ __launch_bounds__(BB) void k_paint_rows(const uint32_t *__restrict__ gs,
                                                   const uint32_t *__restrict__ ge,
                                                   const uint32_t *__restrict__ tstart, int64_t n,
                                                   uint64_t *__restrict__ words, int64_t n_words,
                                                   uint64_t *__restrict__ cross,
                                                   unsigned int *__restrict__ ncross) {
    static_assert((int64_t)BT * 64 == (1ll << (BINSH + 2)), "tile = 4 bins");
    __shared__ unsigned long long img[BT];
    const int64_t w0 = (int64_t)blockIdx.x * BT;
    const uint64_t blo = (uint64_t)w0 * 64, bhi = blo + (uint64_t)BT * 64;
    for (int i = threadIdx.x; i < BT; i += BB) img[i] = 0ull;
    const int64_t r0 = tstart[blockIdx.x], r1 = tstart[blockIdx.x + 1];
    __syncthreads();
    for (int64_t r = r0 + threadIdx.x; r < r1; r += BB) {
        const uint64_t g0 = gs[r], g1 = ge[r];
        if (g1 <= g0) continue;
        paint_lds(img, g0 - blo, min(g1, bhi) - blo);
        if (g1 > bhi) cross[atomicAdd(ncross, 1u)] = (bhi << 32) | g1;  // remainder [bhi, g1)
    }
    __syncthreads();
    const int cnt = (int)min((int64_t)BT, n_words - w0);
    for (int i = threadIdx.x; i < cnt; i += BB) words[w0 + i] = img[i];
}

// bits [s, e) of global words (after every tile is stored)
__device__ __forceinline__ void paint_global(uint64_t *words, uint64_t s, uint64_t e) {
    const uint64_t a = s >> 6, b = (e - 1) >> 6;
    for (uint64_t w = a; w <= b; ++w) {
        const uint64_t lo = w == a ? (s & 63) : 0;
        const uint64_t hi = w == b ? ((e - 1) & 63) : 63;
        const uint64_t m = (hi == 63 ? ~0ull : ((1ull << (hi + 1)) - 1)) & (~0ull << lo);
        if (m == ~0ull)
            words[w] = m;  // full word: idempotent plain store
        else
            atomicOr((unsigned long long *)&words[w], (unsigned long long)m);
    }
}

__global__ __launch_bounds__(BB) void k_paint_cross(const uint64_t *__restrict__ cross,
                                                    const unsigned int *__restrict__ ncross,
                                                    uint64_t *__restrict__ words) {
    const int64_t nx = *ncross;
    for (int64_t i = (int64_t)blockIdx.x * BB + threadIdx.x; i < nx; i += (int64_t)gridDim.x * BB)
        paint_global(words, cross[i] >> 32, cross[i] & 0xffffffffull);
}

struct OpArgs {
    const uint64_t *w[MAXK];
    int k;
    int op;  // 0 a, 1 not a, 2 a & b, 3 a & ~b, 4 and of k
    int64_t n_words;
    int64_t span;
    const uint32_t *pad;  // pad bit position of every contig (sorted), nc entries
    int32_t nc;
};

__device__ __forceinline__ uint64_t op_raw(const OpArgs &a, int64_t w) {
    switch (a.op) {
        case 0: return a.w[0][w];
        case 1: return ~a.w[0][w];
        case 2: return a.w[0][w] & a.w[1][w];
        case 3: return a.w[0][w] & ~a.w[1][w];
        default: {
            uint64_t x = ~0ull;
            for (int i = 0; i < a.k; ++i) x &= a.w[i][w];
            return x;
        }
    }
}

__device__ __forceinline__ void events_of(uint64_t x, uint64_t prev, uint64_t &st, uint64_t &en) {
    const uint64_t sh = (x << 1) | (prev >> 63);
    st = x & ~sh;
    en = ~x & sh;
}

// Stage op(words) of tile [w0, w0 + BT) plus the word before it into LDS
// (img[0] = word w0 - 1).  NOT clears pad bits and bits beyond the span.
__device__ __forceinline__ void stage_tile(const OpArgs &a, int64_t w0, unsigned long long *img,
                                           uint32_t *s_pad, int *s_npad) {
    if (a.op == 1 && threadIdx.x == 0) {
        const int64_t lo = (w0 > 0 ? w0 - 1 : 0) * 64, hi = (w0 + BT) * 64;
        int64_t c = dev::lower_bound(a.pad, 0, (int64_t)a.nc, (uint32_t)min(lo, (int64_t)0xffffffff));
        int np = 0;
        for (; c < a.nc && (int64_t)a.pad[c] < hi && np < MAXPAD; ++c) s_pad[np++] = a.pad[c];
        *s_npad = np;
    }
    __syncthreads();
    for (int i = threadIdx.x; i <= BT; i += BB) {
        const int64_t w = w0 - 1 + i;
        uint64_t x = 0;
        if (w >= 0 && w < a.n_words) {
            x = op_raw(a, w);
            if (a.op == 1) {
                const int64_t b0 = w * 64;
                if (b0 + 64 > a.span) {
                    const int64_t keep = a.span - b0;
                    x &= keep <= 0 ? 0ull : (keep >= 64 ? ~0ull : ((1ull << keep) - 1));
                }
                for (int p = 0; p < *s_npad; ++p) {
                    const int64_t d = (int64_t)s_pad[p] - b0;
                    if (d >= 0 && d < 64) x &= ~(1ull << d);
                }
            }
        }
        img[i] = x;
    }
    __syncthreads();
}

__global__ __launch_bounds__(BB) void k_ev_count(OpArgs a, uint32_t *__restrict__ tcnt) {
    __shared__ unsigned long long img[BT + 1];
    __shared__ uint32_t s_pad[MAXPAD];
    __shared__ int s_npad;
    __shared__ uint32_t ws[BB / 64];
    const int64_t w0 = (int64_t)blockIdx.x * BT;
    stage_tile(a, w0, img, s_pad, &s_npad);
    uint32_t c = 0;
    for (int i = threadIdx.x; i < BT; i += BB) {
        uint64_t st, en;
        events_of(img[i + 1], img[i], st, en);
        c += __popcll(st) + __popcll(en);
    }
    c = dev::wave_reduce_sum(c);
    if (dev::lane_id() == 0) ws[threadIdx.x / 64] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
        for (int i = 0; i < BB / 64; ++i) t += ws[i];
        tcnt[blockIdx.x] = t;
    }
}

__global__ __launch_bounds__(BB) void k_ev_write(OpArgs a, const uint32_t *__restrict__ toff,
                                                 uint32_t *__restrict__ rgs,
                                                 uint32_t *__restrict__ rge) {
    __shared__ unsigned long long img[BT + 1];
    __shared__ uint32_t s_pad[MAXPAD];
    __shared__ int s_npad;
    __shared__ uint32_t scratch[BB / 64 + 1];
    const int64_t w0 = (int64_t)blockIdx.x * BT;
    stage_tile(a, w0, img, s_pad, &s_npad);
    // blocked: thread t owns tile words t*BW .. t*BW + BW - 1 (position order)
    const int q0 = threadIdx.x * BW;
    uint32_t c = 0;
#pragma unroll
    for (int k = 0; k < BW; ++k) {
        uint64_t st, en;
        events_of(img[q0 + k + 1], img[q0 + k], st, en);
        c += __popcll(st) + __popcll(en);
    }
    uint32_t tot;
    uint32_t ev = toff[blockIdx.x] + dev::block_exclusive_sum<BB>(c, scratch, &tot);
#pragma unroll
    for (int k = 0; k < BW; ++k) {
        uint64_t st, en;
        events_of(img[q0 + k + 1], img[q0 + k], st, en);
        uint64_t all = st | en;
        const uint32_t base = (uint32_t)((w0 + q0 + k) * 64);
        while (all) {
            const int b = __builtin_ctzll(all);
            all &= all - 1;
            const uint32_t p = base + (uint32_t)b;
            if (ev & 1u)
                rge[ev >> 1] = p;
            else
                rgs[ev >> 1] = p;
            ++ev;
        }
    }
}

__global__ __launch_bounds__(BB) void k_popcount(const uint64_t *__restrict__ w, int64_t n,
                                                 unsigned long long *out) {
    uint64_t c = 0;
    for (int64_t i = (int64_t)blockIdx.x * BB + threadIdx.x; i < n; i += (int64_t)gridDim.x * BB)
        c += __popcll(w[i]);
    c = dev::wave_reduce_sum(c);
    if (dev::lane_id() == 0) atomicAdd(out, (unsigned long long)c);
}

// Single pass (count + write) when the run count has a known bound: tiles
// in ticket order, the event offset of a tile by decoupled look-back over
// the per-tile status words (flag in bits 62-63, value below), and events
// past the capacity only counted (the caller then falls back to two passes).
constexpr uint64_t EV_AGG = 1ull << 62, EV_INC = 2ull << 62, EV_VAL = (1ull << 62) - 1;

__global__ __launch_bounds__(BB) void k_ev_fused(OpArgs a, uint64_t *__restrict__ status,
                                                 unsigned int *__restrict__ ticket,
                                                 int64_t cap_events, uint32_t *__restrict__ rgs,
                                                 uint32_t *__restrict__ rge,
                                                 unsigned long long *__restrict__ total) {
    __shared__ unsigned long long img[BT + 1];
    __shared__ uint32_t s_pad[MAXPAD];
    __shared__ int s_npad;
    __shared__ uint32_t scratch[BB / 64 + 1];
    __shared__ uint32_t s_tile;
    __shared__ uint64_t s_excl;
    if (threadIdx.x == 0) s_tile = atomicAdd(ticket, 1u);
    __syncthreads();
    const uint32_t tile = s_tile;
    const int64_t w0 = (int64_t)tile * BT;
    stage_tile(a, w0, img, s_pad, &s_npad);
    const int q0 = threadIdx.x * BW;
    uint32_t c = 0;
#pragma unroll
    for (int k = 0; k < BW; ++k) {
        uint64_t st, en;
        events_of(img[q0 + k + 1], img[q0 + k], st, en);
        c += __popcll(st) + __popcll(en);
    }
    uint32_t tot;
    const uint32_t mine = dev::block_exclusive_sum<BB>(c, scratch, &tot);
    if (threadIdx.x < 64) {  // one wave publishes and looks back
        const int lane = dev::lane_id();
        if (tile == 0) {
            if (lane == 0) {
                __hip_atomic_store(status, EV_INC | tot, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
                s_excl = 0;
            }
        } else {
            if (lane == 0)
                __hip_atomic_store(status + tile, EV_AGG | tot, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            uint64_t acc = 0;
            for (int64_t base = (int64_t)tile - 1; base >= 0; base -= 64) {
                const int64_t t = base - lane;
                uint64_t v = EV_INC;  // before tile 0: the inclusive identity
                if (t >= 0) {
                    v = __hip_atomic_load(status + t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    while ((v >> 62) == 0) {
                        __builtin_amdgcn_s_sleep(1);
                        v = __hip_atomic_load(status + t, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
                    }
                }
                const uint64_t inc = __ballot((v >> 62) == 2);
                uint64_t val = v & EV_VAL;
                if (inc && lane > __builtin_ctzll(inc)) val = 0;
                acc += dev::wave_reduce_sum(val);
                if (inc) break;
            }
            if (lane == 0) {
                __hip_atomic_store(status + tile, EV_INC | (acc + tot), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
                s_excl = acc;
            }
        }
    }
    __syncthreads();
    const uint64_t excl = s_excl;
    if (tile == gridDim.x - 1 && threadIdx.x == 0) *total = excl + tot;
    uint64_t ev = excl + mine;
#pragma unroll
    for (int k = 0; k < BW; ++k) {
        uint64_t st, en;
        events_of(img[q0 + k + 1], img[q0 + k], st, en);
        uint64_t all = st | en;
        const uint32_t base = (uint32_t)((w0 + q0 + k) * 64);
        while (all) {
            const int b = __builtin_ctzll(all);
            all &= all - 1;
            if ((int64_t)ev < cap_events) {
                const uint32_t p = base + (uint32_t)b;
                if (ev & 1u)
                    rge[ev >> 1] = p;
                else
                    rgs[ev >> 1] = p;
            }
            ++ev;
        }
    }
}

}  // namespace

int merge_runs(lime_ctx *ctx, const lime_set *set, lime_result *res, bool want_run_ids);

int bitset_build(lime_ctx *ctx, const lime_set *a, lime_bitset *bs) {
    lime_result runs;
    runs.ctx = ctx;
    LIME_TRY(merge_runs(ctx, a, &runs, false));
    bs->runs_bound = runs.n;
    const int64_t span = (int64_t)a->off[a->n_contigs];
    bs->span = span;
    bs->n_words = (span + 63) / 64;
    LIME_TRY(alloc(ctx, &bs->words, (size_t)bs->n_words));
    const int64_t nt = (bs->n_words + BT - 1) / BT;
    if (nt > 0)
        hipLaunchKernelGGL(k_paint, dim3((unsigned)nt), dim3(BB), 0, S(ctx), runs.gs, runs.ge,
                           runs.n, bs->words, bs->n_words);
    LIME_HIP(hipGetLastError());
    release(ctx, runs.gs);
    release(ctx, runs.ge);
    return LIME_OK;
}

// bits of a BINNED set (min_shift == 16): no merge, no full sort
int bitset_build_binned(lime_ctx *ctx, const lime_set *a, lime_bitset *bs) {
    const int64_t span = (int64_t)a->off[a->n_contigs];
    bs->runs_bound = a->n;  // the union of n rows has at most n runs
    bs->span = span;
    bs->n_words = (span + 63) / 64;
    LIME_TRY(alloc(ctx, &bs->words, (size_t)bs->n_words));
    const int64_t nt = (bs->n_words + BT - 1) / BT;
    uint64_t *cross;
    unsigned int *ncross;
    LIME_TRY(alloc(ctx, &cross, (size_t)std::max<int64_t>(a->n, 1)));
    LIME_TRY(alloc(ctx, &ncross, 1));
    LIME_HIP(hipMemsetAsync(ncross, 0, sizeof(unsigned int), S(ctx)));
    uint32_t *tstart;
    LIME_TRY(alloc(ctx, &tstart, (size_t)nt + 1));
    if (nt > 0) {
        hipLaunchKernelGGL(k_tile_starts, dim3(blocks_for(nt + 1, BB)), dim3(BB), 0, S(ctx),
                           a->gs, a->n, nt, tstart);
        hipLaunchKernelGGL(k_paint_rows, dim3((unsigned)nt), dim3(BB), 0, S(ctx), a->gs, a->ge,
                           (const uint32_t *)tstart, a->n, bs->words, bs->n_words, cross, ncross);
    }
    if (a->n > 0)
        hipLaunchKernelGGL(k_paint_cross, dim3(std::min<unsigned>(blocks_for(a->n, BB), 2048u)),
                           dim3(BB), 0, S(ctx),
                           (const uint64_t *)cross, (const unsigned int *)ncross, bs->words);
    LIME_HIP(hipGetLastError());
    release(ctx, cross);
    release(ctx, ncross);
    release(ctx, tstart);
    return LIME_OK;
}

int bitset_runs(lime_ctx *ctx, int op, int k, const lime_bitset *const *sets, lime_result *res) {
    const lime_bitset *a = sets[0];
    if (k > MAXK) return fail(LIME_ERR_ARG, "at most 16 bitsets per op");
    OpArgs oa;
    for (int i = 0; i < MAXK; ++i) oa.w[i] = i < k ? sets[i]->words : nullptr;
    oa.k = k;
    oa.op = op;
    oa.n_words = a->n_words;
    oa.span = a->span;
    oa.nc = a->n_contigs;
    // pad positions: off[c+1] - 1
    std::vector<uint32_t> pad(a->n_contigs);
    for (int c = 0; c < a->n_contigs; ++c) pad[c] = a->off[c + 1] - 1;
    uint32_t *d_pad;
    LIME_TRY(alloc(ctx, &d_pad, pad.size() + 1));
    if (!pad.empty()) {
        LIME_HIP(hipMemcpyAsync(d_pad, pad.data(), pad.size() * 4, hipMemcpyHostToDevice, S(ctx)));
        LIME_HIP(hipStreamSynchronize(S(ctx)));
    }
    oa.pad = d_pad;
    const int64_t nt = (a->n_words + BT - 1) / BT;
    // bound on the result's runs: each run starts at a run start of one
    // operand (AND / ANDN also at a run end of B); NOT adds one gap per contig
    bool known = true;
    int64_t sum = 0;
    for (int i = 0; i < k; ++i) {
        known = known && sets[i]->runs_bound >= 0;
        sum += sets[i]->runs_bound;
    }
    const int64_t bound = op == 1 ? a->runs_bound + a->n_contigs + 1 : sum + 1;
    if (known && nt > 0 && bound < (int64_t)0x7fffffff) {
        uint64_t *status;
        unsigned int *ticket;
        unsigned long long *tot64;
        LIME_TRY(alloc(ctx, &status, (size_t)nt));
        LIME_TRY(alloc(ctx, &ticket, 1));
        LIME_TRY(alloc(ctx, &tot64, 1));
        LIME_TRY(alloc(ctx, &res->gs, (size_t)bound));
        LIME_TRY(alloc(ctx, &res->ge, (size_t)bound));
        LIME_HIP(hipMemsetAsync(status, 0, sizeof(uint64_t) * (size_t)nt, S(ctx)));
        LIME_HIP(hipMemsetAsync(ticket, 0, sizeof(unsigned int), S(ctx)));
        hipLaunchKernelGGL(k_ev_fused, dim3((unsigned)nt), dim3(BB), 0, S(ctx), oa, status,
                           ticket, 2 * bound, res->gs, res->ge, tot64);
        LIME_HIP(hipGetLastError());
        unsigned long long nev = 0;
        LIME_TRY(read_back(ctx, &nev, tot64, sizeof(nev)));
        release(ctx, status);
        release(ctx, ticket);
        release(ctx, tot64);
        if ((int64_t)nev <= 2 * bound) {
            release(ctx, d_pad);
            if (nev & 1u) return fail(LIME_ERR_DEVICE, "bitset run extraction: odd event count");
            const int64_t nr = (int64_t)nev / 2;
            if (nr < bound / 2) {  // keep the result's memory to its size
                uint32_t *gs, *ge;
                LIME_TRY(alloc(ctx, &gs, (size_t)nr));
                LIME_TRY(alloc(ctx, &ge, (size_t)nr));
                if (nr > 0) {
                    LIME_HIP(hipMemcpyAsync(gs, res->gs, 4 * (size_t)nr, hipMemcpyDeviceToDevice,
                                            S(ctx)));
                    LIME_HIP(hipMemcpyAsync(ge, res->ge, 4 * (size_t)nr, hipMemcpyDeviceToDevice,
                                            S(ctx)));
                }
                release(ctx, res->gs);
                release(ctx, res->ge);
                res->gs = gs;
                res->ge = ge;
            }
            res->n = nr;
            return LIME_OK;
        }
        // the bound did not hold (it always should): count first, then write
        release(ctx, res->gs);
        release(ctx, res->ge);
    }
    uint32_t *tcnt, *toff, *total;
    LIME_TRY(alloc(ctx, &tcnt, (size_t)nt));
    LIME_TRY(alloc(ctx, &toff, (size_t)nt));
    LIME_TRY(alloc(ctx, &total, 1));
    hipLaunchKernelGGL(k_ev_count, dim3((unsigned)nt), dim3(BB), 0, S(ctx), oa, tcnt);
    LIME_HIP(hipGetLastError());
    LIME_TRY(scan_exclusive_u32(ctx, tcnt, toff, nt, total));
    uint32_t nev = 0;
    LIME_TRY(read_back(ctx, &nev, total, sizeof(nev)));
    if (nev & 1u) return fail(LIME_ERR_DEVICE, "bitset run extraction: odd event count");
    const int64_t nr = nev / 2;
    LIME_TRY(alloc(ctx, &res->gs, (size_t)nr));
    LIME_TRY(alloc(ctx, &res->ge, (size_t)nr));
    hipLaunchKernelGGL(k_ev_write, dim3((unsigned)nt), dim3(BB), 0, S(ctx), oa,
                       (const uint32_t *)toff, res->gs, res->ge);
    LIME_HIP(hipGetLastError());
    release(ctx, tcnt);
    release(ctx, toff);
    release(ctx, total);
    release(ctx, d_pad);
    res->n = nr;
    return LIME_OK;
}

int64_t bitset_popcount(lime_ctx *ctx, const lime_bitset *a) {
    unsigned long long *d;
    if (alloc(ctx, &d, 1)) return -1;
    if (hipMemsetAsync(d, 0, 8, S(ctx)) != hipSuccess) return -1;
    unsigned grid = blocks_for(a->n_words, BB);
    if (grid > 8192) grid = 8192;
    if (grid == 0) grid = 1;
    hipLaunchKernelGGL(k_popcount, dim3(grid), dim3(BB), 0, S(ctx), a->words, a->n_words, d);
    unsigned long long h = 0;
    if (read_back(ctx, &h, d, 8)) return -1;
    release(ctx, d);
    return (int64_t)h;
}

}  // namespace lime

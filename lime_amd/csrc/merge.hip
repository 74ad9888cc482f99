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
// Kernels (tile = 4096 rows):
//   k_tile_max    per-tile max of ge                               4 B/row
//   k_scan_max    exclusive max over tiles (one block)
//   k_runs_count  M_i, flags, runs per tile                        8 B/row
//   scan          exclusive sum of runs per tile
//   k_runs_write  run starts/ends + run id of every row            8 B/row + 4 B/row + 8 B/run
// The same scan gives the inclusive prefix max used by subtract.
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

// Per tile: exclusive prefix max M of every row; returns flags as a bitmask.
__device__ __forceinline__ uint32_t tile_flags(const uint32_t *__restrict__ gs,
                                               const uint32_t *__restrict__ ge, int64_t base,
                                               int64_t n, uint32_t carry, uint32_t *lds,
                                               uint32_t *scratch, uint32_t (&M)[MITEMS],
                                               uint32_t (&s)[MITEMS], uint32_t (&e)[MITEMS]) {
    load_blocked(gs, base, n, 0xffffffffu, lds, s);
    load_blocked(ge, base, n, 0u, lds, e);
    uint32_t agg = 0;
#pragma unroll
    for (int k = 0; k < MITEMS; ++k) agg = max(agg, e[k]);
    uint32_t tot;
    uint32_t pre = dev::block_exclusive_max<MB>(agg, 0u, scratch, &tot);
    uint32_t run = max(pre, carry);
    uint32_t flags = 0;
#pragma unroll
    for (int k = 0; k < MITEMS; ++k) {
        M[k] = run;
        int64_t i = base + threadIdx.x * MITEMS + k;
        if (i < n && run <= s[k]) flags |= 1u << k;
        run = max(run, e[k]);
    }
    return flags;
}

__global__ __launch_bounds__(MB) void k_runs_count(const uint32_t *__restrict__ gs,
                                                   const uint32_t *__restrict__ ge, int64_t n,
                                                   const uint32_t *__restrict__ tpre,
                                                   uint32_t *__restrict__ tcnt) {
    __shared__ uint32_t lds[MTILE];
    __shared__ uint32_t scratch[MB / 64 + 1];
    const int64_t base = (int64_t)blockIdx.x * MTILE;
    uint32_t M[MITEMS], s[MITEMS], e[MITEMS];
    uint32_t f = tile_flags(gs, ge, base, n, tpre[blockIdx.x], lds, scratch, M, s, e);
    uint32_t c = __popc(f);
    c = dev::wave_reduce_sum(c);
    __shared__ uint32_t ws[MB / 64];
    if (dev::lane_id() == 0) ws[threadIdx.x / 64] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
        for (int i = 0; i < MB / 64; ++i) t += ws[i];
        tcnt[blockIdx.x] = t;
    }
}

__global__ __launch_bounds__(MB) void k_runs_write(
    const uint32_t *__restrict__ gs, const uint32_t *__restrict__ ge, int64_t n,
    const uint32_t *__restrict__ tpre, const uint32_t *__restrict__ toff,
    uint32_t *__restrict__ run_gs, uint32_t *__restrict__ run_ge,
    uint32_t *__restrict__ run_of_sorted) {
    __shared__ uint32_t lds[MTILE];
    __shared__ uint32_t scratch[MB / 64 + 1];
    const int64_t base = (int64_t)blockIdx.x * MTILE;
    uint32_t M[MITEMS], s[MITEMS], e[MITEMS];
    uint32_t f = tile_flags(gs, ge, base, n, tpre[blockIdx.x], lds, scratch, M, s, e);
    uint32_t tot;
    uint32_t r = toff[blockIdx.x] + dev::block_exclusive_sum<MB>((uint32_t)__popc(f), scratch, &tot);
    uint32_t rid[MITEMS];
#pragma unroll
    for (int k = 0; k < MITEMS; ++k) {
        int64_t i = base + threadIdx.x * MITEMS + k;
        if (i < n) {
            if (f & (1u << k)) {
                run_gs[r] = s[k];
                if (r > 0) run_ge[r - 1] = M[k];
                ++r;
            }
            if (i == n - 1) run_ge[r - 1] = max(M[k], e[k]);
        }
        rid[k] = r - 1;
    }
    if (run_of_sorted) {
        // blocked -> striped through LDS for coalesced stores
#pragma unroll
        for (int k = 0; k < MITEMS; ++k) lds[threadIdx.x * MITEMS + k] = rid[k];
        __syncthreads();
#pragma unroll
        for (int k = 0; k < MITEMS; ++k) {
            int64_t i = base + k * MB + threadIdx.x;
            if (i < n) run_of_sorted[i] = lds[k * MB + threadIdx.x];
        }
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

int build_prefix_max(lime_ctx *ctx, const lime_set *set) {
    if (set->pmax) return LIME_OK;
    const int64_t n = set->n;
    uint32_t *pm;
    LIME_TRY(alloc(ctx, &pm, (size_t)n));
    if (n > 0) {
        uint32_t *tpre;
        LIME_TRY(tile_prefix(ctx, set->ge, n, &tpre));
        const int64_t nt = (n + MTILE - 1) / MTILE;
        hipLaunchKernelGGL(k_prefix_max, dim3((unsigned)nt), dim3(MB), 0, S(ctx), set->ge, n,
                           (const uint32_t *)tpre, pm);
        LIME_HIP(hipGetLastError());
        release(ctx, tpre);
    }
    set->pmax = pm;
    return LIME_OK;
}

// merge runs of a sorted set; result owns run_gs / run_ge / run_of_sorted
int merge_runs(lime_ctx *ctx, const lime_set *set, lime_result *res, bool want_run_ids) {
    const int64_t n = set->n;
    res->n = 0;
    if (n == 0) {
        LIME_TRY(alloc(ctx, &res->gs, 1));
        LIME_TRY(alloc(ctx, &res->ge, 1));
        return LIME_OK;
    }
    const int64_t nt = (n + MTILE - 1) / MTILE;
    uint32_t *tpre, *tcnt, *toff, *total;
    LIME_TRY(tile_prefix(ctx, set->ge, n, &tpre));
    LIME_TRY(alloc(ctx, &tcnt, (size_t)nt));
    LIME_TRY(alloc(ctx, &toff, (size_t)nt));
    LIME_TRY(alloc(ctx, &total, 1));
    hipLaunchKernelGGL(k_runs_count, dim3((unsigned)nt), dim3(MB), 0, S(ctx), set->gs, set->ge, n,
                       (const uint32_t *)tpre, tcnt);
    LIME_HIP(hipGetLastError());
    LIME_TRY(scan_exclusive_u32(ctx, tcnt, toff, nt, total));
    uint32_t nr = 0;
    LIME_TRY(read_back(ctx, &nr, total, sizeof(nr)));
    LIME_TRY(alloc(ctx, &res->gs, nr));
    LIME_TRY(alloc(ctx, &res->ge, nr));
    if (want_run_ids) LIME_TRY(alloc(ctx, &res->run_of_sorted, (size_t)n));
    hipLaunchKernelGGL(k_runs_write, dim3((unsigned)nt), dim3(MB), 0, S(ctx), set->gs, set->ge, n,
                       (const uint32_t *)tpre, (const uint32_t *)toff, res->gs, res->ge,
                       res->run_of_sorted);
    LIME_HIP(hipGetLastError());
    release(ctx, tpre);
    release(ctx, tcnt);
    release(ctx, toff);
    release(ctx, total);
    res->n = nr;
    return LIME_OK;
}

}  // namespace lime

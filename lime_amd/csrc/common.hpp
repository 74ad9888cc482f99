// common.hpp -- internal types shared by the engine's translation units:
// context (device, stream, caching pool), coordinate space, device sets and
// results, error plumbing, and the wave/block primitives the kernels use.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <limits>

#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/lime_amd.h"

namespace lime {

// ------------------------------------------------------------------ errors
void set_error(const std::string &msg);
int fail(int code, const std::string &msg);

#define LIME_HIP(expr)                                                                          \
    do {                                                                                        \
        hipError_t _e = (expr);                                                                 \
        if (_e != hipSuccess)                                                                   \
            return ::lime::fail(LIME_ERR_DEVICE, std::string(#expr) + ": " + hipGetErrorString(_e)); \
    } while (0)

#define LIME_TRY(expr)                \
    do {                              \
        int _s = (expr);              \
        if (_s != LIME_OK) return _s; \
    } while (0)

// ------------------------------------------------------------- device pool
// Grow-only caching allocator: blocks are recycled by exact (rounded) size so
// that repeated operator calls of the same shape never hit hipMalloc.
// Caching device allocator of one context.  A released block is reused at
// once by work on the stream that released it (stream order).  Once the
// context has run on more than one stream (lime_ctx_set_stream), each release
// also records an event, and work on another stream takes the block only
// after that event has completed -- so e.g. the next batch's sort can run on
// a second stream while this batch's fill streams, sharing one pool.
struct Pool {
    struct Block {
        void *p;
        hipStream_t s;   // stream current at release
        hipEvent_t ev;   // completion of the releasing stream's work (or null)
    };
    std::multimap<size_t, Block> free_blocks;
    std::map<void *, size_t> live;
    std::vector<hipEvent_t> spare_events;
    const hipStream_t *stream = nullptr;  // the owning context's current stream
    bool multi_stream = false;
    int64_t held = 0;
    int64_t in_use = 0, peak = 0;  // bytes of live blocks; their high-water mark
    void *get(size_t bytes);
    void put(void *p);
    void release_all();
};

// A space's contig offsets and lengths on the device, cached per context
// (space_device) and shared by the sets created in it
struct SpaceDev {
    lime_ctx *ctx = nullptr;
    uint32_t *off = nullptr, *len = nullptr;
    ~SpaceDev();
};

}  // namespace lime

struct lime_ctx {
    int device = 0;
    hipStream_t own_stream = nullptr;
    hipStream_t stream = nullptr;
    lime::Pool pool;
    std::mutex mu;
    // small pinned scratch for scalar read-backs
    void *pinned = nullptr;
    // device copies of the spaces' (off, len) used with this context, keyed
    // by the offsets (which determine the lengths): uploaded once, so an
    // operator never drains the stream to upload them (space_device).
    // Bounded: past SPACE_CACHE entries, the ones no live set holds are
    // dropped (ad-hoc spaces no longer accumulate)
    std::map<std::vector<uint32_t>, std::shared_ptr<lime::SpaceDev>> spaces;
    static constexpr size_t SPACE_CACHE = 8;
    hipEvent_t ev = nullptr;
    // bit-per-base builds: after an optimistic (uncounted) binning overflowed
    // its regions, this many later builds take the counted path first
    int bin_pessimism = 0;
};

struct lime_space {
    int32_t n = 0;
    std::vector<int64_t> len;   // contig lengths
    std::vector<uint32_t> off;  // n + 1 entries; off[c+1] = off[c] + len[c] + 1
    int64_t span = 0;           // off[n]
};

// Device-resident sorted set: canonical order (gstart, zero-width first).
struct lime_set {
    lime_ctx *ctx = nullptr;
    int64_t n = 0;
    uint32_t *gs = nullptr;   // global start
    uint32_t *ge = nullptr;   // global end
    uint32_t *row = nullptr;  // input row
    // device copy of the space offsets (n_contigs + 1), borrowed from the
    // context's cache entry `space_keep` (held while the set lives)
    uint32_t *d_off = nullptr;
    std::shared_ptr<lime::SpaceDev> space_keep;
    int32_t n_contigs = 0;
    std::vector<uint32_t> off;  // host copy
    std::vector<int64_t> len;
    // statistics gathered during creation
    uint32_t min_width = 0, max_width = 0;
    bool has_zero_width = false;
    // lazily built: inclusive prefix max of ge (for subtract)
    mutable uint32_t *pmax = nullptr;
    // stranded sets (lime_set_create_host_stranded): strand code per INPUT
    // row; the set is sorted by (gs, ge, strand) and merge breaks runs at
    // strand changes (the reference fold's overlaps test)
    int8_t *strand_in = nullptr;
    bool strand_uniform = false;  // every row has the same strand code
    // strand_in indexed by SORTED position instead of row id (global
    // stranded sets, whose row ids are the caller's)
    bool strand_sorted = false;
    // sort by (gs, ge, row) (subtract's tie index, a temporary set)
    bool row_ties = false;
    // lazily built: the rows of B's multi-row same-start groups sorted by
    // (gs, ge, row) -- subtract's block head among many same-start hits
    mutable uint32_t *tie_gs = nullptr, *tie_ge = nullptr, *tie_row = nullptr;
    mutable int64_t tie_n = -1;  // -1: not built
    // binned sets (bitset painting from unsorted rows): only the gs digits
    // at shifts >= min_shift are sorted, i.e. rows grouped by gs >> min_shift
    int min_shift = 0;
};

struct lime_result {
    lime_ctx *ctx = nullptr;
    int64_t n = 0;
    uint32_t *gs = nullptr;   // global start
    uint32_t *ge = nullptr;   // global end
    uint32_t *a_row = nullptr;  // may be null
    uint32_t *b_row = nullptr;  // may be null (0xffffffff = None)
    uint32_t *run_of_sorted = nullptr;  // merge only (per sorted input)
    int8_t *run_strand = nullptr;       // merge of a stranded set: strand per run
    const lime_set *src = nullptr;      // merge only
    uint32_t *d_off = nullptr;          // contig offsets used to localise
    int32_t n_contigs = 0;
    std::vector<uint32_t> off;
};

struct lime_bitset {
    lime_ctx *ctx = nullptr;
    uint64_t *words = nullptr;
    int64_t n_words = 0;
    int64_t runs_bound = -1;  // upper bound on its runs (rows painted), -1 unknown
    int64_t word0 = 0;        // global index of words[0] (a coordinate shard's window)
    int64_t hi_bit = 0;       // end of the window (global bits): bits >= hi_bit are outside
    int64_t span = 0;
    uint32_t *d_off = nullptr;
    int32_t n_contigs = 0;
    std::vector<uint32_t> off;
    std::vector<int64_t> len;
    // binned form (bitset_build_rows, bitset_and_rows): the bits are the AND
    // of these row sets, each grouped by paint tile; words painted on first
    // need (null until then) or never, when an op's runs are extracted
    // straight from the bins (k_paint_ev)
    struct Bins {
        uint32_t *slab2 = nullptr;   // packed rows, tile order
        uint32_t *tstart = nullptr;  // nt + 1 tile starts
        uint2 *xl = nullptr;         // tile-bucketed cross pieces (null: none)
        uint32_t *xb = nullptr;      // [bucket starts | full-tile scan | fill] x (nt + 1)
        bool own_tstart = true;      // (else inside the first set's block)
    };
    std::vector<Bins> bins;
    int64_t nt = 0;  // paint tiles of the bins
};

namespace lime {

inline hipStream_t S(lime_ctx *c) { return c->stream; }

template <typename T>
inline int alloc(lime_ctx *c, T **p, size_t count) {
    size_t bytes = count * sizeof(T);
    if (bytes == 0) bytes = 256;
    void *v = c->pool.get(bytes);
    if (!v) return fail(LIME_ERR_NOMEM, "device allocation of " + std::to_string(bytes) + " bytes failed");
    *p = reinterpret_cast<T *>(v);
    return LIME_OK;
}
template <typename T>
inline void release(lime_ctx *c, T *&p) {
    if (p) c->pool.put(reinterpret_cast<void *>(p));
    p = nullptr;
}

// RAII release of a pool block on every return path
template <typename T>
struct PoolGuard {
    lime_ctx *ctx;
    T *&p;
    ~PoolGuard() { release(ctx, p); }
};

// read a device scalar back to the host (synchronises the context stream)
int read_back(lime_ctx *c, void *host, const void *dev, size_t bytes);

// the context's device copy of a space's contig offsets (n + 1 entries) and
// lengths (n + 1, the last 0), owned by the context's cache: never released
// by callers; valid for the call, or as long as `keep` is held
int space_device(lime_ctx *c, const std::vector<uint32_t> &off, const uint32_t **d_off,
                 const uint32_t **d_len, std::shared_ptr<SpaceDev> *keep = nullptr);

// grid helper
inline unsigned blocks_for(int64_t n, int64_t per_block) {
    return (unsigned)((n + per_block - 1) / per_block);
}

// ------------------------------------------------------ kernel entry points
// (defined in the .hip translation units)
int sort_set(lime_ctx *ctx, lime_set *set, const int32_t *d_contig, const uint32_t *d_start,
             const uint32_t *d_end, const uint32_t *d_len);
int scan_exclusive_u32(lime_ctx *ctx, const uint32_t *in, uint32_t *out, int64_t n,
                       uint32_t *total_dev);
int scan_exclusive_u32_pair(lime_ctx *ctx, const uint32_t *in0, uint32_t *out0, int64_t n0,
                            const uint32_t *in1, uint32_t *out1, int64_t n1);
int scan_exclusive_u64(lime_ctx *ctx, const uint64_t *in, uint64_t *out, int64_t n,
                       uint64_t *total_dev);
int build_prefix_max(lime_ctx *ctx, const lime_set *set);
// inclusive prefix max of a u32 array (out may alias in)
int prefix_max_u32(lime_ctx *ctx, const uint32_t *in, uint32_t *out, int64_t n);

}  // namespace lime

// ====================================================================== device
// Wave (64-lane) and block primitives.  Block size is a multiple of 64.
#ifdef __HIPCC__
namespace lime {
namespace dev {

constexpr int WAVE = 64;

__device__ __forceinline__ int lane_id() { return __lane_id(); }

__device__ __forceinline__ uint64_t lanemask_lt() {
    int l = __lane_id();
    return l == 0 ? 0ull : (~0ull >> (64 - l));
}

// Wave scans and reductions on DPP (data-parallel primitives: a VALU
// operand read from another lane of the row / wave, no LDS crossbar): row_shr
// 1, 2, 4, 8 scan each 16-lane row, row_bcast:15 / :31 carry the row totals
// into the rows above (rows 1, 3 then rows 2, 3).  Lanes whose source is
// outside the row or whose row is masked off get `ident`.  A reduction is the
// scan's lane 63, read into a scalar register (v_readlane).  (The
// ds_bpermute-based __shfl_up / __shfl_xor version cost an LDS round trip per
// step.)
template <int CTRL, int ROWS = 0xf>
__device__ __forceinline__ uint32_t dpp32(uint32_t ident, uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)ident, (int)v, CTRL, ROWS, 0xf, false);
}
template <int CTRL, int ROWS = 0xf, typename T>
__device__ __forceinline__ T dpp_move(T ident, T v) {
    if constexpr (sizeof(T) == 8) {
        const uint64_t a = (uint64_t)ident, b = (uint64_t)v;
        const uint32_t lo = dpp32<CTRL, ROWS>((uint32_t)a, (uint32_t)b);
        const uint32_t hi = dpp32<CTRL, ROWS>((uint32_t)(a >> 32), (uint32_t)(b >> 32));
        return (T)(((uint64_t)hi << 32) | lo);
    } else {
        return (T)dpp32<CTRL, ROWS>((uint32_t)ident, (uint32_t)v);
    }
}
template <typename T, typename Op>
__device__ __forceinline__ T wave_scan_dpp(T x, T ident, Op op) {
    x = op(x, dpp_move<0x111>(ident, x));        // row_shr:1
    x = op(x, dpp_move<0x112>(ident, x));        // row_shr:2
    x = op(x, dpp_move<0x114>(ident, x));        // row_shr:4
    x = op(x, dpp_move<0x118>(ident, x));        // row_shr:8
    x = op(x, dpp_move<0x142, 0xa>(ident, x));   // row_bcast:15 -> rows 1, 3
    x = op(x, dpp_move<0x143, 0xc>(ident, x));   // row_bcast:31 -> rows 2, 3
    return x;
}
// the value of lane 63, wave-uniform
template <typename T>
__device__ __forceinline__ T lane63(T v) {
    if constexpr (sizeof(T) == 8) {
        const uint64_t b = (uint64_t)v;
        const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)b, 63);
        const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), 63);
        return (T)(((uint64_t)hi << 32) | lo);
    } else {
        return (T)__builtin_amdgcn_readlane((int)v, 63);
    }
}
// lane l gets lane l - 1's value (lane 0: ident): DPP wave_shr:1
template <typename T>
__device__ __forceinline__ T wave_shr1(T v, T ident) {
    return dpp_move<0x138>(ident, v);
}

template <typename T>
__device__ __forceinline__ T wave_inclusive_sum(T v) {
    return wave_scan_dpp(v, (T)0, [](T a, T b) { return a + b; });
}
template <typename T>
__device__ __forceinline__ T wave_inclusive_max(T v) {
    return wave_scan_dpp(v, std::numeric_limits<T>::lowest(), [](T a, T b) { return a > b ? a : b; });
}
template <typename T>
__device__ __forceinline__ T wave_reduce_sum(T v) {
    return lane63(wave_inclusive_sum(v));
}
template <typename T>
__device__ __forceinline__ T wave_reduce_max(T v) {
    return lane63(wave_inclusive_max(v));
}
template <typename T>
__device__ __forceinline__ T wave_reduce_or(T v) {
    return lane63(wave_scan_dpp(v, (T)0, [](T a, T b) { return a | b; }));
}
template <typename T>
__device__ __forceinline__ T wave_reduce_xor(T v) {
    return lane63(wave_scan_dpp(v, (T)0, [](T a, T b) { return a ^ b; }));
}
template <typename T>
__device__ __forceinline__ T wave_reduce_min(T v) {
    return lane63(wave_scan_dpp(v, std::numeric_limits<T>::max(), [](T a, T b) { return a < b ? a : b; }));
}

// Block-wide exclusive sum. `scratch` holds >= BLOCK/64 + 1 T's.  Returns the
// exclusive prefix; *total receives the block total.  Contains barriers.
template <int BLOCK, typename T>
__device__ __forceinline__ T block_exclusive_sum(T v, T *scratch, T *total) {
    constexpr int NW = BLOCK / WAVE;
    const int w = threadIdx.x / WAVE;
    T inc = wave_inclusive_sum(v);
    if (__lane_id() == WAVE - 1) scratch[w] = inc;
    __syncthreads();
    if (threadIdx.x == 0) {
        T run = 0;
#pragma unroll
        for (int i = 0; i < NW; ++i) {
            T t = scratch[i];
            scratch[i] = run;
            run += t;
        }
        scratch[NW] = run;
    }
    __syncthreads();
    T res = scratch[w] + inc - v;
    *total = scratch[NW];
    __syncthreads();
    return res;
}

// Block-wide exclusive max with identity `ident`.
template <int BLOCK, typename T>
__device__ __forceinline__ T block_exclusive_max(T v, T ident, T *scratch, T *total) {
    constexpr int NW = BLOCK / WAVE;
    const int w = threadIdx.x / WAVE;
    T inc = wave_inclusive_max(v);
    T exc = wave_shr1(inc, ident);
    if (__lane_id() == WAVE - 1) scratch[w] = inc;
    __syncthreads();
    if (threadIdx.x == 0) {
        T run = ident;
#pragma unroll
        for (int i = 0; i < NW; ++i) {
            T t = scratch[i];
            scratch[i] = run;
            run = run > t ? run : t;
        }
        scratch[NW] = run;
    }
    __syncthreads();
    T pre = scratch[w];
    T res = pre > exc ? pre : exc;
    *total = scratch[NW];
    __syncthreads();
    return res;
}

// first index in [lo, hi) with a[i] >= key (a sorted ascending)
template <typename T, typename K>
__device__ __forceinline__ int64_t lower_bound(const T *a, int64_t lo, int64_t hi, K key) {
    while (lo < hi) {
        int64_t mid = lo + ((hi - lo) >> 1);
        if ((K)a[mid] < key)
            lo = mid + 1;
        else
            hi = mid;
    }
    return lo;
}
// first index in [lo, hi) with a[i] > key
template <typename T, typename K>
__device__ __forceinline__ int64_t upper_bound(const T *a, int64_t lo, int64_t hi, K key) {
    while (lo < hi) {
        int64_t mid = lo + ((hi - lo) >> 1);
        if ((K)a[mid] <= key)
            lo = mid + 1;
        else
            hi = mid;
    }
    return lo;
}

// lower bounds of N keys each among w[0, n) (w sorted ascending, in LDS) by
// binary lifting in lockstep, branch-free: a step's N reads are all issued
// (the index clamped into the window) before any is compared, so they
// overlap; past the window (b + step > n) the read is w[n - 1], and a key
// above it lifts b to n, its lower bound, where it stays.  (The guarded form, `b + step <= n && w[b + step - 1] < key`,
// compiles to a branch per read, each with its own LDS wait: 8 serial waits
// per step in k_sub_fused, 31 % of its wave time at 1e9 rows.)
template <int N, typename K>
__device__ __forceinline__ void lds_lower_bounds(const uint32_t *w, int n, const K (&key)[N],
                                                 int (&b)[N]) {
#pragma unroll
    for (int k = 0; k < N; ++k) b[k] = 0;
    for (int step = n > 0 ? (1 << (31 - __clz(n))) : 0; step > 0; step >>= 1) {
        uint32_t v[N];
#pragma unroll
        for (int k = 0; k < N; ++k) v[k] = w[min(b[k] + step, n) - 1];
#pragma unroll
        for (int k = 0; k < N; ++k) b[k] = min(b[k] + ((K)v[k] < key[k] ? step : 0), n);
    }
}

// 65-ary search by one wave: every step probes 64 evenly spaced rows at once
// and keeps the gap the key falls in, so a lower_bound over 1e8 rows takes
// 5 dependent memory round trips instead of 27.  Wave-uniform result.
__device__ __forceinline__ int64_t wave_lower_bound(const uint32_t *__restrict__ a, int64_t n,
                                                    int64_t key) {
    int64_t lo = 0, hi = n;  // answer in [lo, hi]
    const int lane = __lane_id();
    while (hi - lo > 64) {
        const int64_t step = (hi - lo + 64) / 65;  // probes lo + step*(l+1) - 1, l < 64
        const int64_t idx = lo + step * (lane + 1) - 1;
        const bool less = idx < hi && (int64_t)a[idx] < key;
        const uint64_t m = __ballot(less);
        const int c = __popcll(m);  // probes below key (a prefix, a is sorted)
        const int64_t nlo = c == 0 ? lo : lo + step * c;
        const int64_t nhi = c == 64 ? hi : min(hi, lo + step * (c + 1) - 1);
        lo = nlo;
        hi = nhi;
    }
    // final: at most 64 candidates [lo, hi)
    const int64_t idx = lo + lane;
    const bool less = idx < hi && (int64_t)a[idx] < key;
    return lo + __popcll(__ballot(less));
}

// Decoupled look-back over per-tile status words (u64: 2 flag bits + a
// 62-bit value), tiles numbered in ticket order (an atomic counter read at
// the start of each workgroup).  A tile publishes its aggregate (ST_AGG |
// value), looks back, then publishes its inclusive prefix (ST_INC | value).
constexpr uint64_t ST_AGG = 1ull << 62;  // tile aggregate published
constexpr uint64_t ST_INC = 2ull << 62;  // inclusive prefix published
constexpr uint64_t ST_VAL = (1ull << 62) - 1;

__device__ __forceinline__ void st_publish(uint64_t *p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t st_poll(const uint64_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Decoupled look-back by one wave: combine (max or sum) of the values of
// every tile before `tile`.  Lane l inspects tile base - l; a window of 64
// predecessors is consumed once all of them have published at least an
// aggregate, and the walk stops at the nearest inclusive prefix.  Tiles are
// numbered in ticket order, so every predecessor is already running and
// publishes without waiting on this tile: the spin always ends.
template <bool MAX>
__device__ __forceinline__ uint64_t lookback(const uint64_t *st, int64_t tile) {
    const int lane = __lane_id();
    uint64_t acc = 0;
    for (int64_t base = tile - 1; base >= 0; base -= 64) {
        const int64_t i = base - lane;
        uint64_t v = ST_INC;  // before tile 0: inclusive identity
        if (i >= 0) {
            v = st_poll(st + i);
            while ((v >> 62) == 0) {
                __builtin_amdgcn_s_sleep(1);
                v = st_poll(st + i);
            }
        }
        const uint64_t inc = __ballot((v >> 62) == 2);
        uint64_t val = v & ST_VAL;
        if (inc) {
            const int first = __ffsll((unsigned long long)inc) - 1;
            if (lane > first) val = 0;
        }
        const uint64_t r = MAX ? wave_reduce_max(val) : wave_reduce_sum(val);
        acc = MAX ? (acc > r ? acc : r) : acc + r;
        if (inc) break;
    }
    return acc;
}

// a value the caller knows to be wave-uniform, moved to SGPRs so that what
// is indexed by it (kernel-argument structs, table entries) is read by
// scalar loads, outside the vector memory counter
__device__ __forceinline__ int64_t uni64(int64_t v) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)((uint64_t)v >> 32));
    return (int64_t)(((uint64_t)hi << 32) | lo);
}

// splitmix64 finaliser (shared with oracle/lime_oracle.c lo_pair_hash)
__host__ __device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
}
__host__ __device__ __forceinline__ uint64_t pair_hash(uint32_t s, uint32_t e, uint32_t a,
                                                       uint32_t b) {
    uint64_t x = ((uint64_t)s << 32) | e;
    uint64_t y = ((uint64_t)a << 32) | b;
    return mix64(x ^ mix64(y));
}

}  // namespace dev
}  // namespace lime
#endif

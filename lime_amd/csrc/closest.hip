// closest.hip -- SingleClosest (lime-core Closest.scala:34-214, the CLI's
// `closest`, cli/Closest.scala:45-58) on the device, exactly as the
// reference's sweep computes it on one partition: left rows in RegionOrdering,
// a right pointer j advanced while advanceCacheCondition holds (each success
// sets the mutable currentClosest C to the candidate, so C = R[j-1]), a cache
// R[p, j) trimmed at its head by pruneCacheCondition (with SetTheory.scala
// :131-141's "index <= 0 -> trim nothing"), and processHits emitting every
// cached R at the same unstrandedDistance from L as C.
//
// The sweep is sequential; its state (j, p) is recovered here in parallel.
//
// Right pointer.  Within contig c (rights [r0, r1)), for left L the advance
// stops at position k in (r0, r1) iff dist(L, R[k]) > dist(L, R[k-1]).  With
// A(L) = first right starting at or after L.end, a stop below A(L) is a "jag"
// (R[k-1].end > R[k].end) whose R[k] lies wholly before L -- and stays before
// every later left, so once the pointer halts at one it never moves again on
// this contig.  Without such a halt the pointer after left i is
//     U_i = max_{i' <= i} N_{i'},
// N = the left's own stop at or after A (A itself when dist grows there, else
// the next distinct start).  So: N per left, one prefix max, then per left
// "is there an active jag in [U_{i-1}, A_i)?"; the first such left fixes the
// contig's stuck position.  The pointer crosses into the next left contig only
// if it reached r1 and no rights lie on contigs in between; otherwise the
// sweep is stuck on another contig for good and emits nothing more
// (contig liveness, a host pass over <= n_contigs entries).
//
// Cache head.  p_i = first k in [p_{i-1}, j_i) with dist(L_i, R[k]) <= D_i
// (D_i = dist(L_i, C)), else p_{i-1}.  The map x -> F_i(x) is monotone, so
// starting from the prefix max of F_i(r0) (a lower bound) and applying
// p_i <- F_i(p_{i-1}) for all lefts at once converges upwards to the exact
// chain; on the inputs tried it is exact after the first round, which the
// next round confirms.  F_i(r0) is one binary search of the right set's
// prefix max of ends; F_i(x) scans the ends with a two-level block-max skip.
//
// Output per left: every k in [p_i, j_i) with dist(L_i, R[k]) == D_i, in
// index order (= cache order), as (L, (L.row, R.row)) records.
#include <algorithm>

#include "common.hpp"

namespace lime {

int sort_set_global(lime_ctx *ctx, lime_set *set, const uint32_t *d_gs, const uint32_t *d_ge,
                    const uint32_t *d_row, const uint32_t *d_len);

struct ClosestPlan {
    lime_ctx *ctx = nullptr;
    const lime_set *A = nullptr, *B = nullptr;
    int64_t nl = 0;
    uint32_t *jp = nullptr;    // per left: right pointer j after the left
    uint32_t *pp = nullptr;    // per left: cache head p after the left
    uint32_t *dd = nullptr;    // per left: D (0xffffffff: no output)
    uint64_t *off = nullptr;   // per left: exclusive output offsets
    uint32_t *rb = nullptr;    // n_contigs + 1 right contig bounds
    uint32_t *aa = nullptr;    // per left: A, the first right starting at or after its end
    uint32_t *eg = nullptr;    // the rights' ends, ascending (end index) ...
    uint32_t *ek = nullptr;    // ... and the right index of each, ascending among equal ends
    uint32_t *deg = nullptr;   // directory of eg
    int64_t nb = 0;            // directory entries - 1
    int64_t total = 0;
    int rounds = 0;            // cache-head rounds run (Jacobi, capped)
    bool sequential = false;   // the in-order recursion finished the chain
    bool alive_in = true;      // the sweep enters this space live (chained spaces)
    bool alive_out = true;     // ... and leaves it live
};

namespace {

constexpr int CB = 256;
constexpr int MAX_ROUNDS = 32;  // Jacobi cache-head rounds before the in-order recursion
constexpr uint32_t NONE = 0xffffffffu;
constexpr int OCAP = 4096;  // contig offsets staged in LDS
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int contig_of(const uint32_t *off, int32_t nc, uint32_t g) {
    int lo = 0, hi = nc;  // largest c with off[c] <= g
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (off[mid] <= g)
            lo = mid;
        else
            hi = mid;
    }
    return lo;
}

// ADAM unstrandedDistance for rows of one contig: 0 if covering, else gap + 1
__device__ __forceinline__ uint32_t udist(uint32_t ls, uint32_t le, uint32_t rs, uint32_t re) {
    if (le > rs && ls < re) return 0u;
    return rs >= le ? rs - le + 1u : ls - re + 1u;
}

struct Rights {
    const uint32_t *gs, *ge, *row, *pmax;
    const uint32_t *jag;            // per right: end if a jag, else NONE
    const uint32_t *jmin1, *jmin2;  // block minima of jag (64, 4096 rows)
    const uint32_t *gmax1, *gmax2;  // block maxima of ge
    int64_t n;
    const uint32_t *dgs, *dpm;      // directories of gs and pmax
    int64_t nb;
};

struct Lefts {
    const uint32_t *gs, *ge, *row;
    int64_t n;
    const uint32_t *off;  // space offsets
    int32_t nc;
    const uint32_t *rb;   // right contig bounds
};

// first k in [lo, hi) with v[k] <= t (MIN) / v[k] >= t (!MIN), hi if none;
// whole 64- and 4096-row blocks are skipped by their minimum / maximum
template <bool MIN>
__device__ __forceinline__ int64_t first_hit(const uint32_t *v, const uint32_t *l1,
                                             const uint32_t *l2, int64_t lo, int64_t hi,
                                             uint64_t t) {
    auto hit = [&](uint32_t x) { return MIN ? (uint64_t)x <= t : (uint64_t)x >= t; };
    int64_t k = lo;
    while (k < hi && (k & 63)) {
        if (hit(v[k])) return k;
        ++k;
    }
    while (k < hi) {
        if (!(k & 4095) && !hit(l2[k >> 12])) {
            k += 4096;
            continue;
        }
        if (!hit(l1[k >> 6])) {
            k += 64;
            continue;
        }
        const int64_t e = min(k + 64, hi);
        for (; k < e; ++k)
            if (hit(v[k])) return k;
    }
    return hi;
}

// Coarse directory of a sorted u32 array: dir[b] = first index with
// a[idx] >= b << DSH.  A lower_bound then searches only [dir[b], dir[b+1]]
// (~130 rows at C2's density) instead of the whole array: 8 dependent loads
// instead of 27.
constexpr int DSH = 12;

struct Dir {
    const uint32_t *a, *d;
    int64_t n, nb;  // array length, directory entries - 1
};

// first index in [lo, hi) with a[i] >= key (hi if none)
__device__ __forceinline__ int64_t dlb(const Dir &D, int64_t lo, int64_t hi, uint64_t key) {
    const uint64_t b = key >> DSH;
    int64_t g;
    if (b >= (uint64_t)D.nb)
        g = D.n;
    else
        g = dev::lower_bound(D.a, (int64_t)D.d[b], (int64_t)D.d[b + 1], key);
    return min(max(g, lo), hi);
}

__global__ __launch_bounds__(CB) void k_dir(const uint32_t *__restrict__ a, int64_t n,
                                            uint32_t *__restrict__ d, int64_t nb) {
    const int64_t b = (int64_t)blockIdx.x * CB + threadIdx.x;
    if (b > nb) return;
    d[b] = (uint32_t)dev::lower_bound(a, 0, n, (uint64_t)b << DSH);
}

__global__ __launch_bounds__(CB) void k_bounds(const uint32_t *__restrict__ gs, int64_t n,
                                               const uint32_t *__restrict__ off, int32_t nc,
                                               uint32_t *__restrict__ rb) {
    const int c = blockIdx.x * CB + threadIdx.x;
    if (c > nc) return;
    rb[c] = (uint32_t)dev::lower_bound(gs, 0, n, off[c]);
}

__global__ __launch_bounds__(CB) void k_iota(uint32_t *__restrict__ v, int64_t n) {
    const int64_t k = (int64_t)blockIdx.x * CB + threadIdx.x;
    if (k < n) v[k] = (uint32_t)k;
}

// U at the last left of each contig with lefts
__global__ __launch_bounds__(CB) void k_last(const uint32_t *__restrict__ lb,
                                             const uint32_t *__restrict__ U, int32_t nc,
                                             uint32_t *__restrict__ last) {
    const int c = blockIdx.x * CB + threadIdx.x;
    if (c >= nc) return;
    last[c] = lb[c + 1] > lb[c] ? U[lb[c + 1] - 1] : 0u;
}

// jag[k] = R[k].end when R[k-1] (same contig) ends later, else NONE
__global__ __launch_bounds__(CB) void k_jags(const uint32_t *__restrict__ gs,
                                             const uint32_t *__restrict__ ge, int64_t n,
                                             const uint32_t *__restrict__ off, int32_t nc,
                                             uint32_t *__restrict__ jag) {
    __shared__ uint32_t s_off[OCAP];
    if (nc + 1 <= OCAP)
        for (int i = threadIdx.x; i <= nc; i += CB) s_off[i] = off[i];
    __syncthreads();
    const uint32_t *o = nc + 1 <= OCAP ? s_off : off;
    const int64_t k = (int64_t)blockIdx.x * CB + threadIdx.x;
    if (k >= n) return;
    uint32_t v = NONE;
    if (k > 0) {
        const int c = contig_of(o, nc, gs[k]);
        if (gs[k - 1] >= o[c] && ge[k - 1] > ge[k]) v = ge[k];
    }
    jag[k] = v;
}

// one block-min / block-max level: 64 inputs per output, one wave each
template <bool MIN>
__global__ __launch_bounds__(CB) void k_level(const uint32_t *__restrict__ v, int64_t n,
                                              uint32_t *__restrict__ out, int64_t m) {
    const int64_t b = (int64_t)blockIdx.x * (CB / 64) + threadIdx.x / 64;
    if (b >= m) return;
    const int64_t i = b * 64 + dev::lane_id();
    uint32_t x = i < n ? v[i] : (MIN ? NONE : 0u);
    x = MIN ? dev::wave_reduce_min(x) : dev::wave_reduce_max(x);
    if (dev::lane_id() == 0) out[b] = x;
}

// per left: A (first right starting at or after L.end) and N (the left's
// own stop at or after A)
__global__ __launch_bounds__(CB) void k_stops(Lefts L, Rights R, uint32_t *__restrict__ Aout,
                                              uint32_t *__restrict__ Nout) {
    __shared__ uint32_t s_off[OCAP];
    if (L.nc + 1 <= OCAP)
        for (int i = threadIdx.x; i <= L.nc; i += CB) s_off[i] = L.off[i];
    __syncthreads();
    const uint32_t *o = L.nc + 1 <= OCAP ? s_off : L.off;
    const int64_t i = (int64_t)blockIdx.x * CB + threadIdx.x;
    if (i >= L.n) return;
    const uint32_t ls = L.gs[i], le = L.ge[i];
    const int c = contig_of(o, L.nc, ls);
    const int64_t lo = L.rb[c], hi = L.rb[c + 1];
    const Dir G{R.gs, R.dgs, R.n, R.nb};
    const int64_t a = dlb(G, lo, hi, le);
    int64_t nn;
    if (a == hi)
        nn = hi;
    else if (a > lo && udist(ls, le, R.gs[a - 1], R.ge[a - 1]) < udist(ls, le, R.gs[a], R.ge[a]))
        nn = a;
    else
        nn = dlb(G, a, hi, (uint64_t)R.gs[a] + 1);
    Aout[i] = (uint32_t)a;
    Nout[i] = (uint32_t)nn;
}

// per left: the first active jag in [max(U_{i-1}, r0 + 1), A_i); the
// smallest such left of each contig (and its jag) is kept per contig
__global__ __launch_bounds__(CB) void k_stuck(Lefts L, Rights R, const uint32_t *__restrict__ A,
                                              const uint32_t *__restrict__ U,
                                              unsigned long long *__restrict__ stuck) {
    __shared__ uint32_t s_off[OCAP];
    if (L.nc + 1 <= OCAP)
        for (int i = threadIdx.x; i <= L.nc; i += CB) s_off[i] = L.off[i];
    __syncthreads();
    const uint32_t *o = L.nc + 1 <= OCAP ? s_off : L.off;
    const int64_t i = (int64_t)blockIdx.x * CB + threadIdx.x;
    if (i >= L.n) return;
    const uint32_t ls = L.gs[i];
    const int c = contig_of(o, L.nc, ls);
    const int64_t r0 = L.rb[c];
    const int64_t lo = max((int64_t)(i > 0 ? U[i - 1] : 0u), r0 + 1);
    const int64_t a = A[i];
    if (lo >= a) return;
    const int64_t k = first_hit<true>(R.jag, R.jmin1, R.jmin2, lo, a, ls);
    if (k < a) atomicMin(&stuck[c], ((unsigned long long)i << 32) | (unsigned long long)k);
}

struct State {
    const uint32_t *A, *U;
    const unsigned long long *stuck;
    const uint8_t *live;
};

__device__ __forceinline__ uint32_t pointer_of(const State &s, int c, int64_t i) {
    const unsigned long long st = s.stuck[c];
    if (st != ~0ull && (uint64_t)i >= (st >> 32)) return (uint32_t)(st & 0xffffffffu);
    return s.U[i];
}

// F_i(x): first k in [x, j) with dist(L, R[k]) <= D, else x.  Below A that
// is R.end >= L.start + 1 - D; from A on it is R.start <= L.end + D - 1,
// which holds for a prefix of [A, j) (starts ascend), so only A is tested.
__device__ __forceinline__ int64_t near_from(const Rights &R, uint32_t ls, uint32_t le,
                                             uint32_t D, int64_t a, int64_t j, int64_t x,
                                             bool fresh) {
    const int64_t T = (int64_t)ls + 1 - (int64_t)D;
    const int64_t hi = min(a, j);
    if (x < hi) {
        int64_t k;
        if (T <= 0)
            k = x;
        else if (fresh)  // prefix max of ends: exact from the contig start
            k = dlb(Dir{R.pmax, R.dpm, R.n, R.nb}, x, hi, (uint64_t)T);
        else
            k = first_hit<false>(R.ge, R.gmax1, R.gmax2, x, hi, (uint64_t)T);
        if (k < hi) return k;
    }
    const int64_t k = max(x, a);
    if (k < j && (int64_t)R.gs[k] <= (int64_t)le + (int64_t)D - 1) return k;
    return x;
}

// per left: j, D and the fresh cache head F_i(r0)
__global__ __launch_bounds__(CB) void k_fresh(Lefts L, Rights R, State s,
                                              uint32_t *__restrict__ jp, uint32_t *__restrict__ dd,
                                              uint32_t *__restrict__ P) {
    __shared__ uint32_t s_off[OCAP];
    if (L.nc + 1 <= OCAP)
        for (int i = threadIdx.x; i <= L.nc; i += CB) s_off[i] = L.off[i];
    __syncthreads();
    const uint32_t *o = L.nc + 1 <= OCAP ? s_off : L.off;
    const int64_t i = (int64_t)blockIdx.x * CB + threadIdx.x;
    if (i >= L.n) return;
    const uint32_t ls = L.gs[i], le = L.ge[i];
    const int c = contig_of(o, L.nc, ls);
    const int64_t r0 = L.rb[c];
    const int64_t j = pointer_of(s, c, i);
    jp[i] = (uint32_t)j;
    if (!s.live[c] || j <= r0) {
        dd[i] = NONE;
        P[i] = (uint32_t)r0;
        return;
    }
    const uint32_t D = udist(ls, le, R.gs[j - 1], R.ge[j - 1]);
    dd[i] = D;
    P[i] = (uint32_t)near_from(R, ls, le, D, s.A[i], j, r0, true);
}

// one round of p_i <- max(p_i, F_i(p_{i-1}))
__global__ __launch_bounds__(CB) void k_prune_round(Lefts L, Rights R, State s,
                                                    const uint32_t *__restrict__ jp,
                                                    const uint32_t *__restrict__ dd,
                                                    const uint32_t *__restrict__ pin,
                                                    uint32_t *__restrict__ pout,
                                                    unsigned int *__restrict__ changed) {
    __shared__ uint32_t s_off[OCAP];
    if (L.nc + 1 <= OCAP)
        for (int i = threadIdx.x; i <= L.nc; i += CB) s_off[i] = L.off[i];
    __syncthreads();
    const uint32_t *o = L.nc + 1 <= OCAP ? s_off : L.off;
    const int64_t i = (int64_t)blockIdx.x * CB + threadIdx.x;
    if (i >= L.n) return;
    const uint32_t cur = pin[i];
    uint32_t nv = cur;
    const uint32_t D = dd[i];
    if (D != NONE) {
        const uint32_t ls = L.gs[i], le = L.ge[i];
        const int c = contig_of(o, L.nc, ls);
        const int64_t r0 = L.rb[c];
        const int64_t x = max((int64_t)(i > 0 ? pin[i - 1] : 0u), r0);
        const int64_t f = near_from(R, ls, le, D, s.A[i], jp[i], x, false);
        nv = (uint32_t)max((int64_t)cur, f);
    }
    pout[i] = nv;
    if (nv != cur) atomicOr(changed, 1u);
}

// The same fixed point in order, one thread per contig: F_i is monotone in
// its argument (the first hit at or after x), so the recursion p_i =
// max(p_i, F_i(p_{i-1})) taken left to right reaches the rounds' least fixed
// point.  Used past the round cap: an adversarial chain needs O(n) rounds of
// the full grid, the recursion O(n log n) work.  A contig's first left starts
// from r0 (every earlier contig's heads lie below it), so contigs are
// independent.
__global__ __launch_bounds__(CB) void k_seq_prune(Lefts L, Rights R, State s,
                                                  const uint32_t *__restrict__ lb,
                                                  const uint32_t *__restrict__ jp,
                                                  const uint32_t *__restrict__ dd,
                                                  uint32_t *__restrict__ p) {
    const int c = blockIdx.x * CB + threadIdx.x;
    if (c >= L.nc) return;
    const int64_t r0 = L.rb[c], i0 = lb[c], i1 = lb[c + 1];
    int64_t prev = r0;
    for (int64_t i = i0; i < i1; ++i) {
        int64_t v = p[i];
        const uint32_t D = dd[i];
        if (D != NONE) {
            const int64_t f = near_from(R, L.gs[i], L.ge[i], D, s.A[i], jp[i], max(prev, r0),
                                        false);
            v = max(v, f);
            p[i] = (uint32_t)v;
        }
        prev = v;
    }
}

// SingleClosestSingleOverlap (Closest.scala:216-268): its advance also stops
// inside the covering zone where the covered length drops, and its prune
// drops covering rows shorter than a covering current closest.  Those stops
// depend on each left, so its (j, p) chain is run in order -- one wave per
// contig, the wave testing 64 candidates per step -- and the output pass is
// the shared one.  (Used by the reference's suite only; its CLI runs
// SingleClosest.)
__device__ __forceinline__ bool covers(uint32_t ls, uint32_t le, uint32_t rs, uint32_t re) {
    return le > rs && ls < re;
}
__device__ __forceinline__ uint32_t cover_len(uint32_t ls, uint32_t le, uint32_t rs, uint32_t re) {
    return min(le, re) - max(ls, rs);
}

__global__ __launch_bounds__(64) void k_seq_single(Lefts L, Rights R,
                                                   const uint32_t *__restrict__ lb,
                                                   uint32_t *__restrict__ jp,
                                                   uint32_t *__restrict__ pp,
                                                   uint32_t *__restrict__ dd) {
    const int c = blockIdx.x;
    const int lane = threadIdx.x;
    const int64_t i0 = lb[c], i1 = lb[c + 1];
    const int64_t r0 = L.rb[c], r1 = L.rb[c + 1];
    int64_t j = r0, p = r0;
    for (int64_t i = i0; i < i1; ++i) {
        const uint32_t ls = L.gs[i], le = L.ge[i];
        // advanceCache (:251-267): C = R[k-1]; the contig's first row always
        // advances (the current closest lies on another contig)
        for (;;) {
            const int64_t k = j + lane;
            bool stop = k >= r1;
            if (!stop && k > r0) {
                const uint32_t cs = R.gs[k], ce = R.ge[k], ps = R.gs[k - 1], pe = R.ge[k - 1];
                bool adv;
                if (covers(ls, le, cs, ce))
                    adv = !covers(ls, le, ps, pe) ||
                          cover_len(ls, le, cs, ce) >= cover_len(ls, le, ps, pe);
                else
                    adv = udist(ls, le, cs, ce) <= udist(ls, le, ps, pe);
                stop = !adv;
            }
            const uint64_t b = __ballot(stop);
            if (b) {
                j += __builtin_ctzll(b);
                break;
            }
            j += 64;
        }
        // pruneCache (:230-241) with SetTheory.scala:131-141's index rule
        uint32_t D = NONE;
        if (j > r0) {
            const uint32_t Cs = R.gs[j - 1], Ce = R.ge[j - 1];
            D = udist(ls, le, Cs, Ce);
            const bool cc = covers(ls, le, Cs, Ce);
            const uint32_t cbC = cc ? cover_len(ls, le, Cs, Ce) : NONE;
            for (int64_t q = p; q < j; q += 64) {
                const int64_t k = q + lane;
                bool keep = false;
                if (k < j) {
                    const uint32_t rs = R.gs[k], re = R.ge[k];
                    const bool cv = covers(ls, le, rs, re);
                    keep = !((cv && cover_len(ls, le, rs, re) < cbC) || udist(ls, le, rs, re) > D);
                }
                const uint64_t b = __ballot(keep);
                if (b) {
                    p = q + __builtin_ctzll(b);
                    break;
                }
            }
        }
        if (lane == 0) {
            jp[i] = (uint32_t)j;
            pp[i] = (uint32_t)p;
            dd[i] = D;
        }
    }
}

// lefts of contigs the sweep never enters: no output
__global__ __launch_bounds__(CB) void k_kill(Lefts L, const uint8_t *__restrict__ live,
                                             uint32_t *__restrict__ dd) {
    __shared__ uint32_t s_off[OCAP];
    if (L.nc + 1 <= OCAP)
        for (int i = threadIdx.x; i <= L.nc; i += CB) s_off[i] = L.off[i];
    __syncthreads();
    const uint32_t *o = L.nc + 1 <= OCAP ? s_off : L.off;
    const int64_t i = (int64_t)blockIdx.x * CB + threadIdx.x;
    if (i >= L.n) return;
    if (!live[contig_of(o, L.nc, L.gs[i])]) dd[i] = NONE;
}

// Output pass.  A match is k in [p, j) with dist(L, R[k]) == D.
//  D > 0: below A that means R[k].end == L.start + 1 - D exactly, above A
//    R[k].start == L.end + D - 1 exactly: one run of the end index (rights by
//    end, index ascending) and one run of the starts, each cut to its index
//    range by binary search -- no scan.  Before-side matches (k < A) precede
//    after-side ones, so index order is kept.
//  D == 0 (L covered by the current closest): the covering rights of
//    [p, min(A, j)); one wave per 64 consecutive lefts tests 64 candidates at
//    once (coalesced loads), so matches come out as contiguous runs.
// Matches are counted (SCAN_COUNT), written as 16-B records at their output
// offsets (SCAN_FILL, only those inside [first, first + count)) or hashed
// (SCAN_SUM).
enum { SCAN_COUNT = 0, SCAN_FILL = 1, SCAN_SUM = 2 };
constexpr int SWIN = 2048;  // rights staged per block for the covering scan (24 KiB)

struct EndIndex {
    const uint32_t *eg, *ek;  // ends ascending, right index ascending among equal ends
    const uint32_t *aa;       // per left A
    int64_t n;
    const uint32_t *deg;      // directory of eg
    int64_t nb;
};

template <int MODE>
__global__ __launch_bounds__(CB) void k_scan(Lefts L, Rights R, EndIndex E,
                                             const uint32_t *__restrict__ jp,
                                             const uint32_t *__restrict__ pp,
                                             const uint32_t *__restrict__ dd,
                                             const uint64_t *__restrict__ off, int64_t first,
                                             int64_t count, uint64_t *__restrict__ cnt,
                                             lime_pair *__restrict__ out,
                                             unsigned long long *__restrict__ ck) {
    __shared__ uint32_t s_off[OCAP];
    // the block's covering-candidate window of rights [min p, max min(j, A)):
    // consecutive lefts share most of their candidates (each right is tested
    // by ~every left it covers, ~160 at C2's depth), so the count pass loads
    // the window once into LDS instead of re-reading it from L2 per left
    // (count pass only: the fill is store-bound and keeps its occupancy)
    constexpr bool USEWIN = MODE == SCAN_COUNT;
    __shared__ uint32_t w_gs[USEWIN ? SWIN : 1], w_ge[USEWIN ? SWIN : 1];
    __shared__ uint32_t s_lo[CB / 64], s_hi[CB / 64];
    if (L.nc + 1 <= OCAP)
        for (int i = threadIdx.x; i <= L.nc; i += CB) s_off[i] = L.off[i];
    const uint32_t *o = L.nc + 1 <= OCAP ? s_off : L.off;
    const int lane = dev::lane_id();
    const int64_t i = ((int64_t)blockIdx.x * (CB / 64) + threadIdx.x / 64) * 64 + lane;
    if (USEWIN) {
        uint32_t lo = 0xffffffffu, hi = 0;
        if (i < L.n && dd[i] == 0u) {
            lo = pp[i];
            hi = min(jp[i], E.aa[i]);
        }
        lo = dev::wave_reduce_min(lo);
        hi = dev::wave_reduce_max(hi);
        if (lane == 0) {
            s_lo[threadIdx.x / 64] = lo;
            s_hi[threadIdx.x / 64] = hi;
        }
    }
    __syncthreads();
    uint32_t wlo = 0xffffffffu, whi = 0;
    if (USEWIN)
#pragma unroll
        for (int w = 0; w < CB / 64; ++w) {
            wlo = min(wlo, s_lo[w]);
            whi = max(whi, s_hi[w]);
        }
    const bool win = USEWIN && whi > wlo && whi - wlo <= (uint32_t)SWIN;
    if (win)
        for (uint32_t k = threadIdx.x; k < whi - wlo; k += CB) {
            w_gs[k] = R.gs[wlo + k];
            w_ge[k] = R.ge[wlo + k];
        }
    __syncthreads();
    uint32_t ls = 0, le = 0, D = NONE, p = 0, j = 0, s0 = 0, e0 = 0, ar = 0;
    uint64_t pos0 = 0;
    bool valid = i < L.n && dd[i] != NONE;
    if (valid) {
        ls = L.gs[i];
        le = L.ge[i];
        D = dd[i];
        p = pp[i];
        j = jp[i];
        if (MODE != SCAN_COUNT) {
            const int c = contig_of(o, L.nc, ls);
            s0 = ls - o[c];
            e0 = le - o[c];
            ar = L.row[i];
            pos0 = off[i];
            if (MODE == SCAN_FILL)
                valid = off[i + 1] > (uint64_t)first && pos0 < (uint64_t)(first + count);
        }
    }
    uint64_t mine = 0, hs = 0, hx = 0;
    uint32_t a = 0;
    if (valid) a = E.aa[i];
    if (valid && D > 0) {
        // before-side run: rights ending exactly at T with index in [p, min(A, j))
        uint64_t pos = pos0;
        auto emit = [&](int64_t k) {
            if (MODE == SCAN_FILL && (int64_t)pos >= first && (int64_t)pos < first + count) {
                u32x4 v = {s0, e0, ar, R.row[k]};
                *reinterpret_cast<u32x4 *>(out + (pos - first)) = v;
            }
            if (MODE == SCAN_SUM) {
                const uint64_t h = dev::pair_hash(s0, e0, ar, R.row[k]);
                hs += h;
                hx ^= h;
            }
            ++pos;
            ++mine;
        };
        const int64_t T = (int64_t)ls + 1 - (int64_t)D;
        const int64_t hb = min((int64_t)a, (int64_t)j);
        if (T >= 0 && (int64_t)p < hb) {
            const Dir ED{E.eg, E.deg, E.n, E.nb};
            const int64_t e0r = dlb(ED, 0, E.n, (uint64_t)T);
            const int64_t e1r = dlb(ED, e0r, E.n, (uint64_t)T + 1);
            for (int64_t e = dev::lower_bound(E.ek, e0r, e1r, p); e < e1r && (int64_t)E.ek[e] < hb;
                 ++e)
                emit(E.ek[e]);
        }
        // after-side run: rights starting exactly at V with index in [max(p, A), j)
        const int64_t V = (int64_t)le + (int64_t)D - 1;
        const int64_t lo = max((int64_t)p, (int64_t)a);
        if (V <= (int64_t)NONE && lo < (int64_t)j)
            for (int64_t k = dev::lower_bound(R.gs, lo, (int64_t)j, (uint64_t)V);
                 k < (int64_t)j && R.gs[k] == (uint32_t)V; ++k)
                emit(k);
    }
    const uint64_t below = dev::lanemask_lt();
    for (uint64_t todo = __ballot(valid && D == 0); todo; todo &= todo - 1) {
        const int l = __builtin_ctzll(todo);
        const uint32_t bls = __shfl(ls, l), ble = __shfl(le, l), bD = __shfl(D, l);
        const uint32_t bj = min(__shfl(j, l), __shfl(a, l));  // covering rights lie below A
        uint32_t bs0 = 0, be0 = 0, bar = 0;
        uint64_t pos = 0;
        if (MODE != SCAN_COUNT) {
            bs0 = __shfl(s0, l);
            be0 = __shfl(e0, l);
            bar = __shfl(ar, l);
            pos = __shfl(pos0, l);
        }
        uint64_t total = 0;
        // software-pipelined: the next chunk's coordinates and payload rows
        // are loaded while this chunk is tested and stored
        int64_t k0 = __shfl(p, l);
        uint32_t cs = 0, ce = 0, cr = 0;
        auto fetch = [&](int64_t kk, uint32_t &fs, uint32_t &fe, uint32_t &fr) {
            if (kk < (int64_t)bj) {
                if (win) {  // (every covering candidate of the block lies in the window)
                    fs = w_gs[kk - wlo];
                    fe = w_ge[kk - wlo];
                } else {
                    fs = R.gs[kk];
                    fe = R.ge[kk];
                    if (MODE != SCAN_COUNT) fr = R.row[kk];
                }
            }
        };
        fetch(k0 + lane, cs, ce, cr);
        for (; k0 < (int64_t)bj; k0 += 64) {
            uint32_t ns = 0, ne = 0, nr = 0;
            fetch(k0 + 64 + lane, ns, ne, nr);
            const bool m = k0 + lane < (int64_t)bj && udist(bls, ble, cs, ce) == bD;
            const uint64_t bm = __ballot(m);
            if (MODE == SCAN_FILL && m) {
                const int64_t idx = (int64_t)(pos + __popcll(bm & below)) - first;
                if (idx >= 0 && idx < count) {
                    u32x4 v = {bs0, be0, bar, cr};
                    *reinterpret_cast<u32x4 *>(out + idx) = v;
                }
            }
            if (MODE == SCAN_SUM && m) {
                const uint64_t h = dev::pair_hash(bs0, be0, bar, cr);
                hs += h;
                hx ^= h;
            }
            pos += __popcll(bm);
            total += __popcll(bm);
            cs = ns;
            ce = ne;
            cr = nr;
        }
        if (lane == l) mine = total;
    }
    if (MODE == SCAN_COUNT && i < L.n) cnt[i] = valid ? mine : 0;
    if (MODE == SCAN_SUM) {
        hs = dev::wave_reduce_sum(hs);
        hx = dev::wave_reduce_xor(hx);
        if (lane == 0) {
            atomicAdd(&ck[0], (unsigned long long)hs);
            atomicXor(&ck[1], (unsigned long long)hx);
        }
    }
}

}  // namespace

void closest_free(ClosestPlan *pl) {
    if (!pl) return;
    lime_ctx *ctx = pl->ctx;
    release(ctx, pl->jp);
    release(ctx, pl->pp);
    release(ctx, pl->dd);
    release(ctx, pl->off);
    release(ctx, pl->rb);
    release(ctx, pl->aa);
    release(ctx, pl->eg);
    release(ctx, pl->ek);
    release(ctx, pl->deg);
    delete pl;
}

int64_t closest_total(const ClosestPlan *pl) { return pl->total; }
int closest_rounds(const ClosestPlan *pl, bool *sequential) {
    if (sequential) *sequential = pl->sequential;
    return pl->rounds;
}

namespace {

// Scratch buffers of one plan build, returned to the pool however it ends.
struct Scratch {
    lime_ctx *ctx;
    std::vector<void *> held;
    template <typename T>
    int get(T **p, size_t n) {
        LIME_TRY(alloc(ctx, p, n));
        held.push_back(*p);
        return LIME_OK;
    }
    ~Scratch() {
        for (void *q : held) ctx->pool.put(q);
    }
};

int plan_body(lime_ctx *ctx, const lime_set *A, const lime_set *B, int mode, ClosestPlan *pl) {
    const int64_t nl = A->n, nr = B->n;
    const int32_t nc = A->n_contigs;
    Scratch sc{ctx, {}};
#define CL_TRY LIME_TRY
    CL_TRY(alloc(ctx, &pl->rb, (size_t)nc + 1));
    CL_TRY(alloc(ctx, &pl->jp, (size_t)std::max<int64_t>(nl, 1)));
    CL_TRY(alloc(ctx, &pl->pp, (size_t)std::max<int64_t>(nl, 1)));
    CL_TRY(alloc(ctx, &pl->dd, (size_t)std::max<int64_t>(nl, 1)));
    CL_TRY(alloc(ctx, &pl->off, (size_t)nl + 1));
    if (nl == 0) {
        LIME_HIP(hipMemsetAsync(pl->off, 0, sizeof(uint64_t), S(ctx)));
        // no lefts: the sweep passes on only over a space without rights
        pl->alive_out = pl->alive_in && nr == 0;
        return LIME_OK;
    }
    hipLaunchKernelGGL(k_bounds, dim3(blocks_for(nc + 1, CB)), dim3(CB), 0, S(ctx), B->gs, nr,
                       B->d_off, nc, pl->rb);
    LIME_HIP(hipGetLastError());
    CL_TRY(build_prefix_max(ctx, B));
    // right-side search levels
    const int64_t m1 = (nr + 63) / 64, m2 = (m1 + 63) / 64;
    uint32_t *jag, *jmin1, *jmin2, *gmax1, *gmax2;
    CL_TRY(sc.get(&jag, (size_t)std::max<int64_t>(nr, 1)));
    CL_TRY(sc.get(&jmin1, (size_t)std::max<int64_t>(m1, 1)));
    CL_TRY(sc.get(&jmin2, (size_t)std::max<int64_t>(m2, 1)));
    CL_TRY(sc.get(&gmax1, (size_t)std::max<int64_t>(m1, 1)));
    CL_TRY(sc.get(&gmax2, (size_t)std::max<int64_t>(m2, 1)));
    if (nr > 0) {
        hipLaunchKernelGGL(k_jags, dim3(blocks_for(nr, CB)), dim3(CB), 0, S(ctx), B->gs, B->ge,
                           nr, B->d_off, nc, jag);
        hipLaunchKernelGGL(k_level<true>, dim3(blocks_for(m1, CB / 64)), dim3(CB), 0, S(ctx),
                           (const uint32_t *)jag, nr, jmin1, m1);
        hipLaunchKernelGGL(k_level<true>, dim3(blocks_for(m2, CB / 64)), dim3(CB), 0, S(ctx),
                           (const uint32_t *)jmin1, m1, jmin2, m2);
        hipLaunchKernelGGL(k_level<false>, dim3(blocks_for(m1, CB / 64)), dim3(CB), 0, S(ctx),
                           B->ge, nr, gmax1, m1);
        hipLaunchKernelGGL(k_level<false>, dim3(blocks_for(m2, CB / 64)), dim3(CB), 0, S(ctx),
                           (const uint32_t *)gmax1, m1, gmax2, m2);
        LIME_HIP(hipGetLastError());
    }
    // coarse directories of the starts and of the prefix max of ends
    pl->nb = ((int64_t)B->off[nc] >> DSH) + 1;
    uint32_t *dgs, *dpm;
    CL_TRY(sc.get(&dgs, (size_t)pl->nb + 1));
    CL_TRY(sc.get(&dpm, (size_t)pl->nb + 1));
    hipLaunchKernelGGL(k_dir, dim3(blocks_for(pl->nb + 1, CB)), dim3(CB), 0, S(ctx), B->gs, nr,
                       dgs, pl->nb);
    hipLaunchKernelGGL(k_dir, dim3(blocks_for(pl->nb + 1, CB)), dim3(CB), 0, S(ctx),
                       (const uint32_t *)B->pmax, nr, dpm, pl->nb);
    LIME_HIP(hipGetLastError());
    Rights R{B->gs, B->ge, B->row, B->pmax, jag,       jmin1, jmin2,
             gmax1, gmax2, nr,     dgs,     dpm, pl->nb};
    Lefts L{A->gs, A->ge, A->row, nl, A->d_off, nc, pl->rb};
    // right pointer: stops, prefix max, stuck positions
    uint32_t *Aa, *Nn, *U, *P, *p2;
    unsigned long long *stuck;
    uint8_t *live;
    unsigned int *changed;
    CL_TRY(alloc(ctx, &pl->aa, (size_t)nl));
    Aa = pl->aa;
    CL_TRY(sc.get(&Nn, (size_t)nl));
    CL_TRY(sc.get(&U, (size_t)nl));
    CL_TRY(sc.get(&P, (size_t)nl));
    CL_TRY(sc.get(&p2, (size_t)nl));
    CL_TRY(sc.get(&stuck, (size_t)nc));
    CL_TRY(sc.get(&live, (size_t)nc));
    CL_TRY(sc.get(&changed, 1));
    const unsigned gl = blocks_for(nl, CB);
    hipLaunchKernelGGL(k_stops, dim3(gl), dim3(CB), 0, S(ctx), L, R, Aa, Nn);
    LIME_HIP(hipGetLastError());
    LIME_HIP(hipMemsetAsync(stuck, 0xff, sizeof(unsigned long long) * (size_t)nc, S(ctx)));
    uint32_t *lbd;
    CL_TRY(sc.get(&lbd, (size_t)nc + 1));
    hipLaunchKernelGGL(k_bounds, dim3(blocks_for(nc + 1, CB)), dim3(CB), 0, S(ctx), A->gs, nl,
                       A->d_off, nc, lbd);
    LIME_HIP(hipGetLastError());
    if (mode == 0) {
        CL_TRY(prefix_max_u32(ctx, Nn, U, nl));
        hipLaunchKernelGGL(k_stuck, dim3(gl), dim3(CB), 0, S(ctx), L, R, (const uint32_t *)Aa,
                           (const uint32_t *)U, stuck);
    } else {
        // the chain in order, one wave per contig; exit pointers from jp
        hipLaunchKernelGGL(k_seq_single, dim3(nc), dim3(64), 0, S(ctx), L, R,
                           (const uint32_t *)lbd, pl->jp, pl->pp, pl->dd);
    }
    LIME_HIP(hipGetLastError());
    // contig liveness (host, <= n_contigs steps): the sweep enters the next
    // left contig only from the end of this contig's rights, and only if no
    // rights lie on the contigs in between
    {
        uint32_t *lastU;
        CL_TRY(sc.get(&lastU, (size_t)nc));
        hipLaunchKernelGGL(k_last, dim3(blocks_for(nc, CB)), dim3(CB), 0, S(ctx),
                           (const uint32_t *)lbd, (const uint32_t *)(mode == 0 ? U : pl->jp), nc,
                           lastU);
        LIME_HIP(hipGetLastError());
        std::vector<uint32_t> rb(nc + 1), lb(nc + 1), lu(nc);
        std::vector<unsigned long long> st(nc);
        CL_TRY(read_back(ctx, rb.data(), pl->rb, sizeof(uint32_t) * (nc + 1)));
        CL_TRY(read_back(ctx, lb.data(), lbd, sizeof(uint32_t) * (nc + 1)));
        CL_TRY(read_back(ctx, lu.data(), lastU, sizeof(uint32_t) * nc));
        CL_TRY(read_back(ctx, st.data(), stuck, sizeof(unsigned long long) * nc));
        std::vector<uint8_t> lv(nc, 0);
        bool alive = pl->alive_in, first = true;
        for (int32_t c = 0; c < nc; ++c) {
            if (lb[c + 1] <= lb[c]) continue;  // no lefts on c
            if (first) {  // the sweep starts at right row 0 (of this space)
                alive = alive && rb[c] == 0;
                first = false;
            }
            lv[c] = alive ? 1 : 0;
            if (!alive) continue;
            const uint64_t last = lb[c + 1] - 1;
            const uint32_t jl =
                (st[c] != ~0ull && last >= (st[c] >> 32)) ? (uint32_t)(st[c] & 0xffffffffu) : lu[c];
            // the next left contig is entered from the end of c's rights only,
            // and only if no rights lie on the contigs in between (the space's
            // end included: alive_out chains a next space of contigs)
            alive = jl == rb[c + 1];
            int32_t cn = c + 1;
            while (cn < nc && lb[cn + 1] <= lb[cn]) ++cn;
            if (alive) alive = rb[c + 1] == rb[cn];
        }
        pl->alive_out = alive;
        LIME_HIP(hipMemcpyAsync(live, lv.data(), (size_t)nc, hipMemcpyHostToDevice, S(ctx)));
        LIME_HIP(hipStreamSynchronize(S(ctx)));
    }
    // end index for the exact-distance lookups of the output pass
    CL_TRY(alloc(ctx, &pl->eg, (size_t)std::max<int64_t>(nr, 1)));
    CL_TRY(alloc(ctx, &pl->ek, (size_t)std::max<int64_t>(nr, 1)));
    if (nr > 0) {
        uint32_t *idx;
        CL_TRY(sc.get(&idx, (size_t)nr));
        hipLaunchKernelGGL(k_iota, dim3(blocks_for(nr, CB)), dim3(CB), 0, S(ctx), idx, nr);
        LIME_HIP(hipGetLastError());
        lime_set es;  // (ge, ge, k) sorted by ge; ties keep k ascending
        es.ctx = ctx;
        es.n = nr;
        es.d_off = B->d_off;
        es.n_contigs = nc;
        es.off = B->off;
        es.len = B->len;
        CL_TRY(sort_set_global(ctx, &es, B->ge, B->ge, idx, nullptr));
        release(ctx, pl->eg);
        release(ctx, pl->ek);
        pl->eg = es.gs;
        pl->ek = es.row;
        release(ctx, es.ge);
        CL_TRY(alloc(ctx, &pl->deg, (size_t)pl->nb + 1));
        hipLaunchKernelGGL(k_dir, dim3(blocks_for(pl->nb + 1, CB)), dim3(CB), 0, S(ctx),
                           (const uint32_t *)pl->eg, nr, pl->deg, pl->nb);
        LIME_HIP(hipGetLastError());
    }
    State s{Aa, U, stuck, live};
    if (mode != 0) {
        hipLaunchKernelGGL(k_kill, dim3(gl), dim3(CB), 0, S(ctx), L, (const uint8_t *)live,
                           pl->dd);
        LIME_HIP(hipGetLastError());
    } else {
        hipLaunchKernelGGL(k_fresh, dim3(gl), dim3(CB), 0, S(ctx), L, R, s, pl->jp, pl->dd, P);
        LIME_HIP(hipGetLastError());
        // cache head: prefix max of the fresh heads, then rounds to the fixed point
        CL_TRY(prefix_max_u32(ctx, P, pl->pp, nl));
    }
    // Jacobi rounds (each a full-grid pass + one read-back) up to a cap --
    // one round sufficed on every input measured -- then the in-order
    // recursion finishes the chain (k_seq_prune)
    const char *ev = getenv("LIME_CLOSEST_MAX_ROUNDS");  // (tests force the recursion)
    const int env_cap = ev ? atoi(ev) : -1;
    const int64_t cap = env_cap >= 0 ? env_cap : MAX_ROUNDS;
    uint32_t *cur = pl->pp, *nxt = p2;
    bool done = mode != 0;
    for (int64_t r = 0; !done && r < cap; ++r) {
        LIME_HIP(hipMemsetAsync(changed, 0, sizeof(unsigned int), S(ctx)));
        hipLaunchKernelGGL(k_prune_round, dim3(gl), dim3(CB), 0, S(ctx), L, R, s,
                           (const uint32_t *)pl->jp, (const uint32_t *)pl->dd,
                           (const uint32_t *)cur, nxt, changed);
        LIME_HIP(hipGetLastError());
        unsigned int ch = 0;
        LIME_TRY(read_back(ctx, &ch, changed, sizeof(ch)));
        std::swap(cur, nxt);
        ++pl->rounds;
        done = !ch;
    }
    if (cur != pl->pp)
        LIME_HIP(hipMemcpyAsync(pl->pp, cur, sizeof(uint32_t) * (size_t)nl,
                                hipMemcpyDeviceToDevice, S(ctx)));
    if (!done && nl > 0) {
        pl->sequential = true;
        hipLaunchKernelGGL(k_seq_prune, dim3(blocks_for(nc, CB)), dim3(CB), 0, S(ctx), L, R, s,
                           (const uint32_t *)lbd, (const uint32_t *)pl->jp,
                           (const uint32_t *)pl->dd, pl->pp);
        LIME_HIP(hipGetLastError());
    }
    // output counts and offsets
    uint64_t *cnt, *tot;
    CL_TRY(sc.get(&cnt, (size_t)nl));
    CL_TRY(sc.get(&tot, 1));
    const EndIndex E{pl->eg, pl->ek, pl->aa, nr, pl->deg, pl->nb};
    hipLaunchKernelGGL(k_scan<SCAN_COUNT>, dim3(gl), dim3(CB), 0, S(ctx), L, R, E,
                       (const uint32_t *)pl->jp, (const uint32_t *)pl->pp,
                       (const uint32_t *)pl->dd, (const uint64_t *)nullptr, (int64_t)0,
                       (int64_t)0, cnt, (lime_pair *)nullptr, (unsigned long long *)nullptr);
    LIME_HIP(hipGetLastError());
    CL_TRY(scan_exclusive_u64(ctx, cnt, pl->off, nl, tot));
    LIME_HIP(hipMemcpyAsync(pl->off + nl, tot, sizeof(uint64_t), hipMemcpyDeviceToDevice,
                            S(ctx)));
    uint64_t total = 0;
    LIME_TRY(read_back(ctx, &total, tot, sizeof(total)));
    pl->total = (int64_t)total;
#undef CL_TRY
    return LIME_OK;
}

}  // namespace

int closest_plan(lime_ctx *ctx, const lime_set *A, const lime_set *B, int mode, bool alive_in,
                 bool *alive_out, ClosestPlan **out) {
    if (A->n >= (int64_t)NONE || B->n >= (int64_t)NONE)
        return fail(LIME_ERR_RANGE, "closest supports fewer than 2^32 - 1 rows per set");
    ClosestPlan *pl = new ClosestPlan();
    pl->ctx = ctx;
    pl->A = A;
    pl->B = B;
    pl->nl = A->n;
    pl->alive_in = alive_in;
    const int rc = plan_body(ctx, A, B, mode, pl);
    if (rc != LIME_OK) {
        closest_free(pl);
        return rc;
    }
    if (alive_out) *alive_out = pl->alive_out;
    *out = pl;
    return LIME_OK;
}

int closest_fill(ClosestPlan *pl, int64_t first, int64_t count, lime_pair *d_out) {
    lime_ctx *ctx = pl->ctx;
    if (first < 0 || count < 0 || first + count > pl->total)
        return fail(LIME_ERR_ARG, "fill range outside the plan");
    if (count == 0 || pl->nl == 0) return LIME_OK;
    const lime_set *A = pl->A, *B = pl->B;
    Rights R{B->gs,   B->ge,   B->row, B->pmax, nullptr, nullptr, nullptr,
             nullptr, nullptr, B->n,   nullptr, nullptr, 0};
    Lefts L{A->gs, A->ge, A->row, pl->nl, A->d_off, A->n_contigs, pl->rb};
    const EndIndex E{pl->eg, pl->ek, pl->aa, B->n, pl->deg, pl->nb};
    hipLaunchKernelGGL(k_scan<SCAN_FILL>, dim3(blocks_for(pl->nl, CB)), dim3(CB), 0, S(ctx), L,
                       R, E, (const uint32_t *)pl->jp, (const uint32_t *)pl->pp,
                       (const uint32_t *)pl->dd, (const uint64_t *)pl->off, first, count,
                       (uint64_t *)nullptr, d_out, (unsigned long long *)nullptr);
    LIME_HIP(hipGetLastError());
    return LIME_OK;
}

int closest_checksum(ClosestPlan *pl, uint64_t *sum, uint64_t *xr) {
    lime_ctx *ctx = pl->ctx;
    unsigned long long *ck;
    LIME_TRY(alloc(ctx, &ck, 2));
    LIME_HIP(hipMemsetAsync(ck, 0, 2 * sizeof(unsigned long long), S(ctx)));
    if (pl->nl > 0) {
        const lime_set *A = pl->A, *B = pl->B;
        Rights R{B->gs,   B->ge,   B->row, B->pmax, nullptr, nullptr, nullptr,
                 nullptr, nullptr, B->n,   nullptr, nullptr, 0};
        Lefts L{A->gs, A->ge, A->row, pl->nl, A->d_off, A->n_contigs, pl->rb};
        const EndIndex E{pl->eg, pl->ek, pl->aa, B->n, pl->deg, pl->nb};
        hipLaunchKernelGGL(k_scan<SCAN_SUM>, dim3(blocks_for(pl->nl, CB)), dim3(CB), 0,
                           S(ctx), L, R, E, (const uint32_t *)pl->jp, (const uint32_t *)pl->pp,
                           (const uint32_t *)pl->dd, (const uint64_t *)pl->off, (int64_t)0,
                           pl->total, (uint64_t *)nullptr, (lime_pair *)nullptr, ck);
        LIME_HIP(hipGetLastError());
    }
    unsigned long long h[2];
    LIME_TRY(read_back(ctx, h, ck, sizeof(h)));
    release(ctx, ck);
    *sum = h[0];
    *xr = h[1];
    return LIME_OK;
}

}  // namespace lime

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
//   k_bin_*     unsorted rows -> bits without a sort (below)
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

// ------------------------------------------------- rows -> bits, no sort
// Unsorted rows are binned by a two-level counting scatter, then each
// 2^PSH-base paint tile ORs its rows into an LDS image and stores it once:
//   k_bin_count  per chunk of rows (one block, looping): LDS histogram of the
//                rows' paint tiles -> per-bin counts into column `chunk` of
//                the bin-major matrix mat[bin][chunk], tile totals by atomics
//   scan x2      (bin, chunk) segment starts; paint tile starts
//   k_bin_write  the chunks again: per 8192-row step the rows are ranked per
//                bin (LDS atomics), staged in LDS in bin order, and stored as
//                runs, one u32 each (offset in bin << LENB | length); longer
//                rows and rows crossing the bin end leave their remainder to
//                the cross list (bucketed by tile: k_xcount / k_xwrite)
//   k_bin_split_atomic  one block per bin: its rows to its PSUB paint tiles
//                (one returning LDS atomic per row on the tile's cursor: a
//                wave's claims on one cursor come back consecutive, so the
//                stores stay runs), re-packed relative to the tile,
//                tile-crossing remainders to the cross list
//   k_paint_and  one block per paint tile: its rows OR-ed into a 64 KiB LDS
//                image, stored once (every word written exactly once) -- or
//   k_paint_ev   the same image combined with the other operands' and its
//                runs' events extracted in place (no words stored)
// Why two levels: a one-level scatter to 5,900 paint tiles (hg38) keeps
// (destinations x resident blocks) lines open per XCD, far beyond its 4 MiB
// L2, and wrote 3.9x its bytes (profiles/round2_c5_pmc_onelevel.txt); 369
// bins x one block per CU fit.  Staging the step in LDS (runs per bin) beat
// direct per-row stores 0.90 vs 1.38 ms per 1.25e8 rows.
// HBM per row: 8 B (count) + 12 B + 4 B (write) + 4 B + 4 B (split) + 4 B
// (paint), + G/8 bits.
// 2^23-base bins (369 for hg38): the write pass's runs per bin and step are
// twice as long as at 2^22 (737 bins), so its partial lines halve -- C5's
// write pass 661 -> 597 us per set, C4's 59 -> 51, same box; the split then
// fills 16 tiles per bin and takes 16 rows per lane per chunk
// (profiles/round6/c4_c5_bins_2e23_ab.txt).  Lengths in a bin slab: 9 bits
// (rows past 511 bases leave their remainder to the cross list)
#ifndef LIME_BSH
#define LIME_BSH 23
#endif
#ifndef LIME_PSH
#define LIME_PSH 19
#endif
#ifndef LIME_PAINTB
#define LIME_PAINTB 512
#endif
constexpr int BSH = LIME_BSH;            // bin = 2^23 bases
constexpr int PSH = LIME_PSH;            // paint tile = 2^19 bases = 8192 words (64 KiB)
constexpr int PSUB = 1 << (BSH - PSH);   // paint tiles per bin
constexpr int TWORDS = 1 << (PSH - 6);
constexpr int LENB = 32 - BSH;           // packed length bits (bin slab)
constexpr uint32_t LMAX = (1u << LENB) - 1;
constexpr int PLENB = 32 - PSH;          // packed length bits (tile slab)
constexpr int NBMAX = 1 << (32 - BSH);   // bins (span < 2^32)
constexpr int NTMAX = NBMAX * PSUB;      // paint tiles
constexpr int BINB = 1024;               // count / split block
// the write pass: 1024-thread workgroups, one per CU, so a step holds
// 12288 rows and each bin's run per step is twice as long (fewer partial
// lines) as with two 512-thread workgroups per CU: C5's write pass 567 ->
// 519 us per set, same box (profiles/round6/c5_write_1024_threads_ab.txt)
#ifndef LIME_WRB
#define LIME_WRB 1024
#endif
constexpr int WRB = LIME_WRB;            // write block (<= 256 VGPRs: no spills)
constexpr int PAINTB = LIME_PAINTB;

struct BinArgs {
    const int32_t *contig;     // null: start / end are global coordinates
    const uint32_t *start, *end;
    const uint32_t *off, *len;
    int32_t nc;
    int64_t n;
    uint32_t lo, hi;           // the bitset covers global bits [lo, hi), lo % 64 == 0
    uint64_t span;
    int nb;                    // bins
    int64_t chunk_rows;        // R (multiple of STEP)
    uint32_t nchunks;
    uint32_t *mat;             // nb * nchunks + 1 (counts, then scanned starts)
    uint32_t *ttot;            // nb * PSUB + 1 tile totals, then scanned starts
    uint32_t *gsum;            // ngroups x (nb * PSUB): rows per (chunk group, paint tile)
    uint32_t *gpre;            // (nb * PSUB) x ngroups: rows of a tile in earlier chunk groups
    int ngroups;               // split workgroups per bin (chunk groups)
    uint32_t *slab;            // n packed rows, bin order
    uint32_t *slab2;           // n packed rows, paint tile order
    uint64_t *cross;           // remainders (s << 32 | e) in window bits, capacity n
    unsigned int *ncross;
    unsigned int *err;         // bit0 contig, bit1 end < start, bit2 end > length
    uint32_t *dummy;           // sink of the fixed-count store batches (see k_bin_write)
    uint32_t *xbz;             // (may be null) 3 (nb PSUB + 1) words zeroed by k_tile_groups:
                               // the set's cross buckets, so no memset follows the read-back
    uint32_t rcap;             // optimistic binning (no count pass): rows of (bin b, chunk
                               // c) at slab[(b nchunks + c) rcap ...), the rest SLAB_PAD
};
// an unused slot of an optimistic slab region (no packed row has offset
// 2^BSH - 1 with length LMAX: its length is clamped to 1 there)
constexpr uint32_t SLAB_PAD = 0xffffffffu;
constexpr unsigned int ERR_REGION = 256u;  // an optimistic region overflowed

// global start of a row (0 for an invalid contig); every pass derives a
// row's bin and tile from it alone, so they always agree.  u32 arithmetic
// (span < 2^32; an invalid row's start may wrap, identically in every pass,
// and it paints nothing)
__device__ __forceinline__ uint32_t row_gs(const BinArgs &a, const uint32_t *off, int32_t c,
                                           uint32_t s) {
    if (!a.contig) return s;
    return (c >= 0 && c < a.nc) ? off[c] + s : 0u;
}
// bit g of the space -> bit of the bitset's window (clamped into it)
__device__ __forceinline__ uint32_t local_bit(const BinArgs &a, uint32_t g) {
    return (g < a.lo ? a.lo : (g > a.hi ? a.hi : g)) - a.lo;
}
__device__ __forceinline__ int bin_of(const BinArgs &a, uint32_t l) {
    const uint32_t t = l >> BSH;
    return t < (uint32_t)a.nb ? (int)t : a.nb - 1;
}
// paint tile of a window bit, consistent with bin_of and with the offset
// k_bin_write packs (clamped into the bin, see there)
__device__ __forceinline__ int ptile_of(const BinArgs &a, uint32_t l) {
    const int b = bin_of(a, l);
    const uint32_t q = (l - ((uint32_t)b << BSH)) >> PSH;
    return b * PSUB + (q < PSUB ? (int)q : PSUB - 1);
}
// the contig table in LDS when it fits (CMAX contigs: every hg assembly's
// primary contigs), else read through the caches; the row passes gather it
// once per row, a dependent load the prefetch cannot hide
constexpr int CMAX = 1024;
template <bool LC>
__device__ __forceinline__ void stage_contigs(const BinArgs &a, uint32_t *coff, uint32_t *clen,
                                              int nt) {
    if (LC)
        for (int i = threadIdx.x; i < a.nc; i += nt) {
            coff[i] = a.off[i];
            if (clen) clen[i] = a.len[i];
        }
}
// bit g of the space -> bit of the bitset's window (clamped into it)
__device__ __forceinline__ uint64_t local_bit(const BinArgs &a, uint64_t g) {
    return (g < a.lo ? a.lo : (g > a.hi ? a.hi : g)) - a.lo;
}
__device__ __forceinline__ int bin_of(const BinArgs &a, uint64_t l) {
    const uint64_t t = l >> BSH;
    return t < (uint64_t)a.nb ? (int)t : a.nb - 1;
}
// paint tile of a window bit, consistent with bin_of
__device__ __forceinline__ int ptile_of(const BinArgs &a, uint64_t l) {
    const int b = bin_of(a, l);
    const uint64_t q = (l - ((uint64_t)b << BSH)) >> PSH;
    return b * PSUB + (q < PSUB ? (int)q : PSUB - 1);
}
// bijective block -> chunk map: each XCD (blockIdx % 8) takes a contiguous
// range of chunks (speed only)
__device__ __forceinline__ uint32_t xcd_chunk(uint32_t bid, uint32_t nch) {
    const uint32_t q = nch / 8, r = nch % 8, x = bid % 8, i = bid / 8;
    return x * q + (x < r ? x : r) + i;
}

// A step = SROWS rows per lane: groups of 4 consecutive rows, the groups
// BINB * 4 rows apart, so every load is a lane-consecutive 16-B access and a
// step keeps 6-9 loads in flight per lane.
// 12 rows per lane (<= 128 VGPRs): with two 512-thread write workgroups per
// CU, C5 10.8-11.1 -> 10.5-10.8 ms against 16 rows at one per CU (8 rows: no
// gain, shorter runs per bin); now one 1024-thread workgroup (LIME_WRB)
#ifndef LIME_SROWS
#define LIME_SROWS 12
#endif
constexpr int SROWS = LIME_SROWS;  // (a multiple of 4)
constexpr int STEP = SROWS * BINB;    // rows per count step
constexpr int WSTEP = SROWS * WRB;    // rows per write step

template <bool END, int NT = BINB>
__device__ __forceinline__ void load_step(const BinArgs &a, int64_t base, int64_t lim,
                                          int32_t (&c)[SROWS], uint32_t (&s)[SROWS],
                                          uint32_t (&e)[SROWS], uint32_t &valid) {
    valid = 0;
#pragma unroll
    for (int q = 0; q < SROWS / 4; ++q) {
        const int64_t i0 = base + (int64_t)q * 4 * NT + 4 * threadIdx.x;
        if (i0 + 4 <= lim) {
            const int4 cv =
                a.contig ? *reinterpret_cast<const int4 *>(a.contig + i0) : int4{0, 0, 0, 0};
            const uint4 sv = *reinterpret_cast<const uint4 *>(a.start + i0);
            c[4 * q] = cv.x, c[4 * q + 1] = cv.y, c[4 * q + 2] = cv.z, c[4 * q + 3] = cv.w;
            s[4 * q] = sv.x, s[4 * q + 1] = sv.y, s[4 * q + 2] = sv.z, s[4 * q + 3] = sv.w;
            if (END) {
                const uint4 ev = *reinterpret_cast<const uint4 *>(a.end + i0);
                e[4 * q] = ev.x, e[4 * q + 1] = ev.y, e[4 * q + 2] = ev.z, e[4 * q + 3] = ev.w;
            }
            valid |= 0xfu << (4 * q);
        } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const bool v = i0 + j < lim;
                c[4 * q + j] = v && a.contig ? a.contig[i0 + j] : 0;
                s[4 * q + j] = v ? a.start[i0 + j] : 0u;
                if (END) e[4 * q + j] = v ? a.end[i0 + j] : 0u;
                if (v) valid |= 1u << (4 * q + j);
            }
        }
    }
}

// The write pass's prefetch: one step's rows by 16-B buffer loads through
// per-chunk descriptors (bounds = the chunk's bytes), straight into the
// step's registers.  A step past the chunk's last whole one is fetched at an
// out-of-range offset: the loads return zeros and touch no memory, so the
// prefetch needs no branch.  (Behind a per-lane bounds test hipcc joined the
// loaded values into other registers, copying each group -- and so waiting
// for it -- right after issuing it: 3 load latencies per step.)
struct StepRsrc {
    __amdgpu_buffer_rsrc_t c, s, e;
};
template <bool HC>
__device__ __forceinline__ StepRsrc step_rsrc(const BinArgs &a, int64_t r0, int64_t r1) {
    const int nbytes = (int)((r1 - r0) * 4);  // (< 2^31: chunk_rows <= 16 STEP)
    StepRsrc r;
    r.c = __builtin_amdgcn_make_buffer_rsrc(HC ? (void *)(a.contig + r0) : (void *)a.start, (short)0,
                                           HC ? nbytes : 0, 0x00020000);
    r.s = __builtin_amdgcn_make_buffer_rsrc((void *)(a.start + r0), (short)0, nbytes, 0x00020000);
    r.e = __builtin_amdgcn_make_buffer_rsrc((void *)(a.end + r0), (short)0, nbytes, 0x00020000);
    return r;
}
constexpr uint32_t RSRC_OOB = 0x40000000u;  // byte offset past any chunk
template <bool HC, int NT>
__device__ __forceinline__ void load_rsrc(const StepRsrc &r, uint32_t rel, int32_t (&c)[SROWS],
                                          uint32_t (&s)[SROWS], uint32_t (&e)[SROWS]) {
#pragma unroll
    for (int q = 0; q < SROWS / 4; ++q) {
        const uint32_t off = rel + 4u * (q * 4 * NT + 4 * threadIdx.x);  // bytes
        if (HC) {
            const auto cv = __builtin_amdgcn_raw_buffer_load_b128(r.c, (int)off, 0, 0);
            c[4 * q] = (int32_t)cv[0], c[4 * q + 1] = (int32_t)cv[1], c[4 * q + 2] = (int32_t)cv[2],
                  c[4 * q + 3] = (int32_t)cv[3];
        } else {
            c[4 * q] = c[4 * q + 1] = c[4 * q + 2] = c[4 * q + 3] = 0;
        }
        const auto sv = __builtin_amdgcn_raw_buffer_load_b128(r.s, (int)off, 0, 0);
        s[4 * q] = sv[0], s[4 * q + 1] = sv[1], s[4 * q + 2] = sv[2], s[4 * q + 3] = sv[3];
        const auto ev = __builtin_amdgcn_raw_buffer_load_b128(r.e, (int)off, 0, 0);
        e[4 * q] = ev[0], e[4 * q + 1] = ev[1], e[4 * q + 2] = ev[2], e[4 * q + 3] = ev[3];
    }
}

template <bool LC>
__global__ __launch_bounds__(BINB) void k_bin_count(BinArgs a) {
    __shared__ uint32_t hist[NTMAX];
    __shared__ uint32_t coff[LC ? CMAX : 1];
    const uint32_t *off = LC ? coff : a.off;
    const int nt = a.nb * PSUB;
    for (int i = threadIdx.x; i < nt; i += BINB) hist[i] = 0;
    stage_contigs<LC>(a, coff, nullptr, BINB);
    __syncthreads();
    const uint32_t ch = xcd_chunk(blockIdx.x, a.nchunks);
    // the matrix's extra last entry (it receives the total from the scan), and
    // the set's flags (ncross, err: written only by the later passes)
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        a.mat[(int64_t)a.nb * a.nchunks] = 0u;
        *a.ncross = 0u;
        *a.err = 0u;
    }
    const int64_t r0 = (int64_t)ch * a.chunk_rows;
    const int64_t r1 = min(a.n, r0 + a.chunk_rows);
    for (int64_t base = r0; base < r1; base += STEP) {
        int32_t c[SROWS];
        uint32_t s[SROWS], e[SROWS];
        uint32_t valid;
        load_step<false>(a, base, r1, c, s, e, valid);
#pragma unroll
        for (int k = 0; k < SROWS; ++k)
            if (valid & (1u << k))
                atomicAdd(&hist[ptile_of(a, local_bit(a, row_gs(a, off, c[k], s[k])))], 1u);
    }
    __syncthreads();
    for (int b = threadIdx.x; b < a.nb; b += BINB) {
        uint32_t sum = 0;
#pragma unroll
        for (int q = 0; q < PSUB; ++q) sum += hist[b * PSUB + q];
        a.mat[(int64_t)b * a.nchunks + ch] = sum;
    }
    // the chunk's rows per paint tile into its chunk group's totals (the
    // split runs one workgroup per (bin, chunk group))
    uint32_t g = (uint32_t)(((uint64_t)ch * a.ngroups + a.ngroups - 1) / a.nchunks);
    while (g > 0 && (int64_t)(g * (uint64_t)a.nchunks / a.ngroups) > ch) --g;
    while (g + 1 < (uint32_t)a.ngroups && (int64_t)((g + 1) * (uint64_t)a.nchunks / a.ngroups) <= ch)
        ++g;
    for (int t = threadIdx.x; t < nt; t += BINB)
        if (hist[t]) atomicAdd(&a.gsum[(int64_t)g * nt + t], hist[t]);
}

// per paint tile: its rows in the chunk groups before each group (gpre) and
// in all (ttot, scanned next into the tile starts); also zeroes the set's
// cross buckets (a.xbz, 3 (nt + 1) words), so no memset follows the host's
// read-back.  (A one-workgroup form that scanned ttot in the same launch
// made C4's step slower, 0.88 -> 0.93 ms same box: one CU's latency chain.)
__global__ __launch_bounds__(256) void k_tile_groups(BinArgs a) {
    const int nt = a.nb * PSUB;
    const int t = blockIdx.x * 256 + threadIdx.x;
    if (a.xbz && t <= nt) {
        const int64_t ts = (int64_t)nt + 1;
        a.xbz[t] = a.xbz[ts + t] = a.xbz[2 * ts + t] = 0u;
    }
    if (t >= nt) return;
    uint32_t run = 0;
    for (int g = 0; g < a.ngroups; ++g) {
        a.gpre[(int64_t)t * a.ngroups + g] = run;
        run += a.gsum[(int64_t)g * nt + t];
    }
    a.ttot[t] = run;
}

#ifndef LIME_WRITE_BLOCKS
#define LIME_WRITE_BLOCKS 1
#endif
#ifndef LIME_BIN_PREFETCH
#define LIME_BIN_PREFETCH 1
#endif
// LC: the contig table in LDS; HC: rows carry contig ids (else global
// coordinates)
// OPT (optimistic, no count pass): the chunk's rows of bin t go to its
// region slab[(t nchunks + ch) rcap, + rcap) (sized from the window's
// uniform density; rows past a region go to the sink and raise ERR_REGION,
// and the host bins the set again through the counted path); the unused
// rest of each region is filled with SLAB_PAD, and the rows per paint tile
// (LDS, u16 pairs) are added into the chunk group's totals (gsum), which
// k_bin_count made otherwise
template <bool LC, bool HC, bool OPT = false>
__global__ __launch_bounds__(WRB)
__attribute__((amdgpu_waves_per_eu(LIME_WRITE_BLOCKS * WRB / 256, 8))) void k_bin_write(BinArgs a) {
    __shared__ uint32_t stage[WSTEP];
    __shared__ uint16_t sbin[WSTEP];
    __shared__ uint32_t hist[NBMAX], soff[NBMAX], cur[NBMAX];
    __shared__ uint32_t scratch[WRB / 64 + 1];
    __shared__ uint32_t coff[LC ? CMAX : 1], clen[LC ? CMAX : 1];
    __shared__ uint32_t th[OPT ? NTMAX / 2 : 1];  // rows per paint tile, two u16 per word
    const uint32_t *off = LC ? coff : a.off, *len = LC ? clen : a.len;
    stage_contigs<LC>(a, coff, clen, WRB);
    const uint32_t ch = xcd_chunk(blockIdx.x, a.nchunks);
    for (int t = threadIdx.x; t < NBMAX; t += WRB) {
        cur[t] = t < a.nb ? (OPT ? (uint32_t)(((uint64_t)t * a.nchunks + ch) * a.rcap)
                                 : a.mat[(int64_t)t * a.nchunks + ch])
                          : 0u;
        hist[t] = 0;
    }
    if (OPT)
        for (int i = threadIdx.x; i < NTMAX / 2; i += WRB) th[i] = 0u;
    __syncthreads();
    uint32_t ovf = 0;  // (OPT) a row past its region
    const int64_t r0 = (int64_t)ch * a.chunk_rows;
    const int64_t r1 = min(a.n, r0 + a.chunk_rows);
    uint32_t err = 0;
    int32_t c[SROWS];
    uint32_t s[SROWS], e[SROWS];
    // one step: its rows' bins and packed runs from (c, s, e), then NEXT()
    // (the following step's loads: in flight across this step's barriers --
    // plain loads survive __syncthreads), then rank, stage and store
    auto step = [&](int64_t base, uint32_t valid, auto next) {
        // tb[k]: the row's bin, then (bin << RKB | its rank among the step's
        // rows of the bin) once ranked: one register per row for both
        uint32_t tb[SROWS], pk[SROWS];
#pragma unroll
        for (int k = 0; k < SROWS; ++k) {
            const int32_t cc = c[k];
            const uint32_t gs = row_gs(a, off, HC ? cc : 0, s[k]);
            uint32_t ge = gs;
            if (!(valid & (1u << k))) {
            } else if (!HC) {
                if (e[k] < s[k]) err |= 2u;
                else if (e[k] > a.span) err |= 4u;
                else ge = e[k];
            } else if (cc < 0 || cc >= a.nc) {
                err |= 1u;
            } else if (e[k] < s[k]) {
                err |= 2u;
            } else if (e[k] > len[cc]) {
                err |= 4u;
            } else {
                ge = off[cc] + e[k];
            }
            // the row's part inside the window, in window bits
            const uint32_t g0 = local_bit(a, gs), g1 = local_bit(a, ge);
            const int t = bin_of(a, g0);
            // offset in the bin; a row clamped to the end of a window whose
            // width is a multiple of 2^BSH sits at 2^BSH: clamp it into the
            // bin's last tile, where ptile_of counted it (it paints nothing)
            const uint32_t o = min(g0 - ((uint32_t)t << BSH), (1u << BSH) - 1);
            // in-bin piece [g0, g0 + l), l <= LMAX; the rest: cross list
            uint32_t l = g1 > g0 ? g1 - g0 : 0u;
            l = min(min(l, LMAX), (1u << BSH) - o);
            tb[k] = (uint32_t)t;
            pk[k] = (o << LENB) | l;
            if ((valid & (1u << k)) && g1 > g0 + l)
                a.cross[atomicAdd(a.ncross, 1u)] = ((uint64_t)(g0 + l) << 32) | g1;
            if (OPT && (valid & (1u << k))) {  // (the split's tile of the row: bin piece start)
                const uint32_t tile = (uint32_t)t * PSUB + min(o >> PSH, (uint32_t)PSUB - 1);
                atomicAdd(&th[tile >> 1], 1u << ((tile & 1u) << 4));
            }
        }
        next();
        // rank per bin (16 independent LDS atomics), then bin offsets in the
        // step (one scan over <= 1024 bins), then stage in bin order
        constexpr int RKB = WSTEP <= (1 << 13) ? 13 : 14;  // rank bits
        static_assert(WSTEP <= (1 << RKB) && NBMAX <= (1 << (32 - RKB)), "bin / rank packing");
#pragma unroll
        for (int k = 0; k < SROWS; ++k)
            if (valid & (1u << k)) tb[k] = (tb[k] << RKB) | atomicAdd(&hist[tb[k]], 1u);
        __syncthreads();
        {
            // bins BPT t .. BPT t + BPT - 1 per thread (fewer bins than
            // threads: one bin each, the rest idle)
            constexpr int BPT = NBMAX >= WRB ? NBMAX / WRB : 1;
            const int t = BPT * threadIdx.x;
            const bool has = t < NBMAX;
            uint32_t h[BPT], sum = 0;
#pragma unroll
            for (int q = 0; q < BPT; ++q) sum += (h[q] = has ? hist[t + q] : 0u);
            uint32_t tot;
            uint32_t o = dev::block_exclusive_sum<WRB>(sum, scratch, &tot);
#pragma unroll
            for (int q = 0; q < BPT; ++q) {
                if (has) soff[t + q] = o;
                o += h[q];
            }
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < SROWS; ++k)
            if (valid & (1u << k)) {
                const uint32_t t = tb[k] >> RKB;
                const uint32_t j = soff[t] + (tb[k] & ((1u << RKB) - 1u));
                stage[j] = pk[k];
                sbin[j] = (uint16_t)t;
            }
        __syncthreads();
        // runs of a bin are consecutive: lane-consecutive stores.  Every lane
        // issues exactly SROWS stores (positions past the step's rows go to a
        // sink): loads and stores share vmcnt, so with a static store count
        // the next step's first use of its prefetched rows waits for the
        // loads only, not for this step's stores
        const int cnt = (int)min((int64_t)WSTEP, r1 - base);
#pragma unroll
        for (int k = 0; k < SROWS; ++k) {
            const int j = threadIdx.x + k * WRB;
            const uint32_t t = sbin[j];
            const uint32_t pos = cur[t] + (uint32_t)j - soff[t];
            bool in = j < cnt;
            if (OPT && in && pos >= (uint32_t)(((uint64_t)t * a.nchunks + ch + 1) * a.rcap)) {
                in = false;
                ovf = 1;
            }
            uint32_t *dst = in ? a.slab + pos : a.dummy;
            *dst = stage[j];
        }
        __syncthreads();
        for (int t = threadIdx.x; t < NBMAX; t += WRB) {
            cur[t] += hist[t];
            hist[t] = 0;
        }
        __syncthreads();
    };
    constexpr uint32_t ALL = (1u << SROWS) - 1;
    // the chunk's whole steps (every chunk but the set's last has only
    // those: chunk_rows is a multiple of WSTEP), then its partial tail
    const int64_t nfull = (r1 - r0) / WSTEP;
    if (LIME_BIN_PREFETCH) {
        // iteration -1 only fetches step 0: the rows' one load site, so the
        // registers they land in are the ones the next step reads
        const StepRsrc rs = step_rsrc<HC>(a, r0, r1);
        for (int64_t k = -1; k < nfull; ++k) {  // (uniform)
            const int64_t base = r0 + k * WSTEP;
            auto fetch = [&]() {
                const uint32_t rel = k + 1 < nfull ? 4u * (uint32_t)((k + 1) * WSTEP) : RSRC_OOB;
                load_rsrc<HC, WRB>(rs, rel, c, s, e);
            };
            if (k < 0)
                fetch();
            else
                step(base, ALL, fetch);
        }
    } else {
        for (int64_t k = 0; k < nfull; ++k) {
            const int64_t base = r0 + k * WSTEP;
            uint32_t valid;
            load_step<true, WRB>(a, base, r1, c, s, e, valid);
            step(base, valid, [] {});
        }
    }
    const int64_t tail = r0 + nfull * WSTEP;
    if (tail < r1) {
        uint32_t valid;
        load_step<true, WRB>(a, tail, r1, c, s, e, valid);
        step(tail, valid, [] {});
    }
    if (OPT) {
        __syncthreads();  // (cur final, th complete)
        // the regions' unused slots: SLAB_PAD, lane-consecutive per wave
        const int wv = threadIdx.x / 64, lane = dev::lane_id();
        for (int t = wv; t < a.nb; t += WRB / 64) {
            const uint32_t rend = (uint32_t)(((uint64_t)t * a.nchunks + ch + 1) * a.rcap);
            for (uint32_t p = cur[t] + lane; p < rend; p += 64) a.slab[p] = SLAB_PAD;
        }
        // this chunk's rows per paint tile into its chunk group's totals
        uint32_t g = (uint32_t)(((uint64_t)ch * a.ngroups + a.ngroups - 1) / a.nchunks);
        while (g > 0 && (int64_t)(g * (uint64_t)a.nchunks / a.ngroups) > ch) --g;
        while (g + 1 < (uint32_t)a.ngroups &&
               (int64_t)((g + 1) * (uint64_t)a.nchunks / a.ngroups) <= ch)
            ++g;
        const int nt = a.nb * PSUB;
        for (int i = threadIdx.x; i < (nt + 1) / 2; i += WRB) {
            const uint32_t w = th[i];
            if (w & 0xffffu) atomicAdd(&a.gsum[(int64_t)g * nt + 2 * i], w & 0xffffu);
            if ((w >> 16) && 2 * i + 1 < nt) atomicAdd(&a.gsum[(int64_t)g * nt + 2 * i + 1], w >> 16);
        }
        if (ovf) err |= ERR_REGION;
    }
    err = dev::wave_reduce_or(err);
    if (err && dev::lane_id() == 0) atomicOr(a.err, err);
}

// one block per bin: its rows -> its PSUB paint tiles.  The bin's rows go
// in chunks of SPB * PV: every row claims a slot on its WAVE's counter for its
// tile (one returning LDS atomic; 64 lanes over 16 counters, where a counter
// per block took 512), a scan over the 8 waves per tile places the waves'
// slot groups one after the other at the tile's cursor, and the rows are
// stored there (a wave's rows of one tile are consecutive slots).  Claims
// inside a group come back in any order: a tile's rows are ORed in any order.
static_assert(NBMAX % WRB == 0 || WRB % NBMAX == 0, "write-pass bin scan: whole bins per thread");
#ifndef LIME_SPB
#define LIME_SPB 512
#endif
#ifndef LIME_SPLIT_PV
#define LIME_SPLIT_PV 16
#endif
constexpr int SPB = LIME_SPB;  // split block (16 rows per lane: 2 blocks per CU)
#ifndef LIME_SPLIT_BLOCKS
#define LIME_SPLIT_BLOCKS 3072
#endif
// OPT: the bin's rows of chunks [c0, c1) are their regions, SLAB_PAD slots
// skipped
// STAGE: the chunk's rows are staged in LDS tile by tile and stored as one
// contiguous run per tile (~CH / PSUB rows), where each wave's store had
// scattered its 64 lanes over the bin's 16 tiles
#ifndef LIME_SPLIT_STAGE
#define LIME_SPLIT_STAGE 1
#endif
template <bool OPT = false>
__global__ __launch_bounds__(SPB) void k_bin_split_atomic(BinArgs a) {
    constexpr int NWV = SPB / 64, PV = LIME_SPLIT_PV;
    constexpr bool STG = LIME_SPLIT_STAGE != 0;
    __shared__ uint32_t wc[NWV][PSUB], wbase[NWV][PSUB], cur[PSUB];
    __shared__ uint32_t stg[STG ? SPB * PV : 1], sst[PSUB + 1], sgs[PSUB];
    // workgroup (bin b, chunk group g): the bin's rows of chunks [c0, c1),
    // consecutive in the bin-ordered slab; each tile's cursor starts past
    // its rows of the earlier groups (gpre), so the groups split in parallel
    const int b = blockIdx.x / a.ngroups, g = blockIdx.x % a.ngroups;
    const int wv = threadIdx.x / 64, lane = dev::lane_id();
    if (threadIdx.x < PSUB)
        cur[threadIdx.x] = a.ttot[b * PSUB + threadIdx.x] +
                           a.gpre[(int64_t)(b * PSUB + threadIdx.x) * a.ngroups + g];
    if (threadIdx.x < NWV * PSUB) (&wc[0][0])[threadIdx.x] = 0u;
    const int64_t c0 = (int64_t)g * a.nchunks / a.ngroups,
                  c1 = (int64_t)(g + 1) * a.nchunks / a.ngroups;
    const uint32_t r0 = OPT ? (uint32_t)(((uint64_t)b * a.nchunks + c0) * a.rcap)
                            : a.mat[(int64_t)b * a.nchunks + c0],
                   r1 = OPT ? (uint32_t)(((uint64_t)b * a.nchunks + c1) * a.rcap)
                            : a.mat[(int64_t)b * a.nchunks + c1];
    __syncthreads();
    const uint64_t bin0 = (uint64_t)b << BSH;
    constexpr uint32_t CH = SPB * PV;  // rows per chunk
    const uint32_t mine = (uint32_t)wv * 64 * PV + lane;  // the lane's first row in a chunk
    uint32_t pv[PV];
    if (r0 < r1)
#pragma unroll
        for (int k = 0; k < PV; ++k) pv[k] = a.slab[min(r0 + mine + k * 64, r1 - 1)];
    for (uint32_t c0 = r0; c0 < r1; c0 += CH) {  // (uniform over the block)
        uint32_t q[PV], val[PV], rk[PV];
#pragma unroll
        for (int k = 0; k < PV; ++k) {
            const bool v = c0 + mine + k * 64 < r1 && (!OPT || pv[k] != SLAB_PAD);
            const uint32_t o = pv[k] >> LENB, l = pv[k] & LMAX;
            q[k] = v ? min(o >> PSH, (uint32_t)PSUB - 1) : PSUB;  // PSUB: no row
            const uint32_t qend = (q[k] + 1) << PSH;
            const uint32_t l2 = o + l > qend ? qend - o : l;  // clipped at the tile end
            if (v && l2 < l)  // remainder [o + l2, o + l) into the next tile(s)
                a.cross[atomicAdd(a.ncross, 1u)] = ((bin0 + o + l2) << 32) | (bin0 + o + l);
            val[k] = ((o - (q[k] << PSH)) << PLENB) | l2;
            rk[k] = v ? atomicAdd(&wc[wv][q[k]], 1u) : 0u;
        }
        if (c0 + CH < r1)
#pragma unroll
            for (int k = 0; k < PV; ++k) pv[k] = a.slab[min(c0 + CH + mine + k * 64, r1 - 1)];
        __syncthreads();
        if (STG) {
            if (threadIdx.x < 64) {  // wave 0: tile d = lane (PSUB <= 64)
                static_assert(PSUB <= 64, "one tile per lane of wave 0");
                const int d = lane;
                uint32_t run = 0;
                if (d < PSUB)
#pragma unroll
                    for (int w = 0; w < NWV; ++w) {
                        const uint32_t c = wc[w][d];
                        wbase[w][d] = run;  // (relative to the tile's staging start)
                        wc[w][d] = 0u;
                        run += c;
                    }
                // the tiles' staging starts: an exclusive scan over the lanes
                const uint32_t inc = dev::wave_inclusive_sum(run);
                if (d < PSUB) {
                    const uint32_t st0 = inc - run;
                    sst[d] = st0;
                    sgs[d] = cur[d];
                    cur[d] += run;
#pragma unroll
                    for (int w = 0; w < NWV; ++w) wbase[w][d] += st0;
                }
                if (d == PSUB - 1) sst[PSUB] = inc;
            }
            __syncthreads();
#pragma unroll
            for (int k = 0; k < PV; ++k)
                if (q[k] < PSUB) stg[wbase[wv][q[k]] + rk[k]] = val[k];
            __syncthreads();
            // one contiguous run per tile: slot j is tile t's (j - sst[t])-th
            const uint32_t cnt = sst[PSUB];
            for (uint32_t j = threadIdx.x; j < cnt; j += SPB) {
                int t = 0;
#pragma unroll
                for (int h = PSUB / 2; h >= 1; h >>= 1)
                    if (sst[t + h] <= j) t += h;
                a.slab2[sgs[t] + (j - sst[t])] = stg[j];
            }
            __syncthreads();  // (stg and the tables are rewritten by the next chunk)
            continue;
        }
        if (threadIdx.x < PSUB) {  // the waves' groups, one after the other per tile
            const int d = threadIdx.x;
            uint32_t run = cur[d];
#pragma unroll
            for (int w = 0; w < NWV; ++w) {
                const uint32_t c = wc[w][d];
                wbase[w][d] = run;
                wc[w][d] = 0u;
                run += c;
            }
            cur[d] = run;
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < PV; ++k)
            *(q[k] < PSUB ? a.slab2 + wbase[wv][q[k] & (PSUB - 1)] + rk[k] : a.dummy) = val[k];
    }
}

// bits [s0, e0) of a tile image (LDS); rows within two words (C4/C5's
// lengths) take a branch-free path: two masked ORs
#ifndef LIME_PAINT2
#define LIME_PAINT2 1
#endif
__device__ __forceinline__ void paint_lds(unsigned long long *img, uint32_t s0, uint32_t e0) {
    const uint32_t wa = s0 >> 6, wb = (e0 - 1) >> 6;
    if (wb - wa <= 1) {
        const uint64_t head = ~0ull << (s0 & 63), tail = ~0ull >> (63 - ((e0 - 1) & 63));
#if LIME_PAINT2
        // branch-free: two ORs always (the same word twice when the row is
        // inside one), where a lane-divergent one-or-two made a wave of
        // mixed rows issue three (C5's rows span one or two words)
        const bool one = wa == wb;
        atomicOr(&img[wa], (unsigned long long)(one ? head & tail : head));
        atomicOr(&img[wb], (unsigned long long)(one ? head & tail : tail));
#else
        if (wa == wb) {
            atomicOr(&img[wa], (unsigned long long)(head & tail));
        } else {
            atomicOr(&img[wa], (unsigned long long)head);
            atomicOr(&img[wb], (unsigned long long)tail);
        }
#endif
        return;
    }
    // head and tail words by ORs, the whole words between by plain stores
    // (idempotent with the ORs): one store per interior word, no per-word
    // mask arithmetic (C4's rows span ~5 words)
    const uint64_t head = ~0ull << (s0 & 63), tail = ~0ull >> (63 - ((e0 - 1) & 63));
    atomicOr(&img[wa], (unsigned long long)head);
    atomicOr(&img[wb], (unsigned long long)tail);
    for (uint32_t w = wa + 1; w < wb; ++w) img[w] = ~0ull;
}

// ---------------------------------------- k-way AND straight from rows
// The C5 shape: k row sets binned as above, then ONE kernel
// paints every set's rows of a tile into LDS in turn and ANDs the images in
// registers -- one bitset stored instead of k, and no k-operand re-read.
// Cross-list pieces (rows longer than a bin piece, pieces crossing a tile)
// are bucketed by tile first: a piece [s, e) paints its head in tile(s) and
// its tail in tile(e - 1); the tiles strictly between are wholly covered,
// which a difference array records (the set then leaves those tiles' AND
// unchanged).
__global__ __launch_bounds__(BB) void k_xcount(const uint64_t *__restrict__ cross,
                                               const unsigned int *__restrict__ ncross,
                                               uint32_t *__restrict__ xcnt,
                                               uint32_t *__restrict__ diff) {
    const int64_t nx = *ncross;
    for (int64_t i = (int64_t)blockIdx.x * BB + threadIdx.x; i < nx; i += (int64_t)gridDim.x * BB) {
        const uint64_t s = cross[i] >> 32, e = cross[i] & 0xffffffffull;
        const uint32_t t0 = (uint32_t)(s >> PSH), t1 = (uint32_t)((e - 1) >> PSH);
        atomicAdd(&xcnt[t0], 1u);
        if (t1 > t0) atomicAdd(&xcnt[t1], 1u);
        if (t1 > t0 + 1) {
            atomicAdd(&diff[t0 + 1], 1u);
            atomicAdd(&diff[t1], 0xffffffffu);  // -1 (the scan is modulo 2^32)
        }
    }
}

// piece slots: the tile's scanned start xoff[t] + a claim on xfill[t]
// (zeroed with the counters: no copy of the scanned starts to a cursor)
__global__ __launch_bounds__(BB) void k_xwrite(const uint64_t *__restrict__ cross,
                                               const unsigned int *__restrict__ ncross,
                                               const uint32_t *__restrict__ xoff,
                                               uint32_t *__restrict__ xfill,
                                               uint2 *__restrict__ xl) {
    const int64_t nx = *ncross;
    for (int64_t i = (int64_t)blockIdx.x * BB + threadIdx.x; i < nx; i += (int64_t)gridDim.x * BB) {
        const uint64_t s = cross[i] >> 32, e = cross[i] & 0xffffffffull;
        const uint32_t t0 = (uint32_t)(s >> PSH), t1 = (uint32_t)((e - 1) >> PSH);
        const uint64_t b0 = (uint64_t)t0 << PSH;
        const uint64_t h = t1 > t0 ? b0 + (1ull << PSH) : e;  // head [s, h) in tile t0
        xl[xoff[t0] + atomicAdd(&xfill[t0], 1u)] =
            make_uint2((uint32_t)(s - b0), (uint32_t)(h - b0));
        if (t1 > t0) {
            const uint64_t b1 = (uint64_t)t1 << PSH;
            xl[xoff[t1] + atomicAdd(&xfill[t1], 1u)] = make_uint2(0u, (uint32_t)(e - b1));
        }
    }
}

template <int CAP>
struct AndArgsK {
    static constexpr int NCAP = CAP;
    const uint32_t *slab2[CAP];  // tile-ordered packed rows of set i
    const uint32_t *tstart[CAP]; // nt + 1 tile starts
    const uint2 *xl[CAP];        // tile-bucketed cross pieces (null: none)
    const uint32_t *xoff[CAP];   // nt + 1 bucket starts
    const uint32_t *full[CAP];   // nt + 1 exclusive scan of the difference array
    int k;
    int init;  // the AND continues the words already stored (sets past the first 16)
    uint64_t *words;
    int64_t n_words;
};
using AndArgs = AndArgsK<MAXK>;

constexpr int AWPT = TWORDS / PAINTB;  // AND words per thread (registers)
constexpr int APV = 16;                // rows per lane per batch
// acc[j] (word t TWORDS + threadIdx.x + j PAINTB of tile t) &= every set's
// bits of the tile, complemented for the sets in `neg`.  The tile's (set,
// batch) sequence is software-pipelined: the next batch's loads (possibly
// the next set's) are issued before the current batch is painted, so they
// stay in flight across the set's AND barriers.  img: TWORDS words of LDS.
template <class AA>
__device__ __forceinline__ void paint_and_tile(const AA &a, int t, uint32_t neg,
                                               unsigned long long *img, uint64_t (&acc)[AWPT]) {
    constexpr uint32_t B = APV * PAINTB;
    // the tile's per-set table entries (row range, cross-piece range, whole
    // coverage), read once into LDS by one batch of loads: walked from
    // global memory, each was a vector load whose wait also waited for the
    // prefetched batch, ~4 serial round trips per batch (C5: 24 batches a tile)
    __shared__ uint32_t s_r0[AA::NCAP], s_r1[AA::NCAP], s_x0[AA::NCAP], s_x1[AA::NCAP],
        s_full[AA::NCAP];
    if (threadIdx.x < (unsigned)a.k) {
        const int q = threadIdx.x;
        s_r0[q] = a.tstart[q][t];
        s_r1[q] = a.tstart[q][t + 1];
        s_full[q] = a.full[q] ? a.full[q][t + 1] : 0u;
        s_x0[q] = a.xl[q] ? a.xoff[q][t] : 0u;
        s_x1[q] = a.xl[q] ? a.xoff[q][t + 1] : 0u;
    }
#pragma unroll
    for (int j = 0; j < AWPT; ++j) img[threadIdx.x + j * PAINTB] = 0ull;
    __syncthreads();
    // a tile wholly inside one of the set's cross pieces: all ones (AND
    // unchanged, or all zeros complemented)
    bool zero = false;
    auto skip = [&](int i) {
        const bool f = s_full[i] != 0u;
        if (f && ((neg >> i) & 1u)) zero = true;
        return f;
    };
    // a batch of B rows by bounds-checked buffer loads through a descriptor
    // over the batch's rows (past them, and for i = k: no set, zeros, no
    // traffic): no per-lane branch, so painting the current batch does not
    // wait for this one (behind per-lane bounds tests it waited for all)
    auto load = [&](int i, uint32_t rb, uint32_t(&p)[APV]) {
        const bool has = i < a.k;  // (uniform)
        const uint32_t r0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)rb);
        const uint32_t r1 = has ? (uint32_t)__builtin_amdgcn_readfirstlane((int)s_r1[i]) : r0;
        const uint32_t cnt = r1 > r0 ? min(r1 - r0, B) : 0u;
        const uint32_t *base = has ? a.slab2[i] + r0 : a.slab2[0];
        const auto rs = __builtin_amdgcn_make_buffer_rsrc((void *)base, (short)0, (int)(4u * cnt),
                                                          0x00020000);
#pragma unroll
        for (int k = 0; k < APV; ++k)
            p[k] = __builtin_amdgcn_raw_buffer_load_b32(rs, (int)(4u * (k * PAINTB + threadIdx.x)),
                                                         0, 0);
    };
    int i = 0;
    while (i < a.k && skip(i)) ++i;
    uint32_t rb = i < a.k ? s_r0[i] : 0u;
    uint32_t pv[APV];
    if (i < a.k) load(i, rb, pv);
    while (i < a.k) {  // (i, rb) and i2 are uniform over the block
        int i2 = i;
        uint32_t rb2 = rb + B;
        if (rb2 >= s_r1[i]) {
            i2 = i + 1;
            while (i2 < a.k && skip(i2)) ++i2;
            if (i2 < a.k) rb2 = s_r0[i2];
        }
        uint32_t pn[APV];
        load(i2, rb2, pn);  // (i2 = k: zeros)
#pragma unroll
        for (int k = 0; k < APV; ++k) {
            const uint32_t l = pv[k] & ((1u << PLENB) - 1);
            if (l) paint_lds(img, pv[k] >> PLENB, (pv[k] >> PLENB) + l);
        }
        if (i2 != i) {  // set i complete: its cross pieces, then the AND
            if (a.xl[i]) {
                const uint32_t x0 = s_x0[i], x1 = s_x1[i];
                for (uint32_t x = x0 + threadIdx.x; x < x1; x += PAINTB) {
                    const uint2 p = a.xl[i][x];
                    if (p.y > p.x) paint_lds(img, p.x, p.y);
                }
            }
            __syncthreads();
            const uint64_t inv = ((neg >> i) & 1u) ? ~0ull : 0ull;
#pragma unroll
            for (int j = 0; j < AWPT; ++j) acc[j] &= img[threadIdx.x + j * PAINTB] ^ inv;
            if (i2 < a.k) {
                __syncthreads();
#pragma unroll
                for (int j = 0; j < AWPT; ++j) img[threadIdx.x + j * PAINTB] = 0ull;
                __syncthreads();
            }
        }
#pragma unroll
        for (int k = 0; k < APV; ++k) pv[k] = pn[k];
        i = i2;
        rb = rb2;
    }
    if (zero)
#pragma unroll
        for (int j = 0; j < AWPT; ++j) acc[j] = 0ull;
}

__global__ __launch_bounds__(PAINTB) void k_paint_and(AndArgs a) {
    __shared__ unsigned long long img[TWORDS];
    const int t = blockIdx.x;
    uint64_t acc[AWPT];
    const int64_t w0 = (int64_t)t * TWORDS;
#pragma unroll
    for (int j = 0; j < AWPT; ++j) {
        const int64_t w = w0 + threadIdx.x + j * PAINTB;
        acc[j] = a.init ? (w < a.n_words ? a.words[w] : 0ull) : ~0ull;
    }
    paint_and_tile(a, t, 0u, img, acc);
#pragma unroll
    for (int j = 0; j < AWPT; ++j) {
        const int64_t w = w0 + threadIdx.x + j * PAINTB;
        if (w < a.n_words) a.words[w] = acc[j];
    }
}

// words = (init ? words : all ones) & AND of up to MAXK bitsets (chains a
// k-way AND past 16 operands)
struct WordsAnd {
    const uint64_t *w[MAXK];
    int k;
};
__global__ __launch_bounds__(BB) void k_and_words(WordsAnd a, int init, uint64_t *__restrict__ out,
                                                  int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * BB + threadIdx.x; i < n; i += (int64_t)gridDim.x * BB) {
        uint64_t x = init ? out[i] : ~0ull;
        for (int q = 0; q < a.k; ++q) x &= a.w[q][i];
        out[i] = x;
    }
}

struct OpArgs {
    const uint64_t *w[MAXK];
    int k;
    int op;  // 0 a, 1 not a, 2 a & b, 3 a & ~b, 4 and of k
    int64_t n_words;
    int64_t word0;        // global index of word 0 (a shard's window)
    int64_t span;
    const uint32_t *off;  // contig offsets (nc + 1): contig c's pad bit is off[c + 1] - 1
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

// the events of word x after `prev` (whose top bit precedes x's bit 0): bit
// i where x_i != x_(i-1) -- a run start where x_i is set, an end where it is
// clear; starts and ends alternate, so their order tells them apart and one
// mask (one xor, one popcount) serves both)
__device__ __forceinline__ uint64_t event_bits(uint64_t x, uint64_t prev) {
    return x ^ ((x << 1) | (prev >> 63));
}

// NOT within contigs: clear the pad bits and every bit past the window
__device__ __forceinline__ uint64_t not_mask(const OpArgs &a, int64_t w, uint64_t x,
                                             const uint32_t *s_pad, int npad) {
    const int64_t b0 = (a.word0 + w) * 64;
    if (b0 + 64 > a.span) {
        const int64_t keep = a.span - b0;
        x &= keep <= 0 ? 0ull : (keep >= 64 ? ~0ull : ((1ull << keep) - 1));
    }
    for (int p = 0; p < npad; ++p) {
        const int64_t d = (int64_t)s_pad[p] - b0;
        if (d >= 0 && d < 64) x &= ~(1ull << d);
    }
    return x;
}

// word pairs (w, w + 1), w = w0 + 2 (t + j BB): 16-B loads, all issued
// before any is used (0 past the window)
// Tile images in LDS hold word q of [w0 - 1, w0 + TW) at ipad(q): one pad
// word after every 16, so the blocked readers (thread t: words 16 t ..
// 16 t + 16, a 128-B lane stride) spread over the banks instead of all
// hitting one (SQ_LDS_BANK_CONFLICT was 69% of the extraction's LDS cycles)
__device__ __forceinline__ int ipad(int q) { return q + (q >> 4); }
constexpr int img_words(int tw) { return tw + 1 + (tw + 1) / 16 + 1; }

// (NT threads staging a tile of TW words; defaults: the BB x BW tiles)
template <int NT = BB, int TW = BT>
__device__ __forceinline__ void load_pairs(const uint64_t *__restrict__ src, int64_t w0,
                                           int64_t nw, uint64_t (&x0)[TW / (2 * NT)],
                                           uint64_t (&x1)[TW / (2 * NT)]) {
    constexpr int SJ = TW / (2 * NT);
#pragma unroll
    for (int j = 0; j < SJ; ++j) {
        const int64_t w = w0 + 2 * (threadIdx.x + (int64_t)j * NT);
        if (w + 1 < nw) {
            const ulonglong2 v = *reinterpret_cast<const ulonglong2 *>(src + w);
            x0[j] = v.x;
            x1[j] = v.y;
        } else {
            x0[j] = w < nw ? src[w] : 0ull;
            x1[j] = 0ull;
        }
    }
}

// Stage op(words) of tile [w0, w0 + BT) plus the word before it into LDS
// (img[0] = word w0 - 1).  NOT clears pad bits and bits beyond the span.
// Every operand's 16 words per thread are loaded as 8 independent 16-B
// loads, combined in registers, then stored to LDS once.
template <int NT = BB, int TW = BT>
__device__ __forceinline__ void stage_tile(const OpArgs &a, int64_t w0, unsigned long long *img,
                                           uint32_t *s_pad, int *s_npad) {
    constexpr int SJ = TW / (2 * NT);
    if (a.op == 1 && threadIdx.x == 0) {
        const int64_t lo = (a.word0 + (w0 > 0 ? w0 - 1 : 0)) * 64, hi = (a.word0 + w0 + TW) * 64;
        // first contig whose pad bit off[c + 1] - 1 is >= lo
        int64_t c = dev::lower_bound(a.off + 1, 0, (int64_t)a.nc, (uint64_t)lo + 1);
        int np = 0;
        for (; c < a.nc && (int64_t)a.off[c + 1] - 1 < hi && np < MAXPAD; ++c)
            s_pad[np++] = a.off[c + 1] - 1;
        *s_npad = np;
    }
    const int64_t nw = a.n_words;
    uint64_t x0[SJ], x1[SJ];
    load_pairs<NT, TW>(a.w[0], w0, nw, x0, x1);
    const int nops = a.op == 4 ? a.k : (a.op >= 2 ? 2 : 1);
    for (int i = 1; i < nops; ++i) {
        uint64_t y0[SJ], y1[SJ];
        load_pairs<NT, TW>(a.w[i], w0, nw, y0, y1);
#pragma unroll
        for (int j = 0; j < SJ; ++j) {
            x0[j] &= a.op == 3 ? ~y0[j] : y0[j];
            x1[j] &= a.op == 3 ? ~y1[j] : y1[j];
        }
    }
    // the word before the tile (its events' left neighbour)
    uint64_t xb = 0;
    if (threadIdx.x == 0 && w0 > 0 && w0 - 1 < nw) xb = op_raw(a, w0 - 1);
    __syncthreads();  // s_pad
    if (a.op == 1) {
        const int npad = *s_npad;
#pragma unroll
        for (int j = 0; j < SJ; ++j) {
            const int64_t w = w0 + 2 * (threadIdx.x + (int64_t)j * NT);
            x0[j] = w < nw ? not_mask(a, w, ~x0[j], s_pad, npad) : 0ull;
            x1[j] = w + 1 < nw ? not_mask(a, w + 1, ~x1[j], s_pad, npad) : 0ull;
        }
        if (threadIdx.x == 0 && w0 > 0 && w0 - 1 < nw) xb = not_mask(a, w0 - 1, xb, s_pad, npad);
    }
#pragma unroll
    for (int j = 0; j < SJ; ++j) {
        const int q = 2 * (threadIdx.x + j * NT);
        img[ipad(q + 1)] = x0[j];
        img[ipad(q + 2)] = x1[j];
    }
    if (threadIdx.x == 0) img[0] = xb;
    __syncthreads();
}

__global__ __launch_bounds__(BB) void k_ev_count(OpArgs a, uint32_t *__restrict__ tcnt) {
    __shared__ unsigned long long img[img_words(BT)];
    __shared__ uint32_t s_pad[MAXPAD];
    __shared__ int s_npad;
    __shared__ uint32_t ws[BB / 64];
    const int64_t w0 = (int64_t)blockIdx.x * BT;
    stage_tile(a, w0, img, s_pad, &s_npad);
    uint32_t c = 0;
    for (int i = threadIdx.x; i < BT; i += BB) {
        c += __popcll(event_bits(img[ipad(i + 1)], img[ipad(i)]));
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
    __shared__ unsigned long long img[img_words(BT)];
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
        c += __popcll(event_bits(img[ipad(q0 + k + 1)], img[ipad(q0 + k)]));
    }
    uint32_t tot;
    uint32_t ev = toff[blockIdx.x] + dev::block_exclusive_sum<BB>(c, scratch, &tot);
#pragma unroll
    for (int k = 0; k < BW; ++k) {
        uint64_t all = event_bits(img[ipad(q0 + k + 1)], img[ipad(q0 + k)]);
        const uint32_t base = (uint32_t)((a.word0 + w0 + q0 + k) * 64);
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

// Tile geometry of the one-pass extraction: EV_NT threads x EV_W words.
// Fewer, larger tiles mean fewer serial look-backs (as for k_merge_scan)
#ifndef LIME_EV_NT
#define LIME_EV_NT 256
#endif
// 8 words per thread (2048-word tiles, 2048-event slots: the same events per
// word as 16 / 4096): C4's extraction 0.445 -> 0.42 ms (twice the tiles, a
// shorter tail); 32 words: 0.465 ms (profiles/round3l_ev_geometry_ab.txt)
#ifndef LIME_EV_W
#define LIME_EV_W 8
#endif
#ifndef LIME_EVCAP
#define LIME_EVCAP 2048
#endif
constexpr int EV_NT = LIME_EV_NT, EV_W = LIME_EV_W, EV_TW = EV_NT * EV_W;
constexpr int EVCAP = LIME_EVCAP;  // events of a tile staged in LDS
constexpr int EVSLOT_MAX = 2 * TWORDS;  // k_paint_ev's largest slot (staged in its image)

}  // namespace

// Look-back-free extraction: every tile writes its events to its own slot
// of EVCAP events (staged in LDS, stored lane-consecutively) and its count;
// a scan of the counts then places them (k_ev_gather).  Nothing waits on a
// predecessor, so the pass runs at the rate of the count pass; a tile with
// more than EVCAP events raises *oflow and the host takes the two-pass path.
// The tile is held in registers, not staged in LDS: thread t loads its
// EV_W consecutive words (16-B loads, every operand combined as it lands),
// the word before a lane's first is the previous lane's last (DPP shift;
// across waves one LDS word per wave; before the tile one global read), and
// only the events go through LDS (for lane-consecutive slot stores).  (The
// LDS-staged tile image held the kernel to 3 workgroups per CU: 2.3-4.6
// TB/s.)
__global__ __launch_bounds__(EV_NT) void k_ev_local(OpArgs a, uint32_t *__restrict__ tev,
                                                    uint32_t *__restrict__ tcnt,
                                                    unsigned int *__restrict__ oflow) {
    constexpr int NW = EV_NT / 64;
    __shared__ uint32_t s_pad[MAXPAD];
    __shared__ int s_npad;
    __shared__ uint64_t s_last[NW];
    __shared__ uint32_t scratch[EV_NT / 64 + 1];
    __shared__ uint32_t s_ev[EVCAP];
    const uint32_t tile = blockIdx.x;
    const int64_t w0 = (int64_t)tile * EV_TW;
    const int64_t nw = a.n_words;
    const int w = threadIdx.x / 64, lane = dev::lane_id();
    const int64_t q0 = w0 + (int64_t)threadIdx.x * EV_W;  // the thread's first word
    if (a.op == 1 && w == 0) {  // NOT: the contig pads of the tile, by wave 0
        // (a 65-ary search, then lane l tests the l-th pad from there: the
        // serial binary search by one lane cost C4's complement ~15 us)
        const int64_t lo = (a.word0 + (w0 > 0 ? w0 - 1 : 0)) * 64, hi = (a.word0 + w0 + EV_TW) * 64;
        static_assert(MAXPAD == 64, "one pad per lane");
        const int64_t c = dev::wave_lower_bound(a.off + 1, (int64_t)a.nc, lo + 1) + lane;
        const int64_t pad = c < a.nc ? (int64_t)a.off[c + 1] - 1 : INT64_MAX;
        const bool in = pad < hi;  // (pads ascend: a prefix of the lanes)
        const uint64_t m = __ballot(in);
        if (in) s_pad[lane] = (uint32_t)pad;
        if (lane == 0) s_npad = __popcll(m);
    }
    uint64_t x[EV_W];
    const int nops = a.op == 4 ? a.k : (a.op >= 2 ? 2 : 1);
    for (int i = 0; i < nops; ++i) {
        const uint64_t *src = a.w[i];
#pragma unroll
        for (int k = 0; k < EV_W; k += 2) {
            const int64_t wd = q0 + k;
            uint64_t y0, y1;
            if (wd + 1 < nw) {
                const ulonglong2 v = *reinterpret_cast<const ulonglong2 *>(src + wd);
                y0 = v.x;
                y1 = v.y;
            } else {
                y0 = wd < nw ? src[wd] : 0ull;
                y1 = 0ull;
            }
            if (i == 0) {
                x[k] = y0;
                x[k + 1] = y1;
            } else {
                x[k] &= a.op == 3 ? ~y0 : y0;
                x[k + 1] &= a.op == 3 ? ~y1 : y1;
            }
        }
    }
    // the word before the tile (thread 0's left neighbour)
    uint64_t xb = 0;
    if (threadIdx.x == 0 && w0 > 0 && w0 - 1 < nw) xb = op_raw(a, w0 - 1);
    __syncthreads();  // s_pad
    if (a.op == 1) {
        const int npad = s_npad;
#pragma unroll
        for (int k = 0; k < EV_W; ++k)
            x[k] = q0 + k < nw ? not_mask(a, q0 + k, ~x[k], s_pad, npad) : 0ull;
        if (threadIdx.x == 0 && w0 > 0 && w0 - 1 < nw) xb = not_mask(a, w0 - 1, xb, s_pad, npad);
    }
    // left neighbour of the thread's first word
    if (lane == 63) s_last[w] = x[EV_W - 1];
    uint64_t prev = dev::wave_shr1(x[EV_W - 1], (uint64_t)0);
    __syncthreads();
    if (lane == 0) prev = w > 0 ? s_last[w - 1] : xb;
    uint32_t c = 0;
    {
        uint64_t p = prev;
#pragma unroll
        for (int k = 0; k < EV_W; ++k) {
            c += __popcll(event_bits(x[k], p));
            p = x[k];
        }
    }
    uint32_t tot;
    const uint32_t mine = dev::block_exclusive_sum<EV_NT>(c, scratch, &tot);
    if (threadIdx.x == 0) {
        tcnt[tile] = tot;
        if (tot > (uint32_t)EVCAP) atomicOr(oflow, 1u);
    }
    if (tot > (uint32_t)EVCAP) return;
    uint32_t le = mine;
    {
        uint64_t p = prev;
#pragma unroll
        for (int k = 0; k < EV_W; ++k) {
            uint64_t all = event_bits(x[k], p);
            p = x[k];
            const uint32_t base = (uint32_t)((a.word0 + q0 + k) * 64);
            while (all) {
                const int b = __builtin_ctzll(all);
                all &= all - 1;
                s_ev[le++] = base + (uint32_t)b;
            }
        }
    }
    __syncthreads();
    uint32_t *dst = tev + (size_t)tile * EVCAP;
    for (uint32_t i = threadIdx.x; i < tot; i += EV_NT) dst[i] = s_ev[i];
}

// events of tile t (slot t of k_ev_local) -> run starts (even event index)
// and ends (odd) at the tile's scanned offset; one workgroup per tile
// (launched before the host has seen the totals: nothing is written when a
// tile overflowed its slot, hdr[0], or past the result's capacity)
// (k_paint_ev's slots: `slot` events each, the first skipped where skip1)
__global__ __launch_bounds__(256) void k_ev_gather(const uint32_t *__restrict__ tev,
                                                   const uint32_t *__restrict__ tcnt,
                                                   const uint32_t *__restrict__ toff,
                                                   const unsigned int *__restrict__ hdr,
                                                   uint32_t cap_events,
                                                   uint32_t *__restrict__ rgs,
                                                   uint32_t *__restrict__ rge,
                                                   uint32_t slot = EVCAP,
                                                   const uint32_t *__restrict__ skip1 = nullptr) {
    if (hdr[0]) return;
    const uint32_t t = blockIdx.x;
    const uint32_t e0 = toff[t];
    const uint32_t n = min(tcnt[t], e0 < cap_events ? cap_events - e0 : 0u);
    const uint32_t *src = tev + (size_t)t * slot + (skip1 ? skip1[t] : 0u);
    for (uint32_t i = threadIdx.x; i < n; i += 256) {
        const uint32_t e = e0 + i, p = src[i];
        if (e & 1u)
            rge[e >> 1] = p;
        else
            rgs[e >> 1] = p;
    }
}

// --------------------------------- runs straight from binned operands
// Bitsets built from rows stay binned (their rows grouped by paint tile,
// bitset_build_rows) until words are needed; an op's runs over binned
// operands fuse the paint with the extraction: per paint tile the operands'
// rows are painted in LDS and combined in registers (paint_and_tile, the
// complemented operand of a & ~b or ~a entering inverted), the result is
// staged back into LDS and its events found there -- no bitset stored or
// re-read (C4: two 386 MB bitsets written and three read by the two
// extractions).  A tile's events go to its own slot of `cap`, counted with
// the bit before the tile taken as 0 and a run reaching the tile's end
// closed there; k_ev_join then drops the two events of every run that
// crosses a tile boundary (the close and the reopening) before the scan.
struct PaintEvArgs {
    int64_t n_words;      // the window's words
    uint32_t neg;         // bit i: operand i complemented (k_paint_ev)
    int notmask;          // not a: clear the contig pads and the bits past the window
    int64_t word0;        // global index of the window's word 0
    int64_t hi_bit;       // end of the window (global bits)
    const uint32_t *off;  // contig offsets (nc + 1): contig c's pad bit is off[c + 1] - 1
    int32_t nc;
    uint32_t *tev;        // nt slots of `cap` events
    uint32_t cap;
    uint32_t *tcnt;       // events of each tile
    uint32_t *edge;       // bit 0: the tile's first bit, bit 1: its last, bit 2: past `cap`
    unsigned int *oflow;  // zeroed by block 0; k_ev_join raises it (no memset launch)
};
constexpr int PEW = TWORDS / PAINTB;  // consecutive words per thread (extraction)

// One output's events of tile t from its words acc (thread: words
// threadIdx.x + j PAINTB), as described above; img / scratch / s_last: the
// kernel's LDS.  (pc, pad): wave 0's prefetched first 64 contig pads of the
// tile (NOT only).  Ends with a barrier: img is free again.
// (word j of the thread: wj(j))
template <class WJ>
__device__ __forceinline__ void tile_events(const PaintEvArgs &a, int t, WJ wj,
                                            unsigned long long *img, uint32_t *scratch,
                                            uint32_t &s_last, int64_t pc, int64_t pad) {
    const int64_t nw = a.n_words;
    const int64_t w0 = (int64_t)t * TWORDS;
    const int64_t plo = (a.word0 + w0) * 64, phi = plo + (int64_t)TWORDS * 64;
    // (only a tile reaching past the window's last word or bit tests its
    // words: a tile-uniform branch)
    const bool edge = w0 + TWORDS > nw || (a.notmask && (a.word0 + w0 + TWORDS) * 64 > a.hi_bit);
#pragma unroll
    for (int j = 0; j < AWPT; ++j) {
        const int q = threadIdx.x + j * PAINTB;
        uint64_t x = wj(j);
        if (edge) {
            if (w0 + q >= nw) x = 0ull;
            if (a.notmask) {  // nothing past the window
                const int64_t b0 = (a.word0 + w0 + q) * 64;
                if (b0 + 64 > a.hi_bit) {
                    const int64_t keep = a.hi_bit - b0;
                    x &= keep <= 0 ? 0ull : ((1ull << keep) - 1);
                }
            }
        }
        img[ipad(q)] = x;
    }
    __syncthreads();
    if (a.notmask) {
        // the contig pads inside the tile, cleared 64 at a time by wave 0
        // (the pads ascend: a batch not wholly inside the tile is the last)
        if (threadIdx.x < 64) {
            for (int64_t c = pc; c < a.nc; c += 64) {
                if (c != pc) {
                    const int64_t cc = c + threadIdx.x;
                    pad = cc < a.nc ? (int64_t)a.off[cc + 1] - 1 : INT64_MAX;
                }
                const bool in = pad < phi;
                if (in) {
                    const int64_t q = pad - plo;
                    atomicAnd(&img[ipad((int)(q >> 6))], ~(1ull << (q & 63)));
                }
                if (__ballot(in) != ~0ull) break;
            }
        }
        __syncthreads();
    }
    const int q0 = threadIdx.x * PEW;
    uint64_t x[PEW];
#pragma unroll
    for (int k = 0; k < PEW; ++k) x[k] = img[ipad(q0 + k)];
    const uint64_t prev = q0 > 0 ? img[ipad(q0 - 1)] : 0ull;
    uint32_t c = 0;
    {
        uint64_t p = prev;
#pragma unroll
        for (int k = 0; k < PEW; ++k) {
            c += __popcll(event_bits(x[k], p));
            p = x[k];
        }
    }
    // a run reaching the tile's end closes there (k_ev_join reopens it)
    const bool close = threadIdx.x == PAINTB - 1 && (x[PEW - 1] >> 63) != 0;
    if (threadIdx.x == PAINTB - 1) s_last = close;
    c += close;
    uint32_t tot;
    // (its barriers also end every read of img: the events are staged there)
    const uint32_t mine = dev::block_exclusive_sum<PAINTB>(c, scratch, &tot);
    if (threadIdx.x == 0) {
        a.tcnt[t] = tot;
        a.edge[t] = (uint32_t)(x[0] & 1ull) | s_last << 1 | (tot > a.cap ? 4u : 0u);
    }
    if (tot <= a.cap) {  // (block-uniform)
        // events staged in LDS, then stored lane-consecutively
        uint32_t *dst = reinterpret_cast<uint32_t *>(img);
        uint32_t e = mine;
        const uint32_t base = (uint32_t)((a.word0 + w0 + q0) * 64);
        uint64_t p = prev;
#pragma unroll
        for (int k = 0; k < PEW; ++k) {
            uint64_t all = event_bits(x[k], p);
            p = x[k];
            while (all) {
                const int b = __builtin_ctzll(all);
                all &= all - 1;
                dst[e++] = base + (uint32_t)(64 * k + b);
            }
        }
        if (close) dst[e] = (uint32_t)((a.word0 + w0 + TWORDS) * 64);
        __syncthreads();
        uint32_t *slot = a.tev + (size_t)t * a.cap;
        for (uint32_t i = threadIdx.x; i < tot; i += PAINTB) slot[i] = dst[i];
    }
    __syncthreads();
}

// the pads of a NOT (wave 0, before the paint: their round trips overlap it)
__device__ __forceinline__ void prefetch_pads(const PaintEvArgs &a, int t, int64_t &pc,
                                              int64_t &pad) {
    pc = 0;
    pad = INT64_MAX;
    if (threadIdx.x < 64) {
        const int64_t plo = (a.word0 + (int64_t)t * TWORDS) * 64;
        pc = dev::wave_lower_bound(a.off + 1, (int64_t)a.nc, plo + 1);
        const int64_t cc = pc + threadIdx.x;
        pad = cc < a.nc ? (int64_t)a.off[cc + 1] - 1 : INT64_MAX;
    }
}

__global__ __launch_bounds__(PAINTB) void k_paint_ev(PaintEvArgs a, AndArgs s) {
    __shared__ unsigned long long img[img_words(TWORDS)];
    __shared__ uint32_t scratch[PAINTB / 64 + 1];
    __shared__ uint32_t s_last;
    static_assert(EVSLOT_MAX * 4 <= sizeof(img), "the event slot (<= EVSLOT_MAX) staged in img");
    const int t = blockIdx.x;
    if (t == 0 && threadIdx.x == 0) *a.oflow = 0u;  // (raised by k_ev_join, a later launch)
    uint64_t acc[AWPT];
#pragma unroll
    for (int j = 0; j < AWPT; ++j) acc[j] = ~0ull;
    int64_t pc = 0, pad = INT64_MAX;
    if (a.notmask) prefetch_pads(a, t, pc, pad);
    paint_and_tile(s, t, a.neg, img, acc);
    __syncthreads();  // img again, in the extraction's padded layout
    tile_events(a, t, [&](int j) { return acc[j]; }, img, scratch, s_last, pc, pad);
}

// a run crossing the boundary of tiles t and t + 1 was closed at the end of
// t and reopened at the start of t + 1: both events dropped (cnt2 = the
// kept events, skip1 = whether the slot's first event is dropped)
__global__ __launch_bounds__(256) void k_ev_join(const uint32_t *__restrict__ tcnt,
                                                 const uint32_t *__restrict__ edge, int64_t nt,
                                                 uint32_t *__restrict__ cnt2,
                                                 uint32_t *__restrict__ skip1,
                                                 unsigned int *__restrict__ oflow) {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= nt) return;
    const uint32_t e = edge[t];
    if (e & 4u) *oflow = 1u;  // a tile past its slot (plain store: idempotent)
    const uint32_t jp = t > 0 && (edge[t - 1] & 2u) && (e & 1u);
    const uint32_t jn = t + 1 < nt && (e & 2u) && (edge[t + 1] & 1u);
    cnt2[t] = tcnt[t] - jp - jn;
    skip1[t] = jp;
}

int merge_runs(lime_ctx *ctx, const lime_set *set, lime_result *res, bool want_run_ids);

int bitset_build(lime_ctx *ctx, const lime_set *a, lime_bitset *bs) {
    lime_result runs;
    runs.ctx = ctx;
    LIME_TRY(merge_runs(ctx, a, &runs, false));
    bs->runs_bound = runs.n;
    const int64_t span = (int64_t)a->off[a->n_contigs];
    bs->span = span;
    bs->hi_bit = span;
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

namespace {
// pool blocks released on every return path (a set of PoolGuards)
struct PoolBag {
    lime_ctx *ctx;
    std::vector<void *> ps;
    template <typename T>
    int get(T **p, size_t count) {
        LIME_TRY(alloc(ctx, p, count));
        ps.push_back((void *)*p);
        return LIME_OK;
    }
    ~PoolBag() {
        for (void *p : ps) release(ctx, p);
    }
};

int rows_error(unsigned int e) {
    if (e & 1u) return fail(LIME_ERR_CONTIG, "interval contig id outside the space");
    if (e & 2u) return fail(LIME_ERR_RANGE, "interval end < start");
    if (e & 4u) return fail(LIME_ERR_RANGE, "interval end beyond its contig length");
    return LIME_OK;
}

int n_bins(int64_t width) {
    return (int)std::max<int64_t>((width + (1ll << BSH) - 1) >> BSH, 1);
}

// rows -> their paint tiles' packed rows (slab2, tile order) and the tile
// starts (ttot, nt + 1 entries); pieces left to the cross list are appended
// to `cross` (capacity 2 n: a row leaves at most its bin remainder and its
// tile-crossing remainder), flags[0] counts them and flags[1] collects the
// row errors.  Enqueued on the context stream only: no host sync.
int bin_rows(lime_ctx *ctx, const lime_space *sp, int64_t n, const int32_t *d_contig,
             const uint32_t *d_start, const uint32_t *d_end, const uint32_t *d_off,
             const uint32_t *d_len, int64_t lo, int64_t hi, uint32_t *slab2, uint32_t *ttot,
             uint64_t *cross, unsigned int *flags, uint32_t *xbz = nullptr,
             bool allow_opt = true) {
    const int nb = n_bins(hi - lo);
    const int nt = nb * PSUB;
    // chunk: 1..16 count steps; as many chunks as whole rounds of the write
    // pass's resident workgroups (`cus`: per CU x CUs) need, so its last round is not
    // a small tail (1e7 rows: 204 chunks in one round, not 306 in two)
    static const int64_t cus = [] {
        int dev = 0, c = 256, occ = 1;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev);
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_bin_write<true, true>, WRB, 0);
        return (int64_t)(c > 0 ? c : 256) * (occ > 0 ? occ : 1);
    }();
    const int64_t rounds = std::max<int64_t>((n + cus * 16 * STEP - 1) / (cus * 16 * STEP), 1);
    int64_t R = (n + cus * rounds - 1) / (cus * rounds);
    R = std::min<int64_t>(std::max<int64_t>(R, STEP), 16 * (int64_t)STEP);
    R = (R + STEP - 1) / STEP * STEP;
    const uint32_t nch = (uint32_t)std::max<int64_t>((n + R - 1) / R, 1);
    const int64_t mlen = (int64_t)nb * nch + 1;
    // split workgroups per bin: ~LIME_SPLIT_BLOCKS in all (one per bin left
    // the split at 42 serial 4096-row rounds per workgroup on C5's sets)
    const int ng = (int)std::min<int64_t>(std::max<int64_t>((LIME_SPLIT_BLOCKS + nb - 1) / nb, 1),
                                          std::min<int64_t>(nch, 16));
    // optimistic binning (no count pass; opt-in: LIME_BIN_OPTIMISTIC=1) when
    // the rows per (bin, chunk) are many enough that regions of mean + 6
    // sigma under the window's uniform density pad the slab by at most ~1.6x
    // (C5's sets: ~166 rows, 251 slots); rows clustered by input order
    // (sorted BED) overflow a region and the set is binned again through the
    // counted path (the caller sees ERR_REGION in its flags read-back),
    // which then stays the first choice for this context's next builds
    // (bin_pessimism).  Measured on C5, same box: the count pass's 223 us
    // per set went, but the write pass took 636 -> 804 us (a tile count per
    // row, the padding filled, the group totals added) and the split 267 ->
    // 331 us (padding read): 1126 vs 1135 us per set, so it is not the
    // default (profiles/round6/c5_optimistic_binning_*)
    const double E = (double)R * (double)(1ll << BSH) / (double)std::max<int64_t>(hi - lo, 1);
    uint32_t rcap = 0;
    const char *ov = getenv("LIME_BIN_OPTIMISTIC");  // (per call: tests set it at run time)
    const bool opt_on = ov && ov[0] == '1';
    if (allow_opt && opt_on && ctx->bin_pessimism == 0 && nb >= 8 && E >= 128.0) {
        const double c = std::ceil(E + 6.0 * std::sqrt(E)) + 8.0;
        const uint64_t cap = ((uint64_t)c + 3) / 4 * 4;
        if ((uint64_t)nb * nch * cap < 0xffff0000ull) rcap = (uint32_t)cap;
    }
    if (!rcap && ctx->bin_pessimism > 0) --ctx->bin_pessimism;
    if (getenv("LIME_TRACE_BINNING"))  // (read per call: tests set it at run time)
        fprintf(stderr, "lime: bin_rows n=%lld %s (rows per region %.0f, slots %u)\n",
                (long long)n, rcap ? "optimistic" : "counted", E, rcap);
    PoolBag bag{ctx, {}};
    uint32_t *mat, *slab, *dummy, *gsum, *gpre;
    LIME_TRY(bag.get(&mat, rcap ? 1 : (size_t)mlen));
    LIME_TRY(bag.get(&slab, rcap ? (size_t)nb * nch * rcap : (size_t)std::max<int64_t>(n, 1)));
    LIME_TRY(bag.get(&dummy, 64));
    LIME_TRY(bag.get(&gsum, (size_t)ng * (size_t)nt));
    LIME_TRY(bag.get(&gpre, (size_t)nt * (size_t)ng));
    if (n == 0) {
        LIME_HIP(hipMemsetAsync(mat, 0, 4 * (size_t)mlen, S(ctx)));
        LIME_HIP(hipMemsetAsync(ttot, 0, 4 * ((size_t)nt + 1), S(ctx)));
        LIME_HIP(hipMemsetAsync(flags, 0, 8, S(ctx)));
        if (xbz) LIME_HIP(hipMemsetAsync(xbz, 0, 4 * 3 * ((size_t)nt + 1), S(ctx)));
        return LIME_OK;
    }
    BinArgs a;
    a.contig = d_contig;
    a.start = d_start;
    a.end = d_end;
    a.off = d_off;
    a.len = d_len;
    a.nc = sp->n;
    a.n = n;
    a.lo = (uint32_t)lo;
    a.hi = (uint32_t)hi;
    a.span = (uint64_t)sp->span;
    a.nb = nb;
    a.chunk_rows = R;
    a.nchunks = nch;
    a.mat = mat;
    a.ttot = ttot;
    a.gsum = gsum;
    a.gpre = gpre;
    a.ngroups = ng;
    a.slab = slab;
    a.slab2 = slab2;
    a.cross = cross;
    a.ncross = flags;
    a.err = flags + 1;
    a.dummy = dummy;
    a.xbz = xbz;
    a.rcap = rcap;
    const bool lc = d_contig != nullptr && sp->n <= CMAX;
    LIME_HIP(hipMemsetAsync(gsum, 0, 4 * (size_t)ng * (size_t)nt, S(ctx)));
    if (rcap) {
        // write (tile totals counted on the way) -> tile groups -> split
        LIME_HIP(hipMemsetAsync(flags, 0, 8, S(ctx)));  // (k_bin_count zeroes them otherwise)
        if (lc)
            hipLaunchKernelGGL((k_bin_write<true, true, true>), dim3(nch), dim3(WRB), 0, S(ctx), a);
        else if (d_contig)
            hipLaunchKernelGGL((k_bin_write<false, true, true>), dim3(nch), dim3(WRB), 0, S(ctx), a);
        else
            hipLaunchKernelGGL((k_bin_write<false, false, true>), dim3(nch), dim3(WRB), 0, S(ctx), a);
        hipLaunchKernelGGL(k_tile_groups, dim3(blocks_for(nt + 1, 256)), dim3(256), 0, S(ctx), a);
        LIME_TRY(scan_exclusive_u32(ctx, ttot, ttot, (int64_t)nt + 1, nullptr));
        hipLaunchKernelGGL(k_bin_split_atomic<true>, dim3((unsigned)(nb * ng)), dim3(SPB), 0,
                           S(ctx), a);
        LIME_HIP(hipGetLastError());
        return LIME_OK;
    }
    if (lc)
        hipLaunchKernelGGL(k_bin_count<true>, dim3(nch), dim3(BINB), 0, S(ctx), a);
    else
        hipLaunchKernelGGL(k_bin_count<false>, dim3(nch), dim3(BINB), 0, S(ctx), a);
    hipLaunchKernelGGL(k_tile_groups, dim3(blocks_for(nt + 1, 256)), dim3(256), 0, S(ctx), a);
    // (the extra last entries receive the totals)
    LIME_TRY(scan_exclusive_u32(ctx, mat, mat, mlen, nullptr));
    LIME_TRY(scan_exclusive_u32(ctx, ttot, ttot, (int64_t)nt + 1, nullptr));
    if (lc)
        hipLaunchKernelGGL((k_bin_write<true, true>), dim3(nch), dim3(WRB), 0, S(ctx), a);
    else if (d_contig)
        hipLaunchKernelGGL((k_bin_write<false, true>), dim3(nch), dim3(WRB), 0, S(ctx), a);
    else
        hipLaunchKernelGGL((k_bin_write<false, false>), dim3(nch), dim3(WRB), 0, S(ctx), a);
    // the atomic-claim split (C5 12.05 -> 11.73 ms against a ballot-ranked one)
    hipLaunchKernelGGL(k_bin_split_atomic<false>, dim3((unsigned)(nb * ng)), dim3(SPB), 0, S(ctx),
                       a);
    LIME_HIP(hipGetLastError());
    return LIME_OK;
}

void window_of(lime_bitset *bs, const lime_space *sp, int64_t lo, int64_t hi) {
    bs->span = sp->span;
    bs->word0 = lo / 64;
    bs->hi_bit = hi;
    bs->n_words = (hi - lo + 63) / 64;
}
}  // namespace

namespace {
// set's cross pieces (nx, in `cross`) bucketed by paint tile: xb = [bucket
// starts | difference-array scan (tiles wholly covered) | fill claims], each
// tstride long (zeroed here), xl = the 2 nx piece slots
int bucket_cross(lime_ctx *ctx, int64_t tstride, const uint64_t *cross,
                 const unsigned int *d_ncross, unsigned int nx, uint32_t *xb, uint2 *xl,
                 bool zeroed = false) {
    uint32_t *xcnt = xb, *diff = xb + tstride, *xfill = xb + 2 * tstride;
    // (zeroed: by the set's k_tile_groups, before the host's read-back)
    if (!zeroed) LIME_HIP(hipMemsetAsync(xb, 0, 4 * 3 * (size_t)tstride, S(ctx)));
    const unsigned g = std::min<unsigned>(blocks_for(nx, BB), 2048u);
    hipLaunchKernelGGL(k_xcount, dim3(g), dim3(BB), 0, S(ctx), cross, d_ncross, xcnt, diff);
    LIME_TRY(scan_exclusive_u32_pair(ctx, xcnt, xcnt, tstride, diff, diff, tstride));
    hipLaunchKernelGGL(k_xwrite, dim3(g), dim3(BB), 0, S(ctx), cross, d_ncross,
                       (const uint32_t *)xcnt, xfill, xl);
    LIME_HIP(hipGetLastError());
    return LIME_OK;
}

// paint arguments over binned row sets (k <= MAXK, nt tiles each)
template <int CAP = MAXK>
AndArgsK<CAP> binned_args(const lime_bitset::Bins *const *b, int k, int64_t nt, int64_t n_words) {
    AndArgsK<CAP> aa;
    for (int i = 0; i < CAP; ++i) {
        const bool v = i < k;
        aa.slab2[i] = v ? b[i]->slab2 : nullptr;
        aa.tstart[i] = v ? b[i]->tstart : nullptr;
        aa.xl[i] = v ? b[i]->xl : nullptr;
        aa.xoff[i] = v && b[i]->xl ? b[i]->xb : nullptr;
        aa.full[i] = v && b[i]->xl ? b[i]->xb + nt + 1 : nullptr;
    }
    aa.k = k;
    aa.init = 0;
    aa.words = nullptr;
    aa.n_words = n_words;
    return aa;
}

// one row set binned by paint tile into `b` (owned by the bitset): its rows
// grouped (bin_rows), the row errors checked, its cross pieces bucketed
int bin_set(lime_ctx *ctx, const lime_space *sp, int64_t n, const int32_t *d_contig,
            const uint32_t *d_start, const uint32_t *d_end, const uint32_t *d_off,
            const uint32_t *d_len, int64_t lo, int64_t hi, int64_t nt, lime_bitset::Bins &b) {
    LIME_TRY(alloc(ctx, &b.tstart, (size_t)nt + 1));
    LIME_TRY(alloc(ctx, &b.slab2, (size_t)std::max<int64_t>(n, 1)));
    PoolBag bag{ctx, {}};
    uint64_t *cross;
    unsigned int *flags;  // [0] ncross, [1] err (zeroed by k_bin_count)
    LIME_TRY(bag.get(&cross, (size_t)std::max<int64_t>(2 * n, 1)));
    LIME_TRY(bag.get(&flags, 2));
    // the cross buckets allocated (and zeroed on the device) before the
    // read-back: after it only the bucketing launches remain
    LIME_TRY(alloc(ctx, &b.xb, 3 * ((size_t)nt + 1)));
    LIME_TRY(bin_rows(ctx, sp, n, d_contig, d_start, d_end, d_off, d_len, lo, hi, b.slab2,
                      b.tstart, cross, flags, b.xb));
    unsigned int h[2] = {0, 0};
    LIME_TRY(read_back(ctx, h, flags, sizeof(h)));
    LIME_TRY(rows_error(h[1]));
    if (h[1] & ERR_REGION) {  // an optimistic region overflowed: the counted path
        if (getenv("LIME_TRACE_BINNING")) fprintf(stderr, "lime: region overflow, counted again\n");
        ctx->bin_pessimism = 32;
        LIME_TRY(bin_rows(ctx, sp, n, d_contig, d_start, d_end, d_off, d_len, lo, hi, b.slab2,
                          b.tstart, cross, flags, b.xb, false));
        LIME_TRY(read_back(ctx, h, flags, sizeof(h)));
        LIME_TRY(rows_error(h[1]));
    }
    if (h[0]) {
        LIME_TRY(alloc(ctx, &b.xl, 2 * (size_t)h[0]));
        LIME_TRY(bucket_cross(ctx, nt + 1, cross, flags, h[0], b.xb, b.xl, true));
    } else {
        release(ctx, b.xb);  // (stream-ordered; the ops take xb only with xl)
    }
    return LIME_OK;
}
}  // namespace

void bitset_free(lime_bitset *bs) {
    lime_ctx *ctx = bs->ctx;
    release(ctx, bs->words);
    bs->words = nullptr;
    for (auto &b : bs->bins) {
        release(ctx, b.slab2);
        if (b.own_tstart) release(ctx, b.tstart);
        release(ctx, b.xl);
        release(ctx, b.xb);
    }
    bs->bins.clear();
}

// bits straight from UNSORTED device rows, no sort, no merge: the rows are
// binned by paint tile (k_bin_count / k_bin_write / k_bin_split, their cross
// pieces bucketed by tile) and kept so; the words are painted on first need
// (bitset_paint), or never when an op's runs come straight from the bins
// (k_paint_ev).  Window [lo, hi) of the space's global bits (lo % 64 == 0):
// the whole space, or a coordinate shard's range (rows clipped to it)
int bitset_build_rows(lime_ctx *ctx, const lime_space *sp, int64_t n, const int32_t *d_contig,
                      const uint32_t *d_start, const uint32_t *d_end, const uint32_t *d_off,
                      const uint32_t *d_len, int64_t lo, int64_t hi, lime_bitset *bs) {
    window_of(bs, sp, lo, hi);
    bs->runs_bound = n;  // the union of n rows has at most n runs
    bs->nt = n_bins(hi - lo) * PSUB;
    bs->bins.resize(1);
    return bin_set(ctx, sp, n, d_contig, d_start, d_end, d_off, d_len, lo, hi, bs->nt,
                   bs->bins[0]);
}

// the words of a binned bitset, painted once: k_paint_and over its sets
// (groups of MAXK, each ANDing into the words the earlier ones stored)
int bitset_paint(lime_ctx *ctx, const lime_bitset *cbs) {
    lime_bitset *bs = const_cast<lime_bitset *>(cbs);  // (a cache: the bits are unchanged)
    if (bs->words || bs->bins.empty()) return LIME_OK;
    // painted into a local buffer, published only once every group has been
    // queued without error (a failed paint must not leave words that later
    // calls would take as valid)
    uint64_t *words = nullptr;
    LIME_TRY(alloc(ctx, &words, (size_t)std::max<int64_t>(bs->n_words, 1)));
    PoolGuard<uint64_t> guard{ctx, words};
    const int k = (int)bs->bins.size();
    for (int g0 = 0; g0 < k; g0 += MAXK) {
        std::vector<const lime_bitset::Bins *> b;
        for (int i = g0; i < std::min(k, g0 + MAXK); ++i) b.push_back(&bs->bins[i]);
        AndArgs aa = binned_args(b.data(), (int)b.size(), bs->nt, bs->n_words);
        aa.init = g0 > 0;
        aa.words = words;
        if (bs->nt > 0)
            hipLaunchKernelGGL(k_paint_and, dim3((unsigned)bs->nt), dim3(PAINTB), 0, S(ctx), aa);
        LIME_HIP(hipGetLastError());
    }
    bs->words = words;
    guard.p = nullptr;  // (owned by the bitset from here)
    return LIME_OK;
}

// the words painted (if not yet) and the binned rows released: the bitset
// then holds span / 8 bytes, and every op reads its words
int bitset_drop_bins(lime_ctx *ctx, lime_bitset *bs) {
    LIME_TRY(bitset_paint(ctx, bs));
    for (auto &b : bs->bins) {
        release(ctx, b.slab2);
        if (b.own_tstart) release(ctx, b.tstart);
        release(ctx, b.xl);
        release(ctx, b.xb);
    }
    bs->bins.clear();
    return LIME_OK;
}

// the AND of k row sets' bits over window [lo, hi), straight from their
// unsorted rows: every set binned (bin_rows) and kept, so the bitset is
// their AND in binned form -- its runs come from one k_paint_ev over all the
// sets (k <= MAXK), its words, when needed, from k_paint_and (bitset_paint).
// rows[i] = (n, contig or null for global rows, start, end)
int bitset_and_rows(lime_ctx *ctx, const lime_space *sp, int k, const int64_t *n,
                    const int32_t *const *d_contig, const uint32_t *const *d_start,
                    const uint32_t *const *d_end, const uint32_t *d_off, const uint32_t *d_len,
                    int64_t lo, int64_t hi, lime_bitset *bs) {
    if (k < 1) return fail(LIME_ERR_ARG, "at least one row set per AND");
    window_of(bs, sp, lo, hi);
    int64_t nmax = 0, bound = 0;
    for (int i = 0; i < k; ++i) {
        nmax = std::max(nmax, n[i]);
        bound += n[i];
    }
    bs->runs_bound = bound;  // each AND run starts at a run start of some set
    const int64_t nt = n_bins(hi - lo) * PSUB;
    bs->nt = nt;
    bs->bins.resize(k);
    PoolBag keep{ctx, {}};
    // two cross buffers: set q's rows are binned while set q - 1's cross
    // pieces are read back and bucketed, so the host waits on an event of set
    // q - 1 only and the stream never drains between sets
    uint64_t *cross[2];
    unsigned int *flags;
    LIME_TRY(keep.get(&cross[0], (size_t)std::max<int64_t>(2 * nmax, 1)));
    LIME_TRY(keep.get(&cross[1], (size_t)std::max<int64_t>(2 * nmax, 1)));
    LIME_TRY(keep.get(&flags, 2 * (size_t)k));  // (zeroed per set by its k_bin_count)
    // set q's (ncross, err) land in the upper half of the pinned scratch
    // (read_back uses the lower half)
    unsigned int *hflags = reinterpret_cast<unsigned int *>(static_cast<char *>(ctx->pinned) + 2048);
    struct Events {
        hipEvent_t e[2] = {nullptr, nullptr};
        ~Events() {
            for (hipEvent_t x : e)
                if (x) (void)hipEventDestroy(x);
        }
    } ev;
    for (int j = 0; j < 2; ++j)
        LIME_HIP(hipEventCreateWithFlags(&ev.e[j], hipEventDisableTiming));
    // every set's tile starts: one block (owned by set 0)
    const size_t tstride = (size_t)nt + 1;
    uint32_t *ttot_all;
    LIME_TRY(alloc(ctx, &ttot_all, tstride * (size_t)k));
    bs->bins[0].tstart = ttot_all;
    for (int i = 1; i < k; ++i) bs->bins[i].own_tstart = false;
    // bucket set q's cross pieces by tile (its flags were copied to the host
    // behind its binning; wait for that copy only)
    auto bucket = [&](int q) -> int {
        LIME_HIP(hipEventSynchronize(ev.e[q % 2]));
        unsigned int nx = hflags[2 * (q % 2)], err = hflags[2 * (q % 2) + 1];
        LIME_TRY(rows_error(err));
        if (err & ERR_REGION) {  // set q again through the counted path
            if (getenv("LIME_TRACE_BINNING"))
                fprintf(stderr, "lime: region overflow, counted again\n");
            ctx->bin_pessimism = 32;
            lime_bitset::Bins &b = bs->bins[q];
            LIME_TRY(bin_rows(ctx, sp, n[q], d_contig[q], d_start[q], d_end[q], d_off, d_len, lo,
                              hi, b.slab2, b.tstart, cross[q % 2], flags + 2 * q, b.xb, false));
            unsigned int h[2] = {0, 0};
            LIME_TRY(read_back(ctx, h, flags + 2 * q, sizeof(h)));
            LIME_TRY(rows_error(h[1]));
            nx = h[0];
        }
        lime_bitset::Bins &b = bs->bins[q];
        if (nx == 0) {
            release(ctx, b.xb);
            return LIME_OK;
        }
        LIME_TRY(alloc(ctx, &b.xl, 2 * (size_t)nx));
        return bucket_cross(ctx, (int64_t)tstride, cross[q % 2],
                            (const unsigned int *)(flags + 2 * q), nx, b.xb, b.xl, true);
    };
    for (int q = 0; q < k; ++q) {
        lime_bitset::Bins &b = bs->bins[q];
        b.tstart = ttot_all + tstride * (size_t)q;
        LIME_TRY(alloc(ctx, &b.slab2, (size_t)std::max<int64_t>(n[q], 1)));
        LIME_TRY(alloc(ctx, &b.xb, 3 * tstride));
        // (cross[q % 2] was last used by set q - 2, bucketed before this)
        LIME_TRY(bin_rows(ctx, sp, n[q], d_contig[q], d_start[q], d_end[q], d_off, d_len, lo, hi,
                          b.slab2, b.tstart, cross[q % 2], flags + 2 * q, b.xb));
        LIME_HIP(hipMemcpyAsync(hflags + 2 * (q % 2), flags + 2 * q, 8, hipMemcpyDeviceToHost,
                                S(ctx)));
        LIME_HIP(hipEventRecord(ev.e[q % 2], S(ctx)));
        if (q > 0) LIME_TRY(bucket(q - 1));
    }
    return bucket(k - 1);
}

namespace {
// op's runs over binned operands (sets[0..nin)), fused with their paint:
// k_paint_ev, k_ev_join, a scan, k_ev_gather.  *overflow: a tile had more
// events than its slot (the caller paints the operands and takes the words
// path; nothing is returned)
// one op's extraction from bins: its slots, counts and result sizing
// (prepare), then, after its k_paint_ev / k_paint_ev2 launch, the join, the
// scan, the gather and the read-back (finish)
struct EvPlan {
    lime_ctx *ctx;
    PaintEvArgs pa;
    int64_t nt = 0, cap = 0, bound = -1, rcap = -1;
    uint32_t *cnt2 = nullptr, *skip1 = nullptr, *toff = nullptr;
    unsigned int *hdr = nullptr;  // [0] overflow flag, [1] total events
    PoolBag bag;
    explicit EvPlan(lime_ctx *c) : ctx(c), bag{c, {}} {}

    int prepare(int op, int nin, const lime_bitset *const *sets, uint32_t neg) {
        const lime_bitset *a = sets[0];
        nt = a->nt;
        pa.n_words = a->n_words;
        pa.neg = neg;
        pa.notmask = op == 1;
        pa.word0 = a->word0;
        pa.hi_bit = a->hi_bit;
        const uint32_t *d_off = nullptr;
        LIME_TRY(space_device(ctx, a->off, &d_off, nullptr));
        pa.off = d_off;
        pa.nc = a->n_contigs;
        // runs bound (a run starts at a run start of an operand, or a
        // contig's start for NOT) -> a slot of twice the bound's mean events
        // per tile + 2048, within [4096, 16384] (an AND's bound, the sum, is
        // loose: past the slot a tile falls back to the words path)
        bound = op == 1 ? (int64_t)a->n_contigs + 1 : 0;
        for (int i = 0; i < nin && bound >= 0; ++i)
            bound = sets[i]->runs_bound < 0 ? -1 : bound + sets[i]->runs_bound;
        cap = bound < 0 ? 16384 : 2 * (2 * bound / std::max<int64_t>(nt, 1)) + 2048;
        cap = std::min<int64_t>(std::max<int64_t>((cap + 255) / 256 * 256, 4096), EVSLOT_MAX);
        pa.cap = (uint32_t)cap;
        LIME_TRY(bag.get(&pa.tev, (size_t)nt * (size_t)cap));
        LIME_TRY(bag.get(&pa.tcnt, (size_t)nt));
        LIME_TRY(bag.get(&pa.edge, (size_t)nt));
        LIME_TRY(bag.get(&cnt2, (size_t)nt));
        LIME_TRY(bag.get(&skip1, (size_t)nt));
        LIME_TRY(bag.get(&toff, (size_t)nt));
        LIME_TRY(bag.get(&hdr, 2));  // [0] zeroed by k_paint_ev, [1] the scan's total
        pa.oflow = hdr;
        return LIME_OK;
    }

    // everything up to the read-back queued (the gather too when the result
    // can be sized from the bound)
    int queue(lime_result *res) {
        hipLaunchKernelGGL(k_ev_join, dim3(blocks_for(nt, 256)), dim3(256), 0, S(ctx),
                           (const uint32_t *)pa.tcnt, (const uint32_t *)pa.edge, nt, cnt2, skip1,
                           pa.oflow);
        LIME_HIP(hipGetLastError());
        LIME_TRY(scan_exclusive_u32(ctx, cnt2, toff, nt, hdr + 1));
        rcap = bound < 0 ? -1 : std::min<int64_t>(bound, nt * (cap / 2));
        if (rcap >= 0) {
            LIME_TRY(alloc(ctx, &res->gs, (size_t)std::max<int64_t>(rcap, 1)));
            LIME_TRY(alloc(ctx, &res->ge, (size_t)std::max<int64_t>(rcap, 1)));
            gather(res, (uint32_t)std::min<int64_t>(2 * rcap, 0xffffffffll));
        }
        return LIME_OK;
    }

    void gather(lime_result *res, uint32_t cap_events) {
        hipLaunchKernelGGL(k_ev_gather, dim3((unsigned)nt), dim3(256), 0, S(ctx),
                           (const uint32_t *)pa.tev, (const uint32_t *)cnt2,
                           (const uint32_t *)toff, (const unsigned int *)hdr, cap_events, res->gs,
                           res->ge, (uint32_t)cap, (const uint32_t *)skip1);
    }

    int finish(lime_result *res, bool *overflow) {
        *overflow = false;
        unsigned int h[2] = {0, 0};
        LIME_TRY(read_back(ctx, h, hdr, sizeof(h)));
        if (h[0]) {
            if (rcap >= 0) {
                release(ctx, res->gs);
                release(ctx, res->ge);
                res->gs = res->ge = nullptr;
            }
            *overflow = true;
            return LIME_OK;
        }
        if (h[1] & 1u) return fail(LIME_ERR_DEVICE, "bitset run extraction: odd event count");
        const int64_t nr = h[1] / 2;
        if (rcap >= 0) {
            if (nr > rcap) return fail(LIME_ERR_DEVICE, "bitset run extraction: runs past bound");
        } else {
            LIME_TRY(alloc(ctx, &res->gs, (size_t)std::max<int64_t>(nr, 1)));
            LIME_TRY(alloc(ctx, &res->ge, (size_t)std::max<int64_t>(nr, 1)));
            if (nr > 0) gather(res, h[1]);
            LIME_HIP(hipGetLastError());
        }
        res->n = nr;
        return LIME_OK;
    }
};

int runs_binned(lime_ctx *ctx, int op, int nin, const lime_bitset *const *sets, lime_result *res,
                bool *overflow) {
    *overflow = false;
    const lime_bitset *a = sets[0];
    // every operand's binned sets, the complemented operand's (one) marked
    std::vector<const lime_bitset::Bins *> b;
    uint32_t neg = 0;
    for (int i = 0; i < nin; ++i) {
        const bool inv = (op == 1 && i == 0) || (op == 3 && i == 1);
        if (inv) neg |= 1u << b.size();
        for (const auto &x : sets[i]->bins) b.push_back(&x);
    }
    const AndArgs sargs = binned_args(b.data(), (int)b.size(), a->nt, a->n_words);
    EvPlan p(ctx);
    LIME_TRY(p.prepare(op, nin, sets, neg));
    hipLaunchKernelGGL(k_paint_ev, dim3((unsigned)p.nt), dim3(PAINTB), 0, S(ctx), p.pa, sargs);
    LIME_TRY(p.queue(res));
    return p.finish(res, overflow);
}

}  // namespace

int bitset_runs(lime_ctx *ctx, int op, int k, const lime_bitset *const *sets, lime_result *res) {
    const lime_bitset *a = sets[0];
    // binned operands (bitsets from rows): the runs straight from the bins,
    // unless a tile overflows its event slot; else (or then) from words
    const int nin = op == 4 ? k : (op >= 2 ? 2 : 1);
    // (a complemented operand must be ONE binned set: ~(x & y) is not a
    // complement per set; at most MAXK binned sets in all)
    bool binned = a->n_words > 0;
    size_t nb = 0;
    for (int i = 0; i < nin; ++i) {
        const bool inv = (op == 1 && i == 0) || (op == 3 && i == 1);
        binned = binned && !sets[i]->bins.empty() && sets[i]->nt == a->nt &&
                 (!inv || sets[i]->bins.size() == 1);
        nb += sets[i]->bins.size();
    }
    binned = binned && nb <= (size_t)MAXK;
    if (binned) {
        bool overflow = false;
        LIME_TRY(runs_binned(ctx, op, nin, sets, res, &overflow));
        if (!overflow) return LIME_OK;
    }
    for (int i = 0; i < nin; ++i) LIME_TRY(bitset_paint(ctx, sets[i]));
    // an AND of more than MAXK bitsets: their words ANDed group by group into
    // a temporary bitset, whose runs are then extracted (op 0)
    uint64_t *tmp = nullptr;
    PoolGuard<uint64_t> gt{ctx, tmp};
    if (op == 4 && k > MAXK) {
        LIME_TRY(alloc(ctx, &tmp, (size_t)std::max<int64_t>(a->n_words, 1)));
        for (int g0 = 0; g0 < k; g0 += MAXK) {
            WordsAnd wa;
            wa.k = std::min(MAXK, k - g0);
            for (int q = 0; q < MAXK; ++q) wa.w[q] = q < wa.k ? sets[g0 + q]->words : nullptr;
            const unsigned g = std::min<unsigned>(blocks_for(a->n_words, BB), 8192u);
            if (a->n_words > 0)
                hipLaunchKernelGGL(k_and_words, dim3(g), dim3(BB), 0, S(ctx), wa, g0 > 0 ? 1 : 0,
                                   tmp, a->n_words);
        }
        LIME_HIP(hipGetLastError());
    }
    OpArgs oa;
    for (int i = 0; i < MAXK; ++i) oa.w[i] = i < k && i < MAXK ? sets[i]->words : nullptr;
    oa.k = std::min(k, MAXK);
    oa.op = op;
    if (tmp) {
        oa.w[0] = tmp;
        oa.k = 1;
        oa.op = 0;
    }
    oa.n_words = a->n_words;
    oa.word0 = a->word0;
    oa.span = a->hi_bit;  // NOT clears every bit past the window
    oa.nc = a->n_contigs;
    // pad positions off[c + 1] - 1, from the context's cached offsets (no
    // upload, no stream drain per call)
    const uint32_t *d_off = nullptr;
    LIME_TRY(space_device(ctx, a->off, &d_off, nullptr));
    oa.off = d_off;
    // tiles cover one word past the last: a run reaching the window's end
    // closes there (a shard window may end on any word)
    const int64_t nt = a->n_words == 0 ? 0 : a->n_words / BT + 1;
    if (nt == 0) {  // an empty window (e.g. a zero-width shard): no runs
        LIME_TRY(alloc(ctx, &res->gs, 1));
        LIME_TRY(alloc(ctx, &res->ge, 1));
        res->n = 0;
        return LIME_OK;
    }
    // per-tile event slots + scan + gather (no look-back): C4's two
    // extractions 0.61 -> 0.43 ms against a one-pass decoupled look-back
    {
        const int64_t ntl = a->n_words / EV_TW + 1;
        uint32_t *tev, *tcnt, *toff;
        unsigned int *hdr;  // [0] overflow flag, [1] total events
        LIME_TRY(alloc(ctx, &tev, (size_t)ntl * EVCAP));
        PoolGuard<uint32_t> g0{ctx, tev};
        LIME_TRY(alloc(ctx, &tcnt, (size_t)ntl));
        PoolGuard<uint32_t> g1{ctx, tcnt};
        LIME_TRY(alloc(ctx, &toff, (size_t)ntl));
        PoolGuard<uint32_t> g2{ctx, toff};
        LIME_TRY(alloc(ctx, &hdr, 2));
        PoolGuard<unsigned int> g3{ctx, hdr};
        LIME_HIP(hipMemsetAsync(hdr, 0, 8, S(ctx)));
        hipLaunchKernelGGL(k_ev_local, dim3((unsigned)ntl), dim3(EV_NT), 0, S(ctx), oa, tev, tcnt,
                           hdr);
        LIME_HIP(hipGetLastError());
        LIME_TRY(scan_exclusive_u32(ctx, tcnt, toff, ntl, hdr + 1));
        // with a bound on the runs (every operand's runs_bound known) the
        // result is allocated at the bound and the gather queued before the
        // host reads the totals: no drained stream between the two (C4:
        // ~20 us per extraction); else sized exactly from the read-back
        const int nin = op == 4 ? k : (op >= 2 ? 2 : 1);
        int64_t cap = op == 1 ? (int64_t)a->n_contigs + 1 : 0;
        for (int i = 0; i < nin && cap >= 0; ++i)
            cap = sets[i]->runs_bound < 0 ? -1 : cap + sets[i]->runs_bound;
        if (cap >= 0) cap = std::min<int64_t>(cap, ntl * (EVCAP / 2));
        if (cap >= 0) {
            LIME_TRY(alloc(ctx, &res->gs, (size_t)std::max<int64_t>(cap, 1)));
            LIME_TRY(alloc(ctx, &res->ge, (size_t)std::max<int64_t>(cap, 1)));
            hipLaunchKernelGGL(k_ev_gather, dim3((unsigned)ntl), dim3(256), 0, S(ctx),
                               (const uint32_t *)tev, (const uint32_t *)tcnt,
                               (const uint32_t *)toff, (const unsigned int *)hdr,
                               (uint32_t)(2 * cap), res->gs, res->ge);
            LIME_HIP(hipGetLastError());
        }
        unsigned int h[2] = {0, 0};
        LIME_TRY(read_back(ctx, h, hdr, sizeof(h)));
        if (!h[0]) {
            if (h[1] & 1u) return fail(LIME_ERR_DEVICE, "bitset run extraction: odd event count");
            const int64_t nr = h[1] / 2;
            if (cap >= 0) {
                if (nr > cap) return fail(LIME_ERR_DEVICE, "bitset run extraction: runs past bound");
                res->n = nr;
                return LIME_OK;
            }
            LIME_TRY(alloc(ctx, &res->gs, (size_t)std::max<int64_t>(nr, 1)));
            LIME_TRY(alloc(ctx, &res->ge, (size_t)std::max<int64_t>(nr, 1)));
            if (nr > 0)
                hipLaunchKernelGGL(k_ev_gather, dim3((unsigned)ntl), dim3(256), 0, S(ctx),
                                   (const uint32_t *)tev, (const uint32_t *)tcnt,
                                   (const uint32_t *)toff, (const unsigned int *)hdr,
                                   (uint32_t)h[1], res->gs, res->ge);
            LIME_HIP(hipGetLastError());
            res->n = nr;
            return LIME_OK;
        }
        // a tile past EVCAP events: the two-pass path below
        if (cap >= 0) {
            release(ctx, res->gs);
            release(ctx, res->ge);
            res->gs = res->ge = nullptr;
        }
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
    res->n = nr;
    return LIME_OK;
}

int64_t bitset_popcount(lime_ctx *ctx, const lime_bitset *a) {
    if (bitset_paint(ctx, a) != LIME_OK) return -1;
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

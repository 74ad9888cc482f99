// capi.hip -- the extern "C" boundary (include/lime_amd.h): contexts, the
// coordinate space, set creation, operator entry points and host copies.
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <vector>

#include "common.hpp"

namespace lime {

static thread_local std::string g_err;

void set_error(const std::string &msg) { g_err = msg; }
int fail(int code, const std::string &msg) {
    g_err = msg;
    return code;
}

void *Pool::get(size_t bytes) {
    bytes = (bytes + 255) & ~(size_t)255;
    const hipStream_t cur = stream ? *stream : nullptr;
    auto range = free_blocks.equal_range(bytes);
    for (auto it = range.first; it != range.second; ++it) {
        Block &b = it->second;
        // same stream: stream order protects the reuse; another stream: the
        // releasing stream's work must be done
        if (b.s != cur && b.ev && hipEventQuery(b.ev) != hipSuccess) continue;
        void *p = b.p;
        if (b.ev) spare_events.push_back(b.ev);
        free_blocks.erase(it);
        live[p] = bytes;
        in_use += (int64_t)bytes;
        peak = std::max(peak, in_use);
        return p;
    }
    void *p = nullptr;
    if (hipMalloc(&p, bytes) != hipSuccess) {
        // give cached blocks back and retry once (hipFree waits for the device)
        for (auto &kv : free_blocks) {
            hipFree(kv.second.p);
            if (kv.second.ev) spare_events.push_back(kv.second.ev);
            held -= (int64_t)kv.first;
        }
        free_blocks.clear();
        (void)hipGetLastError();
        if (hipMalloc(&p, bytes) != hipSuccess) {
            (void)hipGetLastError();
            return nullptr;
        }
    }
    held += (int64_t)bytes;
    live[p] = bytes;
    in_use += (int64_t)bytes;
    peak = std::max(peak, in_use);
    return p;
}
void Pool::put(void *p) {
    auto it = live.find(p);
    if (it == live.end()) return;
    Block b{p, stream ? *stream : nullptr, nullptr};
    if (multi_stream) {
        if (!spare_events.empty()) {
            b.ev = spare_events.back();
            spare_events.pop_back();
        } else if (hipEventCreateWithFlags(&b.ev, hipEventDisableTiming) != hipSuccess) {
            (void)hipGetLastError();
            b.ev = nullptr;
            b.s = nullptr;  // no event: treat as foreign to every stream...
        }
        if (b.ev && hipEventRecord(b.ev, b.s) != hipSuccess) (void)hipGetLastError();
        if (!b.ev) hipStreamSynchronize(stream ? *stream : nullptr);  // ...and drain instead
    }
    free_blocks.emplace(it->second, b);
    in_use -= (int64_t)it->second;
    live.erase(it);
}
void Pool::release_all() {
    for (auto &kv : free_blocks) {
        hipFree(kv.second.p);
        if (kv.second.ev) hipEventDestroy(kv.second.ev);
    }
    for (auto &kv : live) hipFree(kv.first);
    for (hipEvent_t e : spare_events) hipEventDestroy(e);
    free_blocks.clear();
    live.clear();
    spare_events.clear();
    held = in_use = 0;
}

int read_back(lime_ctx *c, void *host, const void *dev, size_t bytes) {
    // the lower half of the pinned scratch (the upper half holds the k-way
    // AND's per-set flags, bitset.hip); larger: pageable copy
    if (bytes > 2048) {
        LIME_HIP(hipMemcpyAsync(host, dev, bytes, hipMemcpyDeviceToHost, S(c)));
        LIME_HIP(hipStreamSynchronize(S(c)));
        return LIME_OK;
    }
    LIME_HIP(hipMemcpyAsync(c->pinned, dev, bytes, hipMemcpyDeviceToHost, S(c)));
    LIME_HIP(hipStreamSynchronize(S(c)));
    memcpy(host, c->pinned, bytes);
    return LIME_OK;
}

// defined in the kernel translation units
struct PairsPlan;
int intersect_plan(lime_ctx *ctx, const lime_set *A, const lime_set *B, int64_t threshold,
                   int64_t a_own, int64_t b_own, PairsPlan **out, const lime_set *A_out = nullptr,
                   int64_t reach = -1);
int window_plan(lime_ctx *ctx, const lime_set *A, const lime_set *B, int64_t d, PairsPlan **out);
int format_bed(lime_ctx *ctx, const std::vector<uint32_t> &off,
               const std::vector<std::string> &names, int64_t n, const uint32_t *gs,
               const uint32_t *ge, const uint32_t *extra, char *out, int64_t cap,
               int64_t *total_len);
struct ClosestPlan;
int closest_plan(lime_ctx *ctx, const lime_set *A, const lime_set *B, int mode, bool alive_in,
                 bool *alive_out, ClosestPlan **out);
int closest_fill(ClosestPlan *pl, int64_t first, int64_t count, lime_pair *d_out);
int closest_checksum(ClosestPlan *pl, uint64_t *sum, uint64_t *xr);
void closest_free(ClosestPlan *pl);
int64_t closest_total(const ClosestPlan *pl);
int closest_rounds(const ClosestPlan *pl, bool *sequential);
int intersect_fill(PairsPlan *pl, int64_t first, int64_t count, lime_pair *d_out);
int intersect_checksum(PairsPlan *pl, uint64_t *sum, uint64_t *xr);
void intersect_free(PairsPlan *pl);
int64_t plan_total(const PairsPlan *pl);
int merge_runs(lime_ctx *ctx, const lime_set *set, lime_result *res, bool want_run_ids);
int subtract_run(lime_ctx *ctx, const lime_set *A, const lime_set *B, int64_t threshold, int mode,
                 lime_result *res);
int complement_run(lime_ctx *ctx, const lime_result *runs, const uint32_t *d_off,
                   const uint32_t *d_len, int32_t nc, lime_result *res, uint32_t wlo = 0,
                   uint32_t whi = 0xffffffffu);
int bitset_build(lime_ctx *ctx, const lime_set *a, lime_bitset *bs);
int bitset_build_rows(lime_ctx *ctx, const lime_space *sp, int64_t n, const int32_t *d_contig,
                      const uint32_t *d_start, const uint32_t *d_end, const uint32_t *d_off,
                      const uint32_t *d_len, int64_t lo, int64_t hi, lime_bitset *bs);
int bitset_and_rows(lime_ctx *ctx, const lime_space *sp, int k, const int64_t *n,
                    const int32_t *const *d_contig, const uint32_t *const *d_start,
                    const uint32_t *const *d_end, const uint32_t *d_off, const uint32_t *d_len,
                    int64_t lo, int64_t hi, lime_bitset *bs);
int sample_starts(lime_ctx *ctx, const lime_space *sp, int64_t n, const int32_t *d_contig,
                  const uint32_t *d_start, int32_t k, uint32_t *d_out);
int route_rows(lime_ctx *ctx, const lime_space *sp, int64_t n, const int32_t *d_contig,
               const uint32_t *d_start, const uint32_t *d_end, uint32_t row_base, int32_t nsh,
               const uint32_t *splits, int clip, int64_t cap, uint32_t *d_gs, uint32_t *d_ge,
               uint32_t *d_row, int64_t *counts, const int8_t *d_strand_in,
               int8_t *d_strand_out, uint32_t *d_iv = nullptr, int32_t ik = 0);
int deinterleave_u32(lime_ctx *ctx, int64_t n, int32_t k, const uint32_t *src, uint32_t *d0,
                     uint32_t *d1, uint32_t *d2);
int bitset_runs(lime_ctx *ctx, int op, int k, const lime_bitset *const *sets, lime_result *res);
int64_t bitset_popcount(lime_ctx *ctx, const lime_bitset *a);
void bitset_free(lime_bitset *bs);
int bitset_drop_bins(lime_ctx *ctx, lime_bitset *bs);
int synth(lime_ctx *ctx, const lime_space *sp, int kind, int64_t first, int64_t n, uint64_t seed,
          uint32_t lo, uint32_t hi, int64_t n_centres, uint32_t sigma, int32_t *d_contig,
          uint32_t *d_start, uint32_t *d_end);

int sort_set_global(lime_ctx *ctx, lime_set *set, const uint32_t *d_gs, const uint32_t *d_ge,
                    const uint32_t *d_row, const uint32_t *d_len);

__global__ void k_set_lower_bound(const uint32_t *gs, int64_t n, uint32_t key, int64_t *out) {
    if (threadIdx.x == 0) *out = dev::lower_bound(gs, 0, n, key);
}

// Order-independent checksum of a result (SURVEY.md 8(d) "Verification at
// scale"), restated by the oracle (oracle.result_checksum / lo_merge_mt):
//   regions   sum / xor over regions of mix64(pair_hash(s, e, a, b) + contig),
//             (s, e) contig-local, a / b the rows or 0xffffffff if absent
//   grouping  (merge) sum / xor over sorted rows j of
//             mix64(row_j << 32 | run_of_sorted_j)
__global__ __launch_bounds__(256) void k_result_checksum(
    const uint32_t *__restrict__ gs, const uint32_t *__restrict__ ge,
    const uint32_t *__restrict__ ar, const uint32_t *__restrict__ br, int64_t n,
    const uint32_t *__restrict__ off, int32_t nc, const uint32_t *__restrict__ row,
    const uint32_t *__restrict__ rid, int64_t nrows, unsigned long long *__restrict__ out) {
    uint64_t rs = 0, rx = 0, gsum = 0, gx = 0;
    const int64_t stride = (int64_t)gridDim.x * 256;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
        const uint32_t g = gs[i];
        const int64_t c = dev::upper_bound(off, 0, (int64_t)nc, g) - 1;
        const uint32_t o = off[c < 0 ? 0 : c];
        const uint64_t h = dev::mix64(dev::pair_hash(g - o, ge[i] - o, ar ? ar[i] : 0xffffffffu,
                                                     br ? br[i] : 0xffffffffu) +
                                      (uint64_t)c);
        rs += h;
        rx ^= h;
    }
    for (int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x; rid && j < nrows; j += stride) {
        const uint64_t h = dev::mix64(((uint64_t)row[j] << 32) | rid[j]);
        gsum += h;
        gx ^= h;
    }
    rs = dev::wave_reduce_sum(rs);
    gsum = dev::wave_reduce_sum(gsum);
    rx = dev::wave_reduce_xor(rx);
    gx = dev::wave_reduce_xor(gx);
    if (dev::lane_id() == 0) {
        atomicAdd(&out[0], (unsigned long long)rs);
        atomicXor(&out[1], (unsigned long long)rx);
        atomicAdd(&out[2], (unsigned long long)gsum);
        atomicXor(&out[3], (unsigned long long)gx);
    }
}

// Order-independent checksum of pair records STORED in device memory (sum /
// xor of pair_hash over every record): the check that the bytes a fill wrote
// hash to what lime_intersect_checksum computes in registers.
__global__ __launch_bounds__(256) void k_pairs_hash(const uint4 *__restrict__ rec, int64_t n,
                                                    unsigned long long *__restrict__ out) {
    uint64_t hs = 0, hx = 0;
    const int64_t stride = (int64_t)gridDim.x * 256;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
        const uint4 r = rec[i];
        const uint64_t h = dev::pair_hash(r.x, r.y, r.z, r.w);
        hs += h;
        hx ^= h;
    }
    hs = dev::wave_reduce_sum(hs);
    hx = dev::wave_reduce_xor(hx);
    if (dev::lane_id() == 0) {
        atomicAdd(&out[0], (unsigned long long)hs);
        atomicXor(&out[1], (unsigned long long)hx);
    }
}

// every set / bitset an operator reads must belong to the operator's context:
// its arrays live in that context's pool and device (a foreign set
// could otherwise be read on another device, or have lazily built state
// allocated from, and freed into, the wrong pool)
static int same_ctx(lime_ctx *ctx, const lime_set *s) {
    if (s && s->ctx != ctx)
        return fail(LIME_ERR_ARG, "set belongs to another context (one context per thread)");
    return LIME_OK;
}

static int32_t contig_of(const std::vector<uint32_t> &off, int32_t nc, uint32_t g) {
    // largest c in [0, nc) with off[c] <= g
    auto it = std::upper_bound(off.begin(), off.begin() + nc, g);
    return (int32_t)(it - off.begin()) - 1;
}

template <typename T>
static int d2h(lime_ctx *ctx, std::vector<T> &v, const T *d, int64_t n) {
    v.resize((size_t)n);
    if (n == 0 || !d) return LIME_OK;
    LIME_HIP(hipMemcpyAsync(v.data(), d, sizeof(T) * (size_t)n, hipMemcpyDeviceToHost, S(ctx)));
    LIME_HIP(hipStreamSynchronize(S(ctx)));
    return LIME_OK;
}

SpaceDev::~SpaceDev() {
    release(ctx, off);
    release(ctx, len);
}

int space_device(lime_ctx *ctx, const std::vector<uint32_t> &off, const uint32_t **d_off,
                 const uint32_t **d_len, std::shared_ptr<SpaceDev> *keep) {
    auto it = ctx->spaces.find(off);
    if (it == ctx->spaces.end()) {
        const size_t n1 = off.size();
        auto sd = std::make_shared<SpaceDev>();
        sd->ctx = ctx;  // (a failed upload releases what it got)
        LIME_TRY(alloc(ctx, &sd->off, n1));
        LIME_TRY(alloc(ctx, &sd->len, n1));
        std::vector<uint32_t> len32(n1, 0);
        for (size_t c = 0; c + 1 < n1; ++c) len32[c] = off[c + 1] - off[c] - 1;
        LIME_HIP(hipMemcpyAsync(sd->off, off.data(), 4 * n1, hipMemcpyHostToDevice, S(ctx)));
        LIME_HIP(hipMemcpyAsync(sd->len, len32.data(), 4 * n1, hipMemcpyHostToDevice, S(ctx)));
        LIME_HIP(hipStreamSynchronize(S(ctx)));  // (once per space and context)
        it = ctx->spaces.emplace(off, sd).first;
        // bound the cache: drop entries no set holds (stream-ordered pool:
        // work already queued on them finishes before the blocks are reused)
        if (ctx->spaces.size() > lime_ctx::SPACE_CACHE)
            for (auto e = ctx->spaces.begin(); e != ctx->spaces.end();)
                e = (e != it && e->second.use_count() == 1) ? ctx->spaces.erase(e) : std::next(e);
    }
    *d_off = it->second->off;
    if (d_len) *d_len = it->second->len;
    if (keep) *keep = it->second;
    return LIME_OK;
}

// the space's cached device arrays (borrowed: owned by the context)
static int upload_space(lime_ctx *ctx, const lime_space *sp, uint32_t **d_off, uint32_t **d_len,
                        std::shared_ptr<SpaceDev> *keep = nullptr) {
    const uint32_t *o = nullptr, *l = nullptr;
    LIME_TRY(space_device(ctx, sp->off, &o, d_len ? &l : nullptr, keep));
    *d_off = const_cast<uint32_t *>(o);
    if (d_len) *d_len = const_cast<uint32_t *>(l);
    return LIME_OK;
}

static lime_set *new_set(lime_ctx *ctx, const lime_space *sp, int64_t n) {
    lime_set *s = new lime_set();
    s->ctx = ctx;
    s->n = n;
    s->n_contigs = sp->n;
    s->off = sp->off;
    s->len = sp->len;
    return s;
}

// d_strand (optional, device, input order, taken over by the set): a
// stranded set, sorted by (gs, ge, strand)
static int create_from_device(lime_ctx *ctx, const lime_space *sp, int64_t n,
                              const int32_t *d_contig, const uint32_t *d_start,
                              const uint32_t *d_end, lime_set **out,
                              int8_t *d_strand = nullptr, int min_shift = 0,
                              bool strand_uniform = false) {
    lime_set *s = new_set(ctx, sp, n);
    s->strand_in = d_strand;
    s->strand_uniform = strand_uniform;
    s->min_shift = min_shift;
    uint32_t *d_len = nullptr;
    int rc = upload_space(ctx, sp, &s->d_off, &d_len, &s->space_keep);
    if (rc == LIME_OK) rc = sort_set(ctx, s, d_contig, d_start, d_end, d_len);
    if (rc != LIME_OK) {
        release(ctx, s->strand_in);
        delete s;
        return rc;
    }
    *out = s;
    return LIME_OK;
}

static lime_result *new_result(lime_ctx *ctx, const lime_set *like) {
    lime_result *r = new lime_result();
    r->ctx = ctx;
    r->off = like->off;
    r->n_contigs = like->n_contigs;
    return r;
}

// Java String.compareTo: lexicographic over UTF-16 code units.
static std::vector<uint16_t> utf16(const char *s) {
    std::vector<uint16_t> out;
    const unsigned char *p = (const unsigned char *)s;
    while (*p) {
        uint32_t cp;
        if (*p < 0x80) {
            cp = *p++;
        } else if ((*p >> 5) == 6 && p[1]) {
            cp = ((p[0] & 0x1f) << 6) | (p[1] & 0x3f);
            p += 2;
        } else if ((*p >> 4) == 14 && p[1] && p[2]) {
            cp = ((p[0] & 0x0f) << 12) | ((p[1] & 0x3f) << 6) | (p[2] & 0x3f);
            p += 3;
        } else if ((*p >> 3) == 30 && p[1] && p[2] && p[3]) {
            cp = ((p[0] & 0x07) << 18) | ((p[1] & 0x3f) << 12) | ((p[2] & 0x3f) << 6) | (p[3] & 0x3f);
            p += 4;
        } else {
            cp = *p++;  // invalid byte: keep as a code unit
        }
        if (cp >= 0x10000) {
            cp -= 0x10000;
            out.push_back((uint16_t)(0xD800 + (cp >> 10)));
            out.push_back((uint16_t)(0xDC00 + (cp & 0x3ff)));
        } else {
            out.push_back((uint16_t)cp);
        }
    }
    return out;
}

}  // namespace lime

using namespace lime;

extern "C" {

const char *lime_last_error(void) { return g_err.c_str(); }
int lime_abi_version(void) { return LIME_ABI_VERSION; }

uint64_t lime_pair_hash(uint32_t start, uint32_t end, uint32_t a_row, uint32_t b_row) {
    return dev::pair_hash(start, end, a_row, b_row);
}

int lime_ctx_create(int device, lime_ctx **out) {
    if (!out) return fail(LIME_ERR_ARG, "out is null");
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) {
        (void)hipGetLastError();
        return fail(LIME_ERR_DEVICE, "no HIP device available");
    }
    if (device < 0 || device >= n) return fail(LIME_ERR_ARG, "device index out of range");
    LIME_HIP(hipSetDevice(device));
    lime_ctx *c = new lime_ctx();
    c->device = device;
    if (hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking) != hipSuccess ||
        hipHostMalloc(&c->pinned, 4096, hipHostMallocDefault) != hipSuccess) {
        delete c;
        return fail(LIME_ERR_DEVICE, "stream / pinned buffer creation failed");
    }
    c->stream = c->own_stream;
    c->pool.stream = &c->stream;
    *out = c;
    return LIME_OK;
}

int lime_ctx_destroy(lime_ctx *ctx) {
    if (!ctx) return LIME_OK;
    hipSetDevice(ctx->device);
    hipStreamSynchronize(ctx->stream);
    ctx->spaces.clear();
    ctx->pool.release_all();
    if (ctx->pinned) hipHostFree(ctx->pinned);
    if (ctx->own_stream) hipStreamDestroy(ctx->own_stream);
    delete ctx;
    return LIME_OK;
}

int lime_ctx_set_stream(lime_ctx *ctx, void *stream) {
    if (!ctx) return fail(LIME_ERR_ARG, "ctx is null");
    hipStream_t s = stream ? (hipStream_t)stream : ctx->own_stream;
    // Work of this context on a second stream: from now on releases are
    // ordered by events.  The blocks cached so far carry none, so the old
    // stream is drained once here.
    const bool used = !ctx->pool.live.empty() || !ctx->pool.free_blocks.empty();
    if (s != ctx->stream && used && !ctx->pool.multi_stream) {
        LIME_HIP(hipStreamSynchronize(ctx->stream));
        ctx->pool.multi_stream = true;
    }
    ctx->stream = s;
    return LIME_OK;
}

int lime_ctx_synchronize(lime_ctx *ctx) {
    if (!ctx) return fail(LIME_ERR_ARG, "ctx is null");
    LIME_HIP(hipStreamSynchronize(ctx->stream));
    return LIME_OK;
}

int64_t lime_ctx_pool_bytes(const lime_ctx *ctx) { return ctx ? ctx->pool.held : 0; }
int64_t lime_ctx_pool_live_bytes(lime_ctx *ctx, int32_t reset_peak, int64_t *peak) {
    if (!ctx) return 0;
    if (peak) *peak = ctx->pool.peak;
    if (reset_peak) ctx->pool.peak = ctx->pool.in_use;
    return ctx->pool.in_use;
}

// ------------------------------------------------------------------- space
int lime_space_create(int32_t n, const int64_t *lengths, lime_space **out) {
    if (!out || n < 0 || (n > 0 && !lengths)) return fail(LIME_ERR_ARG, "bad space arguments");
    lime_space *sp = new lime_space();
    sp->n = n;
    sp->len.assign(lengths, lengths + n);
    sp->off.resize((size_t)n + 1);
    int64_t o = 0;
    for (int32_t c = 0; c < n; ++c) {
        if (lengths[c] < 0) {
            delete sp;
            return fail(LIME_ERR_RANGE, "negative contig length");
        }
        sp->off[c] = (uint32_t)o;
        o += lengths[c] + 1;
        if (o > 0xffffffffLL) {
            delete sp;
            return fail(LIME_ERR_RANGE, "coordinate span sum(len + 1) exceeds 2^32");
        }
    }
    sp->off[n] = (uint32_t)o;
    sp->span = o;
    *out = sp;
    return LIME_OK;
}
int lime_space_destroy(lime_space *sp) {
    delete sp;
    return LIME_OK;
}
int32_t lime_space_contigs(const lime_space *sp) { return sp ? sp->n : 0; }
int64_t lime_space_span(const lime_space *sp) { return sp ? sp->span : 0; }
int64_t lime_space_offset(const lime_space *sp, int32_t c) {
    return (sp && c >= 0 && c <= sp->n) ? (int64_t)sp->off[c] : -1;
}

// -------------------------------------------------------------------- sets
static int create_host(lime_ctx *ctx, const lime_space *sp, int64_t n, const int32_t *contig,
                       const int64_t *start, const int64_t *end, const int8_t *strand,
                       lime_set **out);

int lime_set_create_host(lime_ctx *ctx, const lime_space *sp, int64_t n, const int32_t *contig,
                         const int64_t *start, const int64_t *end, lime_set **out) {
    return create_host(ctx, sp, n, contig, start, end, nullptr, out);
}

int lime_set_create_host_stranded(lime_ctx *ctx, const lime_space *sp, int64_t n,
                                  const int32_t *contig, const int64_t *start,
                                  const int64_t *end, const int8_t *strand, lime_set **out) {
    if (n > 0 && !strand) return fail(LIME_ERR_ARG, "bad set arguments");
    return create_host(ctx, sp, n, contig, start, end, strand, out);
}

static int create_host(lime_ctx *ctx, const lime_space *sp, int64_t n, const int32_t *contig,
                       const int64_t *start, const int64_t *end, const int8_t *strand,
                       lime_set **out) {
    if (!ctx || !sp || !out || n < 0 || (n > 0 && (!contig || !start || !end)))
        return fail(LIME_ERR_ARG, "bad set arguments");
    if (n > 0xffffffffLL) return fail(LIME_ERR_RANGE, "more than 2^32 rows in one set");
    hipSetDevice(ctx->device);
    std::vector<uint32_t> s32((size_t)n), e32((size_t)n);
    for (int64_t i = 0; i < n; ++i) {
        if (contig[i] < 0 || contig[i] >= sp->n)
            return fail(LIME_ERR_CONTIG, "row " + std::to_string(i) + ": contig id not in space");
        if (start[i] < 0 || end[i] < start[i])
            return fail(LIME_ERR_RANGE, "row " + std::to_string(i) + ": invalid region");
        if (end[i] > sp->len[contig[i]])
            return fail(LIME_ERR_RANGE, "row " + std::to_string(i) + ": end beyond contig length");
        s32[i] = (uint32_t)start[i];
        e32[i] = (uint32_t)end[i];
    }
    int32_t *dc;
    uint32_t *ds, *de;
    LIME_TRY(alloc(ctx, &dc, (size_t)n));
    LIME_TRY(alloc(ctx, &ds, (size_t)n));
    LIME_TRY(alloc(ctx, &de, (size_t)n));
    if (n > 0) {
        LIME_HIP(hipMemcpyAsync(dc, contig, 4 * (size_t)n, hipMemcpyHostToDevice, S(ctx)));
        LIME_HIP(hipMemcpyAsync(ds, s32.data(), 4 * (size_t)n, hipMemcpyHostToDevice, S(ctx)));
        LIME_HIP(hipMemcpyAsync(de, e32.data(), 4 * (size_t)n, hipMemcpyHostToDevice, S(ctx)));
        LIME_HIP(hipStreamSynchronize(S(ctx)));
    }
    int8_t *dst = nullptr;
    if (strand) {
        LIME_TRY(alloc(ctx, &dst, (size_t)std::max<int64_t>(n, 1)));
        if (n > 0) {
            LIME_HIP(hipMemcpyAsync(dst, strand, (size_t)n, hipMemcpyHostToDevice, S(ctx)));
            LIME_HIP(hipStreamSynchronize(S(ctx)));
        }
    }
    bool uniform = true;
    for (int64_t i = 1; strand && i < n && uniform; ++i) uniform = strand[i] == strand[0];
    int rc = create_from_device(ctx, sp, n, dc, ds, de, out, dst, 0, strand && uniform);
    release(ctx, dc);
    release(ctx, ds);
    release(ctx, de);
    return rc;
}

int lime_set_create_device(lime_ctx *ctx, const lime_space *sp, int64_t n, const int32_t *d_contig,
                           const uint32_t *d_start, const uint32_t *d_end, lime_set **out) {
    if (!ctx || !sp || !out || n < 0 || (n > 0 && (!d_contig || !d_start || !d_end)))
        return fail(LIME_ERR_ARG, "bad set arguments");
    if (n > 0xffffffffLL) return fail(LIME_ERR_RANGE, "more than 2^32 rows in one set");
    hipSetDevice(ctx->device);
    return create_from_device(ctx, sp, n, d_contig, d_start, d_end, out);
}

int lime_set_create_device_stranded(lime_ctx *ctx, const lime_space *sp, int64_t n,
                                    const int32_t *d_contig, const uint32_t *d_start,
                                    const uint32_t *d_end, const int8_t *d_strand,
                                    lime_set **out) {
    if (!ctx || !sp || !out || n < 0 || (n > 0 && (!d_contig || !d_start || !d_end)))
        return fail(LIME_ERR_ARG, "bad set arguments");
    if (n > 0xffffffffLL) return fail(LIME_ERR_RANGE, "more than 2^32 rows in one set");
    hipSetDevice(ctx->device);
    int8_t *dst;  // the set keeps its own copy of the codes
    LIME_TRY(alloc(ctx, &dst, (size_t)std::max<int64_t>(n, 1)));
    if (n > 0) {
        if (d_strand)
            LIME_HIP(hipMemcpyAsync(dst, d_strand, (size_t)n, hipMemcpyDeviceToDevice, S(ctx)));
        else
            LIME_HIP(hipMemsetAsync(dst, 0, (size_t)n, S(ctx)));
    }
    return create_from_device(ctx, sp, n, d_contig, d_start, d_end, out, dst, 0, !d_strand);
}

int lime_set_destroy(lime_set *s) {
    if (!s) return LIME_OK;
    lime_ctx *ctx = s->ctx;
    release(ctx, s->gs);
    release(ctx, s->ge);
    release(ctx, s->row);
    // (s->d_off is the context's cached space array: held by s->space_keep)
    release(ctx, s->pmax);
    release(ctx, s->strand_in);
    release(ctx, s->tie_gs);
    release(ctx, s->tie_ge);
    release(ctx, s->tie_row);
    delete s;
    return LIME_OK;
}

int64_t lime_set_size(const lime_set *s) { return s ? s->n : -1; }

int lime_set_device_arrays(const lime_set *s, const uint32_t **gs, const uint32_t **ge,
                           const uint32_t **row) {
    if (!s) return fail(LIME_ERR_ARG, "set is null");
    if (gs) *gs = s->gs;
    if (ge) *ge = s->ge;
    if (row) *row = s->row;
    return LIME_OK;
}

int lime_set_stats(const lime_set *s, uint32_t *min_width, uint32_t *max_width,
                   int32_t *has_zero_width) {
    if (!s) return fail(LIME_ERR_ARG, "set is null");
    if (min_width) *min_width = s->min_width;
    if (max_width) *max_width = s->max_width;
    if (has_zero_width) *has_zero_width = s->has_zero_width ? 1 : 0;
    return LIME_OK;
}

// Opt-in check of the sorted-concatenation contract (LIME_CHECK_EXTEND=1):
// every row of the new set follows its predecessor in canonical order (gs,
// zero-width first), and the added rows -- [0, a0) and [a1, n) -- lie within
// the declared width bounds.  bit0: order, bit1: width bounds, bit2:
// zero-width row without the flag
__global__ void k_check_join(const uint32_t *__restrict__ gs, const uint32_t *__restrict__ ge,
                             int64_t n, int64_t a0, int64_t a1, uint32_t min_w, uint32_t max_w,
                             int zero_ok, unsigned int *__restrict__ err) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const uint32_t g = gs[i], e = ge[i];
    unsigned int f = 0;
    if (i > 0) {
        const uint32_t pg = gs[i - 1], pe = ge[i - 1];
        // canonical: (gs, zero width before non-zero width); ties beyond that
        // keep input order
        if (pg > g || (pg == g && pe > pg && e == g)) f |= 1u;
    }
    if (i < a0 || i >= a1) {
        const uint32_t w = e - g;
        if (e < g || w < min_w || w > max_w) f |= 2u;
        if (w == 0 && !zero_ok) f |= 4u;
    }
    if (f) atomicOr(err, f);
}

// rows (nl prefix rows) + set + (nr suffix rows), copied device-to-device;
// width statistics: the set's combined with the caller's bounds of the added
// rows.  LIME_CHECK_EXTEND=1 checks the contract at both joins.
static int concat_sorted(lime_ctx *ctx, const lime_set *set, int64_t nl, const uint32_t *l_gs,
                         const uint32_t *l_ge, const uint32_t *l_row, int64_t nr,
                         const uint32_t *r_gs, const uint32_t *r_ge, const uint32_t *r_row,
                         uint32_t min_width, uint32_t max_width, int32_t has_zero_width,
                         lime_set **out) {
    if (!ctx || !set || !out || nl < 0 || nr < 0 || (nl > 0 && (!l_gs || !l_ge || !l_row)) ||
        (nr > 0 && (!r_gs || !r_ge || !r_row)))
        return fail(LIME_ERR_ARG, "bad set arguments");
    if (set->ctx != ctx) return fail(LIME_ERR_ARG, "set belongs to another context");
    if (set->strand_in || set->row_ties || set->min_shift)
        return fail(LIME_ERR_ARG, "only plain sets extend");
    const int64_t m = nl + set->n + nr, added = nl + nr;
    if (m > 0xffffffffLL) return fail(LIME_ERR_RANGE, "more than 2^32 rows in one set");
    hipSetDevice(ctx->device);
    lime_set *s = new lime_set();
    s->ctx = ctx;
    s->n = m;
    s->n_contigs = set->n_contigs;
    s->off = set->off;
    s->len = set->len;
    s->d_off = set->d_off;
    s->space_keep = set->space_keep;
    s->min_width = set->n ? set->min_width : min_width;
    s->max_width = set->max_width;
    s->has_zero_width = set->has_zero_width;
    if (added > 0) {
        if (set->n) s->min_width = std::min(s->min_width, min_width);
        s->max_width = std::max(s->max_width, max_width);
        s->has_zero_width = s->has_zero_width || has_zero_width != 0;
    }
    int rc = alloc(ctx, &s->gs, (size_t)std::max<int64_t>(m, 1));
    if (rc == LIME_OK) rc = alloc(ctx, &s->ge, (size_t)std::max<int64_t>(m, 1));
    if (rc == LIME_OK) rc = alloc(ctx, &s->row, (size_t)std::max<int64_t>(m, 1));
    if (rc != LIME_OK) {
        lime_set_destroy(s);
        return rc;
    }
    hipError_t e = hipSuccess;
    auto part = [&](int64_t at, int64_t cnt, const uint32_t *g, const uint32_t *x,
                    const uint32_t *r) {
        const size_t bytes = 4 * (size_t)cnt;
        if (!cnt || e != hipSuccess) return;
        e = hipMemcpyAsync(s->gs + at, g, bytes, hipMemcpyDeviceToDevice, S(ctx));
        if (e == hipSuccess) e = hipMemcpyAsync(s->ge + at, x, bytes, hipMemcpyDeviceToDevice, S(ctx));
        if (e == hipSuccess) e = hipMemcpyAsync(s->row + at, r, bytes, hipMemcpyDeviceToDevice, S(ctx));
    };
    part(0, nl, l_gs, l_ge, l_row);
    part(nl, set->n, set->gs, set->ge, set->row);
    part(nl + set->n, nr, r_gs, r_ge, r_row);
    if (e != hipSuccess) {
        lime_set_destroy(s);
        return fail(LIME_ERR_DEVICE, std::string("lime_set_extend_sorted copy: ") + hipGetErrorString(e));
    }
    static const bool check = [] {
        const char *v = getenv("LIME_CHECK_EXTEND");
        return v && v[0] && v[0] != '0';
    }();
    if (check && added > 0) {
        // one pass over the whole new set: order everywhere, and the width
        // bounds over the added rows (the set's own rows are canonical)
        unsigned int *err = nullptr, herr = 0;
        rc = alloc(ctx, &err, 1);
        if (rc == LIME_OK && hipMemsetAsync(err, 0, 4, S(ctx)) != hipSuccess) rc = LIME_ERR_DEVICE;
        if (rc == LIME_OK) {
            hipLaunchKernelGGL(k_check_join, dim3(blocks_for(m, 256)), dim3(256), 0, S(ctx), s->gs,
                               s->ge, m, nl, nl + set->n, min_width, max_width,
                               has_zero_width ? 1 : 0, err);
            rc = read_back(ctx, &herr, err, sizeof(herr));
        }
        release(ctx, err);
        if (rc == LIME_OK && herr) rc = fail(LIME_ERR_ARG, herr & 1u ? "extend: rows out of canonical order"
                                                          : herr & 2u ? "extend: a width outside the bounds"
                                                                      : "extend: a zero-width row without the flag");
        if (rc != LIME_OK) {
            lime_set_destroy(s);
            return rc;
        }
    }
    *out = s;
    return LIME_OK;
}

int lime_set_extend_sorted(lime_ctx *ctx, const lime_set *set, int64_t n, const uint32_t *d_gs,
                           const uint32_t *d_ge, const uint32_t *d_row, uint32_t min_width,
                           uint32_t max_width, int32_t has_zero_width, lime_set **out) {
    return concat_sorted(ctx, set, 0, nullptr, nullptr, nullptr, n, d_gs, d_ge, d_row, min_width,
                         max_width, has_zero_width, out);
}

int lime_set_concat_sorted(lime_ctx *ctx, const lime_set *set, int64_t n_before,
                           const uint32_t *b_gs, const uint32_t *b_ge, const uint32_t *b_row,
                           int64_t n_after, const uint32_t *a_gs, const uint32_t *a_ge,
                           const uint32_t *a_row, uint32_t min_width, uint32_t max_width,
                           int32_t has_zero_width, lime_set **out) {
    return concat_sorted(ctx, set, n_before, b_gs, b_ge, b_row, n_after, a_gs, a_ge, a_row,
                         min_width, max_width, has_zero_width, out);
}

int lime_set_create_global(lime_ctx *ctx, const lime_space *sp, int64_t n, const uint32_t *d_gs,
                           const uint32_t *d_ge, const uint32_t *d_row, lime_set **out) {
    if (!ctx || !sp || !out || n < 0 || (n > 0 && (!d_gs || !d_ge || !d_row)))
        return fail(LIME_ERR_ARG, "bad set arguments");
    if (n > 0xffffffffLL) return fail(LIME_ERR_RANGE, "more than 2^32 rows in one set");
    hipSetDevice(ctx->device);
    lime_set *s = new_set(ctx, sp, n);
    uint32_t *d_len = nullptr;
    int rc = upload_space(ctx, sp, &s->d_off, &d_len, &s->space_keep);
    if (rc == LIME_OK) rc = sort_set_global(ctx, s, d_gs, d_ge, d_row, d_len);
    if (rc != LIME_OK) {
        delete s;
        return rc;
    }
    *out = s;
    return LIME_OK;
}

__global__ void k_positions(uint32_t *__restrict__ p, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) p[i] = (uint32_t)i;
}
// sorted positions -> the caller's row ids and strand codes of those rows
__global__ void k_rows_of_positions(const uint32_t *__restrict__ pos,
                                    const uint32_t *__restrict__ crow,
                                    const int8_t *__restrict__ cstr, uint32_t *__restrict__ orow,
                                    int8_t *__restrict__ ostr, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const uint32_t p = pos[i];
    orow[i] = crow[p];
    ostr[i] = cstr ? cstr[p] : (int8_t)0;
}

int lime_set_create_global_stranded(lime_ctx *ctx, const lime_space *sp, int64_t n,
                                    const uint32_t *d_gs, const uint32_t *d_ge,
                                    const uint32_t *d_row, const int8_t *d_strand,
                                    lime_set **out) {
    if (!ctx || !sp || !out || n < 0 || (n > 0 && (!d_gs || !d_ge || !d_row)))
        return fail(LIME_ERR_ARG, "bad set arguments");
    if (n > 0xffffffffLL) return fail(LIME_ERR_RANGE, "more than 2^32 rows in one set");
    hipSetDevice(ctx->device);
    // sorted with positions as the row ids (so the strand pass and the
    // merge's strand lookups index the caller's codes), then the caller's row
    // ids and the codes gathered per sorted row
    uint32_t *pos;
    int8_t *st;
    LIME_TRY(alloc(ctx, &pos, (size_t)std::max<int64_t>(n, 1)));
    PoolGuard<uint32_t> g0{ctx, pos};
    LIME_TRY(alloc(ctx, &st, (size_t)std::max<int64_t>(n, 1)));
    if (n > 0) {
        hipLaunchKernelGGL(k_positions, dim3(blocks_for(n, 256)), dim3(256), 0, S(ctx), pos, n);
        if (d_strand)
            LIME_HIP(hipMemcpyAsync(st, d_strand, (size_t)n, hipMemcpyDeviceToDevice, S(ctx)));
        else
            LIME_HIP(hipMemsetAsync(st, 0, (size_t)n, S(ctx)));
    }
    lime_set *s = new_set(ctx, sp, n);
    s->strand_in = st;
    s->strand_uniform = !d_strand;
    uint32_t *d_len = nullptr;
    int rc = upload_space(ctx, sp, &s->d_off, &d_len, &s->space_keep);
    if (rc == LIME_OK) rc = sort_set_global(ctx, s, d_gs, d_ge, pos, d_len);
    uint32_t *row = nullptr;
    int8_t *sst = nullptr;
    if (rc == LIME_OK) rc = alloc(ctx, &row, (size_t)std::max<int64_t>(n, 1));
    if (rc == LIME_OK) rc = alloc(ctx, &sst, (size_t)std::max<int64_t>(n, 1));
    if (rc == LIME_OK && n > 0) {
        hipLaunchKernelGGL(k_rows_of_positions, dim3(blocks_for(n, 256)), dim3(256), 0, S(ctx),
                           (const uint32_t *)s->row, d_row, (const int8_t *)st, row, sst, n);
        if (hipGetLastError() != hipSuccess) rc = fail(LIME_ERR_DEVICE, "row gather failed");
    }
    if (rc != LIME_OK) {
        release(ctx, row);
        release(ctx, sst);
        lime_set_destroy(s);
        return rc;
    }
    release(ctx, s->row);
    release(ctx, s->strand_in);
    s->row = row;
    s->strand_in = sst;
    s->strand_sorted = true;
    *out = s;
    return LIME_OK;
}

int64_t lime_set_lower_bound(const lime_set *s, uint32_t gkey) {
    if (!s) return -(int64_t)fail(LIME_ERR_ARG, "set is null");
    lime_ctx *ctx = s->ctx;
    hipSetDevice(ctx->device);
    int64_t *d = nullptr;
    if (int rc = alloc(ctx, &d, 1)) return -(int64_t)rc;
    PoolGuard<int64_t> guard{ctx, d};
    hipLaunchKernelGGL(k_set_lower_bound, dim3(1), dim3(64), 0, S(ctx), (const uint32_t *)s->gs,
                       s->n, gkey, d);
    if (hipError_t e = hipGetLastError())
        return -(int64_t)fail(LIME_ERR_DEVICE, std::string("lower_bound launch: ") +
                                                   hipGetErrorString(e));
    int64_t h = -1;
    if (int rc = read_back(ctx, &h, d, 8)) return -(int64_t)rc;
    return h;
}

__global__ void k_first_reaching(const uint32_t *pmax, int64_t n, uint32_t key, int64_t *out) {
    // first j with pmax[j] > key (pmax non-decreasing); n if none
    if (threadIdx.x == 0) *out = dev::upper_bound(pmax, 0, n, key);
}

int64_t lime_set_first_reaching(const lime_set *s, uint32_t gkey) {
    if (!s) return -(int64_t)fail(LIME_ERR_ARG, "set is null");
    lime_ctx *ctx = s->ctx;
    hipSetDevice(ctx->device);
    if (s->n == 0) return 0;
    if (int rc = build_prefix_max(ctx, s)) return -(int64_t)rc;
    int64_t *d = nullptr;
    if (int rc = alloc(ctx, &d, 1)) return -(int64_t)rc;
    PoolGuard<int64_t> guard{ctx, d};
    hipLaunchKernelGGL(k_first_reaching, dim3(1), dim3(64), 0, S(ctx), (const uint32_t *)s->pmax,
                       s->n, gkey, d);
    if (hipError_t e = hipGetLastError())
        return -(int64_t)fail(LIME_ERR_DEVICE, std::string("first_reaching launch: ") +
                                                   hipGetErrorString(e));
    int64_t h = -1;
    if (int rc = read_back(ctx, &h, d, 8)) return -(int64_t)rc;
    return h;
}

// k searches in one launch (thread i: key i) and one read-back: the
// sharded halos look up one bound per shard
__global__ void k_bounds(const uint32_t *arr, int64_t n, const uint32_t *keys, int k, int upper,
                         int64_t *out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < k) out[i] = upper ? dev::upper_bound(arr, 0, n, keys[i]) : dev::lower_bound(arr, 0, n, keys[i]);
}

static int set_bounds(const lime_set *s, int32_t k, const uint32_t *keys, int64_t *out,
                      bool reaching) {
    if (!s || k < 0 || (k > 0 && (!keys || !out))) return fail(LIME_ERR_ARG, "bad bounds arguments");
    if (k == 0) return LIME_OK;
    lime_ctx *ctx = s->ctx;
    hipSetDevice(ctx->device);
    if (s->n == 0) {
        for (int i = 0; i < k; ++i) out[i] = 0;
        return LIME_OK;
    }
    if (reaching) LIME_TRY(build_prefix_max(ctx, s));
    uint32_t *d_keys = nullptr;
    int64_t *d_out = nullptr;
    LIME_TRY(alloc(ctx, &d_keys, (size_t)k));
    PoolGuard<uint32_t> g0{ctx, d_keys};
    LIME_TRY(alloc(ctx, &d_out, (size_t)k));
    PoolGuard<int64_t> g1{ctx, d_out};
    LIME_HIP(hipMemcpyAsync(d_keys, keys, 4 * (size_t)k, hipMemcpyHostToDevice, S(ctx)));
    hipLaunchKernelGGL(k_bounds, dim3(blocks_for(k, 64)), dim3(64), 0, S(ctx),
                       (const uint32_t *)(reaching ? s->pmax : s->gs), s->n,
                       (const uint32_t *)d_keys, (int)k, reaching ? 1 : 0, d_out);
    LIME_HIP(hipGetLastError());
    return read_back(ctx, out, d_out, 8 * (size_t)k);
}

int lime_set_lower_bounds(const lime_set *s, int32_t k, const uint32_t *gkeys, int64_t *out) {
    return set_bounds(s, k, gkeys, out, false);
}

int lime_set_first_reachings(const lime_set *s, int32_t k, const uint32_t *gkeys, int64_t *out) {
    return set_bounds(s, k, gkeys, out, true);
}

int lime_set_copy_rows_device(const lime_set *s, int64_t first, int64_t count, uint32_t *d_gs,
                              uint32_t *d_ge, uint32_t *d_row) {
    if (!s || first < 0 || count < 0 || first + count > s->n)
        return fail(LIME_ERR_ARG, "row range outside the set");
    lime_ctx *ctx = s->ctx;
    hipSetDevice(ctx->device);
    if (count == 0) return LIME_OK;
    const size_t b = 4 * (size_t)count;
    if (d_gs) LIME_HIP(hipMemcpyAsync(d_gs, s->gs + first, b, hipMemcpyDeviceToDevice, S(ctx)));
    if (d_ge) LIME_HIP(hipMemcpyAsync(d_ge, s->ge + first, b, hipMemcpyDeviceToDevice, S(ctx)));
    if (d_row) LIME_HIP(hipMemcpyAsync(d_row, s->row + first, b, hipMemcpyDeviceToDevice, S(ctx)));
    return LIME_OK;
}

int lime_result_copy_range(const lime_result *r, int64_t first, int64_t count, uint32_t *gs,
                           uint32_t *ge) {
    if (!r || first < 0 || count < 0 || first + count > r->n)
        return fail(LIME_ERR_ARG, "range outside the result");
    lime_ctx *ctx = r->ctx;
    hipSetDevice(ctx->device);
    if (count == 0) return LIME_OK;
    const size_t b = 4 * (size_t)count;
    if (gs) LIME_HIP(hipMemcpyAsync(gs, r->gs + first, b, hipMemcpyDeviceToHost, S(ctx)));
    if (ge) LIME_HIP(hipMemcpyAsync(ge, r->ge + first, b, hipMemcpyDeviceToHost, S(ctx)));
    LIME_HIP(hipStreamSynchronize(S(ctx)));
    return LIME_OK;
}

int lime_set_fill_host(const lime_set *s, int32_t *contig, int64_t *start, int64_t *end,
                       int64_t *row) {
    if (!s) return fail(LIME_ERR_ARG, "set is null");
    lime_ctx *ctx = s->ctx;
    std::vector<uint32_t> gs, ge, rw;
    LIME_TRY(d2h(ctx, gs, (const uint32_t *)s->gs, s->n));
    LIME_TRY(d2h(ctx, ge, (const uint32_t *)s->ge, s->n));
    LIME_TRY(d2h(ctx, rw, (const uint32_t *)s->row, s->n));
    for (int64_t i = 0; i < s->n; ++i) {
        int32_t c = contig_of(s->off, s->n_contigs, gs[i]);
        if (contig) contig[i] = c;
        if (start) start[i] = (int64_t)gs[i] - s->off[c];
        if (end) end[i] = (int64_t)ge[i] - s->off[c];
        if (row) row[i] = rw[i];
    }
    return LIME_OK;
}

static bool same_space(const lime_set *a, const lime_set *b) {
    return a->n_contigs == b->n_contigs && a->off == b->off;
}

// --------------------------------------------------------------- intersect
struct lime_pairs {
    PairsPlan *plan;
    lime_ctx *ctx;
    ClosestPlan *closest = nullptr;  // set instead of plan for lime_closest_count
};

static int pairs_fill(lime_pairs *p, int64_t first, int64_t count, lime_pair *d_out) {
    return p->closest ? closest_fill(p->closest, first, count, d_out)
                      : intersect_fill(p->plan, first, count, d_out);
}

int lime_intersect_count(lime_ctx *ctx, const lime_set *a, const lime_set *b, int64_t threshold,
                         lime_pairs **plan, int64_t *n_pairs) {
    return lime_intersect_count_owned(ctx, a, b, threshold, -1, -1, plan, n_pairs);
}

int lime_intersect_count_owned(lime_ctx *ctx, const lime_set *a, const lime_set *b,
                               int64_t threshold, int64_t a_owned, int64_t b_owned,
                               lime_pairs **plan, int64_t *n_pairs) {
    if (!ctx || !a || !b || !plan) return fail(LIME_ERR_ARG, "bad intersect arguments");
    if (!same_space(a, b)) return fail(LIME_ERR_ARG, "sets live in different coordinate spaces");
    if (a_owned > a->n || b_owned > b->n) return fail(LIME_ERR_ARG, "owned rows exceed set size");
    LIME_TRY(same_ctx(ctx, a));
    LIME_TRY(same_ctx(ctx, b));
    hipSetDevice(ctx->device);
    PairsPlan *pl = nullptr;
    LIME_TRY(intersect_plan(ctx, a, b, threshold, a_owned, b_owned, &pl));
    lime_pairs *p = new lime_pairs{pl, ctx};
    *plan = p;
    if (n_pairs) *n_pairs = plan_total(pl);
    return LIME_OK;
}

int lime_window_count(lime_ctx *ctx, const lime_set *a, const lime_set *b, int64_t distance,
                      lime_pairs **plan, int64_t *n_pairs) {
    if (!ctx || !a || !b || !plan) return fail(LIME_ERR_ARG, "bad window arguments");
    if (!same_space(a, b)) return fail(LIME_ERR_ARG, "sets live in different coordinate spaces");
    if (distance < 0) return fail(LIME_ERR_ARG, "window distance must be >= 0");
    LIME_TRY(same_ctx(ctx, a));
    LIME_TRY(same_ctx(ctx, b));
    hipSetDevice(ctx->device);
    PairsPlan *pl = nullptr;
    LIME_TRY(window_plan(ctx, a, b, distance, &pl));
    *plan = new lime_pairs{pl, ctx};
    if (n_pairs) *n_pairs = plan_total(pl);
    return LIME_OK;
}

int lime_closest_count(lime_ctx *ctx, const lime_set *a, const lime_set *b, int mode,
                       lime_pairs **plan, int64_t *n_pairs) {
    return lime_closest_count_chained(ctx, a, b, mode, 1, nullptr, plan, n_pairs);
}

int lime_closest_count_chained(lime_ctx *ctx, const lime_set *a, const lime_set *b, int mode,
                               int32_t alive_in, int32_t *alive_out, lime_pairs **plan,
                               int64_t *n_pairs) {
    if (!ctx || !a || !b || !plan) return fail(LIME_ERR_ARG, "bad closest arguments");
    if (!same_space(a, b)) return fail(LIME_ERR_ARG, "sets live in different coordinate spaces");
    if (mode != LIME_CLOSEST && mode != LIME_CLOSEST_SINGLE_OVERLAP)
        return fail(LIME_ERR_ARG, "closest mode must be LIME_CLOSEST or LIME_CLOSEST_SINGLE_OVERLAP");
    if (!a->strand_in || !b->strand_in || a->min_shift || b->min_shift)
        return fail(LIME_ERR_ARG,
                    "closest needs sets in full RegionOrdering (lime_set_create_host_stranded)");
    LIME_TRY(same_ctx(ctx, a));
    LIME_TRY(same_ctx(ctx, b));
    hipSetDevice(ctx->device);
    ClosestPlan *cl = nullptr;
    bool out_live = false;
    LIME_TRY(closest_plan(ctx, a, b, mode, alive_in != 0, &out_live, &cl));
    if (alive_out) *alive_out = out_live ? 1 : 0;
    lime_pairs *p = new lime_pairs{nullptr, ctx};
    p->closest = cl;
    *plan = p;
    if (n_pairs) *n_pairs = closest_total(cl);
    return LIME_OK;
}

int lime_closest_rounds(const lime_pairs *plan, int32_t *rounds, int32_t *sequential) {
    if (!plan || !plan->closest) return fail(LIME_ERR_ARG, "not a closest plan");
    bool seq = false;
    const int r = closest_rounds(plan->closest, &seq);
    if (rounds) *rounds = r;
    if (sequential) *sequential = seq ? 1 : 0;
    return LIME_OK;
}

int lime_intersect_fill_device(lime_pairs *plan, int64_t first, int64_t count, lime_pair *d_out) {
    if (!plan || (count > 0 && !d_out)) return fail(LIME_ERR_ARG, "bad fill arguments");
    hipSetDevice(plan->ctx->device);
    return pairs_fill(plan, first, count, d_out);
}

int lime_intersect_fill_host(lime_pairs *plan, int64_t first, int64_t count, lime_pair *out) {
    if (!plan || (count > 0 && !out)) return fail(LIME_ERR_ARG, "bad fill arguments");
    lime_ctx *ctx = plan->ctx;
    hipSetDevice(ctx->device);
    const int64_t chunk = 1 << 24;
    lime_pair *stage = nullptr;
    LIME_TRY(alloc(ctx, &stage, (size_t)std::min(chunk, std::max(count, (int64_t)1))));
    PoolGuard<lime_pair> guard{ctx, stage};  // released on every return path
    for (int64_t f = 0; f < count; f += chunk) {
        const int64_t c = std::min(chunk, count - f);
        LIME_TRY(pairs_fill(plan, first + f, c, stage));
        LIME_HIP(hipMemcpyAsync(out + f, stage, sizeof(lime_pair) * (size_t)c,
                                hipMemcpyDeviceToHost, S(ctx)));
        LIME_HIP(hipStreamSynchronize(S(ctx)));
    }
    return LIME_OK;
}

int lime_intersect_checksum(lime_pairs *plan, uint64_t *sum, uint64_t *xr) {
    if (!plan || !sum || !xr) return fail(LIME_ERR_ARG, "bad checksum arguments");
    hipSetDevice(plan->ctx->device);
    if (plan->closest) return closest_checksum(plan->closest, sum, xr);
    return intersect_checksum(plan->plan, sum, xr);
}

int lime_pairs_checksum_device(lime_ctx *ctx, const lime_pair *d_pairs, int64_t count,
                               uint64_t *sum, uint64_t *xr) {
    if (!ctx || count < 0 || (count > 0 && !d_pairs) || !sum || !xr)
        return fail(LIME_ERR_ARG, "bad checksum arguments");
    hipSetDevice(ctx->device);
    unsigned long long *d_out = nullptr;
    LIME_TRY(alloc(ctx, &d_out, 2));
    PoolGuard<unsigned long long> g{ctx, d_out};
    LIME_HIP(hipMemsetAsync(d_out, 0, 16, S(ctx)));
    if (count > 0)
        hipLaunchKernelGGL(k_pairs_hash, dim3(std::min<unsigned>(blocks_for(count, 256), 8192u)),
                           dim3(256), 0, S(ctx), reinterpret_cast<const uint4 *>(d_pairs), count,
                           d_out);
    LIME_HIP(hipGetLastError());
    uint64_t h[2];
    LIME_TRY(read_back(ctx, h, d_out, 16));
    *sum = h[0];
    *xr = h[1];
    return LIME_OK;
}

int lime_pairs_destroy(lime_pairs *plan) {
    if (!plan) return LIME_OK;
    if (plan->closest)
        closest_free(plan->closest);
    else
        intersect_free(plan->plan);
    delete plan;
    return LIME_OK;
}

// ----------------------------------------------------------------- results
int lime_merge(lime_ctx *ctx, const lime_set *a, lime_result **out, int64_t *n_runs) {
    if (!ctx || !a || !out) return fail(LIME_ERR_ARG, "bad merge arguments");
    LIME_TRY(same_ctx(ctx, a));
    hipSetDevice(ctx->device);
    lime_result *r = new_result(ctx, a);
    r->src = a;
    int rc = merge_runs(ctx, a, r, true);
    if (rc != LIME_OK) {
        delete r;
        return rc;
    }
    *out = r;
    if (n_runs) *n_runs = r->n;
    return LIME_OK;
}

int lime_subtract(lime_ctx *ctx, const lime_set *a, const lime_set *b, int64_t threshold, int mode,
                  lime_result **out, int64_t *n) {
    if (!ctx || !a || !b || !out) return fail(LIME_ERR_ARG, "bad subtract arguments");
    if (mode != LIME_SUBTRACT_LIME && mode != LIME_SUBTRACT_SET)
        return fail(LIME_ERR_ARG, "unknown subtract mode");
    if (!same_space(a, b)) return fail(LIME_ERR_ARG, "sets live in different coordinate spaces");
    LIME_TRY(same_ctx(ctx, a));
    LIME_TRY(same_ctx(ctx, b));
    hipSetDevice(ctx->device);
    lime_result *r = new_result(ctx, a);
    int rc = subtract_run(ctx, a, b, threshold, mode, r);
    if (rc != LIME_OK) {
        delete r;
        return rc;
    }
    *out = r;
    if (n) *n = r->n;
    return LIME_OK;
}

int lime_complement(lime_ctx *ctx, const lime_space *genome, const lime_set *a, lime_result **out,
                    int64_t *n) {
    if (!ctx || !genome || !a || !out) return fail(LIME_ERR_ARG, "bad complement arguments");
    if (genome->n != a->n_contigs || genome->off != a->off)
        return fail(LIME_ERR_CONTIG, "set was not created in the genome's coordinate space");
    LIME_TRY(same_ctx(ctx, a));
    hipSetDevice(ctx->device);
    lime_result runs;
    runs.ctx = ctx;
    LIME_TRY(merge_runs(ctx, a, &runs, false));
    uint32_t *d_len = nullptr;
    uint32_t *d_off = nullptr;
    LIME_TRY(upload_space(ctx, genome, &d_off, &d_len));
    lime_result *r = new_result(ctx, a);
    int rc = complement_run(ctx, &runs, d_off, d_len, genome->n, r);
    release(ctx, runs.gs);
    release(ctx, runs.ge);

    if (rc != LIME_OK) {
        delete r;
        return rc;
    }
    *out = r;
    if (n) *n = r->n;
    return LIME_OK;
}

int lime_complement_runs(lime_ctx *ctx, const lime_space *genome, int64_t n, const uint32_t *d_gs,
                         const uint32_t *d_ge, int64_t lo, int64_t hi, lime_result **out,
                         int64_t *n_regions) {
    if (!ctx || !genome || !out || n < 0 || (n > 0 && (!d_gs || !d_ge)) || lo < 0 || hi < lo)
        return fail(LIME_ERR_ARG, "bad complement arguments");
    if (n > 0xffffffffLL) return fail(LIME_ERR_RANGE, "more than 2^32 runs");
    hipSetDevice(ctx->device);
    uint32_t *d_len = nullptr, *d_off = nullptr;
    LIME_TRY(upload_space(ctx, genome, &d_off, &d_len));
    lime_result runs;  // (borrowed arrays)
    runs.ctx = ctx;
    runs.n = n;
    runs.gs = const_cast<uint32_t *>(d_gs);
    runs.ge = const_cast<uint32_t *>(d_ge);
    lime_result *r = new lime_result();
    r->ctx = ctx;
    r->off = genome->off;
    r->n_contigs = genome->n;
    const uint32_t whi = hi >= 0xffffffffLL ? 0xffffffffu : (uint32_t)hi;
    int rc = complement_run(ctx, &runs, d_off, d_len, genome->n, r, (uint32_t)std::min<int64_t>(lo, whi), whi);
    runs.gs = runs.ge = nullptr;
    if (rc != LIME_OK) {
        lime_result_destroy(r);
        return rc;
    }
    *out = r;
    if (n_regions) *n_regions = r->n;
    return LIME_OK;
}

// merge results: the run of every sorted input row and that row's id,
// copied to caller device buffers (n = the merged set's rows)
int lime_result_copy_run_ids_device(const lime_result *r, uint32_t *d_run, uint32_t *d_row) {
    if (!r) return fail(LIME_ERR_ARG, "result is null");
    if (!r->run_of_sorted || !r->src) return fail(LIME_ERR_ARG, "not a merge result");
    lime_ctx *ctx = r->ctx;
    hipSetDevice(ctx->device);
    const size_t b = 4 * (size_t)r->src->n;
    if (b && d_run)
        LIME_HIP(hipMemcpyAsync(d_run, r->run_of_sorted, b, hipMemcpyDeviceToDevice, S(ctx)));
    if (b && d_row) LIME_HIP(hipMemcpyAsync(d_row, r->src->row, b, hipMemcpyDeviceToDevice, S(ctx)));
    return LIME_OK;
}

int lime_result_copy_rows_device(const lime_result *r, int64_t first, int64_t count,
                                 uint32_t *d_gs, uint32_t *d_ge) {
    if (!r || first < 0 || count < 0 || first + count > r->n)
        return fail(LIME_ERR_ARG, "bad copy range");
    lime_ctx *ctx = r->ctx;
    hipSetDevice(ctx->device);
    if (count && d_gs)
        LIME_HIP(hipMemcpyAsync(d_gs, r->gs + first, 4 * (size_t)count, hipMemcpyDeviceToDevice,
                                S(ctx)));
    if (count && d_ge)
        LIME_HIP(hipMemcpyAsync(d_ge, r->ge + first, 4 * (size_t)count, hipMemcpyDeviceToDevice,
                                S(ctx)));
    return LIME_OK;
}

// strand codes of runs [first, first + count) of a stranded merge (host)
int lime_result_run_strands(const lime_result *r, int64_t first, int64_t count, int8_t *out) {
    if (!r || !out || first < 0 || count < 0 || first + count > r->n)
        return fail(LIME_ERR_ARG, "bad strand range");
    if (!r->run_strand) {
        memset(out, 0, (size_t)count);
        return LIME_OK;
    }
    lime_ctx *ctx = r->ctx;
    hipSetDevice(ctx->device);
    if (count) LIME_TRY(read_back(ctx, out, r->run_strand + first, (size_t)count));
    return LIME_OK;
}

int64_t lime_result_size(const lime_result *r) { return r ? r->n : -1; }

int lime_result_fill_host(const lime_result *r, int32_t *contig, int64_t *start, int64_t *end,
                          int64_t *a_row, int64_t *b_row) {
    if (!r) return fail(LIME_ERR_ARG, "result is null");
    lime_ctx *ctx = r->ctx;
    hipSetDevice(ctx->device);
    std::vector<uint32_t> gs, ge, ar, br;
    LIME_TRY(d2h(ctx, gs, (const uint32_t *)r->gs, r->n));
    LIME_TRY(d2h(ctx, ge, (const uint32_t *)r->ge, r->n));
    if (a_row) LIME_TRY(d2h(ctx, ar, (const uint32_t *)r->a_row, r->a_row ? r->n : 0));
    if (b_row) LIME_TRY(d2h(ctx, br, (const uint32_t *)r->b_row, r->b_row ? r->n : 0));
    for (int64_t i = 0; i < r->n; ++i) {
        int32_t c = contig_of(r->off, r->n_contigs, gs[i]);
        if (contig) contig[i] = c;
        if (start) start[i] = (int64_t)gs[i] - r->off[c];
        if (end) end[i] = (int64_t)ge[i] - r->off[c];
        if (a_row) a_row[i] = r->a_row ? (int64_t)ar[i] : -1;
        if (b_row) b_row[i] = r->b_row ? (br[i] == 0xffffffffu ? -1 : (int64_t)br[i]) : -1;
    }
    return LIME_OK;
}

int lime_result_run_of_row(const lime_result *r, int64_t *run_of_row) {
    if (!r || !run_of_row) return fail(LIME_ERR_ARG, "bad arguments");
    if (!r->run_of_sorted || !r->src) return fail(LIME_ERR_ARG, "not a merge result");
    lime_ctx *ctx = r->ctx;
    std::vector<uint32_t> rid, row;
    LIME_TRY(d2h(ctx, rid, (const uint32_t *)r->run_of_sorted, r->src->n));
    LIME_TRY(d2h(ctx, row, (const uint32_t *)r->src->row, r->src->n));
    for (int64_t i = 0; i < r->src->n; ++i) run_of_row[row[i]] = rid[i];
    return LIME_OK;
}

static int names_of(const char *const *names, int32_t n, std::vector<std::string> &v) {
    if (n > 0 && !names) return fail(LIME_ERR_ARG, "contig names are null");
    for (int32_t i = 0; i < n; ++i) {
        if (!names[i]) return fail(LIME_ERR_ARG, "contig name is null");
        v.emplace_back(names[i]);
    }
    return LIME_OK;
}

int lime_set_format_bed(const lime_set *s, const char *const *names, char *out, int64_t cap,
                        int64_t *len) {
    if (!s || !len) return fail(LIME_ERR_ARG, "bad format arguments");
    std::vector<std::string> nm;
    LIME_TRY(names_of(names, s->n_contigs, nm));
    hipSetDevice(s->ctx->device);
    return format_bed(s->ctx, s->off, nm, s->n, s->gs, s->ge, nullptr, out, cap, len);
}

int lime_result_format_bed(const lime_result *r, const char *const *names, char *out,
                           int64_t cap, int64_t *len) {
    if (!r || !len) return fail(LIME_ERR_ARG, "bad format arguments");
    std::vector<std::string> nm;
    LIME_TRY(names_of(names, r->n_contigs, nm));
    hipSetDevice(r->ctx->device);
    return format_bed(r->ctx, r->off, nm, r->n, r->gs, r->ge, nullptr, out, cap, len);
}

int lime_result_device_arrays(const lime_result *r, const uint32_t **gs, const uint32_t **ge) {
    if (!r) return fail(LIME_ERR_ARG, "result is null");
    if (gs) *gs = r->gs;
    if (ge) *ge = r->ge;
    return LIME_OK;
}

int lime_result_checksum(const lime_result *r, uint64_t *reg_sum, uint64_t *reg_xor,
                         uint64_t *grp_sum, uint64_t *grp_xor) {
    if (!r || !reg_sum || !reg_xor) return fail(LIME_ERR_ARG, "bad checksum arguments");
    lime_ctx *ctx = r->ctx;
    hipSetDevice(ctx->device);
    uint32_t *d_off = nullptr;
    unsigned long long *d_out = nullptr;
    LIME_TRY(alloc(ctx, &d_off, (size_t)r->n_contigs + 1));
    PoolGuard<uint32_t> g1{ctx, d_off};
    LIME_TRY(alloc(ctx, &d_out, 4));
    PoolGuard<unsigned long long> g2{ctx, d_out};
    LIME_HIP(hipMemcpyAsync(d_off, r->off.data(), 4 * ((size_t)r->n_contigs + 1),
                            hipMemcpyHostToDevice, S(ctx)));
    LIME_HIP(hipMemsetAsync(d_out, 0, 32, S(ctx)));
    const bool grp = r->run_of_sorted && r->src;
    const int64_t nrows = grp ? r->src->n : 0;
    const int64_t work = std::max<int64_t>(std::max<int64_t>(r->n, nrows), 1);
    const unsigned grid = std::min<unsigned>(blocks_for(work, 256), 4096u);
    hipLaunchKernelGGL(k_result_checksum, dim3(grid), dim3(256), 0, S(ctx),
                       (const uint32_t *)r->gs, (const uint32_t *)r->ge,
                       (const uint32_t *)r->a_row, (const uint32_t *)r->b_row, r->n,
                       (const uint32_t *)d_off, r->n_contigs,
                       grp ? (const uint32_t *)r->src->row : nullptr,
                       grp ? (const uint32_t *)r->run_of_sorted : nullptr, nrows, d_out);
    LIME_HIP(hipGetLastError());
    // (hipMemcpy from pageable memory would not order against the stream: the
    // pinned-scratch read_back does)
    uint64_t h[4];
    LIME_TRY(read_back(ctx, h, d_out, 32));
    *reg_sum = h[0];
    *reg_xor = h[1];
    if (grp_sum) *grp_sum = h[2];
    if (grp_xor) *grp_xor = h[3];
    return LIME_OK;
}

int lime_result_destroy(lime_result *r) {
    if (!r) return LIME_OK;
    lime_ctx *ctx = r->ctx;
    release(ctx, r->gs);
    release(ctx, r->ge);
    release(ctx, r->a_row);
    release(ctx, r->b_row);
    release(ctx, r->run_of_sorted);
    release(ctx, r->run_strand);
    delete r;
    return LIME_OK;
}

// ------------------------------------------------------------------ bitset
int lime_bitset_from_set(lime_ctx *ctx, const lime_set *a, lime_bitset **out) {
    if (!ctx || !a || !out) return fail(LIME_ERR_ARG, "bad bitset arguments");
    LIME_TRY(same_ctx(ctx, a));
    hipSetDevice(ctx->device);
    lime_bitset *bs = new lime_bitset();
    bs->ctx = ctx;
    bs->n_contigs = a->n_contigs;
    bs->off = a->off;
    bs->len = a->len;
    int rc = bitset_build(ctx, a, bs);
    if (rc != LIME_OK) {
        delete bs;
        return rc;
    }
    *out = bs;
    return LIME_OK;
}

int lime_bitset_from_device(lime_ctx *ctx, const lime_space *sp, int64_t n,
                            const int32_t *d_contig, const uint32_t *d_start,
                            const uint32_t *d_end, lime_bitset **out) {
    if (!ctx || !sp || !out || n < 0 || (n > 0 && (!d_contig || !d_start || !d_end)))
        return fail(LIME_ERR_ARG, "bad bitset arguments");
    if (n > 0xffffffffLL) return fail(LIME_ERR_RANGE, "more than 2^32 rows in one set");
    hipSetDevice(ctx->device);
    // rows binned by tile in one counting scatter, painted tile by tile
    uint32_t *d_off = nullptr, *d_len = nullptr;
    LIME_TRY(upload_space(ctx, sp, &d_off, &d_len));  // (borrowed)
    lime_bitset *bs = new lime_bitset();
    bs->ctx = ctx;
    bs->n_contigs = sp->n;
    bs->off = sp->off;
    bs->len = sp->len;
    int rc = bitset_build_rows(ctx, sp, n, d_contig, d_start, d_end, d_off, d_len, 0, sp->span,
                               bs);
    if (rc != LIME_OK) {
        bitset_free(bs);
        delete bs;
        return rc;
    }
    *out = bs;
    return LIME_OK;
}

int lime_bitset_from_global(lime_ctx *ctx, const lime_space *sp, int64_t lo, int64_t hi,
                            int64_t n, const uint32_t *d_gs, const uint32_t *d_ge,
                            lime_bitset **out) {
    if (!ctx || !sp || !out || n < 0 || (n > 0 && (!d_gs || !d_ge)))
        return fail(LIME_ERR_ARG, "bad bitset arguments");
    if (lo < 0 || hi < lo || hi > sp->span || lo % 64 != 0)
        return fail(LIME_ERR_ARG, "window must satisfy 0 <= lo <= hi <= span, lo % 64 == 0");
    if (n > 0xffffffffLL) return fail(LIME_ERR_RANGE, "more than 2^32 rows in one set");
    hipSetDevice(ctx->device);
    lime_bitset *bs = new lime_bitset();
    bs->ctx = ctx;
    bs->n_contigs = sp->n;
    bs->off = sp->off;
    bs->len = sp->len;
    int rc = bitset_build_rows(ctx, sp, n, nullptr, d_gs, d_ge, nullptr, nullptr, lo, hi, bs);
    if (rc != LIME_OK) {
        bitset_free(bs);
        delete bs;
        return rc;
    }
    *out = bs;
    return LIME_OK;
}

// k row sets -> the bits of their AND, one fused paint (bitset.hip)
static int bitset_and_entry(lime_ctx *ctx, const lime_space *sp, int64_t lo, int64_t hi,
                            int32_t k, const int64_t *n, const int32_t *const *d_contig,
                            const uint32_t *const *d_start, const uint32_t *const *d_end,
                            bool global, lime_bitset **out) {
    if (!ctx || !sp || !out || !n || k < 1 || !d_start || !d_end ||
        (!global && !d_contig))
        return fail(LIME_ERR_ARG, "bad bitset and arguments");
    for (int i = 0; i < k; ++i) {
        if (n[i] < 0 || (n[i] > 0 && (!d_start[i] || !d_end[i] || (!global && !d_contig[i]))))
            return fail(LIME_ERR_ARG, "bad bitset and arguments");
        if (n[i] > 0xffffffffLL) return fail(LIME_ERR_RANGE, "more than 2^32 rows in one set");
    }
    hipSetDevice(ctx->device);
    uint32_t *d_off = nullptr, *d_len = nullptr;
    if (!global) LIME_TRY(upload_space(ctx, sp, &d_off, &d_len));  // (borrowed)
    std::vector<const int32_t *> contig(k, nullptr);
    if (!global)
        for (int i = 0; i < k; ++i) contig[i] = d_contig[i];
    lime_bitset *bs = new lime_bitset();
    bs->ctx = ctx;
    bs->n_contigs = sp->n;
    bs->off = sp->off;
    bs->len = sp->len;
    int rc = bitset_and_rows(ctx, sp, k, n, contig.data(), d_start, d_end, d_off, d_len, lo, hi,
                             bs);
    if (rc != LIME_OK) {
        bitset_free(bs);
        delete bs;
        return rc;
    }
    *out = bs;
    return LIME_OK;
}

int lime_bitset_and_from_device(lime_ctx *ctx, const lime_space *sp, int32_t k, const int64_t *n,
                                const int32_t *const *d_contig, const uint32_t *const *d_start,
                                const uint32_t *const *d_end, lime_bitset **out) {
    if (!sp) return fail(LIME_ERR_ARG, "bad bitset and arguments");
    return bitset_and_entry(ctx, sp, 0, sp->span, k, n, d_contig, d_start, d_end, false, out);
}

int lime_bitset_and_from_global(lime_ctx *ctx, const lime_space *sp, int64_t lo, int64_t hi,
                                int32_t k, const int64_t *n, const uint32_t *const *d_gstart,
                                const uint32_t *const *d_gend, lime_bitset **out) {
    if (!sp) return fail(LIME_ERR_ARG, "bad bitset and arguments");
    if (lo < 0 || hi < lo || hi > sp->span || lo % 64 != 0)
        return fail(LIME_ERR_ARG, "window must satisfy 0 <= lo <= hi <= span, lo % 64 == 0");
    return bitset_and_entry(ctx, sp, lo, hi, k, n, nullptr, d_gstart, d_gend, true, out);
}

int lime_bitset_window(const lime_bitset *bs, int64_t *lo, int64_t *n_words) {
    if (!bs) return fail(LIME_ERR_ARG, "bitset is null");
    if (lo) *lo = bs->word0 * 64;
    if (n_words) *n_words = bs->n_words;
    return LIME_OK;
}

int lime_route_rows(lime_ctx *ctx, const lime_space *sp, int64_t n, const int32_t *d_contig,
                    const uint32_t *d_start, const uint32_t *d_end, uint32_t row_base,
                    int32_t n_shards, const uint32_t *splits, int clip, int64_t cap,
                    uint32_t *d_gs, uint32_t *d_ge, uint32_t *d_row, int64_t *counts,
                    const int8_t *d_strand_in, int8_t *d_strand_out) {
    if (!ctx || !sp || !splits || !counts || n < 0 || (n > 0 && (!d_start || !d_end)))
        return fail(LIME_ERR_ARG, "bad route arguments");
    if (n > 0xffffffffLL) return fail(LIME_ERR_RANGE, "more than 2^32 rows in one call");
    hipSetDevice(ctx->device);
    return route_rows(ctx, sp, n, d_contig, d_start, d_end, row_base, n_shards, splits, clip, cap,
                      d_gs, d_ge, d_row, counts, d_strand_in, d_strand_out);
}

int lime_route_rows_interleaved(lime_ctx *ctx, const lime_space *sp, int64_t n,
                                const int32_t *d_contig, const uint32_t *d_start,
                                const uint32_t *d_end, uint32_t row_base, int32_t n_shards,
                                const uint32_t *splits, int clip, int64_t cap, int32_t k,
                                uint32_t *d_rows, int64_t *counts) {
    if (!ctx || !sp || !splits || !counts || n < 0 || (n > 0 && (!d_start || !d_end)) ||
        (k != 2 && k != 3) || (cap > 0 && !d_rows))
        return fail(LIME_ERR_ARG, "bad route arguments");
    if (n > 0xffffffffLL) return fail(LIME_ERR_RANGE, "more than 2^32 rows in one call");
    hipSetDevice(ctx->device);
    uint32_t dummy = 0;  // (the column pointers are unused in interleaved mode)
    return route_rows(ctx, sp, n, d_contig, d_start, d_end, row_base, n_shards, splits, clip, cap,
                      &dummy, &dummy, nullptr, counts, nullptr, nullptr, d_rows, k);
}

int lime_deinterleave_u32(lime_ctx *ctx, int64_t n, int32_t k, const uint32_t *d_src,
                          uint32_t *d_dst0, uint32_t *d_dst1, uint32_t *d_dst2) {
    if (!ctx) return fail(LIME_ERR_ARG, "bad deinterleave arguments");
    hipSetDevice(ctx->device);
    return deinterleave_u32(ctx, n, k, d_src, d_dst0, d_dst1, d_dst2);
}

int lime_sample_starts(lime_ctx *ctx, const lime_space *sp, int64_t n, const int32_t *d_contig,
                       const uint32_t *d_start, int32_t k, uint32_t *d_out) {
    if (!ctx || !sp || n < 0 || k < 0 || (n > 0 && k > 0 && (!d_start || !d_out)))
        return fail(LIME_ERR_ARG, "bad sample arguments");
    hipSetDevice(ctx->device);
    return sample_starts(ctx, sp, n, d_contig, d_start, k, d_out);
}

static lime_result *bitset_result(lime_ctx *ctx, const lime_bitset *b) {
    lime_result *r = new lime_result();
    r->ctx = ctx;
    r->off = b->off;
    r->n_contigs = b->n_contigs;
    return r;
}

int lime_bitset_runs(lime_ctx *ctx, int op, const lime_bitset *a, const lime_bitset *b,
                     lime_result **out, int64_t *n) {
    if (!ctx || !a || !out || op < 0 || op > 3 || ((op == 2 || op == 3) && !b))
        return fail(LIME_ERR_ARG, "bad bitset op arguments");
    if (b && (b->off != a->off || b->word0 != a->word0 || b->n_words != a->n_words))
        return fail(LIME_ERR_ARG, "bitsets over different spaces / windows");
    if (a->ctx != ctx || (b && b->ctx != ctx))
        return fail(LIME_ERR_ARG, "bitset belongs to another context (one context per thread)");
    hipSetDevice(ctx->device);
    const lime_bitset *sets[2] = {a, b};
    lime_result *r = bitset_result(ctx, a);
    int rc = bitset_runs(ctx, op, b ? 2 : 1, sets, r);
    if (rc != LIME_OK) {
        delete r;
        return rc;
    }
    *out = r;
    if (n) *n = r->n;
    return LIME_OK;
}

int lime_bitset_and_runs(lime_ctx *ctx, int k, const lime_bitset *const *sets, lime_result **out,
                         int64_t *n) {
    if (!ctx || k < 1 || !sets || !out) return fail(LIME_ERR_ARG, "bad bitset and arguments");
    for (int i = 0; i < k; ++i) {
        if (!sets[i]) return fail(LIME_ERR_ARG, "bitset is null");
        if (sets[i]->off != sets[0]->off || sets[i]->word0 != sets[0]->word0 ||
            sets[i]->n_words != sets[0]->n_words)
            return fail(LIME_ERR_ARG, "bitsets over different spaces / windows");
        if (sets[i]->ctx != ctx)
            return fail(LIME_ERR_ARG, "bitset belongs to another context (one context per thread)");
    }
    hipSetDevice(ctx->device);
    lime_result *r = bitset_result(ctx, sets[0]);
    int rc = bitset_runs(ctx, 4, k, sets, r);
    if (rc != LIME_OK) {
        delete r;
        return rc;
    }
    *out = r;
    if (n) *n = r->n;
    return LIME_OK;
}

int64_t lime_bitset_popcount(lime_ctx *ctx, const lime_bitset *a) {
    if (!ctx || !a || a->ctx != ctx) return -1;
    hipSetDevice(ctx->device);
    return bitset_popcount(ctx, a);
}

int lime_bitset_drop_bins(lime_ctx *ctx, lime_bitset *bs) {
    if (!ctx || !bs || bs->ctx != ctx) return fail(LIME_ERR_ARG, "bad bitset");
    hipSetDevice(ctx->device);
    return bitset_drop_bins(ctx, bs);
}

int lime_bitset_destroy(lime_bitset *bs) {
    if (!bs) return LIME_OK;
    bitset_free(bs);
    delete bs;
    return LIME_OK;
}

// ------------------------------------------------------------------- synth
int lime_synth_uniform(lime_ctx *ctx, const lime_space *sp, int64_t n, uint64_t seed,
                       uint32_t lo, uint32_t hi, int32_t *d_contig, uint32_t *d_start,
                       uint32_t *d_end) {
    if (!ctx || !sp) return fail(LIME_ERR_ARG, "bad synth arguments");
    hipSetDevice(ctx->device);
    return synth(ctx, sp, 0, 0, n, seed, lo, hi, 0, 0, d_contig, d_start, d_end);
}

int lime_synth_uniform_rows(lime_ctx *ctx, const lime_space *sp, int64_t first, int64_t n,
                            uint64_t seed, uint32_t lo, uint32_t hi, int32_t *d_contig,
                            uint32_t *d_start, uint32_t *d_end) {
    if (!ctx || !sp) return fail(LIME_ERR_ARG, "bad synth arguments");
    hipSetDevice(ctx->device);
    return synth(ctx, sp, 0, first, n, seed, lo, hi, 0, 0, d_contig, d_start, d_end);
}

int lime_synth_pileup(lime_ctx *ctx, const lime_space *sp, int64_t n, uint64_t seed,
                      int64_t n_centres, uint32_t sigma, uint32_t lo, uint32_t hi,
                      int32_t *d_contig, uint32_t *d_start, uint32_t *d_end) {
    if (!ctx || !sp) return fail(LIME_ERR_ARG, "bad synth arguments");
    hipSetDevice(ctx->device);
    return synth(ctx, sp, 1, 0, n, seed, lo, hi, n_centres, sigma, d_contig, d_start, d_end);
}

int lime_synth_pileup_rows(lime_ctx *ctx, const lime_space *sp, int64_t first, int64_t n,
                           uint64_t seed, int64_t n_centres, uint32_t sigma, uint32_t lo,
                           uint32_t hi, int32_t *d_contig, uint32_t *d_start, uint32_t *d_end) {
    if (!ctx || !sp) return fail(LIME_ERR_ARG, "bad synth arguments");
    hipSetDevice(ctx->device);
    return synth(ctx, sp, 1, first, n, seed, lo, hi, n_centres, sigma, d_contig, d_start, d_end);
}

// ----------------------------------------------------------- host helpers
int lime_contig_rank(int32_t n, const char *const *names, int32_t *rank_out) {
    if (n < 0 || (n > 0 && (!names || !rank_out))) return fail(LIME_ERR_ARG, "bad rank arguments");
    std::vector<std::vector<uint16_t>> u(n);
    for (int32_t i = 0; i < n; ++i) {
        if (!names[i]) return fail(LIME_ERR_ARG, "null contig name");
        u[i] = utf16(names[i]);
    }
    std::vector<int32_t> idx(n);
    for (int32_t i = 0; i < n; ++i) idx[i] = i;
    std::stable_sort(idx.begin(), idx.end(), [&](int32_t x, int32_t y) { return u[x] < u[y]; });
    int32_t rank = -1;
    for (int32_t k = 0; k < n; ++k) {
        if (k == 0 || u[idx[k]] != u[idx[k - 1]]) ++rank;
        rank_out[idx[k]] = rank;
    }
    return LIME_OK;
}

}  // extern "C"

// bedparse.hip -- BED text -> interval arrays on the device (the ADAM
// sc.loadBed replacement of SURVEY.md 8(f) row 1: cli/Intersection.scala:42-45,
// cli/Merge.scala:37, cli/Complement.scala:42).  Same record rules as the host
// reader (bed.cpp): tab-separated fields (runs of spaces if a line has no
// tab); empty, '#', "track" and "browser" lines skipped; chrom, start, end
// [, name [, score [, strand]]]; strand '+' 1, '-' 2, '?' 3, else 0; contig
// ids in order of first appearance.
//
// Kernels (the text is read 3 times: HBM / L2-bound byte work, no MFMA):
//   k_nl_count   '\n' per 16 KiB tile (16-B loads, zero-byte bit trick)
//   scan         tile offsets
//   k_nl_write   start offset of every line
//   k_parse      thread per line: classify, split, parse start / end /
//                strand, hash the chrom field (FNV-1a 64) into an
//                open-addressing contig table; first line per name by atomicMin
//   scan         record index of every record line
//   k_emit       compaction + contig id from the table; the chrom bytes are
//                compared with the table's representative line, so a hash
//                collision is an error, never a silent merge of two names
#include <algorithm>

#include "common.hpp"

struct lime_dbed {
    lime_ctx *ctx = nullptr;
    int64_t n = 0;
    std::vector<std::string> names;
    int32_t *contig = nullptr;
    uint32_t *start = nullptr, *end = nullptr;
    int8_t *strand = nullptr;
    int64_t *name_off = nullptr;  // byte offset of the 4th column in the text
    uint32_t *name_len = nullptr;
    bool remapped = false;  // contig ids rewritten by lime_dbed_remap_contigs
};

namespace lime {
void bed_free_device(lime_dbed *d);
namespace {

constexpr int PB = 256;
constexpr int PBYTES = 64;            // bytes per thread in the newline passes
constexpr int PTILE = PB * PBYTES;    // 16 KiB
constexpr uint32_t HCAP = 1u << 16;   // contig table slots

struct LineOut {
    uint32_t *flag;  // 1 = record
    uint32_t *slot;  // contig table slot
    uint32_t *start, *end;
    int8_t *strand;
    int64_t *name_off;
    uint32_t *name_len;
    int64_t *chrom_off;
    uint32_t *chrom_len;
};

__device__ __forceinline__ uint32_t count_nl16(uint4 v) {
    uint32_t c = 0;
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        // bytes equal to 0x0a: zero-byte test on w ^ 0x0a0a0a0a (exact when
        // counted per byte with the borrow-free form below)
        const uint32_t x = w[k] ^ 0x0a0a0a0au;
        const uint32_t z = ~(((x & 0x7f7f7f7fu) + 0x7f7f7f7fu) | x | 0x7f7f7f7fu);
        c += __popc(z);
    }
    return c;
}

__global__ __launch_bounds__(PB) void k_nl_count(const uint8_t *__restrict__ t, int64_t n,
                                                 uint32_t *__restrict__ tcnt) {
    const int64_t tile0 = (int64_t)blockIdx.x * PTILE;
    uint32_t c = 0;
#pragma unroll
    for (int k = 0; k < PBYTES / 16; ++k) {
        const int64_t p = tile0 + ((int64_t)k * PB + threadIdx.x) * 16;  // lane-consecutive
        if (p + 16 <= n) {
            c += count_nl16(*reinterpret_cast<const uint4 *>(t + p));
        } else {
            for (int64_t q = p; q < n && q < p + 16; ++q) c += t[q] == '\n';
        }
    }
    c = dev::wave_reduce_sum(c);
    __shared__ uint32_t ws[PB / 64];
    if (dev::lane_id() == 0) ws[threadIdx.x / 64] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t s = 0;
        for (int i = 0; i < PB / 64; ++i) s += ws[i];
        tcnt[blockIdx.x] = s;
    }
}

// line_start[0] = 0; line_start[1 + k] = offset after the k-th '\n'
__global__ __launch_bounds__(PB) void k_nl_write(const uint8_t *__restrict__ t, int64_t n,
                                                 const uint32_t *__restrict__ toff,
                                                 int64_t *__restrict__ line_start) {
    __shared__ uint32_t scratch[PB / 64 + 1];
    const int64_t tile0 = (int64_t)blockIdx.x * PTILE;
    uint32_t base = toff[blockIdx.x];
    if (blockIdx.x == 0 && threadIdx.x == 0) line_start[0] = 0;
    // chunk k of thread t is tile chunk k * PB + t: count in tile order
#pragma unroll
    for (int k = 0; k < PBYTES / 16; ++k) {
        const int64_t p = tile0 + ((int64_t)k * PB + threadIdx.x) * 16;
        uint8_t b[16];
        if (p + 16 <= n) {
            const uint4 v = *reinterpret_cast<const uint4 *>(t + p);
            const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int i = 0; i < 16; ++i) b[i] = (uint8_t)(w[i / 4] >> (8 * (i % 4)));
        } else {
#pragma unroll
            for (int i = 0; i < 16; ++i) b[i] = p + i < n ? t[p + i] : 0;
        }
        uint32_t c = 0;
#pragma unroll
        for (int i = 0; i < 16; ++i) c += b[i] == '\n';
        uint32_t tot;
        uint32_t o = base + dev::block_exclusive_sum<PB>(c, scratch, &tot);
#pragma unroll
        for (int i = 0; i < 16; ++i)
            if (b[i] == '\n') line_start[1 + (int64_t)(o++)] = p + i + 1;
        base += tot;
    }
}

__device__ __forceinline__ bool is_digit(uint8_t c) { return c >= '0' && c <= '9'; }

// [b, e) as a signed integer with surrounding spaces; false if malformed
__device__ bool parse_int(const uint8_t *t, int64_t b, int64_t e, int64_t &v) {
    while (b < e && t[b] == ' ') ++b;
    while (e > b && t[e - 1] == ' ') --e;
    if (b >= e) return false;
    bool neg = false;
    if (t[b] == '-' || t[b] == '+') {
        neg = t[b] == '-';
        ++b;
    }
    if (b >= e || e - b > 18) return false;
    int64_t x = 0;
    for (; b < e; ++b) {
        if (!is_digit(t[b])) return false;
        x = x * 10 + (t[b] - '0');
    }
    v = neg ? -x : x;
    return true;
}

__device__ __forceinline__ bool starts_with(const uint8_t *t, int64_t b, int64_t e, const char *p,
                                            int len) {
    if (e - b < len) return false;
    for (int i = 0; i < len; ++i)
        if (t[b + i] != (uint8_t)p[i]) return false;
    return true;
}

__global__ __launch_bounds__(PB) void k_parse(const uint8_t *__restrict__ t, int64_t n,
                                              const int64_t *__restrict__ line_start,
                                              int64_t lines, int64_t nl, LineOut o,
                                              unsigned long long *__restrict__ hkeys,
                                              unsigned long long *__restrict__ hfirst,
                                              unsigned long long *__restrict__ err) {
    const int64_t j = (int64_t)blockIdx.x * PB + threadIdx.x;
    if (j >= lines) return;
    const int64_t lb = line_start[j];
    int64_t le = j < nl ? line_start[j + 1] - 1 : n;  // exclusive of its '\n'
    if (le > lb && t[le - 1] == '\r') --le;
    o.flag[j] = 0;
    if (le <= lb || t[lb] == '#' || starts_with(t, lb, le, "track", 5) ||
        starts_with(t, lb, le, "browser", 7))
        return;
    bool tab = false;
    for (int64_t p = lb; p < le && !tab; ++p) tab = t[p] == '\t';
    int64_t fb[6], fe[6];  // the first six fields
    int nf = 0;
    int64_t p = lb;
    if (tab) {
        while (nf < 6) {
            int64_t q = p;
            while (q < le && t[q] != '\t') ++q;
            fb[nf] = p;
            fe[nf] = q;
            ++nf;
            if (q >= le) break;
            p = q + 1;
        }
    } else {
        while (nf < 6) {
            while (p < le && t[p] == ' ') ++p;
            if (p >= le) break;
            int64_t q = p;
            while (q < le && t[q] != ' ') ++q;
            fb[nf] = p;
            fe[nf] = q;
            ++nf;
            p = q;
        }
    }
    int64_t s = 0, e = 0;
    if (nf < 3 || !parse_int(t, fb[1], fe[1], s) || !parse_int(t, fb[2], fe[2], e)) {
        atomicMin(err, (unsigned long long)j);  // malformed record
        return;
    }
    if (s < 0 || e < 0 || s > 0xffffffffll || e > 0xffffffffll) {
        atomicMin(err + 1, (unsigned long long)j);  // coordinate outside [0, 2^32)
        return;
    }
    // FNV-1a 64 of the chrom field; 0 marks an empty slot
    unsigned long long h = 0xcbf29ce484222325ull;
    for (int64_t q = fb[0]; q < fe[0]; ++q) h = (h ^ t[q]) * 0x100000001b3ull;
    if (h == 0) h = 1;
    uint32_t slot = (uint32_t)(h ^ (h >> 32)) & (HCAP - 1);
    for (uint32_t probe = 0;; ++probe) {
        const unsigned long long old = atomicCAS(&hkeys[slot], 0ull, h);
        if (old == 0ull || old == h) break;
        slot = (slot + 1) & (HCAP - 1);
        if (probe + 1 >= HCAP) {
            atomicMin(err + 2, (unsigned long long)j);  // table full
            return;
        }
    }
    atomicMin(&hfirst[slot], (unsigned long long)j);
    o.flag[j] = 1;
    o.slot[j] = slot;
    o.start[j] = (uint32_t)s;
    o.end[j] = (uint32_t)e;
    o.chrom_off[j] = fb[0];
    o.chrom_len[j] = (uint32_t)(fe[0] - fb[0]);
    o.name_off[j] = nf > 3 ? fb[3] : fe[2];
    o.name_len[j] = nf > 3 ? (uint32_t)(fe[3] - fb[3]) : 0u;
    int8_t st = 0;
    if (nf > 5 && fe[5] > fb[5]) {
        const uint8_t c = t[fb[5]];
        st = c == '+' ? 1 : c == '-' ? 2 : c == '?' ? 3 : 0;
    }
    o.strand[j] = st;
}

__global__ __launch_bounds__(PB) void k_emit(const uint8_t *__restrict__ t, int64_t lines,
                                             LineOut o, const uint32_t *__restrict__ rec,
                                             const int32_t *__restrict__ id_of_slot,
                                             const unsigned long long *__restrict__ hfirst,
                                             lime_dbed out, unsigned long long *__restrict__ err) {
    const int64_t j = (int64_t)blockIdx.x * PB + threadIdx.x;
    if (j >= lines || !o.flag[j]) return;
    const uint32_t slot = o.slot[j];
    const int64_t r = (int64_t)hfirst[slot];  // representative line of the slot
    const int64_t a = o.chrom_off[j], b = o.chrom_off[r];
    const uint32_t len = o.chrom_len[j];
    bool same = len == o.chrom_len[r];
    for (uint32_t i = 0; same && i < len; ++i) same = t[a + i] == t[b + i];
    if (!same) {
        atomicMin(err + 3, (unsigned long long)j);
        return;
    }
    const int64_t k = rec[j];
    out.contig[k] = id_of_slot[slot];
    out.start[k] = o.start[j];
    out.end[k] = o.end[j];
    out.strand[k] = o.strand[j];
    out.name_off[k] = o.name_off[j];
    out.name_len[k] = o.name_len[j];
}

__global__ __launch_bounds__(PB) void k_remap(int32_t *__restrict__ contig, int64_t n,
                                              const int32_t *__restrict__ map) {
    const int64_t i = (int64_t)blockIdx.x * PB + threadIdx.x;
    if (i < n) contig[i] = map[contig[i]];
}

}  // namespace

// contig ids (order of first appearance) -> caller's ids, e.g. the rank of
// each name in a lime_space (Java String order), in place on the device
int bed_remap_device(lime_dbed *d, const int32_t *new_id, int32_t n_ids) {
    if (n_ids != (int32_t)d->names.size()) return fail(LIME_ERR_ARG, "remap table size != contigs");
    lime_ctx *ctx = d->ctx;
    if (d->n == 0 || n_ids == 0) return LIME_OK;
    int32_t *dm;
    LIME_TRY(alloc(ctx, &dm, (size_t)n_ids));
    LIME_HIP(hipMemcpyAsync(dm, new_id, sizeof(int32_t) * (size_t)n_ids, hipMemcpyHostToDevice,
                            S(ctx)));
    hipLaunchKernelGGL(k_remap, dim3(blocks_for(d->n, PB)), dim3(PB), 0, S(ctx), d->contig, d->n,
                       (const int32_t *)dm);
    LIME_HIP(hipGetLastError());
    LIME_HIP(hipStreamSynchronize(S(ctx)));
    release(ctx, dm);
    d->remapped = true;
    return LIME_OK;
}

// Parse `nbytes` of BED text held in host memory; the arrays stay in HBM.
int bed_parse_device(lime_ctx *ctx, const char *text, int64_t nbytes, lime_dbed **out) {
    const unsigned long long none = ~0ull;
    uint8_t *dt = nullptr;
    LIME_TRY(alloc(ctx, &dt, (size_t)std::max<int64_t>(nbytes, 16)));
    if (nbytes > 0)
        LIME_HIP(hipMemcpyAsync(dt, text, (size_t)nbytes, hipMemcpyHostToDevice, S(ctx)));
    const int64_t ntiles = std::max<int64_t>((nbytes + PTILE - 1) / PTILE, 1);
    uint32_t *tcnt, *toff, *total;
    LIME_TRY(alloc(ctx, &tcnt, (size_t)ntiles));
    LIME_TRY(alloc(ctx, &toff, (size_t)ntiles));
    LIME_TRY(alloc(ctx, &total, 1));
    hipLaunchKernelGGL(k_nl_count, dim3((unsigned)ntiles), dim3(PB), 0, S(ctx), dt, nbytes, tcnt);
    LIME_HIP(hipGetLastError());
    LIME_TRY(scan_exclusive_u32(ctx, tcnt, toff, ntiles, total));
    uint32_t nl = 0;
    LIME_TRY(read_back(ctx, &nl, total, sizeof(nl)));
    const bool tail = nbytes > 0 && text[nbytes - 1] != '\n';
    const int64_t lines = (int64_t)nl + (tail ? 1 : 0);
    const size_t L = (size_t)std::max<int64_t>(lines, 1);
    int64_t *ls;
    LIME_TRY(alloc(ctx, &ls, L + 1));
    hipLaunchKernelGGL(k_nl_write, dim3((unsigned)ntiles), dim3(PB), 0, S(ctx), dt, nbytes,
                       (const uint32_t *)toff, ls);
    LIME_HIP(hipGetLastError());
    LineOut o;
    LIME_TRY(alloc(ctx, &o.flag, L));
    LIME_TRY(alloc(ctx, &o.slot, L));
    LIME_TRY(alloc(ctx, &o.start, L));
    LIME_TRY(alloc(ctx, &o.end, L));
    LIME_TRY(alloc(ctx, &o.strand, L));
    LIME_TRY(alloc(ctx, &o.name_off, L));
    LIME_TRY(alloc(ctx, &o.name_len, L));
    LIME_TRY(alloc(ctx, &o.chrom_off, L));
    LIME_TRY(alloc(ctx, &o.chrom_len, L));
    unsigned long long *hkeys, *hfirst, *err;
    LIME_TRY(alloc(ctx, &hkeys, HCAP));
    LIME_TRY(alloc(ctx, &hfirst, HCAP));
    LIME_TRY(alloc(ctx, &err, 4));
    LIME_HIP(hipMemsetAsync(hkeys, 0, sizeof(unsigned long long) * HCAP, S(ctx)));
    LIME_HIP(hipMemsetAsync(hfirst, 0xff, sizeof(unsigned long long) * HCAP, S(ctx)));
    LIME_HIP(hipMemsetAsync(err, 0xff, sizeof(unsigned long long) * 4, S(ctx)));
    if (lines > 0)
        hipLaunchKernelGGL(k_parse, dim3(blocks_for(lines, PB)), dim3(PB), 0, S(ctx), dt, nbytes,
                           (const int64_t *)ls, lines, (int64_t)nl, o, hkeys, hfirst, err);
    LIME_HIP(hipGetLastError());
    uint32_t *rec;
    LIME_TRY(alloc(ctx, &rec, L));
    LIME_TRY(scan_exclusive_u32(ctx, o.flag, rec, lines, total));
    uint32_t nrec = 0;
    LIME_TRY(read_back(ctx, &nrec, total, sizeof(nrec)));
    unsigned long long e[4];
    LIME_TRY(read_back(ctx, e, err, sizeof(e)));
    int rc = LIME_OK;
    std::string msg;  // line numbers are 1-based, as bed.cpp's
    if (e[0] != none || e[1] != none) {
        const bool range = e[1] < e[0];
        rc = range ? LIME_ERR_RANGE : LIME_ERR_IO;
        msg = "line " + std::to_string((range ? e[1] : e[0]) + 1) +
              (range ? ": coordinate outside [0, 2^32)" : ": not a BED record");
    } else if (e[2] != none) {
        rc = LIME_ERR_IO;
        msg = "too many distinct contig names";
    }
    lime_dbed *d = new lime_dbed();
    d->ctx = ctx;
    std::vector<int32_t> id_of_slot(HCAP, -1);
    if (rc == LIME_OK && nrec > 0) {
        // contig ids in order of first appearance; names from the host text
        std::vector<unsigned long long> first(HCAP);
        LIME_HIP(hipMemcpyAsync(first.data(), hfirst, sizeof(unsigned long long) * HCAP,
                                hipMemcpyDeviceToHost, S(ctx)));
        LIME_HIP(hipStreamSynchronize(S(ctx)));
        std::vector<std::pair<unsigned long long, uint32_t>> used;
        for (uint32_t s = 0; s < HCAP; ++s)
            if (first[s] != none) used.push_back({first[s], s});
        std::sort(used.begin(), used.end());
        std::vector<int64_t> coff(used.size());
        std::vector<uint32_t> clen(used.size());
        for (size_t i = 0; i < used.size(); ++i) {
            LIME_HIP(hipMemcpyAsync(&coff[i], o.chrom_off + used[i].first, sizeof(int64_t),
                                    hipMemcpyDeviceToHost, S(ctx)));
            LIME_HIP(hipMemcpyAsync(&clen[i], o.chrom_len + used[i].first, sizeof(uint32_t),
                                    hipMemcpyDeviceToHost, S(ctx)));
        }
        LIME_HIP(hipStreamSynchronize(S(ctx)));
        for (size_t i = 0; i < used.size(); ++i) {
            id_of_slot[used[i].second] = (int32_t)i;
            d->names.emplace_back(text + coff[i], text + coff[i] + clen[i]);
        }
    }
    if (rc == LIME_OK) {
        d->n = nrec;
        const size_t R = std::max<size_t>(nrec, 1);
        LIME_TRY(alloc(ctx, &d->contig, R));
        LIME_TRY(alloc(ctx, &d->start, R));
        LIME_TRY(alloc(ctx, &d->end, R));
        LIME_TRY(alloc(ctx, &d->strand, R));
        LIME_TRY(alloc(ctx, &d->name_off, R));
        LIME_TRY(alloc(ctx, &d->name_len, R));
        int32_t *dids;
        LIME_TRY(alloc(ctx, &dids, HCAP));
        LIME_HIP(hipMemcpyAsync(dids, id_of_slot.data(), sizeof(int32_t) * HCAP,
                                hipMemcpyHostToDevice, S(ctx)));
        if (lines > 0)
            hipLaunchKernelGGL(k_emit, dim3(blocks_for(lines, PB)), dim3(PB), 0, S(ctx), dt,
                               lines, o, (const uint32_t *)rec, (const int32_t *)dids,
                               (const unsigned long long *)hfirst, *d, err);
        LIME_HIP(hipGetLastError());
        LIME_TRY(read_back(ctx, e, err, sizeof(e)));
        if (e[3] != none) {
            rc = LIME_ERR_IO;
            msg = "line " + std::to_string(e[3] + 1) + ": contig name hash collision";
        }
        release(ctx, dids);
    }
    for (void *p : {(void *)dt, (void *)tcnt, (void *)toff, (void *)total, (void *)ls,
                    (void *)o.flag, (void *)o.slot, (void *)o.start, (void *)o.end,
                    (void *)o.strand, (void *)o.name_off, (void *)o.name_len,
                    (void *)o.chrom_off, (void *)o.chrom_len, (void *)hkeys, (void *)hfirst,
                    (void *)err, (void *)rec})
        ctx->pool.put(p);
    if (rc != LIME_OK) {
        bed_free_device(d);
        return fail(rc, msg);
    }
    *out = d;
    return LIME_OK;
}

void bed_free_device(lime_dbed *d) {
    if (!d) return;
    lime_ctx *ctx = d->ctx;
    release(ctx, d->contig);
    release(ctx, d->start);
    release(ctx, d->end);
    release(ctx, d->strand);
    release(ctx, d->name_off);
    release(ctx, d->name_len);
    delete d;
}

}  // namespace lime

// ------------------------------------------------------------------- C-ABI
extern "C" {

int lime_bed_parse_device(lime_ctx *ctx, const char *text, int64_t nbytes, lime_dbed **out) {
    if (!ctx || !out || nbytes < 0 || (nbytes > 0 && !text))
        return lime::fail(LIME_ERR_ARG, "bad bed parse arguments");
    hipSetDevice(ctx->device);
    return lime::bed_parse_device(ctx, text, nbytes, out);
}

int64_t lime_dbed_rows(const lime_dbed *d) { return d ? d->n : -1; }
int32_t lime_dbed_contigs(const lime_dbed *d) { return d ? (int32_t)d->names.size() : -1; }
const char *lime_dbed_contig_name(const lime_dbed *d, int32_t i) {
    return (d && i >= 0 && i < (int32_t)d->names.size()) ? d->names[i].c_str() : nullptr;
}

int lime_dbed_device_arrays(const lime_dbed *d, const int32_t **contig, const uint32_t **start,
                            const uint32_t **end, const int8_t **strand) {
    if (!d) return lime::fail(LIME_ERR_ARG, "dbed is null");
    if (contig) *contig = d->contig;
    if (start) *start = d->start;
    if (end) *end = d->end;
    if (strand) *strand = d->strand;
    return LIME_OK;
}

int lime_dbed_fill_host(const lime_dbed *d, int32_t *contig, int64_t *start, int64_t *end,
                        int8_t *strand, int64_t *name_off, int32_t *name_len) {
    if (!d) return lime::fail(LIME_ERR_ARG, "dbed is null");
    lime_ctx *ctx = d->ctx;
    hipSetDevice(ctx->device);
    const size_t n = (size_t)d->n;
    std::vector<uint32_t> s(n), e(n), nl(n);
    auto cp = [&](void *dst, const void *src, size_t bytes) -> int {
        if (dst && bytes) LIME_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, lime::S(ctx)));
        return LIME_OK;
    };
    LIME_TRY(cp(contig, d->contig, n * sizeof(int32_t)));
    LIME_TRY(cp(start ? s.data() : nullptr, d->start, n * sizeof(uint32_t)));
    LIME_TRY(cp(end ? e.data() : nullptr, d->end, n * sizeof(uint32_t)));
    LIME_TRY(cp(strand, d->strand, n));
    LIME_TRY(cp(name_off, d->name_off, n * sizeof(int64_t)));
    LIME_TRY(cp(name_len ? nl.data() : nullptr, d->name_len, n * sizeof(uint32_t)));
    LIME_HIP(hipStreamSynchronize(lime::S(ctx)));
    for (size_t i = 0; i < n; ++i) {
        if (start) start[i] = s[i];
        if (end) end[i] = e[i];
        if (name_len) name_len[i] = (int32_t)nl[i];
    }
    return LIME_OK;
}

int lime_dbed_remap_contigs(lime_dbed *d, const int32_t *new_id_of_contig, int32_t n) {
    if (!d || (n > 0 && !new_id_of_contig)) return lime::fail(LIME_ERR_ARG, "bad remap arguments");
    if (d->remapped) return lime::fail(LIME_ERR_ARG, "contig ids already remapped");
    hipSetDevice(d->ctx->device);
    return lime::bed_remap_device(d, new_id_of_contig, n);
}

void lime_dbed_free(lime_dbed *d) { lime::bed_free_device(d); }

}  // extern "C"

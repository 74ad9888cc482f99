// bedwrite.hip -- sorted interval arrays -> BED text on the device (the writer
// side of SURVEY.md 8(f) row 1; the reference prints each record through
// Spark collect() + println, cli/*.scala).  Rows in GLOBAL coordinates of a
// space (a sorted set, or a merge / subtract / complement result) become
// "chrom<TAB>start<TAB>end[<TAB>extra]\n" lines, in row order.
//
// Kernels (byte output, HBM / PCIe-bound):
//   k_fmt_len    per row: contig by a search of the LDS-staged offsets,
//                line length (name + decimal digits)
//   scan (u64)   line offsets
//   k_fmt_write  per 256-row block: the block's lines assembled in LDS, then
//                written with coalesced stores (rows whose block text exceeds
//                the LDS buffer write their bytes directly)
#include <algorithm>

#include "common.hpp"

namespace lime {
namespace {

constexpr int WB = 256;
constexpr int OCAP = 4096;     // contig offsets staged in LDS
constexpr int TCAP = 24576;    // LDS text buffer per block (bytes)

struct FmtArgs {
    const uint32_t *gs, *ge, *extra;
    int64_t n;
    const uint32_t *off;  // n_contigs + 1 global offsets
    int32_t nc;
    const char *names;    // concatenated contig names
    const uint32_t *name_off;  // n_contigs + 1 byte offsets into names
};

__device__ __forceinline__ int ndigits(uint32_t v) {
    int d = 1;
    while (v >= 10) {
        v /= 10;
        ++d;
    }
    return d;
}

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

__device__ __forceinline__ void stage_offsets(const FmtArgs &a, uint32_t *s_off) {
    if (a.nc + 1 <= OCAP)
        for (int i = threadIdx.x; i <= a.nc; i += WB) s_off[i] = a.off[i];
    __syncthreads();
}

__device__ __forceinline__ uint32_t line_len(const FmtArgs &a, const uint32_t *off, int64_t i,
                                             int &c, uint32_t &s, uint32_t &e) {
    c = contig_of(off, a.nc, a.gs[i]);
    s = a.gs[i] - off[c];
    e = a.ge[i] - off[c];
    uint32_t len = (a.name_off[c + 1] - a.name_off[c]) + 1 + ndigits(s) + 1 + ndigits(e) + 1;
    if (a.extra) len += 1 + ndigits(a.extra[i]);
    return len;
}

__global__ __launch_bounds__(WB) void k_fmt_len(FmtArgs a, uint64_t *__restrict__ len) {
    __shared__ uint32_t s_off[OCAP];
    stage_offsets(a, s_off);
    const uint32_t *off = a.nc + 1 <= OCAP ? s_off : a.off;
    const int64_t i = (int64_t)blockIdx.x * WB + threadIdx.x;
    if (i >= a.n) return;
    int c;
    uint32_t s, e;
    len[i] = line_len(a, off, i, c, s, e);
}

__device__ __forceinline__ int put_uint(char *p, uint32_t v) {
    const int d = ndigits(v);
    for (int k = d - 1; k >= 0; --k) {
        p[k] = (char)('0' + v % 10);
        v /= 10;
    }
    return d;
}

// the line of row i at p (p in LDS or global)
__device__ __forceinline__ void put_line(const FmtArgs &a, char *p, int c, uint32_t s, uint32_t e,
                                         int64_t i) {
    const uint32_t nb = a.name_off[c], ne = a.name_off[c + 1];
    for (uint32_t k = nb; k < ne; ++k) *p++ = a.names[k];
    *p++ = '\t';
    p += put_uint(p, s);
    *p++ = '\t';
    p += put_uint(p, e);
    if (a.extra) {
        *p++ = '\t';
        p += put_uint(p, a.extra[i]);
    }
    *p = '\n';
}

__global__ __launch_bounds__(WB) void k_fmt_write(FmtArgs a, const uint64_t *__restrict__ pos,
                                                  uint64_t total, char *__restrict__ out) {
    __shared__ uint32_t s_off[OCAP];
    __shared__ __attribute__((aligned(16))) char s_txt[TCAP];
    stage_offsets(a, s_off);
    const uint32_t *off = a.nc + 1 <= OCAP ? s_off : a.off;
    const int64_t b0 = (int64_t)blockIdx.x * WB;
    const int64_t b1 = min(b0 + WB, a.n);
    const uint64_t t0 = pos[b0];
    const uint64_t t1 = b1 < a.n ? pos[b1] : total;
    const bool in_lds = t1 - t0 <= (uint64_t)TCAP;
    const int64_t i = b0 + threadIdx.x;
    if (i < a.n) {
        int c;
        uint32_t s, e;
        line_len(a, off, i, c, s, e);
        char *p = in_lds ? s_txt + (pos[i] - t0) : out + pos[i];
        put_line(a, p, c, s, e, i);
    }
    if (!in_lds) return;
    __syncthreads();
    // coalesced copy of the block's text: bytes up to the first 16-B
    // boundary, 16-B chunks, then the tail
    const uint64_t head = std::min<uint64_t>((16 - (t0 & 15)) & 15, t1 - t0);
    for (uint64_t k = threadIdx.x; k < head; k += WB) out[t0 + k] = s_txt[k];
    const uint64_t body = (t1 - t0 - head) / 16;
    for (uint64_t k = threadIdx.x; k < body; k += WB) {
        const char *src = s_txt + head + 16 * k;
        uint4 v;
        char *vb = reinterpret_cast<char *>(&v);
        for (int j = 0; j < 16; ++j) vb[j] = src[j];
        *reinterpret_cast<uint4 *>(out + t0 + head + 16 * k) = v;
    }
    for (uint64_t k = head + 16 * body + threadIdx.x; k < t1 - t0; k += WB) out[t0 + k] = s_txt[k];
}

}  // namespace

// Two-call protocol: cap < total -> only *len is set.  `out` is host memory.
int format_bed(lime_ctx *ctx, const std::vector<uint32_t> &off,
               const std::vector<std::string> &names, int64_t n, const uint32_t *gs,
               const uint32_t *ge, const uint32_t *extra, char *out, int64_t cap,
               int64_t *total_len) {
    const int32_t nc = (int32_t)names.size();
    if ((int32_t)off.size() != nc + 1) return fail(LIME_ERR_ARG, "names do not match the space");
    std::string cat;
    std::vector<uint32_t> noff(1, 0);
    for (auto &s : names) {
        cat += s;
        noff.push_back((uint32_t)cat.size());
    }
    uint32_t *d_off, *d_noff;
    char *d_names;
    uint64_t *len;
    LIME_TRY(alloc(ctx, &d_off, off.size()));
    LIME_TRY(alloc(ctx, &d_noff, noff.size()));
    LIME_TRY(alloc(ctx, &d_names, std::max<size_t>(cat.size(), 1)));
    LIME_TRY(alloc(ctx, &len, (size_t)std::max<int64_t>(n, 1)));
    LIME_HIP(hipMemcpyAsync(d_off, off.data(), 4 * off.size(), hipMemcpyHostToDevice, S(ctx)));
    LIME_HIP(hipMemcpyAsync(d_noff, noff.data(), 4 * noff.size(), hipMemcpyHostToDevice, S(ctx)));
    if (!cat.empty())
        LIME_HIP(hipMemcpyAsync(d_names, cat.data(), cat.size(), hipMemcpyHostToDevice, S(ctx)));
    FmtArgs a{gs, ge, extra, n, d_off, nc, d_names, d_noff};
    uint64_t total = 0;
    if (n > 0) {
        hipLaunchKernelGGL(k_fmt_len, dim3(blocks_for(n, WB)), dim3(WB), 0, S(ctx), a, len);
        LIME_HIP(hipGetLastError());
        uint64_t *tot;
        LIME_TRY(alloc(ctx, &tot, 1));
        LIME_TRY(scan_exclusive_u64(ctx, len, len, n, tot));
        LIME_TRY(read_back(ctx, &total, tot, sizeof(total)));
        release(ctx, tot);
    }
    *total_len = (int64_t)total;
    int rc = LIME_OK;
    if (out && cap >= (int64_t)total && total > 0) {
        char *d_out;
        LIME_TRY(alloc(ctx, &d_out, (size_t)total));
        hipLaunchKernelGGL(k_fmt_write, dim3(blocks_for(n, WB)), dim3(WB), 0, S(ctx), a,
                           (const uint64_t *)len, total, d_out);
        LIME_HIP(hipGetLastError());
        LIME_HIP(hipMemcpyAsync(out, d_out, (size_t)total, hipMemcpyDeviceToHost, S(ctx)));
        LIME_HIP(hipStreamSynchronize(S(ctx)));
        release(ctx, d_out);
    }
    release(ctx, d_off);
    release(ctx, d_noff);
    release(ctx, d_names);
    release(ctx, len);
    return rc;
}

}  // namespace lime

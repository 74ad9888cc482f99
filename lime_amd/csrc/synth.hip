// synth.hip -- counter-based synthetic interval generators.
//
// Every value is a pure function of (seed, row), so the device, the numpy
// restatement in lime_amd/synth.py and any shard count see identical data:
//   rng(seed, i, k) = mix64(seed * 0x9E3779B97F4A7C15 + 8 i + k)   (mod 2^64)
//   mulhi(x, m)     = floor(x * m / 2^64)                          (uniform in [0, m))
// uniform:  pos = mulhi(rng(seed,i,0), G) over the contigs laid end to end
//           (no pads), contig = the one holding pos, len = lo + mulhi(rng(seed,i,1),
//           hi - lo + 1) clipped to the contig, start = min(pos - base, L - len).
// pileup:   centre k = mulhi(rng(seed+1,i,0), K), centre position
//           mulhi(rng(seed,k,0), G), offset ~ N(0, sigma) by an integer
//           Irwin-Hall sum of twelve 16-bit uniforms (rng(seed+1,i,1..3)),
//           len = lo + mulhi(rng(seed+1,i,4), hi - lo + 1).
#include "common.hpp"

namespace lime {
namespace {

constexpr uint64_t GOLD = 0x9E3779B97F4A7C15ULL;

__device__ __forceinline__ uint64_t rng(uint64_t seed, uint64_t i, uint64_t k) {
    return dev::mix64(seed * GOLD + i * 8 + k);
}
__device__ __forceinline__ uint64_t mulhi(uint64_t x, uint64_t m) { return __umul64hi(x, m); }

struct SynthArgs {
    const uint64_t *base;  // nc + 1 cumulative contig lengths (no pads)
    const uint64_t *len;   // nc
    int32_t nc;
    uint64_t G;
    int64_t n;
    int64_t first;  // rows [first, first + n) of the generator's sequence
    uint64_t seed;
    uint32_t len_lo, len_hi;
    int64_t n_centres;
    uint32_t sigma;
    int32_t *contig;
    uint32_t *start, *end;
};

__device__ __forceinline__ void place(const SynthArgs &a, int64_t i, uint64_t pos, uint64_t l) {
    const int32_t c = (int32_t)dev::upper_bound(a.base, 0, (int64_t)a.nc, pos) - 1;
    const uint64_t L = a.len[c];
    if (l > L) l = L;
    uint64_t local = pos - a.base[c];
    if (local > L - l) local = L - l;
    a.contig[i] = c;
    a.start[i] = (uint32_t)local;
    a.end[i] = (uint32_t)(local + l);
}

__global__ __launch_bounds__(256) void k_uniform(SynthArgs a) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t r = (uint64_t)(a.first + i);
        const uint64_t pos = mulhi(rng(a.seed, r, 0), a.G);
        const uint64_t l = a.len_lo + mulhi(rng(a.seed, r, 1), (uint64_t)(a.len_hi - a.len_lo) + 1);
        place(a, i, pos, l);
    }
}

__global__ __launch_bounds__(256) void k_pileup(SynthArgs a) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t s1 = a.seed + 1;
        const uint64_t r = (uint64_t)(a.first + i);
        const uint64_t k = mulhi(rng(s1, r, 0), (uint64_t)a.n_centres);
        const uint64_t cpos = mulhi(rng(a.seed, k, 0), a.G);
        int64_t sum = 0;
#pragma unroll
        for (int q = 1; q <= 3; ++q) {
            uint64_t x = rng(s1, r, q);
#pragma unroll
            for (int h = 0; h < 4; ++h) sum += (int64_t)((x >> (16 * h)) & 0xffff);
        }
        const int64_t off = ((sum - 393210) * (int64_t)a.sigma) >> 16;
        int64_t p = (int64_t)cpos + off;
        if (p < 0) p = 0;
        if (p >= (int64_t)a.G) p = (int64_t)a.G - 1;
        const uint64_t l = a.len_lo + mulhi(rng(s1, r, 4), (uint64_t)(a.len_hi - a.len_lo) + 1);
        place(a, i, (uint64_t)p, l);
    }
}

}  // namespace

int synth(lime_ctx *ctx, const lime_space *sp, int kind, int64_t first, int64_t n, uint64_t seed,
          uint32_t lo, uint32_t hi, int64_t n_centres, uint32_t sigma, int32_t *d_contig,
          uint32_t *d_start, uint32_t *d_end) {
    if (n <= 0) return LIME_OK;
    if (first < 0) return fail(LIME_ERR_ARG, "negative first row");
    if (hi < lo) return fail(LIME_ERR_ARG, "len_hi < len_lo");
    std::vector<uint64_t> base(sp->n + 1), len(sp->n);
    base[0] = 0;
    for (int c = 0; c < sp->n; ++c) {
        len[c] = (uint64_t)sp->len[c];
        base[c + 1] = base[c] + len[c];
    }
    if (base[sp->n] == 0) return fail(LIME_ERR_ARG, "empty genome");
    uint64_t *d_base, *d_len;
    LIME_TRY(alloc(ctx, &d_base, base.size()));
    LIME_TRY(alloc(ctx, &d_len, len.size()));
    LIME_HIP(hipMemcpyAsync(d_base, base.data(), base.size() * 8, hipMemcpyHostToDevice, S(ctx)));
    LIME_HIP(hipMemcpyAsync(d_len, len.data(), len.size() * 8, hipMemcpyHostToDevice, S(ctx)));
    SynthArgs a;
    a.base = d_base;
    a.len = d_len;
    a.nc = sp->n;
    a.G = base[sp->n];
    a.n = n;
    a.first = first;
    a.seed = seed;
    a.len_lo = lo;
    a.len_hi = hi;
    a.n_centres = n_centres > 0 ? n_centres : 1;
    a.sigma = sigma;
    a.contig = d_contig;
    a.start = d_start;
    a.end = d_end;
    unsigned grid = blocks_for(n, 256);
    if (grid > 16384) grid = 16384;
    if (kind == 0)
        hipLaunchKernelGGL(k_uniform, dim3(grid), dim3(256), 0, S(ctx), a);
    else
        hipLaunchKernelGGL(k_pileup, dim3(grid), dim3(256), 0, S(ctx), a);
    LIME_HIP(hipGetLastError());
    // keep the tables alive until the kernel has consumed them
    LIME_HIP(hipStreamSynchronize(S(ctx)));
    release(ctx, d_base);
    release(ctx, d_len);
    return LIME_OK;
}

}  // namespace lime

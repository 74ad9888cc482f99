// bw_probe.hip -- calibration of the HBM write ceiling the fill kernel is
// judged against: streaming stores of N 16-B records in several shapes
// (k_fill's block shape, persistent grid-stride, dword-per-lane, unrolled,
// non-temporal), plus a copy (read + write) reference.
//   ./bw_probe [records]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

template <bool NT>
__global__ __launch_bounds__(256) void k_store(u32x4 *out, long n, long per_block) {
    long b0 = (long)blockIdx.x * per_block;
    long b1 = b0 + per_block < n ? b0 + per_block : n;
    for (long i = b0 + threadIdx.x; i < b1; i += 256) {
        u32x4 v = {(unsigned)i, (unsigned)(i >> 7), (unsigned)blockIdx.x, 7u};
        if (NT)
            __builtin_nontemporal_store(v, out + i);
        else
            out[i] = v;
    }
}

// k_fill's shape: 512-thread workgroup, each wave writes its own contiguous
// chunk of the workgroup's range (per_block / 8 records)
__global__ __launch_bounds__(512) void k_store_wavechunk(u32x4 *out, long n, long per_block) {
    long b0 = (long)blockIdx.x * per_block;
    long b1 = b0 + per_block < n ? b0 + per_block : n;
    long per = ((b1 - b0 + 7) / 8 + 63) & ~63L;
    long w0 = b0 + (threadIdx.x / 64) * per;
    long w1 = w0 + per < b1 ? w0 + per : b1;
    for (long i = w0 + (threadIdx.x & 63); i < w1; i += 64) {
        u32x4 v = {(unsigned)i, (unsigned)(i >> 7), (unsigned)blockIdx.x, 7u};
        out[i] = v;
    }
}

// persistent grid-stride, 16 B per lane
template <int TB>
__global__ __launch_bounds__(TB) void k_store_grid(u32x4 *out, long n) {
    for (long i = (long)blockIdx.x * TB + threadIdx.x; i < n; i += (long)gridDim.x * TB) {
        u32x4 v = {(unsigned)i, (unsigned)(i >> 7), 3u, 7u};
        out[i] = v;
    }
}

// 4 B per lane (256 B per wave instruction), per_block*4 dwords per block
__global__ __launch_bounds__(256) void k_store_dword(unsigned *out, long n, long per_block) {
    long b0 = (long)blockIdx.x * per_block;
    long b1 = b0 + per_block < n ? b0 + per_block : n;
    for (long i = b0 + threadIdx.x; i < b1; i += 256) out[i] = (unsigned)i;
}

// 4 independent 16-B stores in flight per iteration, wave-contiguous
__global__ __launch_bounds__(256) void k_store_unroll4(u32x4 *out, long n, long per_block) {
    long b0 = (long)blockIdx.x * per_block;
    long b1 = b0 + per_block < n ? b0 + per_block : n;
    for (long i = b0 + threadIdx.x; i < b1; i += 1024) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            long j = i + 256 * k;
            if (j < b1) out[j] = u32x4{(unsigned)j, (unsigned)(j >> 7), 5u, 7u};
        }
    }
}

// 512-thread workgroup over per_block records; wave w writes granules of G
// records at w*G, w*G + 8G, ... (G = 64: block-striped; G = per_block/8:
// one chunk per wave)
template <int G>
__global__ __launch_bounds__(512) void k_store_gran(u32x4 *out, long n, long per_block) {
    long b0 = (long)blockIdx.x * per_block;
    long b1 = b0 + per_block < n ? b0 + per_block : n;
    const int w = threadIdx.x / 64, lane = threadIdx.x & 63;
    for (long g = b0 + (long)w * G; g < b1; g += 8L * G)
        for (int k = 0; k < G; k += 64) {
            long i = g + k + lane;
            if (i < b1) out[i] = u32x4{(unsigned)i, (unsigned)(i >> 7), 9u, 7u};
        }
}

// k_fill's exact store shape with constant data: persistent workgroups of
// 512 threads, each over a contiguous range of `per` records cut into
// "tiles" of T records; inside a tile the range is dealt to the 8 waves in
// granules of G records (G >= T/8: one equal chunk per wave).
__global__ __launch_bounds__(512) void k_store_fillshape(u32x4 *out, long n, long per, long T,
                                                         long G) {
    const long b0 = (long)blockIdx.x * per;
    const long b1 = b0 + per < n ? b0 + per : n;
    const int w = threadIdx.x / 64, lane = threadIdx.x & 63;
    for (long t0 = b0; t0 < b1; t0 += T) {
        const long t1 = t0 + T < b1 ? t0 + T : b1;
        long rounds = (t1 - t0 + 8 * G - 1) / (8 * G);
        if (rounds < 1) rounds = 1;
        const long gsz = (((t1 - t0 + 8 * rounds - 1) / (8 * rounds)) + 63) & ~63L;
        for (long g = t0 + w * gsz; g < t1; g += 8 * gsz) {
            const long ge = g + gsz < t1 ? g + gsz : t1;
            for (long i = g + lane; i < ge; i += 64) out[i] = u32x4{(unsigned)i, 1u, 2u, 3u};
        }
        __syncthreads();
    }
}

__global__ __launch_bounds__(256) void k_copy(const u32x4 *in, u32x4 *out, long n) {
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256)
        out[i] = in[i];
}

__global__ __launch_bounds__(256) void k_read(const u32x4 *in, long n, unsigned *sink) {
    unsigned acc = 0;
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
        u32x4 v = in[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

#define CK(x)                                                         \
    do {                                                              \
        hipError_t e = (x);                                           \
        if (e != hipSuccess) {                                        \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));    \
            exit(1);                                                  \
        }                                                             \
    } while (0)

static hipEvent_t ea, eb;

template <class F>
static void timeit(const char *name, long recs, double bytes, F launch) {
    float best = 1e30f;
    for (int r = 0; r < 6; ++r) {
        CK(hipEventRecord(ea));
        launch();
        CK(hipEventRecord(eb));
        CK(hipEventSynchronize(eb));
        float ms;
        CK(hipEventElapsedTime(&ms, ea, eb));
        if (r && ms < best) best = ms;
    }
    CK(hipGetLastError());
    printf("{\"probe\": \"%s\", \"records\": %ld, \"ms\": %.3f, \"GBps\": %.1f}\n", name, recs, best,
           bytes / best / 1e6);
    fflush(stdout);
}

int main(int argc, char **argv) {
    long n = argc > 1 ? atol(argv[1]) : (1L << 31);
    const long per_block = 131072;
    u32x4 *out, *in;
    unsigned *sink;
    CK(hipMalloc(&out, n * 16));
    CK(hipMalloc(&sink, 64));
    CK(hipEventCreate(&ea));
    CK(hipEventCreate(&eb));
    unsigned grid = (unsigned)((n + per_block - 1) / per_block);
    timeit("store16_plain", n, n * 16.0, [&] {
        hipLaunchKernelGGL(k_store<false>, dim3(grid), dim3(256), 0, 0, out, n, per_block);
    });
    timeit("store16_nt", n, n * 16.0, [&] {
        hipLaunchKernelGGL(k_store<true>, dim3(grid), dim3(256), 0, 0, out, n, per_block);
    });
    timeit("store16_wavechunk512", n, n * 16.0, [&] {
        hipLaunchKernelGGL(k_store_wavechunk, dim3(grid), dim3(512), 0, 0, out, n, per_block);
    });
    timeit("store16_unroll4", n, n * 16.0, [&] {
        hipLaunchKernelGGL(k_store_unroll4, dim3(grid), dim3(256), 0, 0, out, n, per_block);
    });
    for (unsigned g : {1024u, 2048u, 4096u, 16384u})
        for (int tb : {256, 1024}) {
            char name[64];
            snprintf(name, sizeof name, "store16_grid%u_tb%d", g, tb);
            timeit(name, n, n * 16.0, [&] {
                if (tb == 256)
                    hipLaunchKernelGGL(k_store_grid<256>, dim3(g), dim3(256), 0, 0, out, n);
                else
                    hipLaunchKernelGGL(k_store_grid<1024>, dim3(g), dim3(1024), 0, 0, out, n);
            });
        }
    timeit("store4_dword", n * 4, n * 16.0, [&] {
        hipLaunchKernelGGL(k_store_dword, dim3(grid), dim3(256), 0, 0, (unsigned *)out, n * 4,
                           per_block * 4);
    });
    for (long pb : {131072L, 524288L}) {
#define GRAN(G)                                                                             \
    {                                                                                       \
        char name[64];                                                                      \
        snprintf(name, sizeof name, "gran%d_wg512_per%ld", G, pb);                          \
        unsigned gg = (unsigned)((n + pb - 1) / pb);                                        \
        timeit(name, n, n * 16.0, [&] {                                                     \
            hipLaunchKernelGGL(k_store_gran<G>, dim3(gg), dim3(512), 0, 0, out, n, pb);     \
        });                                                                                 \
    }
        GRAN(64) GRAN(256) GRAN(512) GRAN(2048) GRAN(8192)
    }
    for (long G : {64L, 2048L, 1L << 40})
        for (int wgs_per_cu : {2, 3}) {
            const unsigned g = 256 * wgs_per_cu;
            const long per = (n + g - 1) / g;
            char name[96];
            snprintf(name, sizeof name, "fillshape_T84000_G%ld_wg%d", G > n ? -1L : G, wgs_per_cu);
            timeit(name, n, n * 16.0, [&] {
                hipLaunchKernelGGL(k_store_fillshape, dim3(g), dim3(512), 0, 0, out, n, per, 84000L, G);
            });
        }
    long nc = n / 2;
    CK(hipMalloc(&in, nc * 16));
    CK(hipMemset(in, 1, nc * 16));
    timeit("copy16", nc, nc * 32.0, [&] {
        hipLaunchKernelGGL(k_copy, dim3(8192), dim3(256), 0, 0, in, out, nc);
    });
    timeit("read16", n, n * 16.0, [&] {
        hipLaunchKernelGGL(k_read, dim3(8192), dim3(256), 0, 0, out, n, sink);
    });
    return 0;
}

// bw_probe.hip -- calibration of the HBM write ceiling the fill kernel is
// judged against: streaming 16-B-per-lane stores of N records, in the same
// block shape as k_fill (one workgroup writes SBLK consecutive records),
// with plain vs non-temporal stores, plus a copy (read + write) reference.
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

__global__ __launch_bounds__(256) void k_copy(const u32x4 *in, u32x4 *out, long n) {
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256)
        out[i] = in[i];
}

#define CK(x)                                                         \
    do {                                                              \
        hipError_t e = (x);                                           \
        if (e != hipSuccess) {                                        \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));    \
            exit(1);                                                  \
        }                                                             \
    } while (0)

int main(int argc, char **argv) {
    long n = argc > 1 ? atol(argv[1]) : (1L << 31);
    const long per_block = 131072;
    u32x4 *out, *in;
    CK(hipMalloc(&out, n * 16));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    unsigned grid = (unsigned)((n + per_block - 1) / per_block);
    for (int variant = 0; variant < 2; ++variant) {
        float best = 1e30f;
        for (int r = 0; r < 6; ++r) {
            CK(hipEventRecord(a));
            if (variant)
                hipLaunchKernelGGL(k_store<true>, dim3(grid), dim3(256), 0, 0, out, n, per_block);
            else
                hipLaunchKernelGGL(k_store<false>, dim3(grid), dim3(256), 0, 0, out, n, per_block);
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            if (r && ms < best) best = ms;
        }
        printf("{\"probe\": \"store16_%s\", \"records\": %ld, \"ms\": %.3f, \"GBps\": %.1f}\n",
               variant ? "nt" : "plain", n, best, n * 16.0 / best / 1e6);
    }
    {
        float best = 1e30f;
        for (int r = 0; r < 6; ++r) {
            CK(hipEventRecord(a));
            hipLaunchKernelGGL(k_store_wavechunk, dim3(grid), dim3(512), 0, 0, out, n, per_block);
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            if (r && ms < best) best = ms;
        }
        printf("{\"probe\": \"store16_wavechunk512\", \"records\": %ld, \"ms\": %.3f, \"GBps\": %.1f}\n",
               n, best, n * 16.0 / best / 1e6);
    }
    long nc = n / 2;
    CK(hipMalloc(&in, nc * 16));
    CK(hipMemset(in, 1, nc * 16));
    float best = 1e30f;
    for (int r = 0; r < 6; ++r) {
        CK(hipEventRecord(a));
        hipLaunchKernelGGL(k_copy, dim3(8192), dim3(256), 0, 0, in, out, nc);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        if (r && ms < best) best = ms;
    }
    printf("{\"probe\": \"copy16\", \"records\": %ld, \"ms\": %.3f, \"GBps\": %.1f}\n", nc, best,
           nc * 32.0 / best / 1e6);
    return 0;
}

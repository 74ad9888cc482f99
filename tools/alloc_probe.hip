// alloc_probe.hip -- does the store ceiling depend on the allocation?  Times
// the plain 16-B store stream (bw_probe's store16_plain shape) into several
// 32 GiB buffers allocated in turn (fresh, second, after a free), each
// timed 5 times, to separate allocation / first-touch effects from the
// kernel, and plain vs hipDeviceMallocContiguous allocations.  One JSON
// line per measurement.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_store(u32x4 *out, long n, long per_block) {
    long b0 = (long)blockIdx.x * per_block;
    long b1 = b0 + per_block < n ? b0 + per_block : n;
    for (long i = b0 + threadIdx.x; i < b1; i += 256) out[i] = u32x4{(unsigned)i, 1u, 2u, 3u};
}

#define CK(x)                                                      \
    do {                                                           \
        hipError_t e = (x);                                        \
        if (e != hipSuccess) {                                     \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); \
            exit(1);                                               \
        }                                                          \
    } while (0)

static void run(const char *tag, u32x4 *buf, long n) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const long per = 131072;
    const unsigned grid = (unsigned)((n + per - 1) / per);
    for (int r = 0; r < 5; ++r) {
        CK(hipEventRecord(a));
        hipLaunchKernelGGL(k_store, dim3(grid), dim3(256), 0, 0, buf, n, per);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        printf("{\"buf\": \"%s\", \"rep\": %d, \"ms\": %.3f, \"GBps\": %.1f}\n", tag, r, ms,
               n * 16.0 / ms / 1e6);
        fflush(stdout);
    }
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
}

int main() {
    const long n = 1L << 31;  // 32 GiB of 16-B records
    u32x4 *A, *B, *C;
    CK(hipMalloc(&A, n * 16));
    run("A_fresh", A, n);
    CK(hipMalloc(&B, n * 16));
    run("B_second", B, n);
    run("A_again", A, n);
    CK(hipFree(A));
    CK(hipMalloc(&C, n * 16));
    run("C_after_free", C, n);
    CK(hipFree(B));
    CK(hipFree(C));
    // physically contiguous allocations (fewer, larger page fragments)
    u32x4 *D, *E;
    CK(hipExtMallocWithFlags((void **)&D, n * 16, hipDeviceMallocContiguous));
    run("D_contiguous", D, n);
    CK(hipExtMallocWithFlags((void **)&E, n * 16, hipDeviceMallocContiguous));
    run("E_contiguous2", E, n);
    CK(hipFree(D));
    CK(hipFree(E));
    return 0;
}

// rocprim_sort_probe.hip -- COMPARISON BAR ONLY: the
// time rocPRIM's device radix sort (onesweep on gfx950) takes for the engine's
// sort stage shapes, so the engine's own sort (lime_amd/csrc/sort.hip) can be
// judged against what a tuned library reaches on this GPU.  Not part of the
// product; built by `make bin/rocprim_sort_probe` only.
//
// Shapes (one JSON line each):
//   pairs12   key u32 (global start) + value u64 (end << 32 | row): the
//             engine's 12 B per row, one LSD sort over 32 key bits
//   pairs8    key u32 + value u32 (row only): 8 B per row
//   keys4     keys only
// Keys: uniform over [0, span) (C2: span = hg38's 3.1e9) or piled up (C3).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <cstring>

#include <rocprim/rocprim.hpp>

#define CK(x)                                                                     \
    do {                                                                          \
        hipError_t e = (x);                                                       \
        if (e != hipSuccess) {                                                    \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                \
            exit(1);                                                              \
        }                                                                         \
    } while (0)

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
}

// kind 0: uniform starts; kind 1: 4e6-centre pile-ups (C3-like)
__global__ void k_gen(uint32_t *k, uint64_t *v, uint32_t *v32, int64_t n, uint64_t span, int kind) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    uint64_t x = mix64(0x5eedULL * 0x9E3779B97F4A7C15ULL + (uint64_t)i);
    uint32_t s;
    if (kind == 0) {
        s = (uint32_t)(((unsigned __int128)x * span) >> 64);
    } else {
        const uint64_t c = mix64((x % 4000000ull) + 77) % (span - 2000);
        s = (uint32_t)(c + (mix64(x) % 900));
    }
    k[i] = s;
    v[i] = ((uint64_t)(s + 50 + (x >> 50) % 4950) << 32) | (uint64_t)i;
    v32[i] = (uint32_t)i;
}

int main(int argc, char **argv) {
    const int64_t n = argc > 1 ? atoll(argv[1]) : 100000000;
    const int kind = argc > 2 ? atoi(argv[2]) : 0;
    const uint64_t span = 3088269832ull;  // hg38 primary + pads
    uint32_t *k0, *k1, *v32a, *v32b;
    uint64_t *v0, *v1;
    CK(hipMalloc(&k0, 4 * n));
    CK(hipMalloc(&k1, 4 * n));
    CK(hipMalloc(&v0, 8 * n));
    CK(hipMalloc(&v1, 8 * n));
    CK(hipMalloc(&v32a, 4 * n));
    CK(hipMalloc(&v32b, 4 * n));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int shape = 0; shape < 3; ++shape) {
        size_t tmp_bytes = 0;
        rocprim::double_buffer<uint32_t> kb(k0, k1);
        rocprim::double_buffer<uint64_t> vb(v0, v1);
        rocprim::double_buffer<uint32_t> wb(v32a, v32b);
        if (shape == 0) CK(rocprim::radix_sort_pairs(nullptr, tmp_bytes, kb, vb, n));
        if (shape == 1) CK(rocprim::radix_sort_pairs(nullptr, tmp_bytes, kb, wb, n));
        if (shape == 2) CK(rocprim::radix_sort_keys(nullptr, tmp_bytes, kb, n));
        void *tmp;
        CK(hipMalloc(&tmp, tmp_bytes));
        float best = 1e30f, sum = 0.f;
        const int reps = 5;
        for (int r = 0; r < reps + 1; ++r) {
            hipLaunchKernelGGL(k_gen, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, k0, v0,
                               v32a, n, span, kind);
            rocprim::double_buffer<uint32_t> kk(k0, k1);
            rocprim::double_buffer<uint64_t> vv(v0, v1);
            rocprim::double_buffer<uint32_t> ww(v32a, v32b);
            CK(hipEventRecord(e0, 0));
            if (shape == 0) CK(rocprim::radix_sort_pairs(tmp, tmp_bytes, kk, vv, n));
            if (shape == 1) CK(rocprim::radix_sort_pairs(tmp, tmp_bytes, kk, ww, n));
            if (shape == 2) CK(rocprim::radix_sort_keys(tmp, tmp_bytes, kk, n));
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms = 0.f;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (r > 0) {  // (the first run pays one-time setup)
                best = ms < best ? ms : best;
                sum += ms;
            }
        }
        CK(hipFree(tmp));
        const int bytes = shape == 0 ? 12 : shape == 1 ? 8 : 4;
        const char *nm = shape == 0 ? "pairs12" : shape == 1 ? "pairs8" : "keys4";
        printf("{\"probe\": \"rocprim_radix_sort\", \"shape\": \"%s\", \"keys\": \"%s\", \"n\": %lld, "
               "\"item_bytes\": %d, \"best_ms\": %.4f, \"avg_ms\": %.4f, \"item_GBps_rw\": %.1f}\n",
               nm, kind ? "pileup" : "uniform", (long long)n, bytes, best, sum / reps,
               2.0 * bytes * n / (best * 1e-3) / 1e9);
        fflush(stdout);
    }
    return 0;
}

// scan.hip -- device-wide exclusive prefix sums (u32 / u64), reduce-then-scan.
//
// Used for the radix-sort digit matrix, per-tile output counts of every
// count/scan/write kernel, and pair offsets.  Three launches: per-block
// reduction, a single-block scan of the block sums (looping in chunks, so any
// n works), and a per-block scan seeded with its block's offset.
#include "common.hpp"

namespace lime {
namespace {

constexpr int SB = 256;
constexpr int SITEMS = 16;
constexpr int STILE = SB * SITEMS;

template <typename T>
__global__ __launch_bounds__(SB) void k_reduce(const T *__restrict__ in, T *__restrict__ part,
                                               int64_t n) {
    const int64_t base = (int64_t)blockIdx.x * STILE;
    T s = 0;
#pragma unroll
    for (int k = 0; k < SITEMS; ++k) {
        int64_t i = base + k * SB + threadIdx.x;
        if (i < n) s += in[i];
    }
    s = dev::wave_reduce_sum(s);
    __shared__ T ws[SB / 64];
    if (dev::lane_id() == 0) ws[threadIdx.x / 64] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        T t = 0;
        for (int i = 0; i < SB / 64; ++i) t += ws[i];
        part[blockIdx.x] = t;
    }
}

// single block: exclusive scan of part[0..m) in place; total -> *total
template <typename T>
__global__ __launch_bounds__(SB) void k_scan_parts(T *part, int64_t m, T *total) {
    __shared__ T scratch[SB / 64 + 1];
    T carry = 0;
    for (int64_t base = 0; base < m; base += SB) {
        int64_t i = base + threadIdx.x;
        T v = i < m ? part[i] : T(0);
        T tot;
        T ex = dev::block_exclusive_sum<SB>(v, scratch, &tot);
        if (i < m) part[i] = carry + ex;
        carry += tot;
    }
    if (threadIdx.x == 0 && total) *total = carry;
}

template <typename T>
__global__ __launch_bounds__(SB) void k_scan_blocks(const T *__restrict__ in, T *__restrict__ out,
                                                    const T *__restrict__ part, int64_t n) {
    // blocked arrangement: thread t owns items [t*SITEMS, (t+1)*SITEMS) of the tile
    __shared__ T tile[STILE];
    __shared__ T scratch[SB / 64 + 1];
    const int64_t base = (int64_t)blockIdx.x * STILE;
#pragma unroll
    for (int k = 0; k < SITEMS; ++k) {
        int64_t i = base + k * SB + threadIdx.x;
        tile[k * SB + threadIdx.x] = i < n ? in[i] : T(0);
    }
    __syncthreads();
    T v[SITEMS];
    T s = 0;
#pragma unroll
    for (int k = 0; k < SITEMS; ++k) {
        v[k] = tile[threadIdx.x * SITEMS + k];
        s += v[k];
    }
    T tot;
    T ex = dev::block_exclusive_sum<SB>(s, scratch, &tot);
    T run = part[blockIdx.x] + ex;
#pragma unroll
    for (int k = 0; k < SITEMS; ++k) {
        tile[threadIdx.x * SITEMS + k] = run;
        run += v[k];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < SITEMS; ++k) {
        int64_t i = base + k * SB + threadIdx.x;
        if (i < n) out[i] = tile[k * SB + threadIdx.x];
    }
}

// small n: ONE launch of one 1024-thread block, looping over 16384-item
// chunks (blocked per thread, staged through LDS): the three-launch path's
// fixed cost (~15-20 us of back-to-back tiny kernels) dominates below ~64k
constexpr int QB = 1024;
// items per thread: a 64 KiB LDS tile for either width (16 u32 / 8 u64), so
// the kernel fits a 64 KiB-LDS target as well as gfx950's 160 KiB
template <typename T>
constexpr int qitems() { return 64 / (int)sizeof(T); }
template <typename T>
constexpr int qtile() { return QB * qitems<T>(); }
static_assert(qtile<uint64_t>() * sizeof(uint64_t) == 65536, "64 KiB small-scan tile");
constexpr int64_t SMALL_SCAN = 4 * QB * 16;
template <typename T>
__device__ __forceinline__ void scan_small_block(const T *in, T *out, int64_t n, T *total);
template <typename T>
__global__ __launch_bounds__(QB) void k_scan_small(const T *in, T *out, int64_t n, T *total) {
    scan_small_block(in, out, n, total);
}
// two independent small scans in one launch (block b scans array b)
template <typename T>
__global__ __launch_bounds__(QB) void k_scan_small2(const T *in0, T *out0, int64_t n0,
                                                    const T *in1, T *out1, int64_t n1) {
    if (blockIdx.x == 0)
        scan_small_block(in0, out0, n0, (T *)nullptr);
    else
        scan_small_block(in1, out1, n1, (T *)nullptr);
}
template <typename T>
__device__ __forceinline__ void scan_small_block(const T *in, T *out, int64_t n, T *total) {
    constexpr int QITEMS = qitems<T>(), QTILE = qtile<T>();
    __shared__ T tile[QTILE];
    __shared__ T scratch[QB / 64 + 1];
    T carry = 0;
    for (int64_t base = 0; base < n; base += QTILE) {
#pragma unroll
        for (int k = 0; k < QITEMS; ++k) {
            const int64_t i = base + k * QB + threadIdx.x;
            tile[k * QB + threadIdx.x] = i < n ? in[i] : T(0);
        }
        __syncthreads();
        T v[QITEMS];
        T s = 0;
#pragma unroll
        for (int k = 0; k < QITEMS; ++k) {
            v[k] = tile[threadIdx.x * QITEMS + k];
            s += v[k];
        }
        T tot;
        T run = carry + dev::block_exclusive_sum<QB>(s, scratch, &tot);
#pragma unroll
        for (int k = 0; k < QITEMS; ++k) {
            tile[threadIdx.x * QITEMS + k] = run;
            run += v[k];
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < QITEMS; ++k) {
            const int64_t i = base + k * QB + threadIdx.x;
            if (i < n) out[i] = tile[k * QB + threadIdx.x];
        }
        carry += tot;
        __syncthreads();
    }
    if (threadIdx.x == 0 && total) *total = carry;
}

template <typename T>
int scan_exclusive(lime_ctx *ctx, const T *in, T *out, int64_t n, T *total_dev) {
    if (n <= 0) {
        if (total_dev) LIME_HIP(hipMemsetAsync(total_dev, 0, sizeof(T), S(ctx)));
        return LIME_OK;
    }
    if (n <= SMALL_SCAN) {
        hipLaunchKernelGGL(k_scan_small<T>, dim3(1), dim3(QB), 0, S(ctx), in, out, n, total_dev);
        LIME_HIP(hipGetLastError());
        return LIME_OK;
    }
    const int64_t nb = (n + STILE - 1) / STILE;
    T *part = nullptr;
    LIME_TRY(alloc(ctx, &part, (size_t)nb));
    hipLaunchKernelGGL(k_reduce<T>, dim3((unsigned)nb), dim3(SB), 0, S(ctx), in, part, n);
    hipLaunchKernelGGL(k_scan_parts<T>, dim3(1), dim3(SB), 0, S(ctx), part, nb, total_dev);
    hipLaunchKernelGGL(k_scan_blocks<T>, dim3((unsigned)nb), dim3(SB), 0, S(ctx), in, out,
                       (const T *)part, n);
    LIME_HIP(hipGetLastError());
    release(ctx, part);
    return LIME_OK;
}

}  // namespace

int scan_exclusive_u32(lime_ctx *ctx, const uint32_t *in, uint32_t *out, int64_t n,
                       uint32_t *total_dev) {
    return scan_exclusive<uint32_t>(ctx, in, out, n, total_dev);
}
// two exclusive u32 scans, in one launch when both are small
int scan_exclusive_u32_pair(lime_ctx *ctx, const uint32_t *in0, uint32_t *out0, int64_t n0,
                            const uint32_t *in1, uint32_t *out1, int64_t n1) {
    if (n0 > 0 && n1 > 0 && n0 <= SMALL_SCAN && n1 <= SMALL_SCAN) {
        hipLaunchKernelGGL(k_scan_small2<uint32_t>, dim3(2), dim3(QB), 0, S(ctx), in0, out0, n0,
                           in1, out1, n1);
        LIME_HIP(hipGetLastError());
        return LIME_OK;
    }
    LIME_TRY(scan_exclusive<uint32_t>(ctx, in0, out0, n0, nullptr));
    return scan_exclusive<uint32_t>(ctx, in1, out1, n1, nullptr);
}
int scan_exclusive_u64(lime_ctx *ctx, const uint64_t *in, uint64_t *out, int64_t n,
                       uint64_t *total_dev) {
    return scan_exclusive<uint64_t>(ctx, in, out, n, total_dev);
}

}  // namespace lime

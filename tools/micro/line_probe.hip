// Random line gather probe (calibrates the k_batch_rows access shape):
// LB-lane groups each read whole random lines (8 B per lane, LB*8 bytes) of
// a large buffer, K independent lines in flight per group; MODE 0 plain
// loads, 1 workgroup-scope atomic loads (sc0, what the kernel uses), 2
// non-temporal loads, 3 sc0 load + no-return 64-bit atomic min on the line.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

template <int K, int LB, int MODE>
__global__ __launch_bounds__(1024) void k_lines(unsigned long long* D, size_t nLines, int iters, unsigned long long* sink) {
    const int l = threadIdx.x % LB;
    const size_t g = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) / LB;
    unsigned long long x = g * 0x9E3779B97F4A7C15ull + 1;
    unsigned long long acc = 0;
    for (int it = 0; it < iters; ++it) {
        size_t idx[K];
        unsigned long long v[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            x ^= x << 13; x ^= x >> 7; x ^= x << 17;
            idx[k] = (x >> 8) % nLines;
        }
#pragma unroll
        for (int k = 0; k < K; ++k) {
            unsigned long long* p = &D[idx[k] * LB + l];
            if (MODE == 0) v[k] = *p;
            else if (MODE == 2) v[k] = __builtin_nontemporal_load(p);
            else v[k] = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
#pragma unroll
        for (int k = 0; k < K; ++k) {
            acc += v[k];
            if (MODE == 3)
                __hip_atomic_fetch_min(&D[idx[k] * LB + l], v[k] - 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    }
    if (acc == 0x123456789ull) sink[0] = acc;
}

// 16 B per lane: LPL lanes cover one line of LPL * 16 bytes (MODE 0 plain
// global_load_dwordx4, 2 non-temporal)
typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));
template <int K, int LPL, int MODE>
__global__ __launch_bounds__(1024) void k_lines16(u64x2* D, size_t nLines, int iters, unsigned long long* sink) {
    const int l = threadIdx.x % LPL;
    const size_t g = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) / LPL;
    unsigned long long x = g * 0x9E3779B97F4A7C15ull + 1;
    unsigned long long acc = 0;
    for (int it = 0; it < iters; ++it) {
        size_t idx[K];
        u64x2 v[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            x ^= x << 13; x ^= x >> 7; x ^= x << 17;
            idx[k] = (x >> 8) % nLines;
        }
#pragma unroll
        for (int k = 0; k < K; ++k) {
            u64x2* p = &D[idx[k] * LPL + l];
            if (MODE == 2) v[k] = __builtin_nontemporal_load(p);
            else v[k] = *p;
        }
#pragma unroll
        for (int k = 0; k < K; ++k) acc += v[k].x + v[k].y;
    }
    if (acc == 0x123456789ull) sink[0] = acc;
}

// 16-lane groups per 128-B line reading it 16 B per lane: MODE 0 every lane
// loads the 16 B holding its own 8-B entry (lanes 2j, 2j+1 share an address),
// MODE 1 only lanes 0..7 load (the others idle)
template <int K, int MODE>
__global__ __launch_bounds__(1024) void k_lines16g(u64x2* D, size_t nLines, int iters, unsigned long long* sink) {
    const int l = threadIdx.x % 16;
    const size_t g = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) / 16;
    unsigned long long x = g * 0x9E3779B97F4A7C15ull + 1;
    unsigned long long acc = 0;
    for (int it = 0; it < iters; ++it) {
        size_t idx[K];
        unsigned long long v[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            x ^= x << 13; x ^= x >> 7; x ^= x << 17;
            idx[k] = (x >> 8) % nLines;
        }
#pragma unroll
        for (int k = 0; k < K; ++k) {
            if (MODE == 0) {
                const u64x2 t = D[idx[k] * 8 + (l >> 1)];
                v[k] = (l & 1) ? t.y : t.x;
            } else {
                v[k] = 0;
                if (l < 8) { const u64x2 t = D[idx[k] * 8 + l]; v[k] = t.x + t.y; }
            }
        }
#pragma unroll
        for (int k = 0; k < K; ++k) acc += v[k];
    }
    if (acc == 0x123456789ull) sink[0] = acc;
}

template <int K, int MODE>
static double run16g(unsigned long long* D, size_t bytes, int grid, int iters, unsigned long long* sink) {
    const size_t nLines = bytes / 128;
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    u64x2* D2 = reinterpret_cast<u64x2*>(D);
    hipLaunchKernelGGL((k_lines16g<K, MODE>), dim3(grid), dim3(1024), 0, 0, D2, nLines, 2, sink);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    hipLaunchKernelGGL((k_lines16g<K, MODE>), dim3(grid), dim3(1024), 0, 0, D2, nLines, iters, sink);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0; CK(hipEventElapsedTime(&ms, a, b));
    const double lines = (double)grid * 1024 / 16 * iters * K;
    CK(hipEventDestroy(a)); CK(hipEventDestroy(b));
    return lines * 128 / (ms * 1e-3) / 1e12;
}

template <int K, int LPL, int MODE>
static double run16(unsigned long long* D, size_t bytes, int grid, int iters, unsigned long long* sink) {
    const size_t nLines = bytes / (LPL * 16);
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    u64x2* D2 = reinterpret_cast<u64x2*>(D);
    hipLaunchKernelGGL((k_lines16<K, LPL, MODE>), dim3(grid), dim3(1024), 0, 0, D2, nLines, 2, sink);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    hipLaunchKernelGGL((k_lines16<K, LPL, MODE>), dim3(grid), dim3(1024), 0, 0, D2, nLines, iters, sink);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0; CK(hipEventElapsedTime(&ms, a, b));
    const double lines = (double)grid * 1024 / LPL * iters * K;
    CK(hipEventDestroy(a)); CK(hipEventDestroy(b));
    return lines * LPL * 16 / (ms * 1e-3) / 1e12;
}

template <int K, int LB, int MODE>
static double run(unsigned long long* D, size_t bytes, int grid, int iters, unsigned long long* sink) {
    const size_t nLines = bytes / (LB * 8);
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    hipLaunchKernelGGL((k_lines<K, LB, MODE>), dim3(grid), dim3(1024), 0, 0, D, nLines, 2, sink);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(a));
    hipLaunchKernelGGL((k_lines<K, LB, MODE>), dim3(grid), dim3(1024), 0, 0, D, nLines, iters, sink);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0; CK(hipEventElapsedTime(&ms, a, b));
    const double lines = (double)grid * 1024 / LB * iters * K;
    CK(hipEventDestroy(a)); CK(hipEventDestroy(b));
    return lines * LB * 8 / (ms * 1e-3) / 1e12;
}

int main() {
    const size_t bytes = (size_t)4 << 30;
    unsigned long long *D, *sink;
    CK(hipMalloc(&D, bytes));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(D, 0x40, bytes));
    int cus = 0; CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const int g = 2 * cus;
    printf("4 GiB buffer, 2 x 1024-thread WGs per CU, K = 8 lines in flight per group (TB/s of line bytes)\n");
    printf("LB16 (128-B lines): plain %.2f  sc0 %.2f  nt %.2f  sc0+atomic %.2f\n",
           run<8, 16, 0>(D, bytes, g, 16, sink), run<8, 16, 1>(D, bytes, g, 16, sink),
           run<8, 16, 2>(D, bytes, g, 16, sink), run<8, 16, 3>(D, bytes, g, 16, sink));
    printf("LB8  (64-B lines):  plain %.2f  sc0 %.2f  nt %.2f  sc0+atomic %.2f\n",
           run<8, 8, 0>(D, bytes, g, 16, sink), run<8, 8, 1>(D, bytes, g, 16, sink),
           run<8, 8, 2>(D, bytes, g, 16, sink), run<8, 8, 3>(D, bytes, g, 16, sink));
    printf("LB32 (256-B lines): plain %.2f  sc0 %.2f  nt %.2f  sc0+atomic %.2f\n",
           run<8, 32, 0>(D, bytes, g, 16, sink), run<8, 32, 1>(D, bytes, g, 16, sink),
           run<8, 32, 2>(D, bytes, g, 16, sink), run<8, 32, 3>(D, bytes, g, 16, sink));
    printf("16 B per lane, 8 lanes per 128-B line: plain K8 %.2f  K4 %.2f  K16 %.2f  nt K8 %.2f\n",
           run16<8, 8, 0>(D, bytes, g, 16, sink), run16<4, 8, 0>(D, bytes, g, 16, sink),
           run16<16, 8, 0>(D, bytes, g, 8, sink), run16<8, 8, 2>(D, bytes, g, 16, sink));
    printf("16 B per lane, 4 lanes per 64-B line: plain K8 %.2f  16 lanes per 256-B line: plain K8 %.2f\n",
           run16<8, 4, 0>(D, bytes, g, 16, sink), run16<8, 16, 0>(D, bytes, g, 16, sink));
    printf("16-lane groups per 128-B line, 16-B loads: shared pair addresses K8 %.2f K4 %.2f, half the lanes K8 %.2f\n",
           run16g<8, 0>(D, bytes, g, 16, sink), run16g<4, 0>(D, bytes, g, 16, sink),
           run16g<8, 1>(D, bytes, g, 16, sink));
    printf("8 B per lane, K16: LB16 plain %.2f sc0 %.2f\n", run<16, 16, 0>(D, bytes, g, 8, sink),
           run<16, 16, 1>(D, bytes, g, 8, sink));
    printf("LB64 (512-B lines): plain %.2f  sc0 %.2f\n",
           run<4, 64, 0>(D, bytes, g, 16, sink), run<4, 64, 1>(D, bytes, g, 16, sink));
    return 0;
}

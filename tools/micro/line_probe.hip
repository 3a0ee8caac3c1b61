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
    printf("LB64 (512-B lines): plain %.2f  sc0 %.2f\n",
           run<4, 64, 0>(D, bytes, g, 16, sink), run<4, 64, 1>(D, bytes, g, 16, sink));
    return 0;
}

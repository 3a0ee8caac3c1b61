// Microbenchmark: cost of one "level" of a workgroup-synchronous gather loop
// (the shape of k_batch_post's level loop) on gfx950, by variant.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

__device__ __forceinline__ double ldwg(const double* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// variant bits: 1 = use ld_wg (atomic relaxed wg) loads, 2 = fence_wg, 4 = store, 8 = barrier only
__global__ __launch_bounds__(1024) void k_levels(const int* __restrict__ idx, double* R, int n,
                                                 int levels, int per, int variant,
                                                 long long* out) {
    long long t0 = clock64();
    for (int d = 0; d < levels; ++d) {
        if (!(variant & 8)) {
            const int base = (d * per) % (n - per);
            for (int q = base + threadIdx.x; q < base + per; q += blockDim.x) {
                const int p = idx[q];
                const double v = (variant & 1) ? ldwg(&R[p]) : R[p];
                if (variant & 4) R[q] = v * 1.0000001;
            }
        }
        if (variant & 2) __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
        __syncthreads();
    }
    if (threadIdx.x == 0) out[blockIdx.x] = clock64() - t0;
}

int main() {
    const int n = 1 << 21;                  // 16 MB of doubles
    std::vector<int> h(n);
    srand(1);
    for (int i = 0; i < n; ++i) h[i] = rand() % n;
    int* di; double* dr; long long* dout;
    hipMalloc(&di, n * 4); hipMalloc(&dr, n * 8); hipMalloc(&dout, 4096 * 8);
    hipMemcpy(di, h.data(), n * 4, hipMemcpyHostToDevice);
    hipMemset(dr, 0, n * 8);
    const int levels = 200;
    for (int grid : {1, 256}) {
        for (int per : {1024, 8192}) {
            for (int variant : {8, 0, 1, 2, 4, 6, 7}) {
                hipLaunchKernelGGL(k_levels, dim3(grid), dim3(1024), 0, 0, di, dr, n, levels, per, variant, dout);
                hipDeviceSynchronize();
                long long c = 0;
                hipMemcpy(&c, dout, 8, hipMemcpyDeviceToHost);
                printf("grid %3d per-level %5d variant %d: %8.0f cycles/level\n", grid, per, variant,
                       (double)c / levels);
            }
        }
    }
    return 0;
}

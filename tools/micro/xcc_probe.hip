// Which XCD (HW_REG_XCC_ID) and CU (HW_REG_HW_ID) each workgroup of a
// persistent grid lands on: checks the blockIdx -> XCD round-robin that a
// cooperative batch relax would group its members by.  (tools only)
// usage: xcc_probe [grid] [threads]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <vector>

__global__ void k(int* out) {
    if (threadIdx.x == 0) {
        unsigned x, h;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(h));
        out[2 * blockIdx.x] = (int)x;
        out[2 * blockIdx.x + 1] = (int)h;
    }
    // stay resident a moment so the whole grid is co-resident
    const long long t0 = clock64();
    while (clock64() - t0 < 2000000) __builtin_amdgcn_s_sleep(10);
}

int main(int argc, char** argv) {
    const int grid = argc > 1 ? atoi(argv[1]) : 256, threads = argc > 2 ? atoi(argv[2]) : 1024;
    int* d;
    if (hipMalloc(&d, grid * 8) != hipSuccess) return 1;
    hipLaunchKernelGGL(k, dim3(grid), dim3(threads), 0, 0, d);
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    std::vector<int> h(2 * grid);
    (void)hipMemcpy(h.data(), d, grid * 8, hipMemcpyDeviceToHost);
    std::map<int, int> perX;
    int rr = 0;
    for (int b = 0; b < grid; ++b) {
        perX[h[2 * b] & 15]++;
        rr += (h[2 * b] & 15) == (b % 8);
    }
    printf("grid %d threads %d: blocks with xcc == blockIdx %% 8: %d of %d; per xcc:", grid, threads, rr, grid);
    for (auto& kv : perX) printf(" %d:%d", kv.first, kv.second);
    printf("\nfirst 24 (xcc, hw_id):");
    for (int b = 0; b < 24 && b < grid; ++b) printf(" (%d,%x)", h[2 * b] & 15, h[2 * b + 1]);
    printf("\n");
    return 0;
}

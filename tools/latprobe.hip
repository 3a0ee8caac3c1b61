// latprobe.hip -- dependent-load latency vs footprint on gfx950 (tool, not
// product).  One wave per CU chases a random permutation cycle of 128-B
// lines inside a buffer of the given size; reports cycles per hop for plain
// loads and for workgroup-scope atomic loads (sc0).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

__global__ void chase(const unsigned long long* __restrict__ buf, int hops, int mode,
                      unsigned long long* out, long long* cyc) {
    unsigned long long idx = (unsigned long long)blockIdx.x * 7919ull * 16ull;
    idx %= 1024ull;     // start somewhere in the cycle
    idx *= 16;          // line-aligned (16 u64 = 128 B)
    const long long t0 = clock64();
    for (int h = 0; h < hops; ++h) {
        unsigned long long nx;
        if (mode == 0) nx = buf[idx];
        else nx = __hip_atomic_load(const_cast<unsigned long long*>(buf + idx), __ATOMIC_RELAXED,
                                    __HIP_MEMORY_SCOPE_WORKGROUP);
        idx = nx;
    }
    const long long t1 = clock64();
    if (threadIdx.x == 0) {
        out[blockIdx.x] = idx;
        cyc[blockIdx.x] = t1 - t0;
    }
}

int main(int argc, char** argv) {
    const int blocks = argc > 1 ? atoi(argv[1]) : 1;
    const size_t sizes[] = {1ull << 20, 4ull << 20, 16ull << 20, 64ull << 20, 256ull << 20,
                            1ull << 30, 4ull << 30};
    for (size_t S : sizes) {
        const size_t lines = S / 128;
        std::vector<unsigned long long> h(S / 8, 0);
        std::vector<size_t> perm(lines);
        for (size_t i = 0; i < lines; ++i) perm[i] = i;
        srand(1);
        for (size_t i = lines - 1; i > 0; --i) {
            size_t j = ((size_t)rand() * 32768ull + rand()) % (i + 1);
            std::swap(perm[i], perm[j]);
        }
        for (size_t i = 0; i < lines; ++i) h[perm[i] * 16] = perm[(i + 1) % lines] * 16;
        unsigned long long *d, *out;
        long long* cyc;
        if (hipMalloc(&d, S) != hipSuccess) { printf("alloc fail %zu\n", S); return 1; }
        (void)hipMalloc(&out, 8 * blocks);
        (void)hipMalloc(&cyc, 8 * blocks);
        (void)hipMemcpy(d, h.data(), S, hipMemcpyHostToDevice);
        for (int mode = 0; mode < 2; ++mode) {
            const int hops = 2000;
            hipLaunchKernelGGL(chase, dim3(blocks), dim3(64), 0, 0, d, 50, mode, out, cyc);
            hipLaunchKernelGGL(chase, dim3(blocks), dim3(64), 0, 0, d, hops, mode, out, cyc);
            (void)hipDeviceSynchronize();
            std::vector<long long> c(blocks);
            (void)hipMemcpy(c.data(), cyc, 8 * blocks, hipMemcpyDeviceToHost);
            double s = 0;
            for (long long x : c) s += x;
            printf("size %6zu MB blocks %4d mode %s: %.0f cycles/hop\n", S >> 20, blocks,
                   mode ? "atomic-wg" : "plain", s / blocks / hops);
        }
        (void)hipFree(d);
        (void)hipFree(out);
        (void)hipFree(cyc);
    }
    return 0;
}

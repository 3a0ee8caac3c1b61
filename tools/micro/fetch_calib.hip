// fetch_calib.hip -- calibrate rocprofv3 FETCH_SIZE / WRITE_SIZE for the
// access shapes of the batched kernel (MI355X guide: "other access widths are
// uncalibrated: calibrate on a known byte count in your own access pattern").
// Each kernel touches a known number of bytes of a 4 GiB buffer (>> the 256
// MiB Infinity Cache, so every access misses on-die):
//   k_stream16   16 B per lane, consecutive           (guide: FETCH = 1/2)
//   k_line128    16 lanes x 8 B = one random 128-B line per lane group
//                (the [v][LB] dist / JH gathers of k_batch_rows)
//   k_word8      8 B per lane, every lane a random line (per-entry gathers)
//   k_store128   16 lanes x 8 B stores to random 128-B lines
// Build: hipcc --offload-arch=gfx950 -O3 fetch_calib.hip -o fetch_calib
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

__device__ __forceinline__ unsigned long long mix(unsigned long long x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull;
    return x ^ (x >> 33);
}

__global__ void k_stream16(const uint4* __restrict__ a, size_t n, unsigned* out) {
    unsigned acc = 0;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
        acc ^= a[i].x ^ a[i].w;
    if (acc == 0x12345u) out[0] = acc;
}

__global__ void k_line128(const unsigned long long* __restrict__ a, size_t nLines, size_t reps,
                          unsigned long long* out) {
    const size_t g = ((size_t)blockIdx.x * 256 + threadIdx.x) >> 4;
    const int l = threadIdx.x & 15;
    unsigned long long acc = 0;
    for (size_t r = 0; r < reps; ++r) {
        const size_t line = mix(g * 1315423911ull + r) % nLines;
        acc ^= a[line * 16 + l];
    }
    if (acc == 0x12345ull) out[0] = acc;
}

__global__ void k_word8(const unsigned long long* __restrict__ a, size_t nLines, size_t reps,
                        unsigned long long* out) {
    const size_t t = (size_t)blockIdx.x * 256 + threadIdx.x;
    unsigned long long acc = 0;
    for (size_t r = 0; r < reps; ++r) {
        const size_t line = mix(t * 2654435761ull + r) % nLines;
        acc ^= a[line * 16 + (t & 15)];
    }
    if (acc == 0x12345ull) out[0] = acc;
}

__global__ void k_store128(unsigned long long* __restrict__ a, size_t nLines, size_t reps) {
    const size_t g = ((size_t)blockIdx.x * 256 + threadIdx.x) >> 4;
    const int l = threadIdx.x & 15;
    for (size_t r = 0; r < reps; ++r) {
        const size_t line = mix(g * 40503ull + r + 7) % nLines;
        a[line * 16 + l] = g + r;
    }
}

int main() {
    const size_t bytes = (size_t)4 << 30;
    const size_t nLines = bytes / 128;
    void* buf;
    unsigned long long* out;
    if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
    (void)hipMemset(buf, 1, bytes);
    const int grid = 256 * 8, reps = 64;
    const size_t threads = (size_t)grid * 256;
    // known bytes per kernel
    const double bStream = (double)bytes;
    const double bLine = (double)(threads / 16) * reps * 128;
    const double bWord = (double)threads * reps * 8;        // useful bytes (lines touched = threads*reps)
    const double bWordLines = (double)threads * reps * 128;
    hipLaunchKernelGGL(k_stream16, dim3(grid), dim3(256), 0, 0, (const uint4*)buf, bytes / 16,
                       (unsigned*)out);
    hipLaunchKernelGGL(k_line128, dim3(grid), dim3(256), 0, 0, (const unsigned long long*)buf,
                       nLines, (size_t)reps, out);
    hipLaunchKernelGGL(k_word8, dim3(grid), dim3(256), 0, 0, (const unsigned long long*)buf,
                       nLines, (size_t)reps, out);
    hipLaunchKernelGGL(k_store128, dim3(grid), dim3(256), 0, 0, (unsigned long long*)buf, nLines,
                       (size_t)reps);
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    std::printf("{\"stream16_bytes\": %.0f, \"line128_bytes\": %.0f, \"word8_useful_bytes\": %.0f, "
                "\"word8_line_bytes\": %.0f, \"store128_bytes\": %.0f}\n",
                bStream, bLine, bWord, bWordLines, bLine);
    (void)hipFree(buf);
    (void)hipFree(out);
    return 0;
}

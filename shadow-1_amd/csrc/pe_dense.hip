// pe_dense.hip -- dense-graph path: blocked min-plus
// row-Bellman-Ford for non-complete dense topologies (isComplete == FALSE,
// so the reference runs igraph Dijkstra per source, topology.c:2030).
//
//   D[s][v] <- min(D[s][v], min_u fl(D[s][u] + W[u][v]))      (in place)
//
// Every relaxation is dist[u] + w, so the fixpoint is bit-identical to
// igraph's left-fold distances; in-place (chaotic)
// updates only change how fast it is reached.  No Floyd-Warshall.
// Predecessors follow igraph's rule (tight in-arc with minimum dist[u]; two
// distinct minima -> tie row, resolved by k_exact_rows on the CSR).
#include <hip/hip_runtime.h>

#include "pe_device.hpp"

namespace shdpe {

constexpr double DINF = __builtin_huge_val();
constexpr int TS = 64;      // output tile (sources x targets)
constexpr int KC = 32;      // K chunk staged in LDS
constexpr int MT = 4;       // micro-tile per thread (MT x MT)

template <class T>
__device__ __forceinline__ T* dglobal(T* p) {
    return (T*)((__attribute__((address_space(1))) T*)p);
}

// W[u][v] = latency of arc u->v (+inf if none, +inf on the diagonal: a
// self-loop never relaxes), Rl[u][v] = its rel.
__global__ __launch_bounds__(256) void k_dense_scatter(DevGraph g, double* W, double* Rl, int64_t n) {
    const int64_t a = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t m = dglobal(g.rowPtr)[n];
    if (a >= m) return;
    // owner row by binary search over rowPtr
    int lo = 0, hi = (int)n;
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (dglobal(g.rowPtr)[mid] <= a) lo = mid; else hi = mid;
    }
    const int64_t v = dglobal(g.col)[a];
    dglobal(W)[(int64_t)lo * n + v] = dglobal(g.lat)[a];
    dglobal(Rl)[(int64_t)lo * n + v] = dglobal(g.rel)[a];
}

__global__ __launch_bounds__(256) void k_dense_fill(double* p, int64_t count, double val) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < count) dglobal(p)[i] = val;
}

// D[b][v] = (v == src) ? 0 : W[src][v]   -- the first relaxation round.
__global__ __launch_bounds__(256) void k_dense_init(DevGraph g, const double* W, double* D,
                                                    const int32_t* rows, int64_t n, int64_t ldD,
                                                    uint8_t* rowActive) {
    const int b = blockIdx.y;
    const int src = dglobal(g.attached)[dglobal(rows)[b]];
    const int64_t v = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (v < n) dglobal(D)[(int64_t)b * ldD + v] = (v == src) ? 0.0 : dglobal(W)[(int64_t)src * n + v];
    if (v == 0) dglobal(rowActive)[b] = 1;
}

// One in-place min-plus sweep over all active row tiles.  Tile = 64 sources
// x 64 targets; 256 threads, 4x4 micro-tile each; K chunks of 32 staged in
// LDS (A transposed).  rowActive: row improved in the previous sweep (a row
// that did not change cannot change again: its update only reads itself).
__global__ __launch_bounds__(256) void k_minplus_sweep(const double* W, double* D, int64_t n,
                                                       int64_t ldD, int32_t nRows,
                                                       const uint8_t* rowActive,
                                                       uint8_t* rowChanged, int32_t* anyChanged) {
    __shared__ double At[KC][TS + 2];
    __shared__ double Bs[KC][TS + 2];
    __shared__ int tileActive;
    const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
    const int64_t v0 = (int64_t)blockIdx.x * TS;
    const int r0 = blockIdx.y * TS;
    const double* __restrict__ Wg = dglobal(W);
    double* Dg = dglobal(D);
    if (threadIdx.x == 0) tileActive = 0;
    __syncthreads();
    if (threadIdx.x < TS && r0 + threadIdx.x < nRows && dglobal(rowActive)[r0 + threadIdx.x])
        tileActive = 1;
    __syncthreads();
    if (!tileActive) return;

    double acc[MT][MT];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < MT; ++j) acc[i][j] = DINF;

    for (int64_t k0 = 0; k0 < n; k0 += KC) {
        // stage A (D rows r0.., cols k0..) transposed and B (W rows k0.., cols v0..)
        for (int e = threadIdx.x; e < TS * KC; e += 256) {
            const int rr = e / KC, kk = e % KC;
            const int64_t u = k0 + kk;
            At[kk][rr] = (r0 + rr < nRows && u < n) ? Dg[(int64_t)(r0 + rr) * ldD + u] : DINF;
            const int kb = e / TS, cc = e % TS;
            const int64_t ub = k0 + kb, vb = v0 + cc;
            Bs[kb][cc] = (ub < n && vb < n) ? Wg[ub * n + vb] : DINF;
        }
        __syncthreads();
#pragma unroll 8
        for (int kk = 0; kk < KC; ++kk) {
            double a[MT], b[MT];
#pragma unroll
            for (int i = 0; i < MT; ++i) a[i] = At[kk][ty * MT + i];
#pragma unroll
            for (int j = 0; j < MT; ++j) b[j] = Bs[kk][tx * MT + j];
#pragma unroll
            for (int i = 0; i < MT; ++i)
#pragma unroll
                for (int j = 0; j < MT; ++j) acc[i][j] = fmin(acc[i][j], a[i] + b[j]);
        }
        __syncthreads();
    }
    int changed = 0;
#pragma unroll
    for (int i = 0; i < MT; ++i) {
        const int r = r0 + ty * MT + i;
        if (r >= nRows) continue;
        int rowCh = 0;
#pragma unroll
        for (int j = 0; j < MT; ++j) {
            const int64_t v = v0 + tx * MT + j;
            if (v >= n) continue;
            double* p = Dg + (int64_t)r * ldD + v;
            if (acc[i][j] < *p) { *p = acc[i][j]; rowCh = 1; }
        }
        if (rowCh) { dglobal(rowChanged)[r] = 1; changed = 1; }
    }
    if (changed) atomicOr(dglobal(anyChanged), 1);
}

// Predecessor pass: for every (source row, target v): among u with
// fl(D[s][u] + W[u][v]) == D[s][v] take the minimum D[s][u]; a second u with
// the same minimum (or a zero-increment u) makes the row tie-ambiguous.
__global__ __launch_bounds__(256) void k_minplus_pred(DevGraph g, const double* W, const double* D,
                                                      int64_t n, int64_t ldD, int32_t nRows,
                                                      const int32_t* rows, int32_t* P,
                                                      uint8_t* rowAmb) {
    __shared__ double At[KC][TS + 2];
    __shared__ double Bs[KC][TS + 2];
    const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
    const int64_t v0 = (int64_t)blockIdx.x * TS;
    const int r0 = blockIdx.y * TS;
    const double* __restrict__ Wg = dglobal(W);
    const double* Dg = dglobal(D);
    double tgt[MT][MT], best[MT][MT];
    int arg[MT][MT], cnt[MT][MT];
#pragma unroll
    for (int i = 0; i < MT; ++i) {
        const int r = r0 + ty * MT + i;
#pragma unroll
        for (int j = 0; j < MT; ++j) {
            const int64_t v = v0 + tx * MT + j;
            tgt[i][j] = (r < nRows && v < n) ? Dg[(int64_t)r * ldD + v] : -1.0;
            best[i][j] = DINF;
            arg[i][j] = -1;
            cnt[i][j] = 0;
        }
    }
    for (int64_t k0 = 0; k0 < n; k0 += KC) {
        for (int e = threadIdx.x; e < TS * KC; e += 256) {
            const int rr = e / KC, kk = e % KC;
            const int64_t u = k0 + kk;
            At[kk][rr] = (r0 + rr < nRows && u < n) ? Dg[(int64_t)(r0 + rr) * ldD + u] : DINF;
            const int kb = e / TS, cc = e % TS;
            const int64_t ub = k0 + kb, vb = v0 + cc;
            Bs[kb][cc] = (ub < n && vb < n) ? Wg[ub * n + vb] : DINF;
        }
        __syncthreads();
        for (int kk = 0; kk < KC; ++kk) {
            double a[MT], b[MT];
#pragma unroll
            for (int i = 0; i < MT; ++i) a[i] = At[kk][ty * MT + i];
#pragma unroll
            for (int j = 0; j < MT; ++j) b[j] = Bs[kk][tx * MT + j];
            const int u = (int)(k0 + kk);
#pragma unroll
            for (int i = 0; i < MT; ++i)
#pragma unroll
                for (int j = 0; j < MT; ++j) {
                    if (a[i] + b[j] == tgt[i][j]) {
                        if (a[i] < best[i][j]) { best[i][j] = a[i]; arg[i][j] = u; cnt[i][j] = 1; }
                        else if (a[i] == best[i][j]) ++cnt[i][j];
                    }
                }
        }
        __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < MT; ++i) {
        const int r = r0 + ty * MT + i;
        if (r >= nRows) continue;
        const int src = dglobal(g.attached)[dglobal(rows)[r]];
        int amb = 0;
#pragma unroll
        for (int j = 0; j < MT; ++j) {
            const int64_t v = v0 + tx * MT + j;
            if (v >= n) continue;
            int p = -1;
            if (v != src && tgt[i][j] < DINF) {
                p = arg[i][j];
                // cnt != 1: two minima, or (tgt == best) a zero-increment arc
                if (cnt[i][j] != 1 || best[i][j] == tgt[i][j]) amb = 1;
            }
            dglobal(P)[(int64_t)r * ldD + v] = p;
        }
        if (amb) dglobal(rowAmb)[r] = 1;
    }
}

// Row writer: lat = D, hops / rel by walking the (short) predecessor chain
// and folding rel in source->target order (topology.c:1430-1499).
__global__ __launch_bounds__(256) void k_dense_write(DevGraph g0, DevTable tab, const double* D,
                                                     const int32_t* P, const double* Rl,
                                                     int64_t n, int64_t ldD, const int32_t* rows,
                                                     const uint8_t* rowAmb) {
    const int b = blockIdx.y;
    if (dglobal(rowAmb)[b]) return;           // resolved by k_exact_rows
    const int j = blockIdx.x * 256 + threadIdx.x;
    DevGraph g = g0;
    if (j >= g.T) return;
    const int r = dglobal(rows)[b];
    const int s = dglobal(g.attached)[r];
    const int t = dglobal(g.attached)[j];
    const double* Dr = dglobal(D) + (int64_t)b * ldD;
    const int32_t* Pr = dglobal(P) + (int64_t)b * ldD;
    const double* R = dglobal(Rl);
    double L = 0.0, Rv = 0.0;
    int h = -1, pv = -1;
    uint8_t f = 0;
    if (t == s) {
        if (dglobal(g.hasSelf)[s]) {
            L = 0.0 + dglobal(g.selfLat)[s];
            Rv = (1.0 * dglobal(g.vrel)[s]) * dglobal(g.selfRel)[s];
            h = 1;
        } else {
            f |= F_NOEDGE;
        }
    } else if (!(Dr[t] < DINF)) {
        f |= F_UNREACHABLE;
    } else {
        L = Dr[t];
        pv = Pr[t];
        // hop count
        int x = t;
        h = 0;
        while (x != s) { x = Pr[x]; ++h; }
        double acc = 1.0 * dglobal(g.vrel)[s];
        acc = acc * dglobal(g.vrel)[t];
        // fold edges from the source end: edge k = (anc(h-k), anc(h-k+1))
        for (int d = h; d >= 1; --d) {
            int y = t;                       // ancestor at distance d-1 from t
            for (int up = 0; up < d - 1; ++up) y = Pr[y];
            acc = acc * R[(int64_t)Pr[y] * n + y];
        }
        Rv = acc;
        if (L == 0.0) { L = 1.0; f |= F_ZEROLAT; }
    }
    const size_t idx = (size_t)r * (size_t)tab.T + j;
    dglobal(tab.lat)[idx] = L;
    dglobal(tab.rel)[idx] = Rv;
    dglobal(tab.hops)[idx] = h;
    dglobal(tab.flags)[idx] = f;
    if (tab.pred) dglobal(tab.pred)[idx] = pv;
}

// ---------------------------------------------------------------------------
void launch_dense_build(const DevGraph& g, double* W, double* Rl, int64_t n, int64_t nArcs,
                        void* stream) {
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const int64_t cells = n * n;
    hipLaunchKernelGGL(k_dense_fill, dim3((unsigned)((cells + 255) / 256)), dim3(256), 0, st, W,
                       cells, DINF);
    hipLaunchKernelGGL(k_dense_fill, dim3((unsigned)((cells + 255) / 256)), dim3(256), 0, st, Rl,
                       cells, 0.0);
    if (nArcs > 0)
        hipLaunchKernelGGL(k_dense_scatter, dim3((unsigned)((nArcs + 255) / 256)), dim3(256), 0, st,
                           g, W, Rl, n);
}

int launch_dense_rows(const DevGraph& g, const DevTable& tab, const double* W, const double* Rl,
                      double* D, int32_t* P, uint8_t* rowActive, uint8_t* rowChanged,
                      uint8_t* rowAmb, int32_t* dAny, const int32_t* dRows, int32_t nRows,
                      int64_t n, void* stream, int* sweepsOut) {
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const int64_t ldD = n;
    hipLaunchKernelGGL(k_dense_init, dim3((unsigned)((n + 255) / 256), nRows), dim3(256), 0, st, g,
                       W, D, dRows, n, ldD, rowActive);
    (void)hipMemsetAsync(rowAmb, 0, nRows, st);
    const dim3 grid((unsigned)((n + TS - 1) / TS), (unsigned)((nRows + TS - 1) / TS));
    int sweeps = 0;
    for (;; ++sweeps) {
        (void)hipMemsetAsync(rowChanged, 0, nRows, st);
        (void)hipMemsetAsync(dAny, 0, 4, st);
        hipLaunchKernelGGL(k_minplus_sweep, grid, dim3(256), 0, st, W, D, n, ldD, nRows, rowActive,
                           rowChanged, dAny);
        int any = 0;
        if (hipMemcpyAsync(&any, dAny, 4, hipMemcpyDeviceToHost, st) != hipSuccess) return -1;
        if (hipStreamSynchronize(st) != hipSuccess) return -1;
        std::swap(rowActive, rowChanged);
        if (!any || sweeps > n) break;
    }
    hipLaunchKernelGGL(k_minplus_pred, grid, dim3(256), 0, st, g, W, D, n, ldD, nRows, dRows, P,
                       rowAmb);
    hipLaunchKernelGGL(k_dense_write, dim3((unsigned)((g.T + 255) / 256), nRows), dim3(256), 0, st,
                       g, tab, D, P, Rl, n, ldD, dRows, rowAmb);
    if (sweepsOut) *sweepsOut = sweeps + 1;
    return 0;
}

}  // namespace shdpe

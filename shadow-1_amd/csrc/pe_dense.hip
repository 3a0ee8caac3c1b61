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

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "pe_device.hpp"

namespace shdpe {

constexpr double DINF = __builtin_huge_val();

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

// Min-plus tiles.  A workgroup (256 threads = 16 x 16) owns 16*MI source
// rows x 128 targets; thread (tx, ty) holds rows ty + 16 i (i < MI) and
// targets tx + 16 j (j < 8), so LDS reads are broadcast (A) or consecutive
// doubles (B) and the D / P stores of a wave are 128-B runs.  K is streamed
// in chunks of 16: D[rows][k0..k0+16) (staged transposed) and
// W[k0..k0+16)[targets] are prefetched into registers while the previous
// chunk is consumed from LDS.
//   SWEEP: acc = min(acc, a + b) -> in-place D update (chaotic Bellman-Ford
//          on rows; every relaxation is dist[u] + w, Appendix B);
//   PRED:  among u with fl(D[s][u] + W[u][v]) == D[s][v] keep the minimum
//          D[s][u] (igraph's first-popped tight predecessor) and its u; a
//          second u at the same minimum, or a zero-increment u, marks the
//          row tie-ambiguous (-> k_exact_rows).  A tight u is rare (about
//          one of n per entry), so the per-chunk test is add + compare and
//          the bookkeeping runs only when some lane of the wave hits.
constexpr int MJ = 8;          // targets per thread
constexpr int TCOL = 16 * MJ;  // 128 targets per tile
constexpr int KB = 16;         // K chunk
constexpr int MAXCH = 4096;    // chunk list capacity (n <= 65536 uses chunk epochs)
enum { MP_SWEEP = 0, MP_PRED = 1 };

template <int MODE, int MI>
__global__ __launch_bounds__(256) void k_minplus(DevGraph g, const double* W, double* D, int64_t n,
                                                 int64_t ldD, int32_t nRows,
                                                 const uint8_t* rowActive, uint8_t* rowChanged,
                                                 int32_t* anyChanged, const int32_t* rows,
                                                 int32_t* P, uint8_t* rowAmb,
                                                 uint8_t* chunkEpoch, int32_t epoch) {
    constexpr int TR = 16 * MI;
    __shared__ double At[KB][TR + 1];
    __shared__ double Bs[KB][TCOL];
    __shared__ int tileActive;
    __shared__ int nAct;
    __shared__ uint16_t actList[MAXCH];
    const int tid = threadIdx.x;
    const int tx = tid & 15, ty = tid >> 4;
    // row tiles vary fastest over the grid: the workgroups dispatched together
    // (round-robin over the XCDs) read the same W column strip, so a K chunk of
    // W is fetched from HBM once per XCD and served from L2 to the other row
    // tiles, instead of once per row tile
    const int rowTile = blockIdx.x;
    const int64_t v0 = (int64_t)blockIdx.y * TCOL;
    const int r0 = rowTile * TR;
    const double* __restrict__ Wg = dglobal(W);
    double* Dg = dglobal(D);
    if (MODE == MP_SWEEP) {
        if (tid == 0) tileActive = 0;
        __syncthreads();
        if (tid < TR && r0 + tid < nRows && dglobal(rowActive)[r0 + tid]) tileActive = 1;
        __syncthreads();
        if (!tileActive) return;
    }
    // K chunks to visit.  SWEEP with chunk epochs (epoch > 0): only chunks u
    // of this row tile whose D[s][u] changed in the previous sweep or in this
    // one (a D[s][u] unchanged since this tile last read it cannot improve
    // D[s][v] again); the visiting order is irrelevant (min is exact and
    // order-free).  Otherwise every chunk, in order.
    const int nch = (int)((n + KB - 1) / KB);
    const bool useList = MODE == MP_SWEEP && epoch > 0;
    if (useList) {
        if (tid == 0) nAct = 0;
        __syncthreads();
        const uint8_t* ce = dglobal(chunkEpoch) + (size_t)rowTile * nch;
        for (int c = tid; c < nch; c += 256)
            if ((int)ce[c] >= epoch - 1) actList[atomicAdd(&nAct, 1)] = (uint16_t)c;
        __syncthreads();
    }
    const int nVisit = useList ? nAct : nch;
    if (nVisit == 0) return;
    // work accounting: visited (row tile, K chunk) pairs (anyChanged[2..3] = u64)
    if (MODE == MP_SWEEP && tid == 0)
        atomicAdd(reinterpret_cast<unsigned long long*>(dglobal(anyChanged) + 2),
                  (unsigned long long)nVisit);
    auto chunkK = [&](int c) -> int64_t { return (int64_t)(useList ? (int)actList[c] : c) * KB; };

    // staging coordinates (fixed per thread); one base pointer per operand,
    // per-chunk offsets are uniform -> few live address registers
    const int aK = tid & 15, aR = tid >> 4;          // A: row aR + 16 q, column k0 + aK
    const int bK = tid >> 7, bC = tid & 127;         // B: row k0 + bK + 2 q, column v0 + bC
    const bool bColOk = v0 + bC < n;
    const double* pA = Dg + (int64_t)(r0 + aR) * ldD + aK;
    const double* pB = Wg + (int64_t)bK * n + v0 + bC;
    int rmask = 0;
#pragma unroll
    for (int q = 0; q < MI; ++q) rmask |= (r0 + aR + 16 * q < nRows) << q;
    double ra[MI], rb[KB / 2];
    auto fetch = [&](int64_t k0) {
        const bool uok = k0 + aK < n;
#pragma unroll
        for (int q = 0; q < MI; ++q) {
            const bool ok = uok && ((rmask >> q) & 1);
            const double x = pA[ok ? (int64_t)q * 16 * ldD + k0 : 0];
            ra[q] = ok ? x : DINF;
        }
#pragma unroll
        for (int q = 0; q < KB / 2; ++q) {
            const int64_t u = k0 + bK + 2 * q;
            const bool ok = u < n && bColOk;
            const double x = pB[ok ? (k0 + 2 * q) * n : 0];
            rb[q] = ok ? x : DINF;
        }
    };

    double acc[MI][MJ];     // SWEEP: running min; PRED: target distance
    double best[MODE == MP_PRED ? MI : 1][MJ];
    int arg[MODE == MP_PRED ? MI : 1][MJ];   // -1 none, >= 0 unique, -2 tie
#pragma unroll
    for (int i = 0; i < MI; ++i) {
        const int r = r0 + ty + 16 * i;
#pragma unroll
        for (int j = 0; j < MJ; ++j) {
            if (MODE == MP_SWEEP) {
                acc[i][j] = DINF;
            } else {
                const int64_t v = v0 + tx + 16 * j;
                acc[i][j] = (r < nRows && v < n) ? Dg[(int64_t)r * ldD + v] : -1.0;
                best[i][j] = DINF;
                arg[i][j] = -1;
            }
        }
    }

    fetch(chunkK(0));
    for (int c = 0; c < nVisit; ++c) {
        const int64_t k0 = chunkK(c);
        __syncthreads();
#pragma unroll
        for (int q = 0; q < MI; ++q) At[aK][aR + 16 * q] = ra[q];
#pragma unroll
        for (int q = 0; q < KB / 2; ++q) Bs[bK + 2 * q][bC] = rb[q];
        __syncthreads();
        if (c + 1 < nVisit) fetch(chunkK(c + 1));
#pragma unroll 4
        for (int kk = 0; kk < KB; ++kk) {
            double a[MI], b[MJ];
#pragma unroll
            for (int i = 0; i < MI; ++i) a[i] = At[kk][ty + 16 * i];
#pragma unroll
            for (int j = 0; j < MJ; ++j) b[j] = Bs[kk][tx + 16 * j];
            if (MODE == MP_SWEEP) {
#pragma unroll
                for (int i = 0; i < MI; ++i)
#pragma unroll
                    for (int j = 0; j < MJ; ++j) acc[i][j] = fmin(acc[i][j], a[i] + b[j]);
            } else {
                bool hit = false;
#pragma unroll
                for (int i = 0; i < MI; ++i)
#pragma unroll
                    for (int j = 0; j < MJ; ++j) hit |= (a[i] + b[j] == acc[i][j]);
                if (__any(hit)) {
                    const int u = (int)(k0 + kk);
#pragma unroll
                    for (int i = 0; i < MI; ++i)
#pragma unroll
                        for (int j = 0; j < MJ; ++j) {
                            if (a[i] + b[j] == acc[i][j]) {
                                if (a[i] < best[i][j]) { best[i][j] = a[i]; arg[i][j] = u; }
                                else if (a[i] == best[i][j]) arg[i][j] = -2;
                            }
                        }
                }
            }
        }
    }

    if (MODE == MP_SWEEP) {
        int changed = 0;
        int colCh = 0;      // bit j: some row of mine changed in chunk v0/16 + j
#pragma unroll
        for (int i = 0; i < MI; ++i) {
            const int r = r0 + ty + 16 * i;
            if (r >= nRows) continue;
            int rowCh = 0;
#pragma unroll
            for (int j = 0; j < MJ; ++j) {
                const int64_t v = v0 + tx + 16 * j;
                if (v >= n) continue;
                double* p = Dg + (int64_t)r * ldD + v;
                if (acc[i][j] < *p) { *p = acc[i][j]; ++rowCh; colCh |= 1 << j; }
            }
            if (rowCh) { dglobal(rowChanged)[r] = 1; changed += rowCh; }
        }
        if (epoch > 0 && colCh) {
            uint8_t* ce = dglobal(chunkEpoch) + (size_t)rowTile * nch + (v0 / KB);
#pragma unroll
            for (int j = 0; j < MJ; ++j)
                if ((colCh >> j) & 1) ce[j] = (uint8_t)epoch;
        }
        // anyChanged counts improved entries (debug statistics; > 0 = not converged)
        if (changed) atomicAdd(dglobal(anyChanged), changed);
    } else {
#pragma unroll
        for (int i = 0; i < MI; ++i) {
            const int r = r0 + ty + 16 * i;
            if (r >= nRows) continue;
            const int src = dglobal(g.attached)[dglobal(rows)[r]];
            int amb = 0;
#pragma unroll
            for (int j = 0; j < MJ; ++j) {
                const int64_t v = v0 + tx + 16 * j;
                if (v >= n) continue;
                int p = -1;
                if (v != src && acc[i][j] < DINF) {
                    p = arg[i][j];
                    // two minima, or (target == best) a zero-increment arc
                    if (p < 0 || best[i][j] == acc[i][j]) amb = 1;
                }
                dglobal(P)[(int64_t)r * ldD + v] = p;
            }
            if (amb) dglobal(rowAmb)[r] = 1;
        }
    }
}

constexpr int MI_SWEEP = 6;
constexpr int MI_PRED = 2;

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
    const size_t idx = (size_t)(r - tab.rowStart) * (size_t)tab.T + j;
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

// Early-stop tie slots of dense tie rows (round 6; undirected graphs, whose
// in-arcs are the vertex's own arc row sorted by neighbour).  From the
// converged distance row and the predecessor pass's choice per entry: the
// row's distances; its parents as in-arc indices -- the unique minimum u's
// arc u -> v, or, where the pass saw equal minima or a zero increment, the
// first tight arc of minimum dist[u] flagged TIE_AMB, whose tied distance
// raises the slot's threshold (atomic max on the f64 bits; the host zeroes
// it first) -- for k_tie_scan, k_exact_dense's early stop and k_tie_write.
// dIdx: the row of D / P per slot, pos: its table position.
__global__ __launch_bounds__(256) void k_dense_tie_export(DevGraph g, const double* D, const int32_t* P,
                                                          int64_t n, int64_t ldD,
                                                          const int32_t* __restrict__ dIdx,
                                                          const int32_t* __restrict__ pos, TieBuf tie) {
    const int sl = blockIdx.y;
    const int64_t v = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (v >= n) return;
    const int64_t b = dglobal(dIdx)[sl];
    const int s = dglobal(g.attached)[dglobal(pos)[sl]];
    const double* Db = dglobal(D) + b * ldD;
    const double d = Db[v];
    const int p = dglobal(P)[b * ldD + v];
    int pe = -1;
    if (v != s && d < DINF) {
        const int a0 = dglobal(g.rowPtr)[v], a1 = dglobal(g.rowPtr)[v + 1];
        if (p >= 0 && !(Db[p] == d)) {                  // unique minimum, positive increment
            if (a1 - a0 == n - 1) {
                pe = a0 + (p < v ? p : p - 1);
            } else {
                int lo = a0, hi = a1;
                while (lo < hi) {
                    const int mid = lo + ((hi - lo) >> 1);
                    if (dglobal(g.col)[mid] < p) lo = mid + 1; else hi = mid;
                }
                pe = lo;
            }
        } else {                                        // ambiguous: the heap decides
            double best = DINF;
            int ba = -1;
            for (int a = a0; a < a1; ++a) {
                const double du = Db[dglobal(g.col)[a]];
                if (du <= d && du + dglobal(g.lat)[a] == d && du < best) {
                    best = du;
                    ba = a;
                }
            }
            pe = TIE_AMB | (ba > 0 ? ba : 0);
            if (best < DINF)
                atomicMax(reinterpret_cast<unsigned long long*>(dglobal(tie.thr) + sl),
                          (unsigned long long)__double_as_longlong(best));
        }
    }
    dglobal(tie.D)[(size_t)sl * (size_t)tie.n + v] = d;
    dglobal(tie.P)[(size_t)sl * (size_t)tie.n + v] = pe;
}

void launch_dense_tie_export(const DevGraph& g, const double* D, const int32_t* P, int64_t n,
                             const int32_t* dIdx, const int32_t* dPos, const TieBuf& tie, int32_t nSlots,
                             void* stream) {
    if (nSlots <= 0) return;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    hipLaunchKernelGGL(k_dense_tie_export, dim3((unsigned)((n + 255) / 256), (unsigned)nSlots), dim3(256), 0,
                       st, g, D, P, n, n, dIdx, dPos, tie);
}

int launch_dense_rows(const DevGraph& g, const DevTable& tab, const double* W, const double* Rl,
                      double* D, int32_t* P, uint8_t* rowActive, uint8_t* rowChanged,
                      uint8_t* rowAmb, int32_t* dAny, uint8_t* chunkEpoch, const int32_t* dRows,
                      int32_t nRows, int64_t n, const Tuning& tu, void* stream, int* sweepsOut,
                      double* flopsOut) {
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const int64_t ldD = n;
    hipLaunchKernelGGL(k_dense_init, dim3((unsigned)((n + 255) / 256), nRows), dim3(256), 0, st, g,
                       W, D, dRows, n, ldD, rowActive);
    (void)hipMemsetAsync(rowAmb, 0, nRows, st);
    const unsigned gx = (unsigned)((n + TCOL - 1) / TCOL);
    const dim3 gridS((unsigned)((nRows + 16 * MI_SWEEP - 1) / (16 * MI_SWEEP)), gx);
    const int miP = tu.densePredMi >= 3 && tu.densePredMi <= 6 && tu.densePredMi != 5 ? tu.densePredMi
                                                                                         : MI_PRED;
    const dim3 gridP((unsigned)((nRows + 16 * miP - 1) / (16 * miP)), gx);
    // chunk epochs (uint8): sweep t visits chunks changed at t-1 or t; the
    // initial rows count as changed at epoch 0.  Off beyond 250 sweeps or
    // when the chunk list would not fit.
    const int64_t nch = (n + KB - 1) / KB;
    const bool epochs = nch <= MAXCH && tu.denseEpochs;
    if (epochs)
        (void)hipMemsetAsync(chunkEpoch, 0, (size_t)gridS.x * (size_t)nch, st);
    int sweeps = 0;
    double visits = 0.0;
    for (;; ++sweeps) {
        (void)hipMemsetAsync(rowChanged, 0, nRows, st);
        (void)hipMemsetAsync(dAny, 0, 16, st);
        const int epoch = (epochs && sweeps + 1 < 250) ? sweeps + 1 : 0;
        hipLaunchKernelGGL((k_minplus<MP_SWEEP, MI_SWEEP>), gridS, dim3(256), 0, st, g, W, D, n,
                           ldD, nRows, rowActive, rowChanged, dAny, dRows, P, rowAmb, chunkEpoch,
                           epoch);
        int32_t cnt[4] = {0, 0, 0, 0};
        if (hipMemcpyAsync(cnt, dAny, 16, hipMemcpyDeviceToHost, st) != hipSuccess) return -1;
        if (hipStreamSynchronize(st) != hipSuccess) return -1;
        const int any = cnt[0];
        unsigned long long vis = 0;
        std::memcpy(&vis, &cnt[2], 8);
        visits += (double)vis;
        std::swap(rowActive, rowChanged);
        if (tu.debug) {
            std::vector<uint8_t> h(nRows);
            (void)hipMemcpy(h.data(), rowActive, nRows, hipMemcpyDeviceToHost);
            long c = 0;
            for (uint8_t x : h) c += x;
            std::fprintf(stderr, "[shdpe] dense sweep %d: rows changed %ld of %d, entries %d\n", sweeps,
                         c, nRows, any);
        }
        if (!any || sweeps > n) break;
    }
    if (miP == 6)
        hipLaunchKernelGGL((k_minplus<MP_PRED, 6>), gridP, dim3(256), 0, st, g, W, D, n, ldD, nRows,
                           rowActive, rowChanged, dAny, dRows, P, rowAmb, chunkEpoch, 0);
    else if (miP == 3)
        hipLaunchKernelGGL((k_minplus<MP_PRED, 3>), gridP, dim3(256), 0, st, g, W, D, n, ldD, nRows,
                           rowActive, rowChanged, dAny, dRows, P, rowAmb, chunkEpoch, 0);
    else if (miP == 4)
        hipLaunchKernelGGL((k_minplus<MP_PRED, 4>), gridP, dim3(256), 0, st, g, W, D, n, ldD, nRows,
                           rowActive, rowChanged, dAny, dRows, P, rowAmb, chunkEpoch, 0);
    else
        hipLaunchKernelGGL((k_minplus<MP_PRED, MI_PRED>), gridP, dim3(256), 0, st, g, W, D, n, ldD,
                           nRows, rowActive, rowChanged, dAny, dRows, P, rowAmb, chunkEpoch, 0);
    hipLaunchKernelGGL(k_dense_write, dim3((unsigned)((g.T + 255) / 256), nRows), dim3(256), 0, st,
                       g, tab, D, P, Rl, n, ldD, dRows, rowAmb);
    if (sweepsOut) *sweepsOut = sweeps + 1;
    // flops: 2 per relaxation; a visit = TR rows x 128 targets x KB u (tile
    // nominal size); the pred pass is one full n x n pass per row
    if (flopsOut)
        *flopsOut = 2.0 * visits * (16.0 * MI_SWEEP) * TCOL * KB + 2.0 * (double)n * n * nRows;
    return 0;
}

}  // namespace shdpe

// pe_aux.hip -- batched per-vertex / per-pair helpers of the path table
// (SURVEY.md §8(f) rank 3): the lookups Shadow otherwise does one at a time
// on the host, with igraph attribute calls per query.
//
//   k_self_paths    _topology_computeShortestPathToSelf  topology.c:1545-1653
//   k_pairs         _topology_lookupDirectPath           topology.c:1877-1927
//                   _topology_verticesAreAdjacent        topology.c:1248-1264
//   k_incident_min  _topology_isComplete                 topology.c:450-552
//
// All are gathers over the CSR (col / lat / rel, rows sorted by neighbour id
// = igraph incidence order): HBM/L2 latency-bound, no arithmetic to speak of.
#include <hip/hip_runtime.h>

#include "pe_device.hpp"
#include "pe_devutil.hpp"
#include "shd_pathengine.h"

namespace shdpe {

// first arc of row s with col >= t (igraph_get_eid on a sorted incidence row)
__device__ __forceinline__ int row_lower_bound(const DevGraph& g, int s, int t) {
    int lo = g.rowPtr[s], hi = g.rowPtr[s + 1];
    while (lo < hi) {
        const int mid = lo + ((hi - lo) >> 1);
        if (g.col[mid] < t) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// One wave per vertex.  The reference walks v's OUT-incident edges in igraph
// order (ascending neighbour, the self-loop in place) and keeps the first
// strict minimum of the latency (the minLatency == 0 sentinel of :1592 only
// seeds it: latencies are > 0).  That is the lexicographic minimum of
// (latency, incidence position): lanes take strided arcs, then a wave
// reduction.  lat = 2 * w_min, rel = r_min * r_min (:1640-1641).
__global__ __launch_bounds__(256) void k_self_paths(DevGraph g0, const int32_t* __restrict__ verts,
                                                    int32_t count, int64_t nEdges,
                                                    double* __restrict__ lat,
                                                    double* __restrict__ rel,
                                                    uint8_t* __restrict__ flags) {
    const DevGraph g = global_view(g0);
    const int w = (int)(((size_t)blockIdx.x * 256 + threadIdx.x) >> 6);
    const int lane = threadIdx.x & 63;
    if (w >= count) return;                                   // uniform per wave
    const int v = verts[w];
    if (v < 0 || v >= g.n) {
        if (lane == 0) { lat[w] = 0.0; rel[w] = 0.0; flags[w] = F_INVALID; }
        return;
    }
    const int b = g.rowPtr[v], e = g.rowPtr[v + 1];
    const int sp = row_lower_bound(g, v, v) - b;               // self-loop's incidence slot
    const bool self = g.hasSelf[v] != 0;
    double bl = INFINITY, br = 0.0;
    int bp = INT32_MAX;
    for (int a = b + lane; a < e; a += 64) {
        const double L = g.lat[a];
        const int pos = (a - b) + ((self && a - b >= sp) ? 1 : 0);
        if (L < bl || (L == bl && pos < bp)) { bl = L; bp = pos; br = g.srel ? g.srel[a] : g.rel[a]; }
    }
    if (lane == 0 && self) {
        const double L = g.selfMinLat[v];
        if (L < bl || (L == bl && sp < bp)) { bl = L; bp = sp; br = g.selfMinRel[v]; }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const double ol = __shfl_xor(bl, o, 64);
        const double orr = __shfl_xor(br, o, 64);
        const int op = __shfl_xor(bp, o, 64);
        if (ol < bl || (ol == bl && op < bp)) { bl = ol; bp = op; br = orr; }
    }
    if (lane == 0) {
        if (bp == INT32_MAX) {
            // no incident edge: minLatency stays 0 (lat 0, rel 0); the
            // reference errors out only on an edgeless graph
            lat[w] = 0.0;
            rel[w] = 0.0;
            flags[w] = nEdges == 0 ? F_NOEDGE : 0;
        } else {
            lat[w] = 2.0 * bl;
            rel[w] = br * br;
            flags[w] = 0;
        }
    }
}

// One thread per pair.  mode 0: direct path (lat = 0.0 + w, rel =
// ((1 * a_s) * a_t) * r_e, flags F_DIRECT or F_NOEDGE); mode 1: adjacency
// only (flags[i] = 1 adjacent, 0 not; s == t adjacent iff it has a loop).
__global__ __launch_bounds__(256) void k_pairs(DevGraph g0, const int32_t* __restrict__ src,
                                               const int32_t* __restrict__ dst, int64_t count,
                                               int mode, double* __restrict__ lat,
                                               double* __restrict__ rel,
                                               uint8_t* __restrict__ flags) {
    const DevGraph g = global_view(g0);
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= count) return;
    const int s = src[i], t = dst[i];
    if (s < 0 || s >= g.n || t < 0 || t >= g.n) {
        if (mode == 0) { lat[i] = 0.0; rel[i] = 0.0; }
        flags[i] = mode == 0 ? F_INVALID : 0;
        return;
    }
    int a = -1;
    bool found;
    if (s == t) {
        found = g.hasSelf[s] != 0;
    } else {
        a = row_lower_bound(g, s, t);
        found = a < g.rowPtr[s + 1] && g.col[a] == t;
    }
    if (mode == 1) {
        flags[i] = found ? 1 : 0;
        return;
    }
    double acc = 1.0 * g.vrel[s];                            // :1901-1907
    acc = acc * g.vrel[t];
    double L = 0.0, R = 0.0;
    uint8_t f = F_NOEDGE;
    if (found) {
        const double w = s == t ? g.selfLat[s] : (g.flat ? g.flat[a] : g.lat[a]);   // get_eid: newest
        const double r = s == t ? g.selfRel[s] : g.rel[a];
        L = 0.0 + w;                                          // :1920
        R = acc * r;                                          // :1921
        f = F_DIRECT;
    }
    lat[i] = L;
    rel[i] = R;
    flags[i] = f;
}

// _topology_isComplete: every vertex's incident count (self-loop counted
// twice undirected, then corrected by one) must reach n.  Minimum count.
// Multigraphs pass the host's per-vertex edge counts (merged rows hold one
// arc per neighbour, the reference counts every parallel edge).
__global__ __launch_bounds__(256) void k_incident_min(DevGraph g0, const int32_t* __restrict__ edgeCount,
                                                      int32_t* out) {
    const DevGraph g = global_view(g0);
    const int v = blockIdx.x * 256 + threadIdx.x;
    int c = INT32_MAX;
    if (v < g.n) {
        if (edgeCount) {
            c = edgeCount[v];
        } else {
            c = g.rowPtr[v + 1] - g.rowPtr[v];
            // a loop counts once directed; twice undirected, minus the one
            // correction of :505-519 -- once either way
            if (g.hasSelf[v]) c += 1;
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) c = min(c, __shfl_xor(c, o, 64));
    if ((threadIdx.x & 63) == 0 && c != INT32_MAX) atomicMin(out, c);
}

// One thread: the igraph path of a row whose per-vertex chosen IN-arcs are in
// P (k_exact_rows' slot after a full emulation), walked from t back to s;
// out[0] = t ... out[len-1] = s in the CALLER's vertex ids.  *len = -1 when a
// vertex on the way has no parent (unreached) or a parent arc outside the
// graph (stale scratch: the caller checks reachability first), -2 when the
// path exceeds cap.
__global__ void k_path_walk(DevGraph g0, const int32_t* __restrict__ P, int s, int t,
                            int32_t* __restrict__ out, int cap, int32_t* __restrict__ len,
                            int32_t nInArcs) {
    const DevGraph g = global_view(g0);
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    int k = 0, v = t;
    while (true) {
        if (k >= cap) { *len = -2; return; }
        if (k > g.n) { *len = -1; return; }
        out[k++] = g.oldId ? g.oldId[v] : v;
        if (v == s) break;
        const int a = P[v];
        if (a < 0 || (a & ~TIE_AMB) >= nInArcs) { *len = -1; return; }
        v = g.inCol[a & ~TIE_AMB];
        if (v < 0 || v >= g.n) { *len = -1; return; }
    }
    *len = k;
}

void launch_path_walk(const DevGraph& g, const int32_t* dP, int32_t s, int32_t t, int32_t* dOut,
                      int32_t cap, int32_t* dLen, int32_t nInArcs, void* stream) {
    hipLaunchKernelGGL(k_path_walk, dim3(1), dim3(64), 0, reinterpret_cast<hipStream_t>(stream), g, dP, s,
                       t, dOut, cap, dLen, nInArcs);
}

void launch_self_paths(const DevGraph& g, const int32_t* dVerts, int32_t count, int64_t nEdges,
                       double* dLat, double* dRel, uint8_t* dFlags, void* stream) {
    if (count <= 0) return;
    const int blocks = (int)(((int64_t)count * 64 + 255) / 256);
    hipLaunchKernelGGL(k_self_paths, dim3(blocks), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), g, dVerts, count, nEdges, dLat,
                       dRel, dFlags);
}

void launch_pairs(const DevGraph& g, const int32_t* dSrc, const int32_t* dDst, int64_t count,
                  int mode, double* dLat, double* dRel, uint8_t* dFlags, void* stream) {
    if (count <= 0) return;
    hipLaunchKernelGGL(k_pairs, dim3((unsigned)((count + 255) / 256)), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), g, dSrc, dDst, count, mode, dLat,
                       dRel, dFlags);
}

void launch_incident_min(const DevGraph& g, const int32_t* dEdgeCount, int32_t* dOut, void* stream) {
    hipLaunchKernelGGL(k_incident_min, dim3((g.n + 255) / 256), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), g, dEdgeCount, dOut);
}

}  // namespace shdpe

namespace shdpe {

// ---------------------------------------------------------------------------
// Row checksums (multi-GPU verification, no reference counterpart): a 64-bit
// fingerprint per table row, the wrapping sum over its entries j and fields f
// of splitmix64(bits(f, j) ^ (j * K + c_f)) -- order-free over j so a
// workgroup reduces it in any order, position-keyed so swapped entries or
// rows change it.  Owners fingerprint their rows before an exchange, every
// rank fingerprints the assembled table after it (bench.py; a numpy twin in
// shdpe/engine.py pins the formula on the CPU).  One 256-thread workgroup per
// row: a coalesced streaming read of the row's 25-29 B per entry.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}
constexpr uint64_t CK_K = 0x9e3779b97f4a7c15ull, CK_C = 0xd1b54a32d192ed03ull;

__global__ __launch_bounds__(256) void k_row_checksums(DevTable tab0, int64_t firstLocal,
                                                       uint64_t* __restrict__ out) {
    const DevTable tab = global_view(tab0);
    __shared__ uint64_t part[4];
    const int64_t T = tab.T;
    const size_t base = (size_t)(firstLocal + blockIdx.x) * (size_t)T;
    uint64_t h = 0;
    for (int64_t j = threadIdx.x; j < T; j += 256) {
        const uint64_t kj = (uint64_t)j * CK_K;
        const size_t o = base + (size_t)j;
        h += mix64((uint64_t)__double_as_longlong(__builtin_nontemporal_load(&tab.lat[o])) ^ (kj + CK_C));
        h += mix64((uint64_t)__double_as_longlong(__builtin_nontemporal_load(&tab.rel[o])) ^ (kj + 2 * CK_C));
        h += mix64((uint64_t)(uint32_t)__builtin_nontemporal_load(&tab.hops[o]) ^ (kj + 3 * CK_C));
        h += mix64((uint64_t)__builtin_nontemporal_load(&tab.flags[o]) ^ (kj + 4 * CK_C));
        if (tab.pred) h += mix64((uint64_t)(uint32_t)__builtin_nontemporal_load(&tab.pred[o]) ^ (kj + 5 * CK_C));
    }
    for (int d = 32; d >= 1; d >>= 1) h += __shfl_xor(h, d, 64);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = h;
    __syncthreads();
    if (threadIdx.x == 0) out[blockIdx.x] = part[0] + part[1] + part[2] + part[3];
}

void launch_row_checksums(const DevTable& tab, int64_t firstLocal, int32_t rows, uint64_t* dOut,
                          void* stream) {
    if (rows <= 0) return;
    hipLaunchKernelGGL(k_row_checksums, dim3(rows), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                       tab, firstLocal, dOut);
}

}  // namespace shdpe

namespace shdpe {

// ---------------------------------------------------------------------------
// Path-cache image (shd_pe_fill_rowstore): the triangular row store of
// pe_rowstore.cpp filled from the whole table exactly as
// shd_rowstore_store_rows over rows 0, 1, ..., T-1 in order would fill it
// (topology.c:1805-1864 per row, :1307-1386 per target, no complete graph,
// no prefersDirectPaths): slot (a, a + k) takes row a's entry a + k when that
// fold succeeded (neither F_UNREACHABLE nor F_NOEDGE), else row a + k's
// entry a (stored under the reversed key), else stays empty.  One workgroup
// per triangular row: coalesced along row a, the reverse column gathered
// only for the (rare) failed forward entries.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_pack_rowstore(DevTable tab0, const int64_t* __restrict__ off,
                                                       uint8_t* __restrict__ img,
                                                       unsigned long long* __restrict__ acc) {
    const DevTable tab = global_view(tab0);
    __shared__ unsigned long long cnt[4], mnb[4];
    const int64_t T = tab.T;
    const int64_t a = blockIdx.x, len = T - a;
    uint8_t* base = img + off[a] + SHD_ROWSTORE_IMAGE_HEADER;
    double* L = reinterpret_cast<double*>(base);
    double* R = L + len;
    uint8_t* S = reinterpret_cast<uint8_t*>(R + len);
    constexpr uint8_t FAILED = F_UNREACHABLE | F_NOEDGE;
    unsigned long long c = 0, mn = INF_BITS;
    for (int64_t k = threadIdx.x; k < len; k += 256) {
        const int64_t b = a + k;
        const size_t fo = (size_t)a * T + b;
        double lat = 0.0, rel = 0.0;
        uint8_t s = 0;
        if (!(tab.flags[fo] & FAILED)) {
            lat = tab.lat[fo];
            rel = tab.rel[fo];
            s = SHD_ROWSTORE_S_STORED;
        } else if (k > 0) {
            const size_t ro = (size_t)b * T + a;
            if (!(tab.flags[ro] & FAILED)) {
                lat = tab.lat[ro];
                rel = tab.rel[ro];
                s = SHD_ROWSTORE_S_STORED | SHD_ROWSTORE_S_REVERSED;
            }
        }
        L[k] = lat;
        R[k] = rel;
        S[k] = s;
        if (s) {
            ++c;
            const unsigned long long lb = (unsigned long long)__double_as_longlong(lat);
            mn = lb < mn ? lb : mn;      // stored latencies are > 0: bit order = value order
        }
    }
    for (int d = 32; d >= 1; d >>= 1) {
        c += __shfl_xor(c, d, 64);
        const unsigned long long o = __shfl_xor(mn, d, 64);
        mn = o < mn ? o : mn;
    }
    if ((threadIdx.x & 63) == 0) { cnt[threadIdx.x >> 6] = c; mnb[threadIdx.x >> 6] = mn; }
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long cc = 0, m = INF_BITS;
        for (int w = 0; w < 4; ++w) { cc += cnt[w]; m = mnb[w] < m ? mnb[w] : m; }
        if (cc) atomicAdd(&acc[0], cc);
        if (m != INF_BITS) atomicMin(&acc[1], m);
    }
}

// per source row: 1 when no target's fold failed (F_NOEDGE; unreachable
// targets do not count), topology.c:1815-1859's isAllSuccess
__global__ __launch_bounds__(256) void k_rows_all_success(DevTable tab0, int32_t* __restrict__ out) {
    const DevTable tab = global_view(tab0);
    __shared__ int bad;
    if (threadIdx.x == 0) bad = 0;
    __syncthreads();
    const size_t base = (size_t)blockIdx.x * (size_t)tab.T;
    int b = 0;
    for (int64_t j = threadIdx.x; j < tab.T; j += 256) b |= (tab.flags[base + j] & F_NOEDGE) != 0;
    if (b) bad = 1;
    __syncthreads();
    if (threadIdx.x == 0) out[blockIdx.x] = bad ? 0 : 1;
}

void launch_pack_rowstore(const DevTable& tab, const int64_t* dOff, uint8_t* dImg,
                          unsigned long long* dAcc, void* stream) {
    if (tab.T <= 0) return;
    hipLaunchKernelGGL(k_pack_rowstore, dim3((unsigned)tab.T), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), tab, dOff, dImg, dAcc);
}

void launch_rows_all_success(const DevTable& tab, int32_t* dOut, void* stream) {
    if (tab.T <= 0) return;
    hipLaunchKernelGGL(k_rows_all_success, dim3((unsigned)tab.T), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), tab, dOut);
}

}  // namespace shdpe

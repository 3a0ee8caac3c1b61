// pe_kernels.hip -- gfx950 kernels of the Shadow path engine.
//
// Reference semantics (Shadow v1.14.0, src/main/routing/topology.c):
//   row      = _topology_computeSourcePaths            :1655-1875
//   SSSP     = igraph_get_shortest_paths_dijkstra      :1765 (igraph 0.7.1)
//   fold     = _topology_computePathProperties         :1407-1523
//   direct   = _topology_lookupDirectPath              :1877-1927
//
// Three kernels:
//   k_sparse_rows  one workgroup per source row: delta-stepping label-
//                  correcting SSSP with dist in LDS (u64 bit patterns of the
//                  positive doubles -> ds_min_rtn_u64), pending bitmask + LDS
//                  frontier queues (thread-per-vertex, wave-per-vertex for
//                  hubs), then a predecessor pass (tight in-arc with minimum
//                  dist[u] = igraph's first-popped tight predecessor), an
//                  equal-distance tie detector, label verification/fix-up and
//                  the row writer.  Relaxations are dist[u] + w (left fold) so
//                  the fixpoint is bit-identical to igraph's distances
//                  (SURVEY.md Appendix B).
//   k_exact_rows   one wavefront per tie-ambiguous row: igraph 0.7.1 2-way
//                  heap Dijkstra emulated exactly (lane 0 owns the heap, the
//                  wave stages the popped vertex's arcs in registers and
//                  broadcasts them with ds_bpermute).
//   k_direct_rows  complete graphs: direct-edge gather (HBM-bound).
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <type_traits>

#include "pe_device.hpp"
#include "pe_devutil.hpp"

namespace shdpe {

constexpr int SP_THREADS = 512;
constexpr int EX_THREADS = 64;

__device__ __forceinline__ unsigned long long ld_relaxed(unsigned long long* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

__device__ __forceinline__ unsigned long long wave_min_u64(unsigned long long x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        unsigned long long y = __shfl_xor(x, o, 64);
        x = y < x ? y : x;
    }
    return x;
}

struct alignas(16) Ctrl {
    int qtail[2];
    int htail[2];
    unsigned long long minNext[2];
    int ambig;
    int mismatch;
    int changed;
    int pad;
    double pad2;
};
static_assert(sizeof(Ctrl) <= 64, "ctrl block");

// Forward fold of reliability with vertex factors (topology.c:1430-1462,
// :1499) for entries where a_s * a_t != 1: walk the chosen predecessor chain
// back to s, then multiply in source->target order.
// (Arrays passed by value: a DevGraph& to a non-inlined callee would force
// the caller's graph descriptor into scratch memory.)
__device__ __noinline__ double fold_rel_general(const double* __restrict__ vrel,
                                                const double* __restrict__ inRel,
                                                const int32_t* __restrict__ inCol,
                                                const int32_t* P, int s, int t, int h) {
    double acc = 1.0 * vrel[s];
    acc = acc * vrel[t];
    if (h <= 64) {
        double fac[64];
        int k = 0, x = t;
        while (x != s && k < 64) {
            int a = P[x];
            fac[k++] = inRel[a];
            x = inCol[a];
        }
        for (int i = k - 1; i >= 0; --i) acc = acc * fac[i];
        return acc;
    }
    // long chains: blocks of 64 factors in source->target order; block k
    // re-walks the h - hi hops above it (O(h^2 / 64) steps, no scratch)
    for (int lo = 0; lo < h; lo += 64) {
        const int hi = h < lo + 64 ? h : lo + 64;
        int x = t;
        for (int up = 0; up < h - hi; ++up) x = inCol[P[x]];
        double fac[64];
        int k = 0;
        while (k < hi - lo) {
            const int a = P[x];
            fac[k++] = inRel[a];
            x = inCol[a];
        }
        for (int i = k - 1; i >= 0; --i) acc = acc * fac[i];
    }
    return acc;
}

// Row writer shared by the sparse and exact kernels (topology.c:1805-1864).
// Targets are processed in groups of 4 so their independent loads overlap.
// NT_OUT: streaming (nontemporal) stores, so the table stream does not evict
// the L2-resident graph.
template <bool NT_OUT = false, class DistOf, class HopOf>
__device__ __forceinline__ void write_row(const DevGraph& g, const DevTable& tab, int r, int s,
                                         DistOf distOf, HopOf hopOf, const double* R,
                                         const int32_t* P, uint8_t extra, int tid, int NT) {
    const int T = (int)tab.T;
    const size_t base = (size_t)(r - tab.rowStart) * (size_t)tab.T;
    double* __restrict__ oLat = tab.lat + base;
    double* __restrict__ oRel = tab.rel + base;
    int32_t* __restrict__ oHops = tab.hops + base;
    uint8_t* __restrict__ oFlags = tab.flags + base;
    int32_t* __restrict__ oPred = tab.pred ? tab.pred + base : nullptr;
    constexpr int G = 4;
    for (int j0 = tid; j0 < T; j0 += NT * G) {
        int tt[G], pa[G], hh[G];
        unsigned long long db[G];
        double rr[G];
#pragma unroll
        for (int k = 0; k < G; ++k) {
            const int j = j0 + k * NT;
            tt[k] = j < T ? g.attached[j] : s;
        }
#pragma unroll
        for (int k = 0; k < G; ++k) {
            const int t = tt[k];
            db[k] = distOf(t);
            if (t != s && db[k] != INF_BITS) { hh[k] = hopOf(t); rr[k] = R[t]; pa[k] = P[t]; }
            else { hh[k] = -1; rr[k] = 0.0; pa[k] = -1; }
        }
#pragma unroll
        for (int k = 0; k < G; ++k) {
            const int j = j0 + k * NT;
            if (j >= T) continue;
            const int t = tt[k];
            double L = 0.0, Rl = 0.0;
            int h = -1, pv = -1;
            uint8_t f = extra;
            if (t == s) {
                // 1-vertex igraph path [s]: the fold uses edge (s,s) (:1469-1488),
                // the destination factor is skipped (:1457).
                if (g.hasSelf[s]) {
                    L = 0.0 + g.selfLat[s];
                    Rl = (1.0 * g.vrel[s]) * g.selfRel[s];
                    h = 1;
                } else {
                    f |= F_NOEDGE;
                }
            } else if (db[k] == INF_BITS) {
                f |= F_UNREACHABLE;
            } else {
                L = b2d(db[k]);
                h = hh[k];
                if (oPred) {
                    pv = g.inCol[pa[k]];
                    if (g.oldId) pv = g.oldId[pv];      // device id -> caller's id
                }
                if (g.vrel[s] == 1.0 && g.vrel[t] == 1.0) Rl = rr[k];
                else Rl = fold_rel_general(g.vrel, g.inRel, g.inCol, P, s, t, h);
                if (L == 0.0) {                    // topology.c:1848-1852
                    L = 1.0;
                    f |= F_ZEROLAT;
                }
            }
            if (NT_OUT) {
                __builtin_nontemporal_store(L, &oLat[j]);
                __builtin_nontemporal_store(Rl, &oRel[j]);
                __builtin_nontemporal_store(h, &oHops[j]);
                __builtin_nontemporal_store(f, &oFlags[j]);
                if (oPred) __builtin_nontemporal_store(pv, &oPred[j]);
            } else {
                oLat[j] = L;
                oRel[j] = Rl;
                oHops[j] = h;
                oFlags[j] = f;
                if (oPred) oPred[j] = pv;
            }
        }
    }
}

constexpr int UNR = 8;   // arcs loaded per batch (independent loads in flight)
// lanes per light frontier vertex: template parameter LPVL of k_sparse_rows
// (4 by default; kflags bits 4-5 select 2 / 1 / 8 for tuning).  Each group
// preloads 16 arcs per batch (UNRG per lane) so a degree <= 16 vertex needs
// one round of independent loads.
template <int LPV>
struct Unr { static constexpr int value = LPV <= 16 ? 16 / LPV : 4; };

// Per-row state placement.  LAYOUT 2: dist, hops (u16), rowPtr in LDS;
// LAYOUT 1: dist in LDS; LAYOUT 0: everything in the workgroup's HBM slot.
template <int LAYOUT>
struct RowCtx {
    using HopT = typename std::conditional<LAYOUT == 2, uint16_t, int32_t>::type;
    unsigned long long* dist;
    HopT* H;
    const int32_t* rp;
    double* R;
    int32_t* P;
    uint32_t* pend;
    const uint32_t* heavyBits;
    // "next" frontier queues (filled on a pending-bit 0 -> 1 transition)
    int32_t* nq;
    int32_t* nhq;
    int* ntail;
    int* nhtail;
    int qcap, hcap;
    double bound;
};

// Lane exchange inside a group: DPP quad permutes for offsets 1 and 2 (a
// few VALU cycles), ds_bpermute for wider groups.
template <int LPV>
__device__ __forceinline__ int gxor(int v, int o) {
    if (LPV <= 4) {
        if (o == 1) return __builtin_amdgcn_update_dpp(v, v, 0xB1, 0xF, 0xF, false);   // [1,0,3,2]
        return __builtin_amdgcn_update_dpp(v, v, 0x4E, 0xF, 0xF, false);               // [2,3,0,1]
    }
    return __shfl_xor(v, o, 64);
}
template <int LPV>
__device__ __forceinline__ unsigned long long gxor64(unsigned long long v, int o) {
    const int lo = gxor<LPV>((int)(unsigned)v, o);
    const int hi = gxor<LPV>((int)(unsigned)(v >> 32), o);
    return ((unsigned long long)(unsigned)hi << 32) | (unsigned)lo;
}

// Process one frontier vertex u with a group of LPV lanes (each lane preloads
// up to UNR of u's arcs): (1) pull -- find the tight in-arc with the minimum
// dist[x] under the CURRENT distances and set u's labels (hops, rel product)
// from it; the candidate labels H[x]+1 and R[x]*r are loaded speculatively
// with the arcs, so no dependent round trip follows the reduction; (2) push
// -- relax u's out-arcs with dist[u] + w (ds_min_u64 on the f64 bit pattern)
// and mark improved vertices pending.  Labels are written only by the group
// leader of u; the final pass re-verifies every label anyway.  All LPV lanes
// of a group call this with the same u (u < 0: idle group, still joins the
// lane exchanges, so the whole wave must be active).
template <int LPV, int LAYOUT, bool QUEUED>
__device__ __forceinline__ void process_group(const DevGraph& g, const RowCtx<LAYOUT>& c, int u,
                                              int s, int sub, int kflags,
                                              long long* st = nullptr) {
    constexpr int UNRG = Unr<LPV>::value;
    long long p0 = st ? clock64() : 0;
    unsigned long long best = INF_BITS;
    int cnt = 0, ba = -1, bh = 0;   // ba: chosen in-arc, bh: its tail vertex
    const bool undirected = g.inCol == g.col;
    if (u >= 0) {
        // u leaves the pending set before its dist is read: an improvement
        // racing with this processing re-sets the bit and re-queues u.
        if (QUEUED && sub == 0) atomicAnd(&c.pend[u >> 5], ~(1u << (u & 31)));
        const unsigned long long dub = ld_relaxed(&c.dist[u]);
        const double du = b2d(dub);
        const int a0 = c.rp[u], a1 = c.rp[u + 1];
        for (int ab = a0 + sub; ab < a1; ab += LPV * UNRG) {
            // Branch-free batch: out-of-range slots re-load arc ab (valid,
            // since ab < a1) and are masked afterwards, so every load of the
            // batch is in flight before the first wait (a branch per slot
            // makes the waitcnt pass serialise them).
            int xs[UNRG];
            double ws[UNRG];
            unsigned long long dx[UNRG];
            bool ok[UNRG];
            if (kflags & 1) {
#pragma unroll
                for (int k = 0; k < UNRG; ++k) {
                    const int a = ab + k * LPV;
                    ok[k] = a < a1;
                    const int ac = ok[k] ? a : ab;
                    xs[k] = g.col[ac];
                    ws[k] = g.lat[ac];
                }
            } else {
                // one 16-B request per arc (lat f64 | col i32); the LPV lanes
                // of a group read consecutive arcs -> one line per group
#pragma unroll
                for (int k = 0; k < UNRG; ++k) {
                    const int a = ab + k * LPV;
                    ok[k] = a < a1;
                    const Arc3 A = g.arc3[ok[k] ? a : ab];
                    xs[k] = A.col;
                    ws[k] = __hiloint2double((int)A.latHi, (int)A.latLo);
                }
            }
#pragma unroll
            for (int k = 0; k < UNRG; ++k) dx[k] = ld_relaxed(&c.dist[xs[k]]);
#pragma unroll
            for (int k = 0; k < UNRG; ++k) {
                if (!ok[k]) continue;
                const int x = xs[k];
                const unsigned long long dxb = dx[k];
                if (undirected && dxb < dub && b2d(dxb) + ws[k] == du) {
                    if (dxb < best) {
                        best = dxb; cnt = 1; ba = ab + k * LPV;
                        bh = x;
                    } else if (dxb == best) ++cnt;
                }
                const double nd = du + ws[k];
                const unsigned long long nb = d2b(nd);
                if (nb < dxb) {
                    // a losing min only leaves a spurious pending vertex
                    // (processed once more, idempotent)
                    atomicMin(&c.dist[x], nb);
                    const uint32_t bit = 1u << (x & 31);
                    if (!QUEUED) {
                        atomicOr(&c.pend[x >> 5], bit);      // fire-and-forget
                        continue;
                    }
                    const uint32_t old = atomicOr(&c.pend[x >> 5], bit);
                    if (!(old & bit) && nd < c.bound) {
                        // newly pending inside the bucket -> next frontier;
                        // on overflow it stays pending for the bucket scan
                        if ((c.heavyBits[x >> 5] >> (x & 31)) & 1u) {
                            const int pos = atomicAdd(c.nhtail, 1);
                            if (pos < c.hcap) c.nhq[pos] = x;
                        } else {
                            const int pos = atomicAdd(c.ntail, 1);
                            if (pos < c.qcap) c.nq[pos] = x;
                        }
                    }
                }
            }
        }
        if (!undirected && u != s) {
            const int b1 = g.inPtr[u + 1];
            for (int a = g.inPtr[u] + sub; a < b1; a += LPV) {
                const int x = g.inCol[a];
                const unsigned long long dxb = ld_relaxed(&c.dist[x]);
                if (dxb < dub && b2d(dxb) + g.inLat[a] == du) {
                    if (dxb < best) {
                        best = dxb; cnt = 1; ba = a;
                        bh = x;
                    } else if (dxb == best) ++cnt;
                }
            }
        }
    }
    long long p1 = st ? clock64() : 0;
#pragma unroll
    for (int o = LPV >> 1; o > 0; o >>= 1) {
        const unsigned long long ob = gxor64<LPV>(best, o);
        const int oc = gxor<LPV>(cnt, o);
        const int oa = gxor<LPV>(ba, o);
        const int oh = gxor<LPV>(bh, o);
        if (ob < best) { best = ob; cnt = oc; ba = oa; bh = oh; }
        else if (ob == best && oa >= 0) {
            cnt += oc;
            if (ba < 0 || oa < ba) { ba = oa; bh = oh; }
        }
    }
    long long p2 = st ? clock64() : 0;
    if (u >= 0 && u != s && ba >= 0 && sub == 0) {
        c.H[u] = (typename RowCtx<LAYOUT>::HopT)(c.H[bh] + 1);
        c.R[u] = c.R[bh] * g.inRel[ba];
    }
    if (st) {
        const long long p3 = clock64();
        st[0] += p1 - p0; st[1] += p2 - p1; st[2] += p3 - p2; st[3] += 1;
    }
}

// ---------------------------------------------------------------------------
// k_sparse_rows
// ---------------------------------------------------------------------------
template <int LAYOUT, int LPV>
__global__ __launch_bounds__(SP_THREADS) void k_sparse_rows(
    DevGraph g0, DevTable tab0, DevScratch sc0, const int32_t* __restrict__ rows, int32_t nRows,
    uint8_t* rowAmbig, double delta, int32_t qcap, int32_t hcap, int32_t heavyDeg, int32_t* dbg,
    int32_t kflags, const TieBuf* __restrict__ tieDesc) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const DevGraph g = global_view(g0);
    const DevTable tab = global_view(tab0);
    const DevScratch sc = global_view(sc0);
    using HopT = typename RowCtx<LAYOUT>::HopT;
    // Frontier: queue-driven (filled by relaxations) when the row lives in
    // HBM (large n: a bitmask scan would read dist from HBM every phase);
    // bitmask scan per phase when dist is in LDS (cheaper relax step).
    constexpr bool QMODE = LAYOUT == 0;
    Ctrl* ctl = reinterpret_cast<Ctrl*>(smem);
    const int n = g.n;
    const int nw = (n + 31) >> 5;
    const int tid = threadIdx.x, NT = blockDim.x;
    const int lane = tid & 63, wave = tid >> 6, NWV = NT >> 6;
    const size_t slot = (size_t)blockIdx.x * (size_t)sc.stride;

    size_t off = 64;
    auto carve = [&](size_t bytes) {
        unsigned char* p = smem + off;
        off += (bytes + 15) & ~(size_t)15;
        return p;
    };
    RowCtx<LAYOUT> c;
    // LAYOUT 3: only dist + pending bits in LDS (2 rows per CU at n = 10k);
    // queues, hops and rowPtr live in the workgroup's HBM slot / the graph.
    if (LAYOUT >= 1) c.dist = reinterpret_cast<unsigned long long*>(carve((size_t)8 * n));
    else c.dist = reinterpret_cast<unsigned long long*>(sc.dist + slot);
    if (LAYOUT == 2) {
        c.H = reinterpret_cast<HopT*>(carve((size_t)2 * n));
        int32_t* rp = reinterpret_cast<int32_t*>(carve((size_t)4 * (n + 1)));
        for (int v = tid; v <= n; v += NT) rp[v] = g.rowPtr[v];
        c.rp = rp;
    } else {
        c.H = reinterpret_cast<HopT*>(sc.hops + slot);
        c.rp = g.rowPtr;
    }
    const uint32_t* heavyBits;
    if (LAYOUT == 3) {
        heavyBits = g.heavyBits;
    } else {
        uint32_t* hb = reinterpret_cast<uint32_t*>(carve((size_t)4 * nw));
        for (int w = tid; w < nw; w += NT) hb[w] = g.heavyBits[w];
        heavyBits = hb;
    }
    c.heavyBits = heavyBits;
    c.pend = reinterpret_cast<uint32_t*>(carve((size_t)4 * nw));
    // ping-pong frontier queues Q[0], Q[1] (light) and HQ[0], HQ[1] (heavy)
    int32_t* Q[2];
    int32_t* HQ[2];
    if (LAYOUT == 3 || LAYOUT == 0) {
        int32_t* base = sc.queue + (size_t)blockIdx.x * (size_t)(2 * (qcap + hcap));
        Q[0] = base;
        Q[1] = base + qcap;
        HQ[0] = base + 2 * qcap;
        HQ[1] = base + 2 * qcap + hcap;
    } else {
        Q[0] = reinterpret_cast<int32_t*>(carve((size_t)4 * qcap));
        Q[1] = reinterpret_cast<int32_t*>(carve((size_t)4 * qcap));
        HQ[0] = reinterpret_cast<int32_t*>(carve((size_t)4 * hcap));
        HQ[1] = reinterpret_cast<int32_t*>(carve((size_t)4 * hcap));
    }
    c.qcap = qcap;
    c.hcap = hcap;
    c.R = sc.rel + slot;
    c.P = sc.pred + slot;

    for (int b = blockIdx.x; b < nRows; b += gridDim.x) {
        const int r = rows[b];
        const int s = g.attached[r];
        for (int v = tid; v < n; v += NT) c.dist[v] = INF_BITS;
        for (int w = tid; w < nw; w += NT) c.pend[w] = 0u;
        if (tid == 0) {
            ctl->qtail[0] = ctl->qtail[1] = 0;
            ctl->htail[0] = ctl->htail[1] = 0;
            ctl->minNext[0] = ctl->minNext[1] = INF_BITS;
            ctl->ambig = 0;
            ctl->mismatch = 0;
            ctl->changed = 0;
        }
        __syncthreads();
        if (tid == 0) {
            c.dist[s] = d2b(0.0);
            c.pend[s >> 5] = 1u << (s & 31);
            if (QMODE) {
                if ((heavyBits[s >> 5] >> (s & 31)) & 1u) { HQ[0][0] = s; ctl->htail[0] = 1; }
                else { Q[0][0] = s; ctl->qtail[0] = 1; }
            }
            c.H[s] = 0;
            c.R[s] = 1.0;
            c.P[s] = -1;
        }
        __syncthreads();

        int phases = 0;
        long long cScan = 0, cRelax = 0, tA = clock64(), tB;
        long long cBits = 0, cResv = 0, cLight = 0, cHeavy = 0, tX;
        long long pst[4] = {0, 0, 0, 0};
        if (QMODE) {
        // ---------------- delta-stepping (label-correcting) ----------------
        // Frontier = queue filled by the previous phase's relaxations; the
        // pending bitmask is scanned only when a bucket's queue runs dry.
        int par = 0;
        double bound = delta;
        for (;;) {
            int qn = min(ctl->qtail[par], qcap);
            int hn = min(ctl->htail[par], hcap);
            if (qn == 0 && hn == 0) {
                // bucket drained: collect pending vertices below the bound
                __syncthreads();
                if (tid == 0) {
                    ctl->qtail[par] = 0;
                    ctl->htail[par] = 0;
                    ctl->minNext[0] = INF_BITS;
                }
                __syncthreads();
                unsigned long long myMin = INF_BITS;
                for (int w0 = wave * 64; w0 < nw; w0 += NT) {
                    const int w = w0 + lane;
                    const uint32_t bits = w < nw ? c.pend[w] : 0u;
                    uint32_t tl = 0, th = 0;
                    if (bits) {
                        const uint32_t hv = heavyBits[w];
                        uint32_t x = bits;
                        while (x) {
                            int pb[4];
                            unsigned long long d[4];
#pragma unroll
                            for (int k = 0; k < 4; ++k) {
                                pb[k] = x ? __ffs(x) - 1 : -1;
                                x &= x - 1;
                            }
#pragma unroll
                            for (int k = 0; k < 4; ++k)
                                d[k] = pb[k] >= 0 ? c.dist[(w << 5) + pb[k]] : INF_BITS;
#pragma unroll
                            for (int k = 0; k < 4; ++k) {
                                if (pb[k] < 0) continue;
                                if (b2d(d[k]) < bound) {
                                    if ((hv >> pb[k]) & 1u) th |= 1u << pb[k];
                                    else tl |= 1u << pb[k];
                                } else {
                                    myMin = d[k] < myMin ? d[k] : myMin;
                                }
                            }
                        }
                    }
                    const int nl = __popc(tl), nh = __popc(th);
                    int pl = nl ? atomicAdd(&ctl->qtail[par], nl) : 0;
                    int ph = nh ? atomicAdd(&ctl->htail[par], nh) : 0;
                    while (tl) {
                        const int bb = __ffs(tl) - 1;
                        tl &= tl - 1;
                        if (pl < qcap) Q[par][pl] = (w << 5) + bb;
                        ++pl;
                    }
                    while (th) {
                        const int bb = __ffs(th) - 1;
                        th &= th - 1;
                        if (ph < hcap) HQ[par][ph] = (w << 5) + bb;
                        ++ph;
                    }
                }
                if (myMin != INF_BITS) atomicMin(&ctl->minNext[0], myMin);
                __syncthreads();
                qn = min(ctl->qtail[par], qcap);
                hn = min(ctl->htail[par], hcap);
                const unsigned long long mn = ctl->minNext[0];
                tB = clock64(); cScan += tB - tA; tA = tB;
                if (qn == 0 && hn == 0) {
                    if (mn == INF_BITS) break;
                    const double m = b2d(mn);
                    bound = (floor(m / delta) + 1.0) * delta;
                    if (!(m < bound)) bound = m + delta;
                    continue;
                }
            }
            c.bound = bound;
            c.nq = Q[par ^ 1];
            c.nhq = HQ[par ^ 1];
            c.ntail = &ctl->qtail[par ^ 1];
            c.nhtail = &ctl->htail[par ^ 1];
            {
                // light vertices: LPV lanes per vertex, 64/LPV vertices per wave
                const int grp = lane / LPV, sub = lane % LPV;
                int32_t* cq = Q[par];
                for (int i0 = wave * (64 / LPV); i0 < qn; i0 += NWV * (64 / LPV)) {
                    const int i = i0 + grp;
                    process_group<LPV, LAYOUT, true>(g, c, i < qn ? cq[i] : -1, s, sub, kflags,
                                               (dbg && tid == 0) ? pst : nullptr);
                }
                tX = clock64(); cLight += tX - tA;
                // heavy vertices: one wave per vertex
                int32_t* chq = HQ[par];
                for (int i = wave; i < hn; i += NWV)
                    process_group<64, LAYOUT, true>(g, c, chq[i], s, lane, kflags);
                tX = clock64(); cHeavy += tX - tA;
            }
            ++phases;
            __syncthreads();
            if (tid == 0) {
                ctl->qtail[par] = 0;
                ctl->htail[par] = 0;
            }
            par ^= 1;
            __syncthreads();
            tB = clock64(); cRelax += tB - tA; tA = tB;
        }

        } else {
        // ---------------- delta-stepping (label-correcting) ----------------
        int par = 0;
        double bound = delta;
        for (;;) {
            unsigned long long myMin = INF_BITS;
            for (int w0 = wave * 64; w0 < nw; w0 += NT) {
                const int w = w0 + lane;
                const uint32_t bits = w < nw ? c.pend[w] : 0u;
                uint32_t tl = 0, th = 0;
                if (bits) {
                    const uint32_t hv = heavyBits[w];
                    uint32_t x = bits;
                    while (x) {
                        // 4 pending bits at a time: independent LDS reads in flight
                        int pb[4];
                        unsigned long long d[4];
#pragma unroll
                        for (int k = 0; k < 4; ++k) {
                            pb[k] = x ? __ffs(x) - 1 : -1;
                            x &= x - 1;
                        }
#pragma unroll
                        for (int k = 0; k < 4; ++k)
                            d[k] = pb[k] >= 0 ? c.dist[(w << 5) + pb[k]] : INF_BITS;
#pragma unroll
                        for (int k = 0; k < 4; ++k) {
                            if (pb[k] < 0) continue;
                            if (b2d(d[k]) < bound) {
                                if ((hv >> pb[k]) & 1u) th |= 1u << pb[k]; else tl |= 1u << pb[k];
                            } else {
                                myMin = d[k] < myMin ? d[k] : myMin;
                            }
                        }
                    }
                }
                tX = clock64(); cBits += tX - tA;
                const int nl = __popc(tl), nh = __popc(th);
                const int basel = nl ? atomicAdd(&ctl->qtail[par], nl) : 0;
                const int baseh = nh ? atomicAdd(&ctl->htail[par], nh) : 0;
                if (tl | th) {
                    uint32_t taken = 0, x = tl;
                    int pos = basel;
                    while (x && pos < qcap) {
                        const int bb = __ffs(x) - 1;
                        x &= x - 1;
                        Q[0][pos++] = (w << 5) + bb;
                        taken |= 1u << bb;
                    }
                    x = th;
                    pos = baseh;
                    while (x && pos < hcap) {
                        const int bb = __ffs(x) - 1;
                        x &= x - 1;
                        HQ[0][pos++] = (w << 5) + bb;
                        taken |= 1u << bb;
                    }
                    c.pend[w] = bits & ~taken;
                }
            }
            tX = clock64(); cResv += tX - tA;
            if (myMin != INF_BITS) atomicMin(&ctl->minNext[par], myMin);
            __syncthreads();
            const int qn = min(ctl->qtail[par], qcap);
            const int hn = min(ctl->htail[par], hcap);
            const unsigned long long mn = ctl->minNext[par];
            if (tid == 0) {
                ctl->qtail[par ^ 1] = 0;
                ctl->htail[par ^ 1] = 0;
                ctl->minNext[par ^ 1] = INF_BITS;
            }
            tB = clock64(); cScan += tB - tA; tA = tB;
            if (qn == 0 && hn == 0) {
                if (mn == INF_BITS) break;
                const double m = b2d(mn);
                bound = (floor(m / delta) + 1.0) * delta;
                if (!(m < bound)) bound = m + delta;
                par ^= 1;
                __syncthreads();
                continue;
            }
            {
                // light vertices: LPV lanes per vertex, 64/LPV vertices per wave
                const int grp = lane / LPV, sub = lane % LPV;
                for (int i0 = wave * (64 / LPV); i0 < qn; i0 += NWV * (64 / LPV)) {
                    const int i = i0 + grp;
                    process_group<LPV, LAYOUT, false>(g, c, i < qn ? Q[0][i] : -1, s, sub, kflags,
                                               (dbg && tid == 0) ? pst : nullptr);
                }
                tX = clock64(); cLight += tX - tA;
                // heavy vertices: one wave per vertex
                for (int i = wave; i < hn; i += NWV)
                    process_group<64, LAYOUT, false>(g, c, HQ[0][i], s, lane, kflags);
                tX = clock64(); cHeavy += tX - tA;
            }
            ++phases;
            par ^= 1;
            __syncthreads();
            tB = clock64(); cRelax += tB - tA; tA = tB;
        }

        }
        // ---------------- predecessor pass + tie detector -------------------
        // igraph sets parent[v] on the first strict improvement to the final
        // distance, i.e. from the first POPPED tight predecessor; pops are in
        // non-decreasing dist, so it is the tight in-arc with minimum dist[u]
        // unless two distinct vertices tie on that minimum (then the heap's
        // pop order decides -> row goes to k_exact_rows).
        int myAmb = 0, myMis = 0;
        if (!(kflags & 8)) {
            for (int v = tid; v < n; v += NT) {
                if (v == s) continue;
                const unsigned long long dvb = c.dist[v];
                if (dvb == INF_BITS) { c.P[v] = -1; continue; }
                const double dv = b2d(dvb);
                unsigned long long best = INF_BITS;
                int cnt = 0, ba = -1, bu = -1;
                const bool undirected = g.inCol == g.col;
                const int a0 = undirected ? c.rp[v] : g.inPtr[v];
                const int a1 = undirected ? c.rp[v + 1] : g.inPtr[v + 1];
                for (int a = a0; a < a1; a += UNR) {
                    int cu[UNR];
                    double lw[UNR];
                    unsigned long long du[UNR];
    #pragma unroll
                    for (int k = 0; k < UNR; ++k) {       // branch-free (see process_group)
                        const int ac = a + k < a1 ? a + k : a;
                        if (undirected) {   // the relax loop's 12-B arcs: one L2 copy of the graph
                            const Arc3 A = g.arc3[ac];
                            cu[k] = A.col;
                            lw[k] = __hiloint2double((int)A.latHi, (int)A.latLo);
                        } else {
                            cu[k] = g.inCol[ac];
                            lw[k] = g.inLat[ac];
                        }
                    }
    #pragma unroll
                    for (int k = 0; k < UNR; ++k) du[k] = c.dist[cu[k]];
    #pragma unroll
                    for (int k = 0; k < UNR; ++k) {
                        if (a + k < a1) {
                            const unsigned long long dub = du[k];
                            if (dub <= dvb && b2d(dub) + lw[k] == dv) {
                                if (dub < best) { best = dub; cnt = 1; ba = a + k; bu = cu[k]; }
                                else if (dub == best) ++cnt;
                            }
                        }
                    }
                }
                // the heap decides: equal-minimum tight predecessors, or the
                // minimum one reaching v by a zero-increment arc (a farther
                // zero-increment predecessor cannot win).  Marked in P's bit
                // 30 for the tie export (the row then never uses P itself).
                if (cnt != 1 || best == dvb) {
                    myAmb = 1;
                    c.P[v] = TIE_AMB | (ba > 0 ? ba : 0);
                    continue;
                }
                c.P[v] = ba;
                if ((int)c.H[v] != (int)c.H[bu] + 1 || c.R[v] != c.R[bu] * g.inRel[ba]) myMis = 1;
            }
        } else {
            // Grouped variant (kflags & 8; measured slower on C2, kept for
            // tuning): PL lanes per vertex read consecutive in-arcs (one line
            // per group per request instead of one per lane), PL*PU arcs per
            // batch, then a DPP merge of (min dist[u], count, first arc).
            constexpr int PL = 4, PU = 4;
            const int grp = tid / PL, sub = tid % PL, NG = NT / PL;
            const bool undirected = g.inCol == g.col;
            for (int v0 = 0; v0 < n; v0 += NG) {
                const int v = v0 + grp;
                const bool inV = v < n && v != s;
                const unsigned long long dvb = inV ? c.dist[v] : INF_BITS;
                const bool act = dvb != INF_BITS;
                const double dv = b2d(dvb);
                unsigned long long best = INF_BITS;
                int cnt = 0, ba = -1, bu = -1;
                if (act) {
                    const int a0 = undirected ? c.rp[v] : g.inPtr[v];
                    const int a1 = undirected ? c.rp[v + 1] : g.inPtr[v + 1];
                    for (int ab = a0 + sub; ab < a1; ab += PL * PU) {
                        int cu[PU];
                        double lw[PU];
                        unsigned long long du[PU];
                        bool ok[PU];
#pragma unroll
                        for (int k = 0; k < PU; ++k) {
                            const int a = ab + k * PL;
                            ok[k] = a < a1;
                            const int ac = ok[k] ? a : ab;
                            if (undirected) { const Arc A = g.arcs[ac]; cu[k] = A.col; lw[k] = A.lat; }
                            else { cu[k] = g.inCol[ac]; lw[k] = g.inLat[ac]; }
                        }
#pragma unroll
                        for (int k = 0; k < PU; ++k) du[k] = c.dist[cu[k]];
#pragma unroll
                        for (int k = 0; k < PU; ++k) {
                            if (!ok[k]) continue;
                            const unsigned long long dub = du[k];
                            if (dub <= dvb && b2d(dub) + lw[k] == dv) {
                                if (dub < best) { best = dub; cnt = 1; ba = ab + k * PL; bu = cu[k]; }
                                else if (dub == best) ++cnt;
                            }
                        }
                    }
                }
#pragma unroll
                for (int o = PL >> 1; o > 0; o >>= 1) {
                    const unsigned long long ob = gxor64<PL>(best, o);
                    const int oc = gxor<PL>(cnt, o);
                    const int oa = gxor<PL>(ba, o);
                    const int ou = gxor<PL>(bu, o);
                    if (ob < best) { best = ob; cnt = oc; ba = oa; bu = ou; }
                    else if (ob == best && oa >= 0) {
                        cnt += oc;
                        if (ba < 0 || oa < ba) { ba = oa; bu = ou; }
                    }
                }
                if (sub != 0 || !inV) continue;
                if (!act) { c.P[v] = -1; continue; }
                if (cnt != 1 || best == dvb) {
                    myAmb = 1;
                    c.P[v] = TIE_AMB | (ba > 0 ? ba : 0);
                    continue;
                }
                c.P[v] = ba;
                if ((int)c.H[v] != (int)c.H[bu] + 1 || c.R[v] != c.R[bu] * g.inRel[ba]) myMis = 1;
            }
        }
        if (myAmb) atomicOr(&ctl->ambig, 1);
        if (myMis) atomicOr(&ctl->mismatch, 1);
        __syncthreads();
        const long long tFinal = clock64();
        if (dbg && tid == 0) {
            dbg[16 * b + 0] = phases;
            dbg[16 * b + 2] = ctl->mismatch;
            dbg[16 * b + 3] = ctl->ambig;
            dbg[16 * b + 4] = (int)(cScan >> 4);
            dbg[16 * b + 5] = (int)(cRelax >> 4);
            dbg[16 * b + 6] = (int)((tFinal - tA) >> 4);
            dbg[16 * b + 8] = (int)(cBits >> 4);
            dbg[16 * b + 9] = (int)(cResv >> 4);
            dbg[16 * b + 10] = (int)(cLight >> 4);
            dbg[16 * b + 11] = (int)(cHeavy >> 4);
            dbg[16 * b + 12] = (int)(pst[0] >> 4);
            dbg[16 * b + 13] = (int)(pst[1] >> 4);
            dbg[16 * b + 14] = (int)(pst[2] >> 4);
            dbg[16 * b + 15] = (int)pst[3];
        }
        if (ctl->ambig) {
            // tie export (as k_batch_rows): final distances, fast-path parents
            // with the ambiguous ones marked, and the largest tied
            // predecessor distance -> early-stop emulation + k_tie_write
            int sl = -1;
            if (tieDesc) {
                const TieBuf tie = *tieDesc;
                if (tid == 0) {
                    const int x = atomicAdd(tie.count, 1);
                    ctl->changed = x < tie.cap ? x : -1;
                    ctl->minNext[0] = 0ull;
                }
                __syncthreads();
                sl = ctl->changed;
                if (sl >= 0) {
                    unsigned long long thr = 0ull;
                    const bool undirected = g.inCol == g.col;
                    const size_t o0 = (size_t)sl * (size_t)tie.n;
                    for (int v = tid; v < n; v += NT) {
                        const unsigned long long dvb = c.dist[v];
                        const int pv = v == s ? -1 : c.P[v];
                        tie.D[o0 + v] = b2d(dvb);
                        tie.P[o0 + v] = pv;
                        if (pv >= 0 && (pv & TIE_AMB)) {   // rare: the tied distance
                            const int a0 = undirected ? c.rp[v] : g.inPtr[v];
                            const int a1 = undirected ? c.rp[v + 1] : g.inPtr[v + 1];
                            unsigned long long mt = INF_BITS;
                            for (int a = a0; a < a1; ++a) {
                                const unsigned long long du = c.dist[g.inCol[a]];
                                if (du <= dvb && d2b(b2d(du) + g.inLat[a]) == dvb && du < mt) mt = du;
                            }
                            if (mt != INF_BITS && mt > thr) thr = mt;
                        }
                    }
                    if (thr) atomicMax(&ctl->minNext[0], thr);
                    __syncthreads();
                    if (tid == 0) tie.thr[sl] = b2d(ctl->minNext[0]);
                }
            }
            if (tid == 0) rowAmbig[b] = sl >= 0 ? (uint8_t)(2 + sl) : (uint8_t)1;
            __syncthreads();
            continue;
        }
        // Labels that raced or were set from a predecessor that later stopped
        // being the chosen one: Jacobi sweeps over the tree until a sweep
        // changes nothing (then every label satisfies its equation).
        int jac = 0;
        if (ctl->mismatch) {
            for (;; ++jac) {
                if (tid == 0) ctl->changed = 0;
                __syncthreads();
                int ch = 0;
                for (int v = tid; v < n; v += NT) {
                    const int a = c.P[v];
                    if (v == s || a < 0) continue;
                    const int u = g.inCol[a];
                    const int eh = (int)c.H[u] + 1;
                    const double er = c.R[u] * g.inRel[a];
                    if ((int)c.H[v] != eh || c.R[v] != er) { c.H[v] = (HopT)eh; c.R[v] = er; ch = 1; }
                }
                if (ch) atomicOr(&ctl->changed, 1);
                __syncthreads();
                if (!ctl->changed) break;
                __syncthreads();
            }
        }
        if (tid == 0) {
            rowAmbig[b] = 0;
            if (dbg) dbg[16 * b + 1] = jac;
        }
        const long long tW = clock64();
        if (kflags & 4)
            write_row<true>(g, tab, r, s, [&](int t) { return c.dist[t]; },
                            [&](int t) { return (int)c.H[t]; }, c.R, c.P, 0, tid, NT);
        else
            write_row(g, tab, r, s, [&](int t) { return c.dist[t]; },
                      [&](int t) { return (int)c.H[t]; }, c.R, c.P, 0, tid, NT);
        __syncthreads();
        if (dbg && tid == 0) dbg[16 * b + 7] = (int)((clock64() - tW) >> 4);
    }
}

// ---------------------------------------------------------------------------
// Early-stop tie rows.  k_batch_rows exported the final distances and the
// fast-path parents of a tie row, TIE_AMB marking the entries whose parent
// the heap decides (equal-minimum tight predecessors / zero-increment arcs),
// and the largest tied predecessor distance thr.  The igraph heap emulation
// stops before the first pop with key > thr: by then every tied predecessor
// was popped, so the emulated parent of each marked entry is final (a later
// pop never improves its distance strictly).  Unmarked entries have a single
// candidate parent, which the emulation would pick too.  tie_finalize merges
// the two parent sets; k_tie_write derives hops / reliability along them.
//
// Consistency check (round 5): every vertex the emulation popped has its
// final igraph distance in Dem, which must equal the exported distance of the
// same row (distances are positive, so equal values are equal bits; the
// source may read -0.0).  A slot holding another source's (or a stale)
// distance array fails it: thr := NaN, k_tie_write leaves the row alone and
// the engine recomputes it with the full emulation (ShdPeStats.rowsTieRepaired,
// zero in every correct run).
// ---------------------------------------------------------------------------
template <class Reached, class Popped>
__device__ __forceinline__ void tie_finalize(const TieBuf& tie, int slot, int n, int lane,
                                             Reached reached, Popped popped, const double* Dem,
                                             const int32_t* P) {
    int32_t* tp = tie.P + (size_t)slot * (size_t)tie.n;
    const double* td = tie.D + (size_t)slot * (size_t)tie.n;
    bool bad = false;
    for (int v = lane; v < n; v += EX_THREADS) {
        const int fp = tp[v];
        if (fp >= 0 && (fp & TIE_AMB))
            tp[v] = reached(v) ? P[v] : -1;   // unreached: off every target's path
        if (popped(v) && Dem[v] != td[v]) bad = true;   // (value compare: the SoA kernel pops the source as -0.0)
    }
    if (__ballot(bad) && lane == 0) tie.thr[slot] = __longlong_as_double(0x7ff8000000000000ll);
}

__device__ __forceinline__ bool tie_slot_bad(const TieBuf& tie, int slot) {
    const double t = tie.thr[slot];
    return t != t;
}

// One workgroup per tie row: is any ambiguous entry on the path to a target?
// A target's igraph path equals its fast-path parent chain up to the first
// ambiguous vertex on it, so if no target chain meets one the fast-path
// parents are exact and the emulation is skipped (thr := -1).  tie.H marks
// vertices whose chain up to the source is known clean (k_tie_write
// re-initialises it).
__global__ __launch_bounds__(1024) void k_tie_scan(DevGraph g0, const int32_t* __restrict__ rows,
                                                   const int32_t* __restrict__ slots, TieBuf tie) {
    const DevGraph g = global_view(g0);
    __shared__ int hit;
    const int n = g.n, T = g.T;
    const int tid = threadIdx.x;
    const int s = g.attached[rows[blockIdx.x]];
    const int sl = slots[blockIdx.x];
    const size_t off = (size_t)sl * (size_t)tie.n;
    const int32_t* P = tie.P + off;
    int32_t* clean = tie.H + off;
    for (int v = tid; v < n; v += 1024) clean[v] = 0;
    if (tid == 0) hit = 0;
    __syncthreads();
    for (int j = tid; j < T; j += 1024) {
        if (ld_wg(&hit)) break;
        const int t = g.attached[j];
        int x = t, bad = 0;
        while (x != s && !ld_wg(&clean[x])) {
            const int p = P[x];
            if (p < 0) break;                          // unreachable
            if (p & TIE_AMB) { bad = 1; break; }
            x = g.inCol[p];
        }
        if (bad) { hit = 1; break; }
        for (int y = t; y != x;) {                     // the walked prefix is clean
            const int p = P[y];
            if (p < 0) break;
            clean[y] = 1;
            y = g.inCol[p];
        }
    }
    __syncthreads();
    if (tid == 0 && !hit) tie.thr[sl] = -1.0;
}

// One workgroup per tie row: hop counts and reliability products level by
// level along the final parent tree (level d reads only level d - 1, written
// before the barrier), then the row writer (topology.c:1805-1864).
constexpr int TW_THREADS = 1024;

__global__ __launch_bounds__(TW_THREADS) void k_tie_write(DevGraph g0, DevTable tab0,
                                                          const int32_t* __restrict__ rows,
                                                          const int32_t* __restrict__ slots,
                                                          TieBuf tie) {
    const DevGraph g = global_view(g0);
    const DevTable tab = global_view(tab0);
    __shared__ int changed;
    const int n = g.n;
    const int tid = threadIdx.x;
    const int r = rows[blockIdx.x];
    const int s = g.attached[r];
    if (tie_slot_bad(tie, slots[blockIdx.x])) return;   // the engine recomputes the row
    const size_t off = (size_t)slots[blockIdx.x] * (size_t)tie.n;
    const double* D = tie.D + off;
    // latency floor: the exported distances must be this row's -- its own
    // source at exactly 0 (latencies are validated > 0, so no other vertex
    // is) -- or the row is not written from them: a slot filled from another
    // source's array (the round-4 wrong-row symptom, latencies below the true
    // distances) is marked bad and the engine recomputes the row with the
    // full emulation (rowsTieRepaired)
    if (D[s] != 0.0) {
        if (tid == 0) tie.thr[slots[blockIdx.x]] = __builtin_nan("");
        return;
    }
    const int32_t* P = tie.P + off;
    int32_t* H = tie.H + off;
    double* R = tie.R + off;
    for (int v = tid; v < n; v += TW_THREADS) {
        H[v] = v == s ? 0 : -1;
        R[v] = 1.0;
    }
    __syncthreads();
    if (tid == 0) changed = 0;
    __syncthreads();
    for (int d = 1;; ++d) {
        int ch = 0;
        for (int v = tid; v < n; v += TW_THREADS) {
            if (H[v] >= 0) continue;
            const int a = P[v];
            if (a < 0) continue;
            const int x = g.inCol[a];
            if (H[x] != d - 1) continue;
            R[v] = R[x] * g.inRel[a];
            H[v] = d;
            ch = 1;
        }
        if (ch) changed = 1;
        __syncthreads();
        const int any = changed;
        __syncthreads();              // everyone has read it before the reset
        if (!any) break;
        if (tid == 0) changed = 0;
        __syncthreads();
    }
    write_row(g, tab, r, s, [&](int t) { return d2b(D[t]); }, [&](int t) { return H[t]; }, R, P,
              F_EXACT, tid, TW_THREADS);
}

// ---------------------------------------------------------------------------
// k_exact_rows: igraph 0.7.1 Dijkstra with the 2-way heap (heap.c), one wave
// per row, for graphs whose heap does not fit LDS (n > EX_SOA_MAXN).
//
// Layout: the heap is structure-of-arrays, key f64 (igraph's -dist) + vertex
// i32; positions < hc in LDS (12 B each: 13.6k entries in 160 KB, the top
// 13 levels), the tail in the workgroup's global slot.  Per vertex (global):
// index2 (0 never reached, 1 popped, >= 2 heap position + 2), the current
// tentative distance (= final distance once popped), labels P/H/R.
//
// The heap operations are wave-parallel but leave exactly igraph's array
// (hence its pop order):
//   sink     (igraph_i_2wheap_sink): the 62 nodes of the 5-level subtree
//            below the hole are loaded at once (one lane each); every lane
//            decides whether it is the child its parent descends to (left
//            when left >= right or no right), a ballot gives the descent
//            path, and the moving key passes the path nodes it is strictly
//            smaller than (a prefix: keys fall along the path).  Those nodes
//            move up one level in parallel; a full 5-level prefix continues
//            below.  A 16-level heap costs 4 dependent rounds, not 16.
//   shift_up (igraph_i_2wheap_shift_up): lane j loads the ancestor j + 1
//            levels up; the key rises past every ancestor it is not strictly
//            smaller than (a prefix: keys grow towards the root); those
//            ancestors move down one level in parallel.
//   modify   (new key > old key, since igraph modifies only on a strictly
//            shorter distance): its sink is a no-op, so shift_up alone.
// The wave pre-checks all arcs of the popped vertex in parallel against
// index2 / the tentative distance (the decision for arc k depends only on
// v_k's own state: no parallel edges, no self-loops in the CSR), writes the
// labels, and the pushes / modifies then run in incidence order.
// A wave's own global stores are seen by its later loads (wavefront-scope
// ordering), so heap operations chain without fences.
// ---------------------------------------------------------------------------

// Heap storage: positions < hc in LDS (dynamic shared memory at offset 0,
// addressed through the __shared__ symbol so accesses stay ds_* -- a flat
// access would also wait for every outstanding global store), the tail in
// the global slot.
extern __shared__ __attribute__((aligned(16))) unsigned char ex_smem[];

// a uniform lane's double, by two v_readlane (no LDS round trip)
__device__ __forceinline__ double readlane_f64(double x, int k) {
    const long long b = __double_as_longlong(x);
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)b, k);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(b >> 32), k);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

struct WHeap {
    double* gkey;     // global tail: position p >= hc at gkey[p - hc]
    int32_t* gidx;
    int32_t* I2;      // index2 (global, per vertex)
    int hc;
    uint32_t* bitw;   // preferred-child bits (LDS, k_exact_rows<.., true>), see below
    __device__ __forceinline__ double* lkey() const { return reinterpret_cast<double*>(ex_smem); }
    __device__ __forceinline__ int32_t* lidx() const {
        return reinterpret_cast<int32_t*>(ex_smem + (size_t)8 * hc);
    }
    // per-lane load / store of position p (LDS or global by lane)
    __device__ __forceinline__ void get(int p, double& k, int& id) const {
        if (p < hc) {
            k = lkey()[p];
            id = lidx()[p];
            asm volatile("" : "+v"(k), "+v"(id));   // no merge of the two branches
        } else {                                      // into one flat load
            k = gkey[p - hc];
            id = gidx[p - hc];
            asm volatile("" : "+v"(k), "+v"(id));
        }
    }
    __device__ __forceinline__ void put(int p, double k, int id) const {
        if (p < hc) {
            lkey()[p] = k;
            lidx()[p] = id;
        } else {
            gkey[p - hc] = k;
            gidx[p - hc] = id;
        }
        I2[id] = p + 2;
    }
    // LDS-only variants for operations whose positions all lie below hc
    // (uniform check): no per-lane LDS/global branches
    __device__ __forceinline__ void put_lds(int p, double k, int id) const {
        lkey()[p] = k;
        lidx()[p] = id;
        I2[id] = p + 2;
    }
    // One round of igraph_i_2wheap_sink of (k, id): the hole at `head` (heap
    // level hl) and up to 5 levels below it.  Returns true once (k, id) is
    // placed; otherwise the hole moved `dd` levels down.  Rounds are cut at
    // the deepest all-LDS level when the rest of the heap then fits one
    // round, so a sift-down touches the global tail once.
    __device__ __forceinline__ bool sink_round(int& head, int& hl, double k, int id, int size,
                                               int ldsLevel, int lane) const {
        // every operand but the lane's own node is wave-uniform: say so, so
        // the descent bookkeeping is scalar code, not exec-masked VALU loops
        head = __builtin_amdgcn_readfirstlane(head);
        hl = __builtin_amdgcn_readfirstlane(hl);
        size = __builtin_amdgcn_readfirstlane(size);
        ldsLevel = __builtin_amdgcn_readfirstlane(ldsLevel);
        k = readlane_f64(k, 0);
        id = __builtin_amdgcn_readfirstlane(id);
        const int bottom = 31 - __builtin_clz(size);       // deepest heap level
        int dd = bottom - hl < 5 ? bottom - hl : 5;
        if (dd <= 0) {
            if (lane == 0) put(head, k, id);
            return true;
        }
        if (hl < ldsLevel && hl + dd > ldsLevel && hl + dd < bottom && bottom - ldsLevel <= 5)
            dd = ldsLevel - hl;
        const int q = lane + 2;                            // subtree node (BFS index, root 1)
        const int d = 31 - __builtin_clz(q);               // its depth below the hole
        const int pos = (head + 1) * (1 << d) - 1 + (q - (1 << d));
        const bool left = (q & 1) == 0;
        const bool valid = d <= dd && pos < size;
        const bool sibValid = d <= dd && (left ? pos + 1 : pos - 1) < size;
        const bool lds = (head + 1) * (1 << dd) + (1 << dd) - 2 < hc;   // deepest node of the round
        double kq = 0.0;
        int iq = -1;
        if (lds) {                                         // branch-free: clamped position
            const int pc = valid ? pos : 0;
            kq = lkey()[pc];
            iq = lidx()[pc];
        } else if (valid) {
            get(pos, kq, iq);
        }
        // sibling (lanes 2i, 2i+1): a DPP quad permute, no LDS round trip
        const double ks = __longlong_as_double(
            (long long)gxor64<4>((unsigned long long)__double_as_longlong(kq), 1));
        // the child its parent descends to: left when left >= right or no right
        const bool chosen = valid && (left ? (!sibValid || kq >= ks) : !(ks >= kq));
        const unsigned long long cm = __ballot(chosen);
        // descent path (scalar): from the hole, the chosen child per level
        unsigned long long path = 0ull;
        for (int x = 1, lv = 0; lv < dd; ++lv) {
            const int c = 2 * x;                           // left child's node index
            if ((cm >> (c - 2)) & 1ull) x = c;
            else if ((cm >> (c - 1)) & 1ull) x = c + 1;
            else break;
            path |= 1ull << (x - 2);
        }
        const bool mv = ((path >> lane) & 1ull) && k < kq;   // passed: a prefix of the path
        const unsigned long long mm = __ballot(mv);
        if (mv) {
            if (lds) put_lds((pos - 1) >> 1, kq, iq);
            else put((pos - 1) >> 1, kq, iq);
        }
        if (mm == 0ull) {
            if (lane == 0) put(head, k, id);
            return true;
        }
        const int hp = __builtin_amdgcn_readlane(pos, 63 - __builtin_clzll(mm));   // deepest passed
        if (__builtin_popcountll(mm) < dd) {
            if (lane == 0) put(hp, k, id);
            return true;
        }
        head = hp;
        hl += dd;
        return false;
    }
    // ---- preferred-child bits (round 5) --------------------------------
    // One bit per internal heap node, 1-based node numbering (node N =
    // position N - 1, children 2N and 2N + 1): set iff the right child
    // exists and its key is strictly larger, i.e. the child igraph's sink
    // descends to from N.  Every operation that changes a key keeps the bits
    // of the changed nodes' parents current (and a pop that removes a right
    // child clears its parent's bit), so a sift-down finds its whole descent
    // path from the bits alone -- six levels per LDS word round and a few
    // scalar instructions per level -- and then loads, compares and moves
    // only the path's nodes in ONE parallel round, instead of loading and
    // ranking every node of each 5-level subtree (62 lanes per round, four
    // rounds for a 16-level heap).  A node's bit is read only while it is
    // internal and every node is re-derived when it gains a child, so the
    // bits need no per-row initialisation.  Updates are LDS atomics (lanes
    // of one operation may share a word).
    __device__ __forceinline__ double get_key(int p) const {
        double k;
        if (p < hc) {
            k = lkey()[p];
            asm volatile("" : "+v"(k));
        } else {
            k = gkey[p - hc];
            asm volatile("" : "+v"(k));
        }
        return k;
    }
    __device__ __forceinline__ void bit_put(int node, bool v) const {
        const uint32_t m = 1u << (node & 31);
        if (v) atomicOr(&bitw[node >> 5], m);
        else atomicAnd(&bitw[node >> 5], ~m);
    }
    // after a pop shrank the heap to `size`: the removed node size + 1, when
    // it was a right child, leaves its parent with the left child only
    __device__ __forceinline__ void bits_removed(int size, int lane) const {
        const int r = size + 1;
        if (lane == 0 && r >= 3 && (r & 1)) bit_put(r >> 1, false);
    }
    // sift-down phase 1: the descent path below the root (nodes of depth
    // 1..K in lanes 0..K-1 of pnode); returns K
    __device__ __forceinline__ int sink_path(int size, int lane, int& pnode) const {
        size = __builtin_amdgcn_readfirstlane(size);
        int cur = 1, K = 0;
        pnode = 1;
        while (2 * cur <= size) {
            // lane d < 6: the bit word of the level d below cur (2^d <= 32
            // consecutive, aligned node numbers: one word)
            const int base = lane < 6 ? cur << lane : 0;
            uint32_t wv = 0u;
            if (lane < 6 && base <= (size >> 1)) wv = bitw[base >> 5];
            int d = 0;
            for (; d < 6 && 2 * cur <= size; ++d) {
                const uint32_t w = (uint32_t)__builtin_amdgcn_readlane((int)wv, d);
                cur = 2 * cur + (int)((w >> (cur & 31)) & 1u);
                pnode = lane == K ? cur : pnode;
                ++K;
            }
        }
        return K;
    }
    // sift-down phase 2: (k, id) passes the path prefix it is strictly
    // smaller than (igraph_i_2wheap_sink); those nodes move up one level.
    // Split in two so the caller can issue the path's loads before it waits
    // for anything else: sink_load issues them, sink_place uses them.
    struct PathVals {
        double kq, ks;
        int iq;
    };
    __device__ __forceinline__ PathVals sink_load(int size, int K, int pnode, int lane) const {
        size = __builtin_amdgcn_readfirstlane(size);
        K = __builtin_amdgcn_readfirstlane(K);
        const bool on = lane < K;
        const int q = on ? pnode : 1;
        const int sb = q ^ 1;
        PathVals pv{0.0, 0.0, -1};
        if (on) get(q - 1, pv.kq, pv.iq);
        if (on && sb <= size) pv.ks = get_key(sb - 1);
        return pv;
    }
    __device__ __forceinline__ void sink_place(double k, int id, int size, int K, int pnode,
                                               const PathVals& pv, int lane) const {
        k = readlane_f64(k, 0);
        id = __builtin_amdgcn_readfirstlane(id);
        size = __builtin_amdgcn_readfirstlane(size);
        K = __builtin_amdgcn_readfirstlane(K);
        const bool on = lane < K;
        const int q = on ? pnode : 1;
        const int sb = q ^ 1;
        const bool sibOk = on && sb <= size;
        const double kq = pv.kq, ks = pv.ks;
        const int iq = pv.iq;
        const unsigned long long mm = __ballot(on && k < kq);   // a prefix of the path
        const int m = __builtin_popcountll(mm);
        if (lane < m) put((q >> 1) - 1, kq, iq);
        const int fin = m == 0 ? 1 : __builtin_amdgcn_readlane(pnode, m - 1);
        if (lane == 0) put(fin - 1, k, id);
        // node q_(t+1) (lane t < m) now holds lane t+1's key, or k
        const double kn = __shfl_down(kq, 1, 64);
        const double nk = lane == m - 1 ? k : kn;
        if (lane < m) bit_put(q >> 1, (q & 1) == 0 ? (sibOk && ks > nk) : (nk > ks));
    }
    // igraph_i_2wheap_shift_up with the bits kept: `size` counts (k, id)
    __device__ __forceinline__ void shift_up_bits(int elem, double k, int id, int size, int lane) const {
        elem = __builtin_amdgcn_readfirstlane(elem);
        k = readlane_f64(k, 0);
        id = __builtin_amdgcn_readfirstlane(id);
        size = __builtin_amdgcn_readfirstlane(size);
        const int e1 = elem + 1;
        const int x = lane < 31 ? e1 >> lane : 0;          // node x_j: e1 and its ancestors
        const int a = lane < 31 ? e1 >> (lane + 1) : 0;    // its parent (0: none)
        const bool valid = a >= 1;
        const int sb = x ^ 1;
        const bool sibOk = valid && sb <= size;
        double ka = 0.0, ks = 0.0;
        int ia = -1;
        if (e1 < hc) {                                     // every node involved in LDS
            const int ac = valid ? a - 1 : 0;
            ka = lkey()[ac];
            ia = lidx()[ac];
            ks = lkey()[sibOk ? sb - 1 : 0];
        } else {
            if (valid) get(a - 1, ka, ia);
            if (sibOk) ks = get_key(sb - 1);
        }
        const unsigned long long sm = __ballot(!valid || k < ka);
        const int c = __builtin_ctzll(sm);                 // ancestors passed (k >= theirs)
        if (lane < c) {
            if (e1 < hc) put_lds(x - 1, ka, ia);
            else put(x - 1, ka, ia);
        }
        if (lane == 0) put((e1 >> c) - 1, k, id);
        // x_j (j <= c) changed: to ancestor j+1's key (j < c) or to k
        if (lane <= c && valid) {
            const double nk = lane < c ? ka : k;
            bit_put(a, (x & 1) == 0 ? (sibOk && ks > nk) : (nk > ks));
        }
    }
    // igraph_i_2wheap_shift_up of (k, id) from the hole at `elem`
    __device__ __forceinline__ void shift_up(int elem, double k, int id, int lane) const {
        elem = __builtin_amdgcn_readfirstlane(elem);
        k = readlane_f64(k, 0);
        id = __builtin_amdgcn_readfirstlane(id);
        const int a = lane < 31 ? ((elem + 1) >> (lane + 1)) - 1 : -1;
        const bool valid = a >= 0;
        const bool lds = elem < hc;                      // every ancestor and the hole
        double ka = 0.0;
        int ia = -1;
        if (lds) {
            const int ac = valid ? a : 0;
            ka = lkey()[ac];
            ia = lidx()[ac];
        } else if (valid) {
            get(a, ka, ia);
        }
        const unsigned long long sm = __ballot(!valid || k < ka);
        const int c = __builtin_ctzll(sm);               // ancestors passed
        if (lane < c) {
            if (lds) put_lds(((elem + 1) >> lane) - 1, ka, ia);
            else put(((elem + 1) >> lane) - 1, ka, ia);
        }
        if (lane == 0) put(c == 0 ? elem : ((elem + 1) >> c) - 1, k, id);
    }
};

// Stream an array through the cache hierarchy once (16-B loads, 8 in flight
// per lane): the exact kernel touches each vertex's arcs once per row in a
// dependent chain, so without this every pop pays HBM latency twice.
__device__ __forceinline__ uint32_t warm_cache(const void* p, size_t bytes, int lane, int nl) {
    const uint4* q = reinterpret_cast<const uint4*>(p);
    const size_t nv = bytes / 16;
    uint32_t acc = 0;
    for (size_t i = lane; i < nv; i += (size_t)nl * 8) {
        uint4 v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const size_t j = i + (size_t)k * nl;
            v[k] = q[j < nv ? j : i];
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) acc ^= v[k].x ^ v[k].w;
    }
    return acc;
}

// XD: per-pop segment counters (SHD_PE_DEBUG_COUNTERS; a separate
// instantiation so the product build carries none of their registers).
// BITS: sift-downs by the preferred-child bits (LDS words after the heap
// head; the engine sizes hc for them), else by 5-level subtree rounds.
template <bool XD, bool BITS>
__global__ __launch_bounds__(EX_THREADS) void k_exact_rows(DevGraph g0, DevTable tab0,
                                                           DevScratch sc0,
                                                           const int32_t* __restrict__ rows,
                                                           int32_t nRows, int32_t hc,
                                                           const int32_t* __restrict__ slots,
                                                           TieBuf tie, long long* xdbg) {
    const DevGraph g = global_view(g0);
    const DevTable tab = global_view(tab0);
    const DevScratch sc = global_view(sc0);
    const int n = g.n;
    const int lane = threadIdx.x;
    const size_t slot = (size_t)blockIdx.x * (size_t)sc.stride;
    double* D = sc.dist + slot;          // tentative distance; final once popped
    int32_t* H = sc.hops + slot;
    double* R = sc.rel + slot;
    int32_t* P = sc.pred + slot;
    // latFold multigraphs (g.flat): the reported latency is the fold of the
    // newest parallel edges' latencies along the path (topology.c:1488-1498),
    // a third label beside hops and reliability
    double* LF = g.flat && sc.lfold ? sc.lfold + slot : nullptr;
    double* tailKey = reinterpret_cast<double*>(sc.heapTail) + (size_t)blockIdx.x * 2 * sc.heapStride;
    const WHeap h{tailKey, reinterpret_cast<int32_t*>(tailKey + sc.heapStride), sc.index2 + slot, hc,
                  reinterpret_cast<uint32_t*>(ex_smem + (((size_t)12 * hc + 15) & ~(size_t)15))};
    {
        const size_t m = (size_t)g.rowPtr[n];
        uint32_t acc = warm_cache(g.rowPtr, (size_t)4 * (n + 1), lane, EX_THREADS);
        acc ^= warm_cache(g.col, 4 * m, lane, EX_THREADS);
        acc ^= warm_cache(g.lat, 8 * m, lane, EX_THREADS);
        acc ^= warm_cache(g.rel, 8 * m, lane, EX_THREADS);
        acc ^= warm_cache(g.outToIn, 4 * m, lane, EX_THREADS);
        acc ^= warm_cache(g.isAttached, (size_t)n, lane, EX_THREADS);
        if (acc == 0x5bd1e995u) D[lane] = 0.0;   // keeps the loads; D is rewritten before use
    }

    for (int b = blockIdx.x; b < nRows; b += gridDim.x) {
        const int r = __builtin_amdgcn_readfirstlane(rows[b]);
        const int s = __builtin_amdgcn_readfirstlane(g.attached[r]);
        const int tslot = __builtin_amdgcn_readfirstlane(slots ? slots[b] : -1);
        const double thr = readlane_f64(tslot >= 0 ? tie.thr[tslot] : 0.0, 0);
        if (tslot < 0 || thr >= 0.0)
            for (int v = lane; v < n; v += EX_THREADS) h.I2[v] = 0;
        __syncthreads();
        if (lane == 0) {
            h.put(0, 0.0, s);
            D[s] = 0.0;
            H[s] = 0;
            R[s] = 1.0;
            P[s] = -1;
            if (LF) LF[s] = 0.0;
        }
        __syncthreads();
        int toReach = g.T;
        int size = 1;                    // uniform
        // SHD_PE_DEBUG_COUNTERS: cycles per pop segment (top+range, sink,
        // arcs+pre-check, pushes), pops, pushes + modifies, heap size at exit
        long long xc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        long long xt = XD ? (long long)clock64() : 0;
        auto xtick = [&](int k) {
            if constexpr (XD) { const long long t = (long long)clock64(); xc[k] += t - xt; xt = t; }
        };
        // early-stop rows need only the parents (k_tie_write derives hops and
        // reliability); a relevance scan may have cleared the row (thr < 0)
        const bool labels = tslot < 0;
        const int ldsLevel = 30 - __builtin_clz(hc + 1);   // deepest heap level wholly in LDS
        if (tslot >= 0 && thr < 0.0) size = 0;
        while (size > 0 && toReach > 0) {
            // pop (igraph_2wheap_delete_max): the vertex record of the top and
            // the last element load together, the sink's LDS rounds overlap them
            const int u = __builtin_amdgcn_readfirstlane(h.lidx()[0]);
            const double mind = -h.lkey()[0];
            if (tslot >= 0 && mind > thr) break;   // early stop: tied predecessors all popped
            const int a0 = g.rowPtr[u], a1 = g.rowPtr[u + 1];
            const int att = g.isAttached[u];
            int hu = 0;
            double ru = 1.0, lfu = 0.0;
            if (labels) { hu = H[u]; ru = R[u]; }
            if (labels && LF) lfu = LF[u];
            size -= 1;
            double km = 0.0;
            int im = 0;
            if (size > 0) h.get(size, km, im);       // uniform position: last element
            if constexpr (XD) { asm volatile("" :: "v"(a0), "v"(a1), "v"(att)); xtick(0); xc[5]++; }
            if (lane == 0) h.I2[u] = 1;
            int head = 0, hl = 0, pK = 0, pnode = 0;
            bool placed = size == 0;
            if constexpr (BITS) {
                h.bits_removed(size, lane);
            } else {
                if (!placed) placed = h.sink_round(head, hl, km, im, size, ldsLevel, lane);
            }
            if (att) --toReach;
            // arcs in chunks of 64; the first chunk's loads and pre-check
            // overlap the remaining sink rounds (the pre-check reads only
            // index2 categories and tentative distances, which a sift-down
            // does not change)
            for (int base = a0; base < a1 || !placed; base += 64) {
                const int a = base + lane;
                const bool valid = a < a1;
                int v = 0, ia = 0;
                double w = 0.0;
                if (valid) {
                    v = g.col[a];
                    w = g.lat[a];
                    ia = g.outToIn[a];
                }
                WHeap::PathVals pv{0.0, 0.0, -1};
                if constexpr (BITS) {
                    if (!placed) {
                        pK = h.sink_path(size, lane, pnode);   // LDS words only
                        pv = h.sink_load(size, pK, pnode, lane);   // in flight under the arc loads' wait
                    }
                } else {
                    if (!placed) placed = h.sink_round(head, hl, km, im, size, ldsLevel, lane);
                }
                // read before the sift-down finished: categories and distances
                // hold, heap positions may not
                const bool posFresh = placed;
                int st = 1;
                double dv = 0.0;
                if (valid) {
                    st = h.I2[v];
                    dv = D[v];
                }
                if constexpr (BITS) {
                    if (!placed) {
                        h.sink_place(km, im, size, pK, pnode, pv, lane);
                        placed = true;
                    }
                } else {
                    while (!placed) placed = h.sink_round(head, hl, km, im, size, ldsLevel, lane);
                }
                xtick(1);
                const double alt = mind + w;
                int need = 0;
                if (st == 0) need = 1;
                else if (st >= 2) need = alt < dv ? 2 : 0;
                if (need) {
                    P[v] = ia;
                    D[v] = alt;
                    if (labels) { H[v] = hu + 1; R[v] = ru * g.rel[a]; }
                    if (labels && LF) LF[v] = lfu + g.flat[a];
                }
                unsigned long long mask = __ballot(need != 0);
                xtick(2);
                if constexpr (XD) xc[6] += __builtin_popcountll(mask);
                bool moved = !posFresh;    // positions read in the pre-check stale?
                while (mask) {
                    const int k = __builtin_ctzll(mask);
                    mask &= mask - 1;
                    const int vk = __builtin_amdgcn_readlane(v, k);
                    const int nk = __builtin_amdgcn_readlane(need, k);
                    const double ak = readlane_f64(alt, k);
                    if (nk == 1) {                    // igraph_2wheap_push_with_index
                        if constexpr (BITS) h.shift_up_bits(size, -ak, vk, size + 1, lane);
                        else h.shift_up(size, -ak, vk, lane);
                        size += 1;
                    } else {                          // igraph_2wheap_modify (sink is a no-op)
                        const int p2 = moved ? h.I2[vk] : __builtin_amdgcn_readlane(st, k);
                        const int pos = __builtin_amdgcn_readfirstlane(p2) - 2;
                        if constexpr (BITS) h.shift_up_bits(pos, -ak, vk, size, lane);
                        else h.shift_up(pos, -ak, vk, lane);
                    }
                    moved = true;
                }
                xtick(3);
            }
        }
        if (XD && lane == 0) {
            xc[7] = size;
            for (int k = 0; k < 8; ++k) xdbg[(size_t)b * 8 + k] = xc[k];
        }
        __syncthreads();
        if (tslot >= 0)
            tie_finalize(tie, tslot, n, lane, [&](int v) { return thr >= 0.0 && h.I2[v] != 0; },
                         [&](int v) { return thr >= 0.0 && h.I2[v] == 1; }, D, P);
        else
            write_row(g, tab, r, s,
                      [&](int t) { return h.I2[t] == 1 ? d2b(LF ? LF[t] : D[t]) : INF_BITS; },
                      [&](int t) { return H[t]; }, R, P, F_EXACT, lane, EX_THREADS);
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------
// k_exact_rows_soa: the same emulation when the whole heap and index2 fit
// LDS (16 B per vertex: n <= 10240).  Structure-of-arrays heap (key f64,
// idx i32) so a sift-down level reads both children's keys with one
// ds_read2_b64 and their ids with one ds_read2_b32 -- one LDS round trip per
// level, no global branch.  Labels are not carried in the heap: the lanes
// that push / modify v write P/H/R[v] (global); the pop reads H/R[u] after
// a workgroup release fence (the writes came from other lanes of this wave).
constexpr int EX_SOA_MAXN = 10240;

__global__ __launch_bounds__(EX_THREADS) void k_exact_rows_soa(DevGraph g0, DevTable tab0,
                                                               DevScratch sc0,
                                                               const int32_t* __restrict__ rows,
                                                               int32_t nRows,
                                                               const int32_t* __restrict__ slots,
                                                               TieBuf tie, long long* xdbg) {
    const DevGraph g = global_view(g0);
    const DevTable tab = global_view(tab0);
    const DevScratch sc = global_view(sc0);
    const int n = g.n;
    const int lane = threadIdx.x;
    const size_t slot = (size_t)blockIdx.x * (size_t)sc.stride;
    double* hkey = reinterpret_cast<double*>(ex_smem);
    int32_t* hidx = reinterpret_cast<int32_t*>(ex_smem + (size_t)8 * n);
    int32_t* index2 = hidx + n;
    double* D = sc.dist + slot;
    int32_t* H = sc.hops + slot;
    double* R = sc.rel + slot;
    int32_t* P = sc.pred + slot;
    double* LF = g.flat && sc.lfold ? sc.lfold + slot : nullptr;   // latFold (k_exact_rows)
    {
        const size_t m = (size_t)g.rowPtr[n];
        uint32_t acc = warm_cache(g.rowPtr, (size_t)4 * (n + 1), lane, EX_THREADS);
        acc ^= warm_cache(g.col, 4 * m, lane, EX_THREADS);
        acc ^= warm_cache(g.lat, 8 * m, lane, EX_THREADS);
        acc ^= warm_cache(g.rel, 8 * m, lane, EX_THREADS);
        acc ^= warm_cache(g.outToIn, 4 * m, lane, EX_THREADS);
        acc ^= warm_cache(g.isAttached, (size_t)n, lane, EX_THREADS);
        if (acc == 0x5bd1e995u) D[lane] = 0.0;   // keeps the loads; D is rewritten before use
    }
    // lane-0 heap primitives (hole moves; igraph heap.c semantics)
    auto place = [&](int p, double k, int id) {
        hkey[p] = k;
        hidx[p] = id;
        index2[id] = p + 2;
    };
    auto sink_hole = [&](int head, double k, int size) -> int {
        for (;;) {
            const int l = 2 * head + 1;
            if (l >= size) return head;
            const bool hasR = l + 1 < size;
            const double kl = hkey[l], kr = hkey[l + 1];   // l + 1 <= n - 1 + 1: inside LDS
            const int il = hidx[l], ir = hidx[l + 1];
            const bool useL = !hasR || kl >= kr;
            const double ck = useL ? kl : kr;
            if (!(k < ck)) return head;
            place(head, ck, useL ? il : ir);
            head = useL ? l : l + 1;
        }
    };
    auto shift_up = [&](int elem, double k, int id) {
        while (elem > 0) {
            const int p = ((elem + 1) >> 1) - 1;
            const double pk = hkey[p];
            if (k < pk) break;
            place(elem, pk, hidx[p]);
            elem = p;
        }
        place(elem, k, id);
    };

    for (int b = blockIdx.x; b < nRows; b += gridDim.x) {
        const int r = rows[b];
        const int s = g.attached[r];
        const int tslot = slots ? slots[b] : -1;
        const double thr = tslot >= 0 ? tie.thr[tslot] : 0.0;
        for (int v = lane; v < n; v += EX_THREADS) index2[v] = 0;   // (LDS: cheap)
        if (lane == 0) {
            place(0, 0.0, s);
            H[s] = 0;
            R[s] = 1.0;
            P[s] = -1;
            if (LF) LF[s] = 0.0;
        }
        __syncthreads();
        int size = tslot >= 0 && thr < 0.0 ? 0 : 1;   // uniform; 0: relevance scan cleared the row
        int toReach = g.T;
        while (size > 0 && toReach > 0) {
            // pop: top known before the sift-down, its arc range loads meanwhile
            const int u = __builtin_amdgcn_readfirstlane(hidx[0]);
            const double mind = -hkey[0];
            if (tslot >= 0 && mind > thr) break;   // early stop (tied preds popped)
            // labels of u were written by lanes of this wave: order their
            // stores, then fetch labels + arc range together (one round trip
            // that overlaps the sift-down)
            __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
            const int a0 = g.rowPtr[u], a1 = g.rowPtr[u + 1];
            const int att = g.isAttached[u];
            const int hu = H[u];
            const double ru = R[u];
            const double lfu = LF ? LF[u] : 0.0;
            size -= 1;
            if (lane == 0) {
                if (size > 0) {
                    const double lk = hkey[size];
                    const int li = hidx[size];
                    const int pos = sink_hole(0, lk, size);
                    place(pos, lk, li);
                }
                index2[u] = 1;
                D[u] = mind;
            }
            if (att) --toReach;
            for (int base = a0; base < a1; base += 64) {
                const int a = base + lane;
                const bool valid = a < a1;
                const int ac = valid ? a : a0;
                const int v = g.col[ac];
                const double w = g.lat[ac];
                const double rw = g.rel[ac];
                const int ia = g.outToIn[ac];
                const int st = valid ? index2[v] : 1;
                const double alt = mind + w;
                int need = 0;
                if (st == 0) need = 1;
                else if (st >= 2) need = (alt < -hkey[st - 2]) ? 2 : 0;
                const int nh = hu + 1;
                const double nr = ru * rw;
                if (need) { P[v] = ia; H[v] = nh; R[v] = nr; }
                if (need && LF) LF[v] = lfu + g.flat[ac];
                unsigned long long mask = __ballot(need != 0);
                while (mask) {
                    const int k = __builtin_ctzll(mask);
                    mask &= mask - 1;
                    const int vk = __builtin_amdgcn_readlane(v, k);
                    const int nk = __builtin_amdgcn_readlane(need, k);
                    const double ak = readlane_f64(alt, k);
                    if (lane == 0) {
                        if (nk == 1) {            // igraph_2wheap_push_with_index
                            shift_up(size, -ak, vk);
                        } else {                  // igraph_2wheap_modify: sink, then shift_up
                            const int pos = index2[vk] - 2;
                            shift_up(sink_hole(pos, -ak, size), -ak, vk);
                        }
                    }
                    size += nk == 1 ? 1 : 0;
                }
            }
        }
        __syncthreads();
        if (tslot >= 0)
            tie_finalize(tie, tslot, n, lane, [&](int v) { return thr >= 0.0 && index2[v] != 0; },
                         [&](int v) { return thr >= 0.0 && index2[v] == 1; }, D, P);
        else
            write_row(g, tab, r, s,
                      [&](int t) { return index2[t] == 1 ? d2b(LF ? LF[t] : D[t]) : INF_BITS; },
                      [&](int t) { return H[t]; }, R, P, F_EXACT, lane, EX_THREADS);
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------
// k_exact_dense: the same igraph 0.7.1 Dijkstra + 2-way heap emulation for
// tie rows of DENSE graphs (mode 3), one 1024-thread workgroup per row.  A
// dense vertex has ~n arcs, so a pop is dominated by the arc scan, which one
// wave (k_exact_rows) walks in dependent 64-arc chunks (~350 us per pop at
// n = 20k).  Here waves 1..15 scan contiguous segments of the popped
// vertex's arcs in parallel (coalesced col / lat / index2 / dist loads; the
// decision for arc k depends only on v_k's own state, as in k_exact_rows)
// while wave 0 sifts the heap down -- the scan reads only categories and
// distances, which a sift-down does not change.  Each scanning wave appends
// its pushes / modifies to a list of its own in incidence order; after a
// barrier wave 0 applies the lists in segment order, i.e. in igraph's
// incidence order, with the wave-parallel WHeap operations.  Same heap array,
// same pop order, same parents as the one-wave kernel.
// ---------------------------------------------------------------------------
constexpr int XD_THREADS = 1024;
constexpr int XD_SCAN_WAVES = XD_THREADS / 64 - 1;

struct alignas(16) XdEntry {
    double alt;      // new tentative distance
    int32_t v;       // vertex
    int32_t st;      // 0: push (never reached), >= 2: modify (index2 at scan time)
};

// slots (round 6): early-stop tie rows of the dense path (k_dense_tie_export
// filled their slots): the emulation stops once the popped key passes the
// slot's threshold and merges its parents into the slot (as k_exact_rows'
// tie_finalize, workgroup-wide); k_tie_write then writes the row.
__global__ __launch_bounds__(XD_THREADS) void k_exact_dense(DevGraph g0, DevTable tab0,
                                                            DevScratch sc0,
                                                            const int32_t* __restrict__ rows,
                                                            int32_t nRows, int32_t hc,
                                                            XdEntry* __restrict__ lists,
                                                            const int32_t* __restrict__ slots,
                                                            TieBuf tie, int32_t* take) {
    const DevGraph g = global_view(g0);
    const DevTable tab = global_view(tab0);
    const DevScratch sc = global_view(sc0);
    const int n = g.n;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const size_t slot = (size_t)blockIdx.x * (size_t)sc.stride;
    double* D = sc.dist + slot;
    int32_t* H = sc.hops + slot;
    double* R = sc.rel + slot;
    int32_t* P = sc.pred + slot;
    double* tailKey = reinterpret_cast<double*>(sc.heapTail) + (size_t)blockIdx.x * 2 * sc.heapStride;
    const WHeap h{tailKey, reinterpret_cast<int32_t*>(tailKey + sc.heapStride), sc.index2 + slot, hc};
    XdEntry* list = as_global(lists) + (size_t)blockIdx.x * (size_t)sc.stride;
    __shared__ int sU, sDone, sSeg, sBad;
    __shared__ double sMind;
    __shared__ int sCnt[XD_SCAN_WAVES];
    const int ldsLevel = 30 - __builtin_clz(hc + 1);
    // rows: static (b = blockIdx.x, + gridDim.x), or taken from a device
    // counter (take, zeroed by the host) when early-stop rows of unequal
    // cost run in one launch
    __shared__ int sB;
    for (int b = blockIdx.x;; b += gridDim.x) {
        if (take) {
            __syncthreads();
            if (tid == 0) sB = atomicAdd(take, 1);
            __syncthreads();
            b = sB;
        }
        if (b >= nRows) break;
        const int r = rows[b];
        const int s = g.attached[r];
        const int tslot = slots ? slots[b] : -1;
        const double thr = tslot >= 0 ? tie.thr[tslot] : 0.0;
        for (int v = tid; v < n; v += XD_THREADS) h.I2[v] = 0;
        __syncthreads();
        if (tid == 0) {
            h.put(0, 0.0, s);
            D[s] = 0.0;
            H[s] = 0;
            R[s] = 1.0;
            P[s] = -1;
        }
        __syncthreads();
        int toReach = g.T;      // wave 0's
        int size = tslot >= 0 && !(thr >= 0.0) ? 0 : 1;   // wave 0's (thr < 0: no relevant tie)
        double km = 0.0;
        int im = 0;
        for (;;) {
            // ---- pop (wave 0): the top, the last element --------------------
            if (wave == 0) {
                int done = size <= 0 || toReach <= 0;
                // early stop: every tied predecessor of the row is popped
                if (!done && tslot >= 0 && -h.lkey()[0] > thr) done = 1;
                if (!done) {
                    const int u = __builtin_amdgcn_readfirstlane(h.lidx()[0]);
                    const double mind = -h.lkey()[0];
                    size -= 1;
                    if (size > 0) h.get(size, km, im);
                    if (lane == 0) {
                        __hip_atomic_store(&h.I2[u], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                        sU = u;
                        sMind = mind;
                        sSeg = (g.rowPtr[u + 1] - g.rowPtr[u] + XD_SCAN_WAVES - 1) / XD_SCAN_WAVES;
                    }
                    if (g.isAttached[u]) --toReach;
                }
                if (lane == 0) sDone = done;
            }
            __syncthreads();
            if (sDone) break;
            const int u = sU;
            const double mind = sMind;
            const int a0 = g.rowPtr[u], a1 = g.rowPtr[u + 1];
            if (wave == 0) {
                // ---- sink (wave 0) while waves 1.. scan ---------------------
                if (size > 0) {
                    int head = 0, hl = 0;
                    bool placed = false;
                    while (!placed) placed = h.sink_round(head, hl, km, im, size, ldsLevel, lane);
                }
            } else {
                // ---- scan: wave w takes arcs [a0 + (w-1) seg, a0 + w seg) -------
                const int seg = sSeg;
                const int lo = a0 + (wave - 1) * seg;
                const int hi = min(a1, lo + seg);
                const int hu = ld_wg(&H[u]);
                const double ru = ld_wg(&R[u]);
                XdEntry* wl = list + (size_t)(wave - 1) * seg;
                int cnt = 0;
                for (int base = lo; base < hi; base += 64) {
                    const int a = base + lane;
                    const bool valid = a < hi;
                    int v = 0, st = 1;
                    double w = 0.0, dv = 0.0;
                    if (valid) {
                        v = g.col[a];
                        w = g.lat[a];
                        st = ld_wg(&h.I2[v]);
                        dv = ld_wg(&D[v]);
                    }
                    const double alt = mind + w;
                    const bool need = valid && (st == 0 || (st >= 2 && alt < dv));
                    if (need) {
                        __hip_atomic_store(&P[v], g.outToIn[a], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                        __hip_atomic_store(&D[v], alt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                        __hip_atomic_store(&H[v], hu + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                        __hip_atomic_store(&R[v], ru * g.rel[a], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    }
                    const unsigned long long m = __ballot(need);
                    if (need) {
                        const int k = cnt + __popcll(m & ((1ull << lane) - 1));
                        wl[k] = XdEntry{alt, v, st};
                    }
                    cnt += __popcll(m);
                }
                if (lane == 0) sCnt[wave - 1] = cnt;
            }
            fence_wg();
            __syncthreads();
            // ---- pushes / modifies in incidence order (wave 0) --------------
            if (wave == 0) {
                const int seg = sSeg;
                for (int w = 0; w < XD_SCAN_WAVES; ++w) {
                    const int cnt = sCnt[w];
                    const XdEntry* wl = list + (size_t)w * seg;
                    for (int c0 = 0; c0 < cnt; c0 += 64) {
                        XdEntry e{0.0, 0, 0};
                        if (c0 + lane < cnt) e = wl[c0 + lane];
                        const int ce = min(64, cnt - c0);
                        for (int k = 0; k < ce; ++k) {
                            const int vk = __builtin_amdgcn_readlane(e.v, k);
                            const int sk = __builtin_amdgcn_readlane(e.st, k);
                            const double ak = readlane_f64(e.alt, k);
                            if (sk == 0) {              // igraph_2wheap_push_with_index
                                h.shift_up(size, -ak, vk, lane);
                                size += 1;
                            } else {                    // igraph_2wheap_modify (sink is a no-op)
                                const int p2 = __builtin_amdgcn_readfirstlane(h.I2[vk]);
                                h.shift_up(p2 - 2, -ak, vk, lane);
                            }
                        }
                    }
                }
            }
        }
        __syncthreads();
        if (tslot >= 0) {
            // tie_finalize, workgroup-wide: the emulated parents of the
            // ambiguous entries, and the popped vertices' distances checked
            // against the slot's (a mismatch: thr := NaN, the engine redoes
            // the row with the full emulation)
            if (tid == 0) sBad = 0;
            __syncthreads();
            int32_t* tp = tie.P + (size_t)tslot * (size_t)tie.n;
            const double* td = tie.D + (size_t)tslot * (size_t)tie.n;
            const bool live = thr >= 0.0;
            int bad = 0;
            for (int v = tid; v < n; v += XD_THREADS) {
                const int fp = tp[v];
                const int st = live ? ld_wg(&h.I2[v]) : 0;
                if (fp >= 0 && (fp & TIE_AMB)) tp[v] = st != 0 ? ld_wg(&P[v]) : -1;
                if (st == 1 && ld_wg(&D[v]) != td[v]) bad = 1;
            }
            if (bad) sBad = 1;
            __syncthreads();
            if (tid == 0 && sBad) tie.thr[tslot] = __longlong_as_double(0x7ff8000000000000ll);
        } else {
            write_row(g, tab, r, s, [&](int t) { return ld_wg(&h.I2[t]) == 1 ? d2b(ld_wg(&D[t])) : INF_BITS; },
                      [&](int t) { return ld_wg(&H[t]); }, R, P, F_EXACT, tid, XD_THREADS);
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------
// k_direct_rows: complete graphs (and prefersDirectPaths pairs): row entry =
// _topology_lookupDirectPath (topology.c:1877-1927).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_direct_rows(DevGraph g0, DevTable tab0,
                                                     const int32_t* __restrict__ rows) {
    const DevGraph g = global_view(g0);
    const DevTable tab = global_view(tab0);
    const int j = blockIdx.x * 256 + threadIdx.x;
    const int r = rows[blockIdx.y];
    if (j >= g.T) return;
    const int s = g.attached[r];
    const int t = g.attached[j];
    double acc = 1.0 * g.vrel[s];
    acc = acc * g.vrel[t];
    double L = 0.0, Rl = acc;
    int h = -1;
    uint8_t f = F_DIRECT;
    if (t == s) {
        if (g.hasSelf[s]) { L = 0.0 + g.selfLat[s]; Rl = acc * g.selfRel[s]; h = 1; }
        else f |= F_NOEDGE;
    } else {
        const int a0 = g.rowPtr[s], a1 = g.rowPtr[s + 1];
        int a = -1;
        if (a1 - a0 == g.n - 1) {
            a = a0 + (t < s ? t : t - 1);
        } else {
            int lo = a0, hi = a1;
            while (lo < hi) {
                const int mid = lo + ((hi - lo) >> 1);
                if (g.col[mid] < t) lo = mid + 1; else hi = mid;
            }
            if (lo < a1 && g.col[lo] == t) a = lo;
        }
        if (a >= 0) { L = 0.0 + (g.flat ? g.flat[a] : g.lat[a]); Rl = acc * g.rel[a]; h = 1; }
        else f |= F_NOEDGE;
    }
    const size_t idx = (size_t)(r - tab.rowStart) * (size_t)tab.T + j;
    tab.lat[idx] = L;
    tab.rel[idx] = Rl;
    tab.hops[idx] = h;
    tab.flags[idx] = f;
    if (tab.pred) tab.pred[idx] = (t == s) ? -1 : s;
}

// ---------------------------------------------------------------------------
int sparse_max_threads() { return SP_THREADS; }

template <int L, int LPV>
static void launch_sparse_lpv(const DevGraph& g, const DevTable& tab, const DevScratch& sc,
                              const int32_t* dRows, int32_t nRows, uint8_t* dRowAmbig,
                              const SparseLaunch& cfg, int32_t* dDbg, const TieBuf* dTie,
                              hipStream_t st, int grid) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_sparse_rows<L, LPV>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, cfg.ldsBytes);
    hipLaunchKernelGGL((k_sparse_rows<L, LPV>), dim3(grid), dim3(cfg.threads), cfg.ldsBytes, st,
                       g, tab, sc, dRows, nRows, dRowAmbig, cfg.delta, cfg.qcap, cfg.hcap,
                       cfg.heavyDeg, dDbg, cfg.kflags, dTie);
}

template <int L>
static void launch_sparse_layout(const DevGraph& g, const DevTable& tab, const DevScratch& sc,
                                 const int32_t* dRows, int32_t nRows, uint8_t* dRowAmbig,
                                 const SparseLaunch& cfg, int32_t* dDbg, const TieBuf* dTie,
                                 hipStream_t st, int grid) {
    if constexpr (L == 3) {
        const int sel = (cfg.kflags >> 4) & 3;
        if (sel == 1)
            return launch_sparse_lpv<L, 2>(g, tab, sc, dRows, nRows, dRowAmbig, cfg, dDbg, dTie, st, grid);
        if (sel == 2)
            return launch_sparse_lpv<L, 1>(g, tab, sc, dRows, nRows, dRowAmbig, cfg, dDbg, dTie, st, grid);
        if (sel == 3)
            return launch_sparse_lpv<L, 8>(g, tab, sc, dRows, nRows, dRowAmbig, cfg, dDbg, dTie, st, grid);
    }
    launch_sparse_lpv<L, 4>(g, tab, sc, dRows, nRows, dRowAmbig, cfg, dDbg, dTie, st, grid);
}

void launch_sparse_rows(const DevGraph& g, const DevTable& tab, const DevScratch& sc,
                        const int32_t* dRows, int32_t nRows, uint8_t* dRowAmbig,
                        const SparseLaunch& cfg, int32_t* dDbg, const TieBuf* dTie,
                        void* stream) {
    if (nRows <= 0) return;
    const int grid = nRows < cfg.grid ? nRows : cfg.grid;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    if (cfg.layout == 3)
        launch_sparse_layout<3>(g, tab, sc, dRows, nRows, dRowAmbig, cfg, dDbg, dTie, st, grid);
    else if (cfg.layout == 2)
        launch_sparse_layout<2>(g, tab, sc, dRows, nRows, dRowAmbig, cfg, dDbg, dTie, st, grid);
    else if (cfg.layout == 1)
        launch_sparse_layout<1>(g, tab, sc, dRows, nRows, dRowAmbig, cfg, dDbg, dTie, st, grid);
    else
        launch_sparse_layout<0>(g, tab, sc, dRows, nRows, dRowAmbig, cfg, dDbg, dTie, st, grid);
}

void launch_tie_scan(const DevGraph& g, const int32_t* dRows, const int32_t* dSlots,
                     int32_t nRows, const TieBuf& tie, void* stream) {
    if (nRows <= 0) return;
    hipLaunchKernelGGL(k_tie_scan, dim3(nRows), dim3(1024), 0,
                       reinterpret_cast<hipStream_t>(stream), g, dRows, dSlots, tie);
}

void launch_tie_write(const DevGraph& g, const DevTable& tab, const int32_t* dRows,
                      const int32_t* dSlots, int32_t nRows, const TieBuf& tie, void* stream) {
    if (nRows <= 0) return;
    hipLaunchKernelGGL(k_tie_write, dim3(nRows), dim3(TW_THREADS), 0,
                       reinterpret_cast<hipStream_t>(stream), g, tab, dRows, dSlots, tie);
}

int exact_soa_max_n() { return EX_SOA_MAXN; }

// LDS bytes of k_exact_rows' preferred-child bits: one bit per 1-based heap
// node 0..n (16-B aligned)
int exact_bits_bytes(int n) { return (int)((((size_t)n + 2 + 31) / 32 * 4 + 15) & ~(size_t)15); }

void launch_exact_rows(const DevGraph& g, const DevTable& tab, const DevScratch& sc,
                       const int32_t* dRows, int32_t nRows, int32_t grid, int32_t hc,
                       bool forceGlobalHeap, const int32_t* dSlots, const TieBuf& tie,
                       long long* dXdbg, void* stream) {
    if (nRows <= 0) return;
    if (grid > nRows) grid = nRows;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    if (g.n <= EX_SOA_MAXN && !forceGlobalHeap) {
        const int sb = (int)(((size_t)16 * g.n + 15) & ~(size_t)15);
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_exact_rows_soa),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, sb);
        hipLaunchKernelGGL(k_exact_rows_soa, dim3(grid), dim3(EX_THREADS), sb, st, g, tab, sc,
                           dRows, nRows, dSlots, tie, dXdbg);
        return;
    }
    // the preferred-child bits follow the heap head when both fit (the
    // engine sizes hc for them, exact_bits_bytes)
    const int head = (int)(((size_t)12 * hc + 15) & ~(size_t)15);
    const int withBits = head + exact_bits_bytes(g.n);
    const bool bits = withBits <= 160 * 1024 - 512;
    const int bytes = bits ? withBits : head;
    auto go = [&](auto kern) {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
        hipLaunchKernelGGL(kern, dim3(grid), dim3(EX_THREADS), bytes, st, g, tab, sc, dRows, nRows, hc,
                           dSlots, tie, dXdbg);
    };
    if (dXdbg) {
        if (bits) go(&k_exact_rows<true, true>);
        else go(&k_exact_rows<true, false>);
    } else {
        if (bits) go(&k_exact_rows<false, true>);
        else go(&k_exact_rows<false, false>);
    }
}

void launch_exact_dense(const DevGraph& g, const DevTable& tab, const DevScratch& sc,
                        const int32_t* dRows, int32_t nRows, int32_t grid, int32_t hc, void* dList,
                        const int32_t* dSlots, const TieBuf& tie, int32_t* dTake, void* stream) {
    if (nRows <= 0) return;
    if (grid > nRows) grid = nRows;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    // (the engine's hc leaves 512 B of LDS for the static shared variables;
    // the heap tail slots are sized for exactly that hc)
    const int bytes = (int)(((size_t)12 * hc + 15) & ~(size_t)15);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_exact_dense),
                              hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    hipLaunchKernelGGL(k_exact_dense, dim3(grid), dim3(XD_THREADS), bytes, st, g, tab, sc, dRows, nRows,
                       hc, reinterpret_cast<XdEntry*>(dList), dSlots, tie, dTake);
}

int exact_dense_list_bytes() { return (int)sizeof(XdEntry); }

void launch_direct_rows(const DevGraph& g, const DevTable& tab, const int32_t* dRows,
                        int32_t nRows, void* stream) {
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const int bx = (g.T + 255) / 256;
    for (int r0 = 0; r0 < nRows; r0 += 65535) {
        const int cnt = (nRows - r0) < 65535 ? (nRows - r0) : 65535;
        hipLaunchKernelGGL(k_direct_rows, dim3(bx, cnt), dim3(256), 0, st, g, tab, dRows + r0);
    }
}

}  // namespace shdpe

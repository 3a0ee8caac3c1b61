// pe_batch.hip -- batched multi-source sparse kernel of the Shadow path
// engine (gfx950).
//
// Reference semantics (Shadow v1.14.0, src/main/routing/topology.c): one
// source row = _topology_computeSourcePaths (:1655-1875) = igraph 0.7.1
// Dijkstra (:1765) + the per-target fold _topology_computePathProperties
// (:1407-1523).  Same contract as k_sparse_rows (pe_kernels.hip); this kernel
// is the layout for graphs whose per-row state does not fit LDS (n of 10^5+).
//
// One workgroup owns a batch of LB sources.  Every per-vertex array is laid
// out [v][LB]: a group of LB lanes handles one vertex for all LB sources
// (lane l = source l), so one arc relaxation dist[u] + w -> dist[v] for LB
// sources is ONE coalesced LB*8-byte access instead of LB random ones.  The
// per-source distance rows (0.8-2 MB each) live in HBM; loaded latency is
// ~1.2 us per dependent access, so every stage keeps several independent
// vertices per group in flight (V-way interleave) and the relaxation phase
// carries no labels at all.  Sources of a batch are chosen close together in
// the graph (host-side BFS rank), so their bucket frontiers coincide.
//
// Per batch:
//   1. label-correcting delta-stepping with a shared bucket bound and
//      double-buffered per-vertex pending lane masks (cur/next); relaxations
//      are dist[u] + w only (left fold -> igraph's distances bit for bit,
//      SURVEY.md Appendix B);
//   2. predecessor pass: tight in-arc with minimum dist[u] per lane = igraph's
//      first-popped tight predecessor; equal minima (or a zero-increment arc)
//      make the row a tie row for k_exact_rows;
//   3. hop counts = depth in the predecessor forest, by pointer jumping
//      (exact integer sums, log2(depth) rounds);
//   4. reliability in depth order: entries bucketed by depth (counting sort
//      in LDS), then level by level R[v] = R[parent] * rel(parent, v) -- the
//      reference's left fold (topology.c:1430, :1499) exactly;
//   5. the row writer (topology.c:1805-1864).
#include <hip/hip_runtime.h>

#include "pe_device.hpp"
#include "pe_devutil.hpp"

namespace shdpe {

constexpr int BT_THREADS = 1024;
constexpr int BK = 4;        // arcs per vertex per load batch
constexpr int BV = 2;        // vertices interleaved per group
constexpr int LMAX = 4096;   // depth levels bucketed in LDS (deeper -> sweeps)

struct alignas(16) BCtrl {
    int qtail;
    int active;
    unsigned long long minNext;
    unsigned int ambMask;
    int changed;
    int maxDepth;
    int pad;
    unsigned long long busyMax;
    unsigned long long busySum;
};

// Forward reliability fold with vertex factors (topology.c:1430-1462, :1499)
// along lane l's predecessor chain, multiplied in source -> target order.
// packed pointer-jumping entry: low word = ancestor J, high word = H
__device__ __forceinline__ int jh_j(unsigned long long w) { return (int)(uint32_t)w; }
__device__ __forceinline__ int jh_h(unsigned long long w) { return (int)(uint32_t)(w >> 32); }
__device__ __forceinline__ void st_jh(unsigned long long* p, int j, int h) {
    const unsigned long long w = (unsigned long long)(uint32_t)j | ((unsigned long long)(uint32_t)h << 32);
    __hip_atomic_store(p, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Wave-aggregated counter add: the lanes of a wave that bump the same
// counter (depth levels: ~20 distinct keys for 10^6 entries) are merged into
// one LDS atomic per distinct key instead of serialising 64 same-address
// atomics.  Returns each participating lane's slot (old value + its rank).
__device__ __forceinline__ int wave_agg_add(int* ctr, int key, bool act) {
    unsigned long long pend = __ballot(act);
    int pos = -1;
    while (pend) {
        const int leader = __ffsll((long long)pend) - 1;
        const int k0 = __shfl(key, leader, 64);
        const bool mine = act && key == k0 && ((pend >> __lane_id()) & 1ull);
        const unsigned long long m = __ballot(mine);
        int base = 0;
        if ((int)__lane_id() == leader) base = atomicAdd(&ctr[k0], __popcll(m));
        base = __shfl(base, leader, 64);
        if (mine)
            pos = base + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                      __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
        pend &= ~m;
    }
    return pos;
}

// Forward reliability fold with vertex factors (topology.c:1430-1462, :1499)
// along lane l's predecessor chain, multiplied in source -> target order:
// the chain is walked in blocks of 64 factors from the source end (O(h)
// loads per block, O(h^2 / 64) in all; no per-thread scratch beyond 64).
template <int LB>
__device__ __noinline__ double fold_rel_batch(const double* __restrict__ vrel,
                                              const double* __restrict__ inRel,
                                              const int32_t* __restrict__ inCol,
                                              const int32_t* P, int l, int s, int t, int h) {
    // (arrays by value: a DevGraph& would pin the caller's descriptor in scratch)
    double acc = 1.0 * vrel[s];
    acc = acc * vrel[t];
    for (int lo = 0; lo < h; lo += 64) {        // hops (lo, hi] counted from the source
        const int hi = min(h, lo + 64);
        int x = t;
        for (int up = 0; up < h - hi; ++up) x = inCol[ld_wg(&P[(size_t)x * LB + l])];
        double fac[64];
        int k = 0;
        while (k < hi - lo) {
            const int a = ld_wg(&P[(size_t)x * LB + l]);
            fac[k++] = inRel[a];
            x = inCol[a];
        }
        for (int i = k - 1; i >= 0; --i) acc = acc * fac[i];
    }
    return acc;
}

template <int LB>
__global__ __launch_bounds__(BT_THREADS) void k_batch_rows(DevGraph g0, DevTable tab0,
                                                           BatchScratch bs,
                                                           const int32_t* __restrict__ batchRows,
                                                           int32_t nBatches, uint8_t* rowAmbig,
                                                           double delta, int32_t* dbg,
                                                           const TieBuf* __restrict__ tieDesc) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    __shared__ int tieSlot[LB];
    __shared__ unsigned long long tieThr[LB];
    const DevGraph g = global_view(g0);
    const DevTable tab = global_view(tab0);
    constexpr unsigned int LBMASK = LB >= 32 ? 0xFFFFFFFFu : ((1u << (LB & 31)) - 1u);
    const int n = g.n;
    const int nw = (n + 31) >> 5;
    const int nwp = (nw + 3) & ~3;
    const int tid = threadIdx.x, NT = blockDim.x;
    const int l = tid % LB;
    const int gid = tid / LB, NG = NT / LB;
    const int gbase = (tid & 63) - l;       // first lane of my group in the wave
    const bool undirected = g.inCol == g.col;
    const size_t NE = (size_t)n * LB;        // (vertex, lane) entries

    BCtrl* ctl = reinterpret_cast<BCtrl*>(smem);
    uint32_t* const any0 = reinterpret_cast<uint32_t*>(smem + 64);
    uint32_t* const any1 = any0 + nwp;
    int32_t* const hist = reinterpret_cast<int32_t*>(any1 + nwp);   // [LMAX + 2]
    int32_t* const cur = hist + (LMAX + 4);                           // [LMAX + 2]

    const size_t slot = blockIdx.x;
    const size_t NS = (size_t)bs.nStride;
    const size_t SE = NS * LB;
    unsigned long long* D = as_global(bs.D + slot * SE);
    double* R = as_global(bs.R + slot * SE);
    int32_t* H = as_global(bs.H + slot * SE);
    int32_t* P = as_global(bs.P + slot * SE);
    int32_t* const X = as_global(bs.X + slot * 4 * SE);
    unsigned long long* JH = reinterpret_cast<unsigned long long*>(X);   // 2 SE words
    int2* LV = reinterpret_cast<int2*>(X + 2 * SE);                     // 2 SE words
    int32_t* Q = as_global(bs.queue + slot * NS);

    for (int b = blockIdx.x; b < nBatches; b += gridDim.x) {
        const int row = batchRows[(size_t)b * LB + l];
        const int src = row >= 0 ? g.attached[row] : -1;
        // ---- init: dist = +inf for all (v, lane); pending sets empty ----
        {
            ulonglong2* D2 = reinterpret_cast<ulonglong2*>(D);
            const size_t cnt2 = NE / 2;
            const ulonglong2 inf2 = make_ulonglong2(INF_BITS, INF_BITS);
            for (size_t i = tid; i < cnt2; i += NT) D2[i] = inf2;
            for (int w = tid; w < nwp; w += NT) { any0[w] = 0u; any1[w] = 0u; }
            if (tid == 0) {
                ctl->qtail = 0;
                ctl->active = 0;
                ctl->minNext = INF_BITS;
                ctl->ambMask = 0u;
                ctl->changed = 0;
                ctl->maxDepth = 0;
                ctl->busyMax = 0;
                ctl->busySum = 0;
            }
        }
        fence_wg();
        __syncthreads();
        if (gid == 0 && src >= 0) {
            D[(size_t)src * LB + l] = d2b(0.0);
            R[(size_t)src * LB + l] = 1.0;
            atomicOr(&any0[src >> 5], 1u << (src & 31));
        }
        fence_wg();
        __syncthreads();

        // ================= 1. delta-stepping over the batch =================
        // Pending state is one bit per VERTEX (LDS): "some lane of u improved".
        // A candidate processes every lane with dist < bound: re-relaxing a
        // lane that did not change costs no memory traffic (the group reads
        // the whole dist[x][0..LB) line anyway) and never improves anything.
        // Lanes at or above the bound keep the vertex pending (deferred);
        // the bound only grows, so such a lane has never been processed at
        // its current value.  Improvements are no-return atomic mins at
        // workgroup scope: the line was just read for the pre-check, so the
        // atomic resolves in L2, and no update is lost.  (Plain stores lost
        // ~1 update per batch to concurrent groups, and the Bellman repair
        // that caught it -- a second relax + predecessor pass -- cost 20% of
        // the relax phase at C4.)  The Bellman check of pass 2 stays as the
        // safety net.
        const long long tPh0 = dbg ? (long long)clock64() : 0;
        long long tPh1 = 0;
        int par = 0, phases = 0, repairs = 0;
        bool failed = false;
        const int phaseCap = 8 * n + 1024;
        long long procs = 0, arcsDone = 0, lanesAct = 0;
        double bound = delta;
        uint32_t ambMask = 0u;
        for (;;) {   // phases + verification until the Bellman check holds
        for (;;) {
            uint32_t* const anyC = par ? any1 : any0;
            uint32_t* const anyN = par ? any0 : any1;
            // candidates = vertices with a pending bit (cur set, consumed)
            for (int w = tid; w < nw; w += NT) {
                uint32_t bits = anyC[w];
                if (bits) {
                    anyC[w] = 0u;
                    int pos = atomicAdd(&ctl->qtail, __popc(bits));
                    while (bits) {
                        const int bb = __ffs(bits) - 1;
                        bits &= bits - 1;
                        Q[pos++] = (w << 5) + bb;
                    }
                }
            }
            fence_wg();
            __syncthreads();
            const int qn = ctl->qtail;
            if (qn == 0) break;
            if (phases > phaseCap) {        // safety net: never spin the GPU
                failed = true;
                break;
            }
            unsigned long long myMin = INF_BITS;
            int myAct = 0;
            const long long tg0 = dbg ? (long long)clock64() : 0;
            // the queue entries of the group's NEXT vertices are loaded one
            // iteration ahead (qn >= 1 here), so a vertex starts with its
            // dist / row-range loads instead of a dependent queue round trip
            int nq[BV];
#pragma unroll
            for (int v = 0; v < BV; ++v) {
                const int idx = gid * BV + v;
                nq[v] = ld_wg(&Q[idx < qn ? idx : qn - 1]);
            }
            for (int i0 = gid * BV; i0 < qn; i0 += NG * BV) {
                int u[BV], a0[BV], a1[BV];
                unsigned long long db[BV], dub[BV];
#pragma unroll
                for (int v = 0; v < BV; ++v) u[v] = i0 + v < qn ? nq[v] : -1;
#pragma unroll
                for (int v = 0; v < BV; ++v) {
                    const int idx = i0 + NG * BV + v;
                    nq[v] = ld_wg(&Q[idx < qn ? idx : qn - 1]);
                }
#pragma unroll
                for (int v = 0; v < BV; ++v) {
                    // branch-free: one round trip for dist[u] and rowPtr[u..u+1]
                    const int uc = u[v] >= 0 ? u[v] : 0;
                    const unsigned long long d0 = ld_wg(&D[(size_t)uc * LB + l]);
                    const int r0 = g.rowPtr[uc], r1 = g.rowPtr[uc + 1];
                    db[v] = u[v] >= 0 ? d0 : INF_BITS;
                    a0[v] = u[v] >= 0 ? r0 : 0;
                    a1[v] = u[v] >= 0 ? r1 : 0;
                }
                int maxd = 0;
#pragma unroll
                for (int v = 0; v < BV; ++v) {
                    const bool act = b2d(db[v]) < bound;
                    const bool defer = !act && db[v] != INF_BITS;
                    const uint32_t amask = (uint32_t)(__ballot(act) >> gbase) & LBMASK;
                    const uint32_t dmask = (uint32_t)(__ballot(defer) >> gbase) & LBMASK;
                    if (l == 0 && dmask) atomicOr(&anyN[u[v] >> 5], 1u << (u[v] & 31));
                    if (defer) myMin = db[v] < myMin ? db[v] : myMin;
                    dub[v] = act ? db[v] : INF_BITS;
                    if (!amask) a1[v] = a0[v];
                    else {
                        ++procs;
                        arcsDone += a1[v] - a0[v];
                        lanesAct += __popc(amask);
                    }
                    maxd = max(maxd, a1[v] - a0[v]);
                }
                // relax u's out-arcs for the lanes below the bound
                for (int t = 0; t < maxd; t += BK) {
                    int xs[BV][BK];
                    double ws[BV][BK];
                    unsigned long long dx[BV][BK];
                    // branch-free: out-of-range slots load arc 0 / vertex 0
                    // and are masked, so all BV*BK loads of a stage are in
                    // flight before the first wait
#pragma unroll
                    for (int v = 0; v < BV; ++v)
#pragma unroll
                        for (int k = 0; k < BK; ++k) {
                            const int a = a0[v] + t + k;
                            const bool ok = a < a1[v];
                            const Arc A = g.arcs[ok ? a : 0];
                            xs[v][k] = ok ? A.col : -1;
                            ws[v][k] = A.lat;
                        }
#pragma unroll
                    for (int v = 0; v < BV; ++v)
#pragma unroll
                        for (int k = 0; k < BK; ++k)
                            dx[v][k] = ld_wg(&D[(size_t)(xs[v][k] >= 0 ? xs[v][k] : 0) * LB + l]);
#pragma unroll
                    for (int v = 0; v < BV; ++v)
#pragma unroll
                        for (int k = 0; k < BK; ++k) {
                            const int x = xs[v][k];
                            bool imp = false;
                            if (x >= 0) {
                                const unsigned long long nb = d2b(b2d(dub[v]) + ws[v][k]);
                                if (nb < dx[v][k]) {
                                    __hip_atomic_fetch_min(&D[(size_t)x * LB + l], nb, __ATOMIC_RELAXED,
                                                           __HIP_MEMORY_SCOPE_WORKGROUP);
                                    imp = true;
                                }
                            }
                            if (__ballot(imp) >> gbase & LBMASK && l == 0) {
                                atomicOr(&anyN[x >> 5], 1u << (x & 31));
                                myAct = 1;
                            }
                        }
                }
            }
            if (dbg && l == 0) {
                const unsigned long long bz = (unsigned long long)((long long)clock64() - tg0);
                atomicMax(&ctl->busyMax, bz);
                atomicAdd(&ctl->busySum, bz);
            }
            if (myMin != INF_BITS) atomicMin(&ctl->minNext, myMin);
            if (myAct) ctl->active = 1;
            fence_wg();
            __syncthreads();
            if (!ctl->active) {
                // no relaxation improved anything: the bucket is settled, jump
                // to the bucket of the smallest deferred distance
                const double mn = b2d(ctl->minNext);
                double nb = (floor(mn / delta) + 1.0) * delta;
                if (!(mn < nb)) nb = mn + delta;
                bound = nb;
            }
            __syncthreads();
            if (tid == 0) {
                ctl->qtail = 0;
                ctl->active = 0;
                ctl->minNext = INF_BITS;
                if (dbg) {
                    dbg[16 * b + 12] += (int)(ctl->busyMax >> 10);
                    dbg[16 * b + 13] += (int)((ctl->busySum / NG) >> 10);
                    dbg[16 * b + 14] += qn;
                    ctl->busyMax = 0;
                    ctl->busySum = 0;
                }
            }
            par ^= 1;
            ++phases;
            __syncthreads();
        }
        if (dbg) tPh1 = (long long)clock64();

        // ================= 2. Bellman check + predecessor pass ===============
        // (a) every entry must satisfy dist[v] <= dist[u] + w for all in-arcs
        //     (a violation = an update lost to a concurrent plain store: fix
        //     it, mark v pending, and go back to phase 1);
        // (b) igraph sets parent[v] from the first POPPED tight predecessor:
        //     the tight in-arc with minimum dist[u]; equal minima from distinct
        //     vertices (or a zero-increment arc) -> the heap decides -> tie
        //     row (k_exact_rows).  Also seeds the pointer jumping: J = parent
        //     vertex (self for roots), depth 1 per tree arc.
        bool amb = false;
        int viol = 0;
        {
            uint32_t* const anyC = par ? any1 : any0;
            for (int v0 = gid * BV; v0 < n; v0 += NG * BV) {
                int a0[BV], a1[BV], ba[BV], cnt[BV], bu[BV];
                unsigned long long dvb[BV], best[BV], mn[BV];
                bool root[BV];
#pragma unroll
                for (int v = 0; v < BV; ++v) {
                    const int vv = v0 + v;
                    if (vv < n) {
                        dvb[v] = ld_wg(&D[(size_t)vv * LB + l]);
                        a0[v] = undirected ? g.rowPtr[vv] : g.inPtr[vv];
                        a1[v] = undirected ? g.rowPtr[vv + 1] : g.inPtr[vv + 1];
                    } else {
                        dvb[v] = INF_BITS;
                        a0[v] = a1[v] = 0;
                    }
                    root[v] = vv == src || src < 0;
                    best[v] = INF_BITS;
                    mn[v] = INF_BITS;
                    cnt[v] = 0;
                    ba[v] = -1;
                    bu[v] = -1;
                }
                int maxd = 0;
#pragma unroll
                for (int v = 0; v < BV; ++v) maxd = max(maxd, a1[v] - a0[v]);
                for (int t = 0; t < maxd; t += BK) {
                    int cu[BV][BK];
                    double lw[BV][BK];
                    unsigned long long du[BV][BK];
#pragma unroll
                    for (int v = 0; v < BV; ++v)
#pragma unroll
                        for (int k = 0; k < BK; ++k) {      // branch-free (see pass 1)
                            const int a = a0[v] + t + k;
                            const bool ok = a < a1[v];
                            const int ac = ok ? a : 0;
                            int c;
                            if (undirected) {
                                const Arc A = g.arcs[ac];
                                c = A.col;
                                lw[v][k] = A.lat;
                            } else {
                                c = g.inCol[ac];
                                lw[v][k] = g.inLat[ac];
                            }
                            cu[v][k] = ok ? c : -1;
                        }
#pragma unroll
                    for (int v = 0; v < BV; ++v)
#pragma unroll
                        for (int k = 0; k < BK; ++k) {
                            const unsigned long long t2 =
                                ld_wg(&D[(size_t)(cu[v][k] >= 0 ? cu[v][k] : 0) * LB + l]);
                            du[v][k] = cu[v][k] >= 0 ? t2 : INF_BITS;
                        }
#pragma unroll
                    for (int v = 0; v < BV; ++v)
#pragma unroll
                        for (int k = 0; k < BK; ++k) {
                            if (cu[v][k] < 0 || root[v]) continue;
                            const double cand = b2d(du[v][k]) + lw[v][k];
                            const unsigned long long cb = d2b(cand);
                            mn[v] = cb < mn[v] ? cb : mn[v];
                            if (dvb[v] != INF_BITS && du[v][k] <= dvb[v] && cand == b2d(dvb[v])) {
                                if (du[v][k] < best[v]) {
                                    best[v] = du[v][k];
                                    cnt[v] = 1;
                                    ba[v] = a0[v] + t + k;
                                    bu[v] = cu[v][k];
                                } else if (du[v][k] == best[v]) {
                                    ++cnt[v];
                                }
                            }
                        }
                }
#pragma unroll
                for (int v = 0; v < BV; ++v) {
                    const int vv = v0 + v;
                    if (vv >= n) continue;
                    const size_t e = (size_t)vv * LB + l;
                    const bool bad = !root[v] && mn[v] < dvb[v];
                    if (bad) {
                        D[e] = mn[v];
                        viol = 1;
                    }
                    const uint32_t bm = (uint32_t)(__ballot(bad) >> gbase) & LBMASK;
                    if (bm && l == 0) atomicOr(&anyC[vv >> 5], 1u << (vv & 31));
                    const bool tree = !root[v] && dvb[v] != INF_BITS && ba[v] >= 0;
                    // an entry whose parent the heap decides: equal minimum
                    // tight predecessors, or the minimum one reaches v by a
                    // zero-increment arc (dist[u] + w == dist[u]: u and v
                    // share a key).  A zero-increment arc from a farther
                    // predecessor cannot win (its relaxation is not strictly
                    // better).  Marked in H (free until the hop counts) for
                    // the tie export below.
                    const bool ea = !root[v] && dvb[v] != INF_BITS &&
                                    (cnt[v] != 1 || best[v] == dvb[v]);
                    amb |= ea;
                    H[e] = ea ? 1 : 0;
                    P[e] = tree ? ba[v] : -1;
                    st_jh(&JH[e], tree ? bu[v] : vv, tree ? 1 : 0);
                }
            }
        }
        if (amb) atomicOr(&ctl->ambMask, 1u << l);
        if (viol) ctl->changed = 1;
        fence_wg();
        __syncthreads();
        const int anyViol = ctl->changed;
        ambMask = ctl->ambMask;
        __syncthreads();
        if (tid == 0) {
            ctl->changed = 0;
            ctl->ambMask = 0u;
        }
        __syncthreads();
        if (!anyViol || failed) break;
        ++repairs;
        }   // verification loop
        // ---- tie export: rows whose parents the igraph heap decides go to
        // k_exact_rows; hand it the final distances, these parents and the
        // ambiguous entries, so it emulates the heap only until the last
        // tied predecessor is popped (tie threshold) ----
        if (ambMask && !failed && tieDesc) {
            // descriptor read from memory here only: as a kernel argument
            // it cost the hot loops registers (SGPR spills)
            const TieBuf tie = *tieDesc;
            if (tid < LB) {
                int sl = -1;
                if ((ambMask >> tid) & 1u) {
                    sl = atomicAdd(tie.count, 1);
                    if (sl >= tie.cap) sl = -1;
                }
                tieSlot[tid] = sl;
                tieThr[tid] = 0ull;
            }
            __syncthreads();
            const int sl = tieSlot[l];
            unsigned long long thr = 0ull;
            for (int v = gid; v < n; v += NG) {
                if (sl < 0) continue;
                const size_t e = (size_t)v * LB + l;
                const int am = ld_wg(&H[e]);
                const size_t o = (size_t)sl * (size_t)tie.n + v;
                tie.D[o] = b2d(ld_wg(&D[e]));
                const int pe = ld_wg(&P[e]);
                tie.P[o] = am ? (TIE_AMB | (pe > 0 ? pe : 0)) : pe;
                if (am) {   // rare: re-derive the tied (minimum tight) predecessor distance
                    const unsigned long long dv = ld_wg(&D[e]);
                    const int a0 = undirected ? g.rowPtr[v] : g.inPtr[v];
                    const int a1 = undirected ? g.rowPtr[v + 1] : g.inPtr[v + 1];
                    unsigned long long mt = INF_BITS;
                    for (int a = a0; a < a1; ++a) {
                        const int u = undirected ? g.col[a] : g.inCol[a];
                        const double w = undirected ? g.lat[a] : g.inLat[a];
                        const unsigned long long du = ld_wg(&D[(size_t)u * LB + l]);
                        if (du <= dv && d2b(b2d(du) + w) == dv && du < mt) mt = du;
                    }
                    if (mt != INF_BITS) thr = mt > thr ? mt : thr;
                }
            }
            if (thr) atomicMax(&tieThr[l], thr);
            fence_wg();
            __syncthreads();
            if (gid == 0 && sl >= 0) tie.thr[sl] = b2d(tieThr[l]);
        } else if (tid < LB) {
            tieSlot[tid] = -1;
        }
        __syncthreads();
        const long long tPh2 = dbg ? (long long)clock64() : 0;

        // ================= 3. hop counts: pointer jumping ====================
        // JH[e] = (J, H) packed in one 8-B word: H = tree distance from v to
        // its ancestor J; roots (and unreached entries) are (v, 0).  Jumping
        // is in place: every read sees SOME consistent pair (single 8-B
        // accesses), each a valid (ancestor, distance), so mixing old and new
        // values only jumps further.  Entries that already point at a root
        // are final and store ~H (negative): later rounds skip them without
        // touching their parent, and children jump straight to the root.
        int rounds = 0;
        for (;;) {
            int ch = 0, dmax = 0;
            for (size_t e0 = (size_t)tid * 4; e0 < NE; e0 += (size_t)NT * 4) {
                unsigned long long p[4], q[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const size_t e = e0 + k;
                    p[k] = e < NE ? ld_wg(&JH[e]) : 0ull;
                }
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const size_t e = e0 + k;
                    const int v = (int)(e / LB), ll = (int)(e % LB);
                    const int j = jh_j(p[k]), h = jh_h(p[k]);
                    const bool live = e < NE && j != v && h >= 0;
                    q[k] = live ? ld_wg(&JH[(size_t)j * LB + ll]) : p[k];
                }
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const size_t e = e0 + k;
                    if (e >= NE) continue;
                    const int v = (int)(e / LB);
                    const int j = jh_j(p[k]), h = jh_h(p[k]);
                    if (j == v) continue;                          // root / unreached
                    if (h < 0) {                                   // final
                        dmax = max(dmax, ~h);
                        continue;
                    }
                    const int jj = jh_j(q[k]), hj = jh_h(q[k]);
                    int nh;
                    if (jj == j) nh = ~h;                          // parent is a root
                    else if (hj < 0) nh = ~(h + ~hj);              // parent final
                    else nh = h + hj;
                    st_jh(&JH[e], jj, nh);
                    ch = 1;
                }
            }
            if (ch) ctl->changed = 1;
            if (dmax) atomicMax(&ctl->maxDepth, dmax);
            fence_wg();
            __syncthreads();
            const int any = ctl->changed;
            __syncthreads();
            if (tid == 0) ctl->changed = 0;
            ++rounds;
            if (!any) break;
            if (tid == 0) ctl->maxDepth = 0;
            __syncthreads();
        }
        const int maxDepth = ctl->maxDepth;
        // unpack the hop counts into H (0 for roots / unreached) and, for the
        // depth-ordered fold, histogram them
        int32_t* const Hc = H;
        if (maxDepth <= LMAX) {
            for (int k = tid; k <= maxDepth + 1; k += NT) hist[k] = 0;
            __syncthreads();
        }
        for (size_t e0 = tid; e0 < NE; e0 += (size_t)NT * 4) {
            int hh[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const size_t e = e0 + (size_t)k * NT;
                hh[k] = e < NE ? jh_h(ld_wg(&JH[e])) : 0;
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const size_t e = e0 + (size_t)k * NT;
                const int d = hh[k] < 0 ? ~hh[k] : 0;
                if (e < NE) Hc[e] = d;
                if (maxDepth <= LMAX) wave_agg_add(hist, d, e < NE && d > 0);
            }
        }
        fence_wg();
        __syncthreads();
        const long long tPh3 = dbg ? (long long)clock64() : 0;

        // ================= 4. reliability in depth order =====================
        if (maxDepth <= LMAX) {
            if (tid < 64) {
                // exclusive scan of hist[1..maxDepth] by one wave
                int carry = 0;
                for (int base = 1; base <= maxDepth; base += 64) {
                    const int k = base + tid;
                    const int x = k <= maxDepth ? hist[k] : 0;
                    int s = x;
#pragma unroll
                    for (int o = 1; o < 64; o <<= 1) {
                        const int y = __shfl_up(s, o, 64);
                        if (tid >= o) s += y;
                    }
                    if (k <= maxDepth) { hist[k] = carry + s - x; cur[k] = carry + s - x; }
                    carry += __shfl(s, 63, 64);
                }
                if (tid == 0) { hist[maxDepth + 1] = carry; cur[maxDepth + 1] = carry; }
            }
            __syncthreads();
            // counting-sort scatter: LV[pos] = (entry, its tree in-arc)
            for (size_t e0 = tid; e0 < NE; e0 += (size_t)NT * 4) {
                int dd[4], aa[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const size_t e = e0 + (size_t)k * NT;
                    dd[k] = e < NE ? ld_wg(&Hc[e]) : 0;
                    aa[k] = e < NE ? ld_wg(&P[e]) : 0;
                }
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const int pos = wave_agg_add(cur, dd[k], dd[k] > 0);
                    if (pos >= 0) LV[pos] = make_int2((int)(e0 + (size_t)k * NT), aa[k]);
                }
            }
            fence_wg();
            __syncthreads();
            // level by level; four entries per thread in flight (the level
            // loop is a chain of dependent gathers, latency-bound otherwise)
            for (int d = 1; d <= maxDepth; ++d) {
                const int q0 = hist[d], q1 = hist[d + 1];
                for (int qb = q0 + tid; qb < q1; qb += NT * 4) {
                    int2 ea[4];
                    int xs[4];
                    double rr[4], rp[4];
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        const int q = qb + k * NT;
                        ea[k] = q < q1 ? LV[q] : make_int2(-1, 0);
                    }
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        const int a = ea[k].x >= 0 ? ea[k].y : 0;
                        xs[k] = g.inCol[a];
                        rr[k] = g.inRel[a];
                    }
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        const int ll = (ea[k].x >= 0 ? ea[k].x : 0) % LB;
                        rp[k] = ld_wg(&R[(size_t)xs[k] * LB + ll]);
                    }
#pragma unroll
                    for (int k = 0; k < 4; ++k)
                        if (ea[k].x >= 0) R[ea[k].x] = rp[k] * rr[k];
                }
                fence_wg();
                __syncthreads();
            }
        } else {
            // very deep trees: Gauss-Seidel sweeps until nothing changes
            for (;;) {
                if (tid == 0) ctl->changed = 0;
                __syncthreads();
                int ch = 0;
                for (size_t e = tid; e < NE; e += NT) {
                    const int a = ld_wg(&P[e]);
                    const int v = (int)(e / LB), ll = (int)(e % LB);
                    if (a < 0 || v == src) continue;
                    const int x = g.inCol[a];
                    const double er = ld_wg(&R[(size_t)x * LB + ll]) * g.inRel[a];
                    if (ld_wg(&R[e]) != er) { R[e] = er; ch = 1; }
                }
                if (ch) ctl->changed = 1;
                fence_wg();
                __syncthreads();
                if (!ctl->changed) break;
                __syncthreads();
            }
        }
        const long long tPh4 = dbg ? (long long)clock64() : 0;
        if (failed) ambMask = LBMASK;     // hand every row to k_exact_rows
        // 0 fast path, 1 full igraph-heap emulation, 2 + slot: early-stop
        // emulation with the exported tie data
        if (gid == 0 && row >= 0)
            rowAmbig[(size_t)b * LB + l] =
                ((ambMask >> l) & 1u) ? (uint8_t)(tieSlot[l] >= 0 ? 2 + tieSlot[l] : 1) : (uint8_t)0;
        if (dbg && tid == 0) {
            dbg[16 * b + 0] = phases;
            dbg[16 * b + 1] = rounds;
            dbg[16 * b + 2] = maxDepth;
            dbg[16 * b + 3] = (int)ambMask;
            dbg[16 * b + 15] = repairs;
            dbg[16 * b + 5] = (int)((tPh1 - tPh0) >> 10);
            dbg[16 * b + 6] = (int)((tPh2 - tPh1) >> 10);
            dbg[16 * b + 7] = (int)((tPh3 - tPh2) >> 10);
            dbg[16 * b + 11] = (int)((tPh4 - tPh3) >> 10);
        }
        if (dbg && l == 0 && procs) {
            atomicAdd(&dbg[16 * b + 4], (int)procs);
            atomicAdd(&dbg[16 * b + 9], (int)(arcsDone >> 4));
            atomicAdd(&dbg[16 * b + 10], (int)lanesAct);
        }

        // ================= 5. row writer (topology.c:1805-1864) ==============
        if (row >= 0 && !((ambMask >> l) & 1u)) {
            const int T = (int)tab.T;
            const size_t base = (size_t)(row - tab.rowStart) * (size_t)tab.T;
            for (int j = gid; j < T; j += NG) {
                const int t = g.attached[j];
                double L = 0.0, Rl = 0.0;
                int h = -1, pv = -1;
                uint8_t f = 0;
                if (t == src) {
                    // 1-vertex igraph path [s]: the fold uses edge (s,s)
                    // (:1469-1488); the destination factor is skipped (:1457)
                    if (g.hasSelf[src]) {
                        L = 0.0 + g.selfLat[src];
                        Rl = (1.0 * g.vrel[src]) * g.selfRel[src];
                        h = 1;
                    } else {
                        f |= F_NOEDGE;
                    }
                } else {
                    const size_t e = (size_t)t * LB + l;
                    const unsigned long long dt = ld_wg(&D[e]);
                    if (dt == INF_BITS) {
                        f |= F_UNREACHABLE;
                    } else {
                        L = b2d(dt);
                        h = ld_wg(&Hc[e]);
                        const int pa = ld_wg(&P[e]);
                        pv = pa >= 0 ? g.inCol[pa] : -1;
                        if (g.vrel[src] == 1.0 && g.vrel[t] == 1.0)
                            Rl = ld_wg(&R[e]);
                        else
                            Rl = fold_rel_batch<LB>(g.vrel, g.inRel, g.inCol, P, l, src, t, h);
                        if (L == 0.0) {                 // topology.c:1848-1852
                            L = 1.0;
                            f |= F_ZEROLAT;
                        }
                    }
                }
                tab.lat[base + j] = L;
                tab.rel[base + j] = Rl;
                tab.hops[base + j] = h;
                tab.flags[base + j] = f;
                if (tab.pred) tab.pred[base + j] = pv;
            }
        }
        fence_wg();
        __syncthreads();
        if (dbg && tid == 0) dbg[16 * b + 8] = (int)(((long long)clock64() - tPh4) >> 10);
    }
}

template <int LB>
static void launch_lb(const DevGraph& g, const DevTable& tab, const BatchScratch& bs,
                      const int32_t* dBatchRows, int32_t nBatches, uint8_t* dRowAmbig,
                      const BatchLaunch& cfg, int32_t* dDbg, const TieBuf* tie, hipStream_t st,
                      int grid) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_batch_rows<LB>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, cfg.ldsBytes);
    hipLaunchKernelGGL(k_batch_rows<LB>, dim3(grid), dim3(cfg.threads), cfg.ldsBytes, st, g, tab,
                       bs, dBatchRows, nBatches, dRowAmbig, cfg.delta, dDbg, tie);
}

int batch_lds_bytes(int n) {
    const int nwp = (((n + 31) >> 5) + 3) & ~3;
    return 64 + 2 * 4 * nwp + 2 * 4 * (LMAX + 4);
}

const void* batch_kernel_ptr(int lb) {
    if (lb == 8) return reinterpret_cast<const void*>(&k_batch_rows<8>);
    if (lb == 32) return reinterpret_cast<const void*>(&k_batch_rows<32>);
    return reinterpret_cast<const void*>(&k_batch_rows<16>);
}

void launch_batch_rows(const DevGraph& g, const DevTable& tab, const BatchScratch& bs,
                       const int32_t* dBatchRows, int32_t nBatches, uint8_t* dRowAmbig,
                       const BatchLaunch& cfg, int32_t* dDbg, const TieBuf* tie, void* stream) {
    if (nBatches <= 0) return;
    const int grid = nBatches < cfg.grid ? nBatches : cfg.grid;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    if (cfg.lb == 8)
        launch_lb<8>(g, tab, bs, dBatchRows, nBatches, dRowAmbig, cfg, dDbg, tie, st, grid);
    else if (cfg.lb == 32)
        launch_lb<32>(g, tab, bs, dBatchRows, nBatches, dRowAmbig, cfg, dDbg, tie, st, grid);
    else
        launch_lb<16>(g, tab, bs, dBatchRows, nBatches, dRowAmbig, cfg, dDbg, tie, st, grid);
}

}  // namespace shdpe

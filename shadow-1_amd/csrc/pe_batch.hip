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
//   1. label-correcting delta-stepping over per-lane keys (dist + the lane's
//      shift: sources of one batch share a nearest hub, and the shift aligns
//      their distances behind it) with one bucket bound, a near and a far
//      pending bitmap (one bit per vertex), and per-ENTRY dirty bits: an entry
//      is relaxed once per value it takes (dirty -> clean by CAS), not once per
//      visit of its vertex; relaxations are dist[u] + w only (left fold ->
//      igraph's distances bit for bit);
//   2. predecessor pass: tight in-arc with minimum dist[u] per lane = igraph's
//      first-popped tight predecessor; equal minima (or a zero-increment arc)
//      mark the entry ambiguous (the row becomes a tie row for k_exact_rows
//      if a target's path meets it);
//   3. labels on demand + the row writer (topology.c:1805-1864): each lane
//      walks its targets' predecessor chains up to the first entry with
//      known labels and unwinds them (hops + 1, rel * r: the reference's left
//      fold, topology.c:1430, :1499, exactly), keeping every label it
//      derives -- only the ~27% of entries on target paths (C4) are touched;
//   4. tie export for rows whose target paths meet an ambiguous entry.
#include <hip/hip_runtime.h>

#include "pe_device.hpp"
#include "pe_devutil.hpp"

namespace shdpe {

constexpr int BT_THREADS = 1024;
constexpr int BK = 3;        // arcs per vertex per load batch (relaxation)
constexpr int BKP = 3;       // in-arcs per vertex per load batch (predecessor pass)
constexpr int PRED_HEAVY = 64;   // predecessor pass: in-degree of a wave-scanned entry
// WPE = waves per SIMD the kernel is compiled for: 4 (128 VGPRs, one
// 1024-thread workgroup per CU, two vertices interleaved per group) or 8
// (64 VGPRs, two workgroups per CU, one vertex per group)
// (experiment knobs for same-box A/B builds, tools/build_variant.sh -D...)
#ifndef SHDPE_W4_BV
#define SHDPE_W4_BV 2
#endif
#ifndef SHDPE_W4_BK
#define SHDPE_W4_BK 3
#endif
template <int WPE> struct BCfg {
    static constexpr int BV = WPE >= 6 ? 1 : SHDPE_W4_BV;   // vertices interleaved per group
    static constexpr int SMAX = WPE >= 6 ? 8 : 16;   // label-walk stack: (entry, arc) pairs per thread
    static constexpr int BKR = WPE >= 6 ? BK : SHDPE_W4_BK;   // dist gathers per vertex in flight
    static constexpr int BKQ = WPE >= 6 ? BKP : SHDPE_W4_BK;
};
constexpr int WALK_BUDGET = 2048;   // walk steps per target before the deep-tree sweeps
// Lane policy of the relaxation: a vertex with ANY dirty lane below the
// bucket bound relaxes ALL its dirty lanes (eager) instead of only those
// below the bound.  The lanes of a batch reach a vertex in different
// buckets; taking the late ones along with the first costs some label-
// correcting re-relaxations but saves whole vertex visits (each visit reads
// one [v][LB] line per arc): C4 schedule simulation (tools/sim) 2.21 -> 1.56
// arc visits per batch, x m_arcs, at a quarter of the bucket width.
constexpr bool EAGER = true;

struct alignas(16) BCtrl {
    int qtail;
    int farAny;       // some vertex waits in the far set
    unsigned long long farMin;   // smallest far key (bits of a non-negative double)
    unsigned int ambMask;
    int changed;
    int htail;        // heavy-vertex list (grows down from the top of the queue)
    int qhead;        // next light-queue entry to take (dynamic distribution)
    unsigned long long busyMax;
    unsigned long long busySum;
    double maxOff;    // largest lane offset of the batch (bits via atomicMax)
    // SHD_PE_DEBUG_COUNTERS only: vertex processings, arcs, active lanes and
    // the relax / predecessor phase timestamps (in LDS, not registers: the
    // relax loop runs at its VGPR cap)
    unsigned int dProcs, dArcs, dLanes;
    unsigned int dWhy;   // SHDPE_DIAG_WHY builds: why the batch's rows left the fast path
    long long t0, t1, t2, t3, t4;
    int pubCnt;          // cooperative relax: near bits this member published this phase
};
static_assert(sizeof(BCtrl) <= 128, "batch control block");
constexpr int BCTRL_BYTES = 128;

// SHDPE_DIAG_WHY (diagnostic builds only, tools/build_variant.sh -D...): per
// batch, the reasons its rows went to the exact kernel, in dbg[16 b + 1]:
// 1 failed, 2 Bellman violation in the on-demand predecessor pass, 4 in the
// full pass, 8 a label walk met an entry without a parent (or the never-spin
// cap), 16 a walk met an ambiguous entry, 32 deep tree (sweeps), 64 the full
// pass ran (attempt 1), 128 the relax kernel flagged the batch (phase cap)
#ifdef SHDPE_DIAG_WHY
#define DIAG_WHY(bit) (why |= (bit))
// the first phase-2 violations of the first batches: entry, stored distance,
// the in-arc minimum that undercuts it (printf; diagnostic builds only)
#define DIAG_VIOL(b, v, lane, dv, mnv, hv)                                                     \
    do {                                                                                    \
        if ((b) < 6 && atomicAdd(&sDiagViol, 1) < 4)                                        \
            printf("[diag] viol batch %d v %d lane %d dist %.17g min %.17g heavy %d attempt %d\n", \
                   (b), (v), (lane), b2d(dv), b2d(mnv), (hv), attempt);                     \
    } while (0)
#else
#define DIAG_WHY(bit) ((void)0)
#define DIAG_VIOL(b, v, lane, dv, mnv, hv) ((void)0)
#endif

// Entry encoding of the [v][LB] distance array: (f64 bits << 1) | dirty.
// Positive doubles have bit 63 clear, so the shift loses nothing and the u64
// order of encodings is the order of distances: an atomic min with a dirty
// encoding of a smaller distance always wins, an equal or larger one never
// changes the entry (an equal distance does not re-dirty a clean entry:
// clean = bit 0 clear is the smaller encoding).  A processor marks the value
// it relaxed clean with a no-return atomic min of e & ~1: if an improvement
// landed in between, its encoding is below e & ~1 and stays, dirty.
__device__ __forceinline__ unsigned long long enc_dirty(unsigned long long bits) { return (bits << 1) | 1ull; }
__device__ __forceinline__ unsigned long long dec(unsigned long long e) { return e >> 1; }
__device__ __forceinline__ bool is_dirty(unsigned long long e) { return (e & 1ull) != 0; }
constexpr unsigned long long INF_ENC = INF_BITS << 1;   // +inf, clean

// (perturbation variants of these three -- plain stores, doubled atomics,
// doubled reads -- are patches under tools/variants/, built by
// tools/build_variant.sh for same-box A/B runs)
// CO = the cooperative relax (PART 3): several workgroups of one XCD share
// the batch's dist array, so its loads are agent scope (past this CU's L1,
// served by the XCD's L2, where a partner's plain stores land and from which
// its memory-side atomics evict the line).  A stale L1 copy would be harmful
// only in one way -- a vertex listed from a partner's near bit, read clean
// or with an older dirty value, relaxed (or skipped) and marked clean while
// the partner's newer value, whose near bit was just consumed, is never
// relaxed -- but it must not happen at all.
template <bool CO = false>
__device__ __forceinline__ unsigned long long ld_d(unsigned long long* p) {
    if constexpr (CO)
        return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else
        return ld_wg(p);
}

template <bool CO = false>
__device__ __forceinline__ void relax_min(unsigned long long* p, unsigned long long v) {
    __hip_atomic_fetch_min(p, v, __ATOMIC_RELAXED, CO ? __HIP_MEMORY_SCOPE_AGENT : __HIP_MEMORY_SCOPE_WORKGROUP);
}

// relax pre-check load
template <bool CO = false>
__device__ __forceinline__ unsigned long long relax_ld(unsigned long long* D, int x, int LB, int l) {
    return ld_d<CO>(&D[(size_t)x * LB + l]);
}

template <bool CO = false>
__device__ __forceinline__ void mark_clean(unsigned long long* p, unsigned long long e) {
    __hip_atomic_fetch_min(p, e & ~1ull, __ATOMIC_RELAXED, CO ? __HIP_MEMORY_SCOPE_AGENT : __HIP_MEMORY_SCOPE_WORKGROUP);
}

// ---- cooperative relax: group formation and the group barrier ----------
// A launch of PART 3 is cooperative (hipLaunchCooperativeKernel: every
// workgroup resident).  Each workgroup registers on its XCD (HW_REG_XCC_ID)
// and waits until all have; the workgroups of one XCD then form groups of K
// (the last one of an XCD may be smaller), so a group's members always share
// the XCD's L2 -- whatever the dispatcher's placement.  Every poll loop
// gives up after bs.coSpin polls and sets the launch's abort word; every
// workgroup that sees it returns at once, and the host recomputes the round
// with the plain relax (never a wrong or a missing row).
__device__ __forceinline__ int co_ld(int* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void co_abort(const BatchScratch& bs) {
    __hip_atomic_store(&bs.coCtl[17], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// lane 0 of a workgroup: out = {group, member, group size, groups}; 0 = abort
__device__ int co_register(const BatchScratch& bs, int* out) {
    unsigned x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
    x &= 15u;
    const int K = bs.coK;
    const int r = __hip_atomic_fetch_add(&bs.coCtl[x], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_fetch_add(&bs.coCtl[16], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (int spin = 0; co_ld(&bs.coCtl[16]) < (int)gridDim.x; ++spin) {
        if (spin > bs.coSpin || co_ld(&bs.coCtl[17])) {
            co_abort(bs);
            return 0;
        }
        __builtin_amdgcn_s_sleep(1);
    }
    int base = 0, total = 0;
    for (int y = 0; y < 16; ++y) {
        const int ng = (co_ld(&bs.coCtl[y]) + K - 1) / K;
        base += y < (int)x ? ng : 0;
        total += ng;
    }
    const int c = co_ld(&bs.coCtl[x]);
    out[0] = base + r / K;
    out[1] = r % K;
    out[2] = min(K, c - (r / K) * K);
    out[3] = total;
    return 1;
}

// group barrier: every wave's memory operations complete, one arrival per
// member on the group's counter, a poll until all K arrived for this epoch;
// false = abort (the poll ran too long, or another workgroup aborted)
__device__ __forceinline__ bool co_barrier(const BatchScratch& bs, int* bar, int K, int& epoch, int* sOk) {
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    ++epoch;
    if (threadIdx.x == 0) {
        __hip_atomic_fetch_add(bar, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int target = epoch * K;
        int ok = 1;
        for (int spin = 0; co_ld(bar) < target; ++spin) {
            if (spin > bs.coSpin || co_ld(&bs.coCtl[17])) {
                ok = 0;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        if (ok && co_ld(&bs.coCtl[17])) ok = 0;
        if (!ok) co_abort(bs);
        *sOk = ok;
    }
    __syncthreads();
    return __builtin_amdgcn_readfirstlane(*sOk) != 0;
}

// Pending bitmaps (one bit per vertex, near + far sets): in LDS when both
// fit beside the control block (n <= ~655k), else in the slot's global
// scratch (GB): same operations at workgroup scope.
template <bool GB> struct Bits;
template <> struct Bits<false> {
    uint32_t* p;
    __device__ __forceinline__ uint32_t ld(int w) const { return p[w]; }
    __device__ __forceinline__ void st(int w, uint32_t v) const { p[w] = v; }
    __device__ __forceinline__ void set(int v) const { atomicOr(&p[v >> 5], 1u << (v & 31)); }
    // sets the bit, returns whether it was set before
    __device__ __forceinline__ bool test_set(int v) const {
        return (atomicOr(&p[v >> 5], 1u << (v & 31)) >> (v & 31)) & 1u;
    }
};
template <> struct Bits<true> {
    uint32_t* p;
    __device__ __forceinline__ uint32_t ld(int w) const { return ld_wg(&p[w]); }
    __device__ __forceinline__ void st(int w, uint32_t v) const {
        __hip_atomic_store(&p[w], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    __device__ __forceinline__ void set(int v) const {
        __hip_atomic_fetch_or(&p[v >> 5], 1u << (v & 31), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    __device__ __forceinline__ bool test_set(int v) const {
        return (__hip_atomic_fetch_or(&p[v >> 5], 1u << (v & 31), __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_WORKGROUP) >> (v & 31)) & 1u;
    }
};

// Wave-aggregated append of `val` (lanes with `want`) to a list whose tail
// counter lives in LDS: one LDS atomic per wave.
__device__ __forceinline__ void wave_append(int32_t* Q, int* tail, bool want, int val) {
    const uint64_t m = __ballot(want);
    if (!m) return;
    const int lane = (int)(threadIdx.x & 63);
    const int leader = __ffsll((unsigned long long)m) - 1;
    int base = 0;
    if (lane == leader) base = atomicAdd(tail, __popcll(m));
    base = __shfl(base, leader, 64);
    if (want) __hip_atomic_store(&Q[base + __popcll(m & ((1ull << lane) - 1))], val, __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_WORKGROUP);
}

// bucket of a key: the smallest multiple of delta above it
__device__ __forceinline__ double next_bound(double mn, double delta) {
    double nb = (floor(mn / delta) + 1.0) * delta;
    if (!(mn < nb)) nb = mn + delta;
    return nb;
}

// workgroup-uniform values read from LDS, pinned to scalar registers (the
// relax loop runs at its VGPR cap)
__device__ __forceinline__ int uni(int x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ double uni(double x) {
    const long long b = __double_as_longlong(x);
    const unsigned lo = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)b);
    const unsigned hi = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)(b >> 32));
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

__device__ __forceinline__ void st_wg(int32_t* p, int v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void st_wg(double* p, double v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void st_wg(unsigned long long* p, unsigned long long v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// label records (BLabel): two 8-B halves of one 16-B slot, loaded / stored
// with relaxed workgroup-scope accesses (walks of other groups race on them:
// a half-written record reads as unresolved -- hop label -1 or rel < 0 --
// and the reader walks on, as the labels are written once with the only
// value the fold can give)
struct Lbl {
    double rel;
    int hops, arc;
};
__device__ __forceinline__ Lbl lbl_ld(BLabel* p) {
    const unsigned long long x = ld_wg(&p->ha);
    return Lbl{ld_wg(&p->rel), (int)(unsigned)x, (int)(unsigned)(x >> 32)};
}
__device__ __forceinline__ int lbl_arc(BLabel* p) { return (int)(unsigned)(ld_wg(&p->ha) >> 32); }
__device__ __forceinline__ void lbl_st(BLabel* p, double rel, int hops, int arc) {
    st_wg(&p->rel, rel);
    st_wg(&p->ha, (unsigned long long)(unsigned)hops | ((unsigned long long)(unsigned)arc << 32));
}
__device__ __forceinline__ bool lbl_known(const Lbl& x) { return x.hops >= 0 && x.rel >= 0.0; }

// Forward reliability fold with vertex factors (topology.c:1430-1462, :1499)
// along lane l's predecessor chain, multiplied in source -> target order:
// the chain is walked in blocks of 64 factors from the source end (O(h)
// loads per block, O(h^2 / 64) in all; no per-thread scratch beyond 64).
template <int LB>
__device__ __noinline__ double fold_rel_batch(const double* __restrict__ vrel,
                                              const double* __restrict__ inRel,
                                              const int32_t* __restrict__ inCol,
                                              BLabel* LBL, int l, int s, int t, int h) {
    // (arrays by value: a DevGraph& would pin the caller's descriptor in scratch)
    double acc = 1.0 * vrel[s];
    acc = acc * vrel[t];
    for (int lo = 0; lo < h; lo += 64) {        // hops (lo, hi] counted from the source
        const int hi = min(h, lo + 64);
        int x = t;
        for (int up = 0; up < h - hi; ++up) x = inCol[lbl_arc(&LBL[(size_t)x * LB + l]) & ~TIE_AMB];
        double fac[64];
        int k = 0;
        while (k < hi - lo) {
            const int a = lbl_arc(&LBL[(size_t)x * LB + l]) & ~TIE_AMB;
            fac[k++] = inRel[a];
            x = inCol[a];
        }
        for (int i = k - 1; i >= 0; --i) acc = acc * fac[i];
    }
    return acc;
}

// PART 0: the whole batch in one kernel (relax, predecessors over every
// vertex, labels + writer, tie export).  PART 1 / 2: the same split in two
// kernels over a round of batches whose dist arrays persist in HBM between
// them (slot = batch index): PART 1 relaxes, PART 2 derives predecessors ON
// DEMAND (only vertices on some target's path in some lane; the full pass only
// for tie rows and trees too deep for the walks), labels, rows and the tie
// export -- each with its own register budget.
template <int LB, int WPE, bool GB, int PART>
__global__ __launch_bounds__(BT_THREADS) __attribute__((amdgpu_waves_per_eu(WPE)))
void k_batch_rows(DevGraph g0, DevTable tab0,
                                                           BatchScratch bs,
                                                           const int32_t* __restrict__ batchRows,
                                                           int32_t nBatches, uint8_t* rowAmbig,
                                                           double delta, int32_t* dbg,
                                                           const TieBuf* __restrict__ tieDesc) {
    // PART 3: the relax (PART 1) shared by K workgroups per batch -- its own
    // instantiation, so the plain relax keeps its code and register budget
    constexpr bool CO = PART == 3;
    constexpr int PT = CO ? 1 : PART;
    constexpr int BV = BCfg<WPE>::BV;
    constexpr int SMAX = BCfg<WPE>::SMAX;
    // the light-vertex relax loop and the predecessor pass are software-
    // pipelined three takes deep with lane-distributed arc records (round 5:
    // C4 N=1 106 -> 98.4 ms, N=8 shards 19.4 -> 18.9 ms same box, r05f;
    // profiles/r05_ab_notes.txt); BKR / BKQ = dist gathers per vertex in flight
    constexpr int BKR = BCfg<WPE>::BKR, BKQ = BCfg<WPE>::BKQ;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    __shared__ int tieSlot[LB];
    __shared__ int laneRow[LB];           // table row of each lane (-1: pad)
    __shared__ unsigned long long tieThr[LB];
    const DevGraph g = global_view(g0);
    const DevTable tab = global_view(tab0);
    constexpr unsigned int LBMASK = LB >= 32 ? 0xFFFFFFFFu : ((1u << (LB & 31)) - 1u);
    const int n = g.n;
    const int nw = (n + 31) >> 5;
    const int nwp = (nw + 3) & ~3;
    // the workgroup size is part of the variant (launch_lb checks it): a
    // compile-time NT makes every stride, group count and LDS tile offset a
    // constant instead of a live register (round 6: fewer spills in the
    // post kernels' loops)
    constexpr int NT = WPE == 6 ? 768 : BT_THREADS;
    const int tid = threadIdx.x;
    const int l = tid % LB;
    const int gid = tid / LB, NG = NT / LB;
    const int gbase = (tid & 63) - l;       // first lane of my group in the wave
    const bool undirected = g.inCol == g.col;
    const size_t NE = (size_t)n * LB;        // (vertex, lane) entries

    BCtrl* ctl = reinterpret_cast<BCtrl*>(smem);
    uint32_t* const bits0 = GB ? as_global(bs.bits) + (size_t)blockIdx.x * 2 * nwp
                               : reinterpret_cast<uint32_t*>(smem + BCTRL_BYTES);
    const Bits<GB> any0{bits0}, any1{bits0 + nwp};

    const size_t slot = blockIdx.x;
    const size_t NS = (size_t)bs.nStride;
    const size_t SE = NS * LB;
    unsigned long long* D = as_global(bs.D + slot * SE);
    BLabel* LBL = as_global(bs.L + slot * SE);
    int32_t* Q = as_global(bs.queue + slot * NS);

    // cooperative relax: this workgroup's group (same XCD), member index and
    // group size; batches are assigned statically, group by group
    int coGroup = 0, coMember = 0, coK = 1, coNG = 1, coEpoch = 0, coPP = 0, coIter = 0;
    int* coBar = nullptr;
    __shared__ int sCo[5];
    if constexpr (CO) {
        if (tid == 0) sCo[4] = co_register(bs, sCo);
        __syncthreads();
        if (!__builtin_amdgcn_readfirstlane(sCo[4])) return;        // abort: the host reruns the round
        coGroup = __builtin_amdgcn_readfirstlane(sCo[0]);
        coMember = __builtin_amdgcn_readfirstlane(sCo[1]);
        coK = __builtin_amdgcn_readfirstlane(sCo[2]);
        coNG = __builtin_amdgcn_readfirstlane(sCo[3]);
        coBar = as_global(bs.coBars) + (size_t)coGroup * 32;
    }

    // batches are taken from a device counter (dynamic: a batch's cost varies
    // by ~20%, and a workgroup finishing early takes the next one)
    __shared__ int nextB;
    for (;;) {
        if (tid == 0) nextB = CO ? coGroup + (coIter++) * coNG : atomicAdd(bs.next, 1);
        __syncthreads();
        const int b = nextB;
        if (b >= nBatches) break;
        const int row = batchRows[(size_t)b * LB + l];
        const int src = row >= 0 ? g.attached[row] : -1;
        if (gid == 0) laneRow[l] = row;
        if constexpr (PT != 0) D = as_global(bs.D + (size_t)b * SE);
        // ---- init: dist = +inf (clean) for all (v, lane); pending sets empty ----
        {
            ulonglong2* D2 = reinterpret_cast<ulonglong2*>(D);
            const size_t cnt2 = NE / 2;
            const ulonglong2 inf2 = make_ulonglong2(INF_ENC, INF_ENC);
            if constexpr (PT != 2) {
                // (cooperative: each member its slice of the shared array)
                const size_t i0 = cnt2 * coMember / coK, i1 = cnt2 * (coMember + 1) / coK;
                for (size_t i = i0 + tid; i < i1; i += NT) D2[i] = inf2;
            }
            for (int w = tid; w < nwp; w += NT) { any0.st(w, 0u); any1.st(w, 0u); }
            if (tid == 0) {
                ctl->qtail = 0;
                ctl->qhead = 0;
                ctl->farAny = 0;
                ctl->farMin = INF_BITS;
                ctl->ambMask = 0u;
                ctl->changed = 0;
                ctl->htail = 0;
                ctl->busyMax = 0;
                ctl->busySum = 0;
                ctl->maxOff = 0.0;
                ctl->dProcs = ctl->dArcs = ctl->dLanes = 0u;
                ctl->dWhy = 0u;
                ctl->pubCnt = 0;
            }
        }
        fence_wg();
        __syncthreads();
        if constexpr (CO)      // every member's slice is +inf before any source entry
            if (!co_barrier(bs, coBar, coK, coEpoch, &sCo[4])) return;
        // lane offset: the source's distance to its nearest hub (host plan);
        // key = dist + (maxOff - off) lines the lanes up behind the hub
        const double off = (row >= 0 && bs.rowOff) ? as_global(bs.rowOff)[row] : 0.0;
        if (gid == 0) atomicMax(reinterpret_cast<unsigned long long*>(&ctl->maxOff), d2b(off));
        if (PT != 2 && gid == 0 && src >= 0 && coMember == 0) {
            D[(size_t)src * LB + l] = enc_dirty(d2b(0.0));
            any0.set(src);
        }
        fence_wg();
        __syncthreads();
        const double sh = uni(ctl->maxOff) - off;      // >= 0: keys are non-negative

        // ================= 1. delta-stepping over the batch =================
        // Pending state is one bit per VERTEX (LDS) in two sets: NEAR (some
        // lane of u has a dirty value below the bound) and FAR (a dirty value
        // at or above it).  A phase lists and clears the near set and
        // processes each listed vertex: its dirty lanes below the bound are
        // marked clean (CAS on the value read) and relaxed, its dirty lanes
        // at or above the bound send it to the far set.  Clean lanes are
        // never re-relaxed (their value already reached every out-neighbour),
        // so a vertex costs arc traffic only when a lane has a new value.
        // When the near set is empty the bound moves to the bucket of the
        // smallest far key and the far set becomes the near set.
        // Improvements are no-return atomic mins at workgroup scope on the
        // encoding (the line was just read for the pre-check, so the atomic
        // resolves in L2, and no update is lost).  The Bellman check of pass
        // 2 stays as the safety net.
        if (dbg && tid == 0) ctl->t0 = (long long)clock64();
        int par = 0, phases = 0, repairs = 0;
        bool failed = false;
        const int phaseCap = 8 * n + 1024;
        double bound = delta;
        unsigned long long myFar = INF_BITS;      // smallest far key this thread added
        if constexpr (PT == 2) failed = as_global(bs.flags)[b] != 0;
#ifdef SHDPE_DIAG_WHY
        uint32_t why = failed ? 128u : 0u;
        __shared__ int sDiagViol;
        if (tid == 0) sDiagViol = 0;
        __syncthreads();
#endif
        uint32_t needMask = 0u;
        bool lastFull = true;     // the final attempt ran the full predecessor pass
        for (int attempt = 0;; ++attempt) {
        const bool fullPred = PT != 2 || attempt > 0;
        if (attempt > 0) DIAG_WHY(64u);
        if (attempt > 0) {
            if (tid == 0) {
                ctl->qtail = 0;
                ctl->changed = 0;
                ctl->ambMask = 0u;
            }
            fence_wg();
            __syncthreads();
        }
        for (;;) {   // phases + verification until the Bellman check holds
        if constexpr (PT != 2) {
        for (;;) {
            if (failed) break;
            const Bits<GB> anyC = par ? any1 : any0;   // near
            const Bits<GB> anyF = par ? any0 : any1;   // far
            // cooperative relax: each member publishes its near bits (set by
            // its own relaxations) and its far state, and after the group
            // barrier lists the group's union of near bits for the words it
            // owns (w = member mod K); the bucket advance and the end follow
            // the group's totals, so every member takes the same decisions
            uint32_t* coPn = nullptr;
            int coNear = 0, coFar = 0;
            unsigned long long coFmin = INF_BITS;
            if constexpr (CO) {
                if (myFar != INF_BITS) {
                    atomicMin(&ctl->farMin, myFar);
                    myFar = INF_BITS;
                }
                coPP ^= 1;      // two buffers: a member publishing phase p + 1 never
                                // overwrites what a partner still reads of phase p
                coPn = as_global(bs.coPub) + ((size_t)coGroup * 2 + coPP) * (size_t)bs.coK * nwp;
                unsigned long long* const ps =
                    as_global(bs.coPubS) + ((size_t)coGroup * 2 + coPP) * (size_t)bs.coK * 2;
                int cnt = 0;
                for (int w = tid; w < nw; w += NT) {
                    const uint32_t bits = anyC.ld(w);
                    __hip_atomic_store(&coPn[(size_t)coMember * nwp + w], bits, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
                    if (bits) {
                        anyC.st(w, 0u);
                        cnt += __popc(bits);
                    }
                }
                if (cnt) atomicAdd(&ctl->pubCnt, cnt);
                fence_wg();
                __syncthreads();
                if (tid == 0) {
                    __hip_atomic_store(&ps[coMember * 2],
                                       (unsigned long long)(unsigned)ctl->pubCnt |
                                           ((unsigned long long)(ctl->farAny != 0) << 32),
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    __hip_atomic_store(&ps[coMember * 2 + 1], ctl->farMin, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
                    ctl->pubCnt = 0;
                }
                if (!co_barrier(bs, coBar, coK, coEpoch, &sCo[4])) return;
                for (int k = 0; k < coK; ++k) {
                    const unsigned long long a =
                        __hip_atomic_load(&ps[k * 2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    const unsigned long long f =
                        __hip_atomic_load(&ps[k * 2 + 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    coNear |= (a & 0xFFFFFFFFull) != 0;
                    coFar |= (int)(a >> 32);
                    coFmin = f < coFmin ? f : coFmin;
                }
                coNear = uni(coNear);
                coFar = uni(coFar);
                coFmin = d2b(uni(b2d(coFmin)));
            }
            // candidates = vertices with a near bit (consumed)
            // (hubs -- degree >= the engine's heavy threshold -- go to a list
            // of their own, processed by whole waves: one 16-lane group on a
            // hub's ~1000 arcs would set the phase's length)
            for (int w = CO ? coMember + tid * coK : tid; w < nw; w += CO ? NT * coK : NT) {
                uint32_t bits = 0u;
                if constexpr (CO) {
                    for (int k = 0; k < coK; ++k)
                        bits |= __hip_atomic_load(&coPn[(size_t)k * nwp + w], __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_AGENT);
                } else {
                    bits = anyC.ld(w);
                }
                if (bits) {
                    if constexpr (!CO) anyC.st(w, 0u);
                    uint32_t hv = bits & g.heavyBits[w];
                    bits &= ~hv;
                    if (bits) {
                        int pos = atomicAdd(&ctl->qtail, __popc(bits));
                        while (bits) {
                            const int bb = __ffs(bits) - 1;
                            bits &= bits - 1;
                            Q[pos++] = (w << 5) + bb;
                        }
                    }
                    if (hv) {
                        int pos = atomicAdd(&ctl->htail, __popc(hv));
                        while (hv) {
                            const int bb = __ffs(hv) - 1;
                            hv &= hv - 1;
                            Q[NS - 1 - pos++] = (w << 5) + bb;
                        }
                    }
                }
            }
            if (myFar != INF_BITS) {
                atomicMin(&ctl->farMin, myFar);
                myFar = INF_BITS;
            }
            fence_wg();
            __syncthreads();
            const int qn = uni(ctl->qtail);
            const int hn = uni(ctl->htail);
            if (CO ? !coNear : qn == 0 && hn == 0) {
                // bucket settled: advance to the far set, or done
                const int farAny = CO ? coFar : uni(ctl->farAny);
                const double fm = CO ? b2d(coFmin) : uni(b2d(ctl->farMin));
                __syncthreads();
                if (!farAny) break;
                bound = uni(fm < b2d(INF_BITS) ? next_bound(fm, delta) : b2d(INF_BITS));
                if (tid == 0) {
                    ctl->farAny = 0;
                    ctl->farMin = INF_BITS;
                }
                par ^= 1;
                ++phases;
                __syncthreads();
                continue;
            }
            if (phases > phaseCap) {        // safety net: never spin the GPU
                failed = true;
                break;
            }
            int farAdd = 0;
            const long long tg0 = dbg ? (long long)clock64() : 0;
            // hubs first (their improvements reach the light vertices in this
            // phase): one wave per hub, its 64 / LB groups interleave the arcs
            {
                constexpr int GPW = 64 / LB;
                const int wv = tid >> 6, NW = NT >> 6, gw = (tid & 63) / LB;
                for (int h = wv; h < hn; h += NW) {
                    const int u = ld_wg(&Q[NS - 1 - h]);
                    unsigned long long* const pu = &D[(size_t)u * LB + l];
                    const unsigned long long e0 = ld_d<CO>(pu);
                    const int a0 = g.rowPtr[u], a1 = g.rowPtr[u + 1];
                    const double k0 = b2d(dec(e0)) + sh;
                    const bool dirty = is_dirty(e0);
                    const bool below = dirty && k0 < bound;
                    const bool act = EAGER ? dirty && __ballot(below) >> gbase & LBMASK : below;
                    const bool defer = dirty && !act;
                    const uint32_t amask = (uint32_t)(__ballot(act) >> gbase) & LBMASK;
                    const uint32_t dmask = (uint32_t)(__ballot(defer) >> gbase) & LBMASK;
                    if (gw == 0 && l == 0 && dmask) anyF.set(u);
                    if (gw == 0 && defer) {
                        myFar = d2b(k0) < myFar ? d2b(k0) : myFar;
                        farAdd = 1;
                    }
                    if (gw == 0 && act) mark_clean<CO>(pu, e0);
                    const unsigned long long dub1 = act ? dec(e0) : INF_BITS;
                    if (!__ballot(amask != 0)) continue;       // wave-uniform
                    if (dbg && gw == 0 && l == 0) {
                        atomicAdd(&ctl->dProcs, 1u);
                        atomicAdd(&ctl->dArcs, (unsigned int)(a1 - a0));
                        atomicAdd(&ctl->dLanes, (unsigned int)__popc(amask));
                    }
                    for (int t = a0 + gw * BK; t < a1; t += GPW * BK) {
                        int xs[BK];
                        double ws[BK];
                        unsigned long long dx[BK];
#pragma unroll
                        for (int k = 0; k < BK; ++k) {
                            const int a = t + k;
                            const bool ok = a < a1;
                            const Arc A = g.arcs[ok ? a : 0];
                            xs[k] = ok ? A.col : -1;
                            ws[k] = A.lat;
                        }
#pragma unroll
                        for (int k = 0; k < BK; ++k)
                            dx[k] = relax_ld<CO>(D, xs[k] >= 0 ? xs[k] : 0, LB, l);
#pragma unroll
                        for (int k = 0; k < BK; ++k) {
                            const int x = xs[k];
                            bool impN = false, impF = false;
                            if (x >= 0) {
                                const double nd = b2d(dub1) + ws[k];
                                const unsigned long long nb = d2b(nd);
                                if (nb < dec(dx[k])) {
                                    relax_min<CO>(&D[(size_t)x * LB + l], enc_dirty(nb));
                                    const double kx = nd + sh;
                                    impN = kx < bound;
                                    impF = !impN;
                                    if (impF) myFar = d2b(kx) < myFar ? d2b(kx) : myFar;
                                }
                            }
                            const uint64_t bn = __ballot(impN), bf = __ballot(impF);
                            if (l == 0) {
                                if ((bn >> gbase) & LBMASK) anyC.set(x);
                                if ((bf >> gbase) & LBMASK) {
                                    anyF.set(x);
                                    farAdd = 1;
                                }
                            }
                        }
                    }
                }
            }
            // Groups take BV queue entries at a time from an LDS counter, so
            // the phase ends when the last entry is done rather than when the
            // unluckiest static share is.  A value loaded ahead may be stale;
            // like any racing read it is only ever larger (entries decrease):
            // relaxing from it is wasted work, and its clean mark (atomic min)
            // leaves a newer dirty value dirty for the next listing round.
            const int qc = qn > 0 ? qn - 1 : 0;
            auto take = [&]() {
                int i = 0;
                if (l == 0) i = atomicAdd(&ctl->qhead, BV);
                return __shfl(i, gbase, 64);
            };
            // A three-stage software pipeline over the group's takes (BV
            // vertices each).  The group's lanes hold ONE arc record per
            // vertex (lane l: arc a0 + l of the vertex's first LB arcs --
            // one coalesced LB x 16-B read per group instead of BK
            // broadcast records per round and a dependent record round
            // trip before every dist gather); the relaxing lanes take the
            // heads by cross-lane reads.  Per take the group issues the
            // records of the next take, the dist lines + row ranges of the
            // one after, and the queue entries of the third, then relaxes
            // the current vertices: their chain is the BKR-wide dist
            // gathers only.  An entry past the queue end is u = -1 (takes
            // rise monotonically, so a take whose first entry is -1 ends).
            auto q_at = [&](int i) { return i < qn ? ld_wg(&Q[min(i, qc)]) : -1; };
            auto ld_head = [&](int uu, unsigned long long& d, int& r0, int& r1) {
                const int uc = uu >= 0 ? uu : 0;
                const unsigned long long d0 = ld_d<CO>(&D[(size_t)uc * LB + l]);
                const int x0 = g.rowPtr[uc], x1 = g.rowPtr[uc + 1];
                d = uu >= 0 ? d0 : INF_ENC;
                r0 = uu >= 0 ? x0 : 0;
                r1 = uu >= 0 ? x1 : 0;
            };
            auto ld_arc = [&](int a, int aEnd, int& c, double& w) {
                const bool ok = a < aEnd;
                const Arc A = g.arcs[ok ? a : 0];
                c = ok ? A.col : -1;
                w = A.lat;
            };
            int uC[BV], u1[BV], u2[BV], a0C[BV], a1C[BV], a01[BV], a11[BV], mcC[BV];
            unsigned long long dbC[BV], db1[BV];
            double mlC[BV];
            {
                const int i0 = take(), i1 = take(), i2 = take();
#pragma unroll
                for (int v = 0; v < BV; ++v) {
                    uC[v] = q_at(i0 + v);
                    u1[v] = q_at(i1 + v);
                    u2[v] = q_at(i2 + v);
                }
            }
#pragma unroll
            for (int v = 0; v < BV; ++v) {
                ld_head(uC[v], dbC[v], a0C[v], a1C[v]);
                ld_head(u1[v], db1[v], a01[v], a11[v]);
            }
#pragma unroll
            for (int v = 0; v < BV; ++v) ld_arc(a0C[v] + l, a1C[v], mcC[v], mlC[v]);
            while (uC[0] >= 0) {
                int mc1[BV], a02[BV], a12[BV], u3[BV];
                double ml1[BV];
                unsigned long long db2[BV];
#pragma unroll
                for (int v = 0; v < BV; ++v) ld_arc(a01[v] + l, a11[v], mc1[v], ml1[v]);
#pragma unroll
                for (int v = 0; v < BV; ++v) ld_head(u2[v], db2[v], a02[v], a12[v]);
                {
                    const int i3 = take();
#pragma unroll
                    for (int v = 0; v < BV; ++v) u3[v] = q_at(i3 + v);
                }
                unsigned long long dub[BV];
                int deg[BV], maxd = 0;
#pragma unroll
                for (int v = 0; v < BV; ++v) {
                    const double k0 = b2d(dec(dbC[v])) + sh;
                    const bool dirty = is_dirty(dbC[v]);
                    const bool below = dirty && k0 < bound;
                    const bool act = EAGER ? dirty && __ballot(below) >> gbase & LBMASK : below;
                    const bool defer = dirty && !act;
                    const uint32_t amask = (uint32_t)(__ballot(act) >> gbase) & LBMASK;
                    const uint32_t dmask = (uint32_t)(__ballot(defer) >> gbase) & LBMASK;
                    if (l == 0 && dmask) anyF.set(uC[v]);
                    if (defer) {
                        myFar = d2b(k0) < myFar ? d2b(k0) : myFar;
                        farAdd = 1;
                    }
                    if (act) mark_clean<CO>(&D[(size_t)uC[v] * LB + l], dbC[v]);
                    dub[v] = act ? dec(dbC[v]) : INF_BITS;
                    deg[v] = amask ? a1C[v] - a0C[v] : 0;          // group-uniform
                    if (amask && dbg && l == 0) {
                        atomicAdd(&ctl->dProcs, 1u);
                        atomicAdd(&ctl->dArcs, (unsigned int)deg[v]);
                        atomicAdd(&ctl->dLanes, (unsigned int)__popc(amask));
                    }
                    maxd = max(maxd, deg[v]);
                }
                // relax the out-arcs for the dirty lanes below the bound
                for (int c0 = 0; c0 < maxd; c0 += LB) {
                    int mc[BV];
                    double ml[BV];
#pragma unroll
                    for (int v = 0; v < BV; ++v) {
                        mc[v] = mcC[v];
                        ml[v] = mlC[v];
                        if (c0 > 0) ld_arc(a0C[v] + c0 + l, a0C[v] + deg[v], mc[v], ml[v]);   // degree > LB
                    }
                    const int cn = min(LB, maxd - c0);
                    for (int t = 0; t < cn; t += BKR) {
                        int xs[BV][BKR];
                        double ws[BV][BKR];
                        unsigned long long dx[BV][BKR];
#pragma unroll
                        for (int v = 0; v < BV; ++v)
#pragma unroll
                            for (int k = 0; k < BKR; ++k) {
                                const int srcL = gbase + min(t + k, LB - 1);   // inside the group
                                const int c = __shfl(mc[v], srcL, 64);
                                ws[v][k] = __shfl(ml[v], srcL, 64);
                                xs[v][k] = t + k < cn && c0 + t + k < deg[v] ? c : -1;   // (the chunk's own records)
                            }
#pragma unroll
                        for (int v = 0; v < BV; ++v)
#pragma unroll
                            for (int k = 0; k < BKR; ++k)
                                dx[v][k] = relax_ld<CO>(D, xs[v][k] >= 0 ? xs[v][k] : 0, LB, l);
#pragma unroll
                        for (int v = 0; v < BV; ++v)
#pragma unroll
                            for (int k = 0; k < BKR; ++k) {
                                const int x = xs[v][k];
                                bool impN = false, impF = false;
                                if (x >= 0) {
                                    const double nd = b2d(dub[v]) + ws[v][k];
                                    const unsigned long long nb = d2b(nd);
                                    if (nb < dec(dx[v][k])) {
                                        relax_min<CO>(&D[(size_t)x * LB + l], enc_dirty(nb));
                                        const double kx = nd + sh;
                                        impN = kx < bound;
                                        impF = !impN;
                                        if (impF) myFar = d2b(kx) < myFar ? d2b(kx) : myFar;
                                    }
                                }
                                const uint64_t bn = __ballot(impN), bf = __ballot(impF);
                                if (l == 0) {
                                    if ((bn >> gbase) & LBMASK) anyC.set(x);
                                    if ((bf >> gbase) & LBMASK) {
                                        anyF.set(x);
                                        farAdd = 1;
                                    }
                                }
                            }
                    }
                }
#pragma unroll
                for (int v = 0; v < BV; ++v) {
                    uC[v] = u1[v]; dbC[v] = db1[v]; a0C[v] = a01[v]; a1C[v] = a11[v];
                    mcC[v] = mc1[v]; mlC[v] = ml1[v];
                    u1[v] = u2[v]; db1[v] = db2[v]; a01[v] = a02[v]; a11[v] = a12[v];
                    u2[v] = u3[v];
                }
            }
            if (dbg && l == 0) {
                const unsigned long long bz = (unsigned long long)((long long)clock64() - tg0);
                atomicMax(&ctl->busyMax, bz);
                atomicAdd(&ctl->busySum, bz);
            }
            if (farAdd) ctl->farAny = 1;
            fence_wg();
            __syncthreads();
            if (tid == 0) {
                ctl->qtail = 0;
                ctl->qhead = 0;
                ctl->htail = 0;
                if (dbg) {
                    atomicAdd(&dbg[16 * b + 12], (int)(ctl->busyMax >> 10));
                    atomicAdd(&dbg[16 * b + 13], (int)((ctl->busySum / NG) >> 10));
                    atomicAdd(&dbg[16 * b + 14], qn);
                    ctl->busyMax = 0;
                    ctl->busySum = 0;
                }
            }
            ++phases;
            __syncthreads();
        }
        }   // PT != 2
        if (dbg && tid == 0) ctl->t1 = (long long)clock64();
        if constexpr (PT == 1) break;

        // ================= 2. Bellman check + predecessor pass ===============
        // (a) every entry must satisfy dist[v] <= dist[u] + w for all in-arcs
        //     (a violation = an update lost to a concurrent plain store: fix
        //     it, mark v pending, and go back to phase 1);
        // (b) igraph sets parent[v] from the first POPPED tight predecessor:
        //     the tight in-arc with minimum dist[u]; equal minima from distinct
        //     vertices (or a zero-increment arc) -> the heap decides -> tie
        //     row (k_exact_rows) if such an entry lies on a target's path.
        int viol = 0;
        {
            const Bits<GB> anyC = par ? any1 : any0;
            // on demand: vertices are claimed in the (empty) far bitmap and
            // listed in Q, targets first, then round by round the tree
            // parents of the last round's entries in every lane
            const Bits<GB> clm = par ? any0 : any1;
            // entries of in-degree >= PRED_HEAVY are set aside per round and
            // scanned by a whole wave each (its groups split the in-arcs and
            // combine by cross-group shuffles): one group on a hub's ~1000
            // in-arcs would set the round's length.  List in the LDS beyond
            // the bitmaps (free until the label walks), capped by that room.
            int* const heavyList = reinterpret_cast<int*>(smem + BCTRL_BYTES + (GB ? 0 : 8 * nwp));
            const int stackB = NT * SMAX * 8, bitsB = GB ? 0 : 8 * nwp;
            const int hcap = min(4096, max(0, stackB - bitsB) / 4);
            int lo = 0, hi = n;
            if (!fullPred) {
                for (int j = tid; j < g.T; j += NT) {
                    const int v = g.attached[j];
                    wave_append(Q, &ctl->qtail, !clm.test_set(v), v);
                }
                fence_wg();
                __syncthreads();
                hi = uni(ctl->qtail);
                __syncthreads();
            }
            while (lo < hi) {
            // the relax loop's three-stage pipeline (BV list entries per
            // group and stride): the group's lanes hold one in-arc record
            // per entry (lane l: in-arc a0 + l, one coalesced read), the
            // scan takes the tails by cross-lane reads, so an entry's
            // chain is its BKQ-wide dist gathers.  Records of the next
            // stride, dist lines + in-arc ranges of the one after, list
            // entries of the third are in flight meanwhile.
            const int S = NG * BV;
            auto item = [&](int i) { return i < hi ? (fullPred ? i : ld_wg(&Q[i])) : -1; };
            auto ld_head = [&](int vv, unsigned long long& d, int& r0, int& r1) {
                const int vc = vv >= 0 ? vv : 0;
                const unsigned long long d0 = dec(ld_wg(&D[(size_t)vc * LB + l]));
                const int x0 = undirected ? g.rowPtr[vc] : g.inPtr[vc];
                const int x1 = undirected ? g.rowPtr[vc + 1] : g.inPtr[vc + 1];
                d = vv >= 0 ? d0 : INF_BITS;
                r0 = vv >= 0 ? x0 : 0;
                r1 = vv >= 0 ? x1 : 0;
            };
            auto ld_rec = [&](int a, int aEnd, int& c, double& w) {
                const bool ok = a < aEnd;
                const int ac = ok ? a : 0;
                if (undirected) {
                    const Arc A = g.arcs[ac];
                    c = A.col;
                    w = A.lat;
                } else {
                    c = g.inCol[ac];
                    w = g.inLat[ac];
                }
                c = ok ? c : -1;
            };
            int v0 = lo + gid * BV;
            int vC[BV], v1[BV], v2[BV], a0C[BV], a1C[BV], a01[BV], a11[BV], mcC[BV];
            unsigned long long dC[BV], d1[BV];
            double mlC[BV];
#pragma unroll
            for (int v = 0; v < BV; ++v) {
                vC[v] = item(v0 + v);
                v1[v] = item(v0 + S + v);
                v2[v] = item(v0 + 2 * S + v);
            }
#pragma unroll
            for (int v = 0; v < BV; ++v) {
                ld_head(vC[v], dC[v], a0C[v], a1C[v]);
                ld_head(v1[v], d1[v], a01[v], a11[v]);
            }
#pragma unroll
            for (int v = 0; v < BV; ++v) ld_rec(a0C[v] + l, a1C[v], mcC[v], mlC[v]);
            for (; v0 < hi; v0 += S) {
                int mc1[BV], a02[BV], a12[BV], v3[BV];
                double ml1[BV];
                unsigned long long d2[BV];
#pragma unroll
                for (int v = 0; v < BV; ++v) ld_rec(a01[v] + l, a11[v], mc1[v], ml1[v]);
#pragma unroll
                for (int v = 0; v < BV; ++v) ld_head(v2[v], d2[v], a02[v], a12[v]);
#pragma unroll
                for (int v = 0; v < BV; ++v) v3[v] = item(v0 + 3 * S + v);
                bool root[BV], hvy[BV];
                unsigned long long best[BV], mn[BV];
                int cnt[BV], ba[BV], bu[BV], deg[BV], maxd = 0;
#pragma unroll
                for (int v = 0; v < BV; ++v) {
                    root[v] = vC[v] == src || src < 0;
                    best[v] = INF_BITS;
                    mn[v] = INF_BITS;
                    cnt[v] = 0;
                    ba[v] = -1;
                    bu[v] = -1;
                    deg[v] = vC[v] >= 0 ? a1C[v] - a0C[v] : 0;   // group-uniform
                    hvy[v] = false;
                    if (deg[v] >= PRED_HEAVY) {                   // -> the round's wave pass
                        int slot = 0;
                        if (l == 0) slot = atomicAdd(&ctl->htail, 1);
                        slot = __shfl(slot, gbase, 64);
                        if (slot < hcap) {
                            if (l == 0) heavyList[slot] = vC[v];
                            hvy[v] = true;
                            deg[v] = 0;
                        }
                    }
                    maxd = max(maxd, deg[v]);
                }
                for (int c0 = 0; c0 < maxd; c0 += LB) {
                    int mc[BV];
                    double ml[BV];
#pragma unroll
                    for (int v = 0; v < BV; ++v) {
                        mc[v] = mcC[v];
                        ml[v] = mlC[v];
                        if (c0 > 0) ld_rec(a0C[v] + c0 + l, a0C[v] + deg[v], mc[v], ml[v]);
                    }
                    const int cn = min(LB, maxd - c0);
                    for (int t = 0; t < cn; t += BKQ) {
                        int cu[BV][BKQ];
                        double lw[BV][BKQ];
                        unsigned long long du[BV][BKQ];
#pragma unroll
                        for (int v = 0; v < BV; ++v)
#pragma unroll
                            for (int k = 0; k < BKQ; ++k) {
                                const int srcL = gbase + min(t + k, LB - 1);
                                const int c = __shfl(mc[v], srcL, 64);
                                lw[v][k] = __shfl(ml[v], srcL, 64);
                                cu[v][k] = t + k < cn && c0 + t + k < deg[v] ? c : -1;   // (a repeat would count as a tie)
                            }
#pragma unroll
                        for (int v = 0; v < BV; ++v)
#pragma unroll
                            for (int k = 0; k < BKQ; ++k) {
                                const unsigned long long t2 =
                                    dec(ld_wg(&D[(size_t)(cu[v][k] >= 0 ? cu[v][k] : 0) * LB + l]));
                                du[v][k] = cu[v][k] >= 0 ? t2 : INF_BITS;
                            }
#pragma unroll
                        for (int v = 0; v < BV; ++v)
#pragma unroll
                            for (int k = 0; k < BKQ; ++k) {
                                if (cu[v][k] < 0 || root[v]) continue;
                                const double cand = b2d(du[v][k]) + lw[v][k];
                                const unsigned long long cb = d2b(cand);
                                mn[v] = cb < mn[v] ? cb : mn[v];
                                if (dC[v] != INF_BITS && du[v][k] <= dC[v] && cand == b2d(dC[v])) {
                                    if (du[v][k] < best[v]) {
                                        best[v] = du[v][k];
                                        cnt[v] = 1;
                                        ba[v] = a0C[v] + c0 + t + k;
                                        bu[v] = cu[v][k];
                                    } else if (du[v][k] == best[v]) {
                                        ++cnt[v];
                                    }
                                }
                            }
                    }
                }
#pragma unroll
                for (int v = 0; v < BV; ++v) {
                    const int vv = vC[v];
                    if (vv < 0 || hvy[v]) continue;
                    const size_t e = (size_t)vv * LB + l;
                    const bool bad = !root[v] && mn[v] < dC[v];
                    if (bad) {
                        D[e] = enc_dirty(mn[v]);
                        viol = 1;
                        DIAG_VIOL(b, vv, l, dC[v], mn[v], 0);
                    }
                    const uint32_t bm = (uint32_t)(__ballot(bad) >> gbase) & LBMASK;
                    if (bm && l == 0) anyC.set(vv);
                    const bool tree = !root[v] && dC[v] != INF_BITS && ba[v] >= 0;
                    // ambiguous (see the generic loop below)
                    const bool ea = !root[v] && dC[v] != INF_BITS && (cnt[v] != 1 || best[v] == dC[v]);
                    const int hx = tree ? ba[v] : -1;
                    const bool isSrc = vv == src;
                    lbl_st(&LBL[e], isSrc ? 1.0 : -1.0, isSrc ? 0 : -1,
                           ea ? (TIE_AMB | (hx > 0 ? hx : 0)) : hx);
                    if (!tree) bu[v] = -1;
                }
                if (!fullPred) {
#pragma unroll
                    for (int v = 0; v < BV; ++v) {
                        const int p = vC[v] >= 0 && !hvy[v] ? bu[v] : -1;
                        wave_append(Q, &ctl->qtail, p >= 0 && !clm.test_set(p), p);
                    }
                }
#pragma unroll
                for (int v = 0; v < BV; ++v) {
                    vC[v] = v1[v]; dC[v] = d1[v]; a0C[v] = a01[v]; a1C[v] = a11[v];
                    mcC[v] = mc1[v]; mlC[v] = ml1[v];
                    v1[v] = v2[v]; d1[v] = d2[v]; a01[v] = a02[v]; a11[v] = a12[v];
                    v2[v] = v3[v];
                }
            }
            {
                // the round's heavy entries, one wave each
                fence_wg();
                __syncthreads();
                const int nh = min(uni(ctl->htail), hcap);
                constexpr int GPW = 64 / LB;
                const int wv = tid >> 6, NW = NT >> 6, gw = (tid & 63) / LB;
                for (int h = wv; h < nh; h += NW) {
                    const int vv = __builtin_amdgcn_readfirstlane(ld_wg(&heavyList[h]));
                    const unsigned long long dv = dec(ld_wg(&D[(size_t)vv * LB + l]));
                    const int a0 = undirected ? g.rowPtr[vv] : g.inPtr[vv];
                    const int a1 = undirected ? g.rowPtr[vv + 1] : g.inPtr[vv + 1];
                    const int deg = a1 - a0;
                    const bool root = vv == src || src < 0;
                    unsigned long long best = INF_BITS, mn = INF_BITS;
                    int cnt = 0, ba = -1, bu = -1;
                    for (int c0 = gw * LB; c0 < deg; c0 += GPW * LB) {
                        int mc;
                        double ml;
                        {
                            const int a = a0 + c0 + l;
                            const bool ok = a < a1;
                            const int ac = ok ? a : 0;
                            if (undirected) {
                                const Arc A = g.arcs[ac];
                                mc = A.col;
                                ml = A.lat;
                            } else {
                                mc = g.inCol[ac];
                                ml = g.inLat[ac];
                            }
                            mc = ok ? mc : -1;
                        }
                        const int cn = min(LB, deg - c0);
                        for (int t = 0; t < cn; t += BKQ) {
                            int cu[BKQ];
                            double lw[BKQ];
                            unsigned long long du[BKQ];
#pragma unroll
                            for (int k = 0; k < BKQ; ++k) {
                                const int srcL = gbase + min(t + k, LB - 1);
                                const int c = __shfl(mc, srcL, 64);
                                lw[k] = __shfl(ml, srcL, 64);
                                cu[k] = t + k < cn ? c : -1;
                            }
#pragma unroll
                            for (int k = 0; k < BKQ; ++k) {
                                const unsigned long long t2 =
                                    dec(ld_wg(&D[(size_t)(cu[k] >= 0 ? cu[k] : 0) * LB + l]));
                                du[k] = cu[k] >= 0 ? t2 : INF_BITS;
                            }
#pragma unroll
                            for (int k = 0; k < BKQ; ++k) {
                                if (cu[k] < 0 || root) continue;
                                const double cand = b2d(du[k]) + lw[k];
                                const unsigned long long cb = d2b(cand);
                                mn = cb < mn ? cb : mn;
                                if (dv != INF_BITS && du[k] <= dv && cand == b2d(dv)) {
                                    if (du[k] < best) {
                                        best = du[k];
                                        cnt = 1;
                                        ba = a0 + c0 + t + k;
                                        bu = cu[k];
                                    } else if (du[k] == best) {
                                        ++cnt;
                                    }
                                }
                            }
                        }
                    }
                    // combine the groups' scans (lane l of every group holds
                    // source l): counts of equal minima add up, so an entry is
                    // ambiguous exactly as after one sequential scan
                    for (int o = LB; o < 64; o <<= 1) {
                        const unsigned long long ob = __shfl_xor(best, o, 64), om = __shfl_xor(mn, o, 64);
                        const int oc = __shfl_xor(cnt, o, 64), oa = __shfl_xor(ba, o, 64), ou = __shfl_xor(bu, o, 64);
                        mn = om < mn ? om : mn;
                        if (ob < best) {
                            best = ob; cnt = oc; ba = oa; bu = ou;
                        } else if (ob == best && ob != INF_BITS) {
                            cnt += oc;
                            if (oa >= 0 && (ba < 0 || oa < ba)) { ba = oa; bu = ou; }
                        }
                    }
                    const size_t e = (size_t)vv * LB + l;
                    const bool bad = !root && mn < dv;
                    if (bad && gw == 0) {
                        D[e] = enc_dirty(mn);
                        viol = 1;
                        DIAG_VIOL(b, vv, l, dv, mn, 1);
                    }
                    const uint32_t bm = (uint32_t)(__ballot(bad) >> gbase) & LBMASK;
                    if (bm && l == 0 && gw == 0) anyC.set(vv);
                    const bool tree = !root && dv != INF_BITS && ba >= 0;
                    const bool ea = !root && dv != INF_BITS && (cnt != 1 || best == dv);
                    const int hx = tree ? ba : -1;
                    if (gw == 0) {
                        const bool isSrc = vv == src;
                        lbl_st(&LBL[e], isSrc ? 1.0 : -1.0, isSrc ? 0 : -1,
                               ea ? (TIE_AMB | (hx > 0 ? hx : 0)) : hx);
                    }
                    if (!fullPred) {
                        const int p = tree ? bu : -1;
                        wave_append(Q, &ctl->qtail, gw == 0 && p >= 0 && !clm.test_set(p), p);
                    }
                }
                fence_wg();
                __syncthreads();
                if (tid == 0) ctl->htail = 0;   // (every thread read it before the barrier)
            }
            if (fullPred) break;
            fence_wg();
            __syncthreads();
            lo = hi;
            hi = uni(ctl->qtail);
            __syncthreads();
            }
            if (!fullPred) {
                for (int w = tid; w < nwp; w += NT) clm.st(w, 0u);
                if (tid == 0) ctl->qtail = 0;
            }
        }
        if (viol) ctl->changed = 1;
        if (viol) DIAG_WHY(attempt ? 4u : 2u);
        fence_wg();
        __syncthreads();
        const int anyViol = uni(ctl->changed);
        __syncthreads();
        if (tid == 0) {
            ctl->changed = 0;
            ctl->ambMask = 0u;
        }
        __syncthreads();
        if (!anyViol || failed) break;
        if constexpr (PT == 2) {   // no relaxation here to repair with: exact path
            failed = true;
            break;
        }
        ++repairs;
        }   // verification loop
        if constexpr (PT == 1) {
            if (tid == 0 && coMember == 0) as_global(bs.flags)[b] = failed ? 1 : 0;
            break;
        }
        if (dbg && tid == 0) ctl->t2 = (long long)clock64();

        // ================= 3. labels on demand + row writer ==================
        // Only entries on some target's path need hops and reliability (27%
        // of the entries at C4).  Each lane resolves a target by walking its
        // predecessor chain up to the first entry with known labels (at the
        // latest the source: hops 0, rel 1) and unwinding the walk:
        // hops[x] = hops[p] + 1, rel[x] = rel[p] * r(p, x) -- the reference's
        // left fold (topology.c:1430, :1499) in path order, exactly.  Unwound
        // entries keep their labels for later walks of the same lane; each
        // label is written once with the only value the fold can give, so a
        // racing reader sees a complete pair (H >= 0 and R >= 0) or an
        // unresolved entry and walks on.  The walk stack holds SMAX
        // (entry, arc) pairs per thread in LDS (the relax bitmaps are dead);
        // a longer chain is resolved from the top, SMAX levels at a time.
        // An ambiguous entry (TIE_AMB) on a walked chain makes the row a tie
        // row; ambiguous entries off every target path never matter.  Very
        // deep trees (a walk over WALK_BUDGET steps: restarts cost
        // O(depth^2 / SMAX)) switch to Gauss-Seidel sweeps over all entries
        // and a second writer pass.
        // latency floor: the lane's own source must sit at distance exactly 0
        // in the array its row is written from (latencies are > 0, so only
        // the source is) -- an array that is not this lane's sends the row to
        // the exact kernel, never to the table
        uint32_t relAmb = row >= 0 && dec(ld_wg(&D[(size_t)(src >= 0 ? src : 0) * LB + l])) != 0ull ? 1u : 0u;
        bool retry = false;
        for (int pass = 0; pass < 2; ++pass) {
        bool deep = false;
        if (!failed && row >= 0) {
            int2* const stk = reinterpret_cast<int2*>(smem + BCTRL_BYTES);
            const int T = (int)tab.T;
            // pass 0: the deep-tree budget; pass 1: only the never-spin net
            // (every consistent entry is resolved by then)
            // (32-bit: the [v][LB] entry indices below are 32-bit already)
            const int stepCap = pass == 0 ? WALK_BUDGET : 4 * n + 64;
            for (int j = gid; j < T; j += NG) {
                const int t = g.attached[j];
                if (t != src) {
                    const size_t e = (size_t)t * LB + l;
                    const unsigned long long dt = dec(ld_wg(&D[(size_t)t * LB + l]));
                    if (dt != INF_BITS) {
                        // one record per step: an entry's record holds its
                        // parent arc, the parent's record its labels and the
                        // next arc up
                        Lbl cr = lbl_ld(&LBL[e]);
                        int steps = 0;
                        int cur = (int)e;
                        while (!lbl_known(cr)) {
                            int sp = 0, x = cur, hp = 0;
                            Lbl xr = cr;
                            double rp = 0.0;
                            bool found = false;
                            while (sp < SMAX) {
                                const int a = xr.arc;
                                if (a < 0 || ++steps > stepCap) {
                                    if (a >= 0 && pass == 0) deep = true;   // -> sweeps
                                    else { relAmb = 1u; DIAG_WHY(8u); }   // no parent / a cycle: exact path
                                    sp = 0;
                                    found = true;
                                    break;
                                }
                                relAmb |= (uint32_t)((a & TIE_AMB) != 0);
                                if (a & TIE_AMB) DIAG_WHY(16u);
                                stk[sp * NT + tid] = make_int2(x, a);
                                ++sp;
                                const int pe = g.inCol[a & ~TIE_AMB] * LB + l;
                                const Lbl pr = lbl_ld(&LBL[pe]);
                                if (lbl_known(pr)) {
                                    hp = pr.hops;
                                    rp = pr.rel;
                                    found = true;
                                    break;
                                }
                                x = pe;
                                xr = pr;
                            }
                            if (!found) {           // chain longer than SMAX: its top first
                                cur = x;
                                cr = xr;
                                continue;
                            }
                            for (int i = sp - 1; i >= 0; --i) {
                                const int2 sx = stk[i * NT + tid];
                                hp += 1;
                                rp = rp * g.inRel[sx.y & ~TIE_AMB];
                                lbl_st(&LBL[sx.x], rp, hp, sx.y);
                            }
                            if (sp == 0) break;     // gave up (deep / inconsistent)
                            if (cur == (int)e) break;
                            cur = (int)e;           // top segment resolved: walk again
                            cr = lbl_ld(&LBL[e]);
                        }
                    }
                }
            }
        }
        if (deep) ctl->changed = 1;
        if (deep) DIAG_WHY(32u);
        fence_wg();
        __syncthreads();
        const int anyDeep = uni(ctl->changed);
        __syncthreads();
        if (tid == 0) ctl->changed = 0;
        __syncthreads();
        if (!anyDeep) break;
        if (!fullPred) {         // the sweeps read every entry's parent
            retry = true;
            break;
        }
        // Gauss-Seidel: every tree entry whose parent has labels takes them
        // (+1, * r) until a sweep changes nothing (<= depth sweeps).  These
        // entries were not walked, so an ambiguous one sends its row to the
        // exact path (conservative).  Cycles of zero-increment parents stay
        // unresolved and the second pass's walks flag them.
        for (int sweep = 0; sweep <= n + 1; ++sweep) {
            int ch = 0;
            for (size_t e = tid; e < NE; e += NT) {
                const Lbl er = lbl_ld(&LBL[e]);
                const int a = er.arc;
                if (a < 0) continue;
                const int ll = (int)(e % LB);
                const int arc = a & ~TIE_AMB;
                const int pe = g.inCol[arc] * LB + ll;
                const Lbl pr = lbl_ld(&LBL[pe]);
                if (!lbl_known(pr)) continue;
                const int hn = pr.hops + 1;
                const double rn = pr.rel * g.inRel[arc];
                if (er.hops != hn || er.rel != rn) {
                    lbl_st(&LBL[e], rn, hn, a);
                    ch = 1;
                    if (a & TIE_AMB) atomicOr(&ctl->ambMask, 1u << ll);
                }
            }
            if (ch) ctl->changed = 1;
            fence_wg();
            __syncthreads();
            const int any = uni(ctl->changed);
            __syncthreads();
            if (tid == 0) ctl->changed = 0;
            __syncthreads();
            if (!any) break;
        }
        }   // label passes
        if (dbg && tid == 0) dbg[16 * b + 2] = (int)(((long long)clock64() - ctl->t2) >> 10);   // walks
        // ---- row writer: the lanes' rows are written target block by
        // target block through an LDS tile (the walk stacks' space): a
        // group holds one target of 16 rows, so direct stores would scatter
        // 16 rows x 8-32 B per wave instruction; from the tile each wave
        // stores a run of consecutive columns of one row (non-temporal:
        // the table is never re-read here)
        if (!failed && !retry) {
            const int T = (int)tab.T;
            // (2 x NT entries of 21 B: inside the walk stacks' SMAX x NT x 8 B)
            double* const tLat = reinterpret_cast<double*>(smem + BCTRL_BYTES);
            double* const tRel = tLat + 2 * NT;
            int32_t* const tHop = reinterpret_cast<int32_t*>(tRel + 2 * NT);
            int32_t* const tPred = tHop + 2 * NT;
            uint8_t* const tFlg = reinterpret_cast<uint8_t*>(tPred + 2 * NT);
            const int wl = tid / NG, wc = tid % NG;     // writer: lane (row), column in block
            const int wrow = laneRow[wl];
            const size_t wbase = (size_t)(wrow >= 0 ? wrow - tab.rowStart : 0) * (size_t)tab.T;
            __syncthreads();                            // walks done: stacks free
            // WQ targets per group per block, their loads issued branch-free
            // level by level (vertex id -> dist + label record + vertex
            // reliability -> parent vertex -> caller id), so WQ dependent
            // chains are in flight per thread and a block's two barriers are
            // shared by WQ x NG targets
            constexpr int WQ = 2;
            const int BW = WQ * NG;
            // the lane's own source (1-vertex igraph path [s]: the fold uses
            // edge (s,s), :1469-1488; the destination factor is skipped, :1457)
            const bool srcSelf = row >= 0 && g.hasSelf[src >= 0 ? src : 0];
            const double srcVrel = row >= 0 ? g.vrel[src >= 0 ? src : 0] : 1.0;
            const double selfL = srcSelf ? 0.0 + g.selfLat[src] : 0.0;
            const double selfR = srcSelf ? (1.0 * srcVrel) * g.selfRel[src] : 0.0;
            for (int j0 = 0; j0 < T; j0 += BW) {
                int tq[WQ], pq[WQ];
                unsigned long long dq[WQ];
                Lbl rq[WQ];
                double vq[WQ];
#pragma unroll
                for (int q = 0; q < WQ; ++q) {
                    const int j = j0 + q * NG + gid;
                    tq[q] = row >= 0 && j < T ? g.attached[j] : -1;
                }
#pragma unroll
                for (int q = 0; q < WQ; ++q) {
                    const int tc = tq[q] >= 0 ? tq[q] : 0;
                    dq[q] = dec(ld_wg(&D[(size_t)tc * LB + l]));
                    rq[q] = lbl_ld(&LBL[(size_t)tc * LB + l]);
                    vq[q] = g.vrel[tc];
                }
#pragma unroll
                for (int q = 0; q < WQ; ++q) {
                    // (an unreachable target's record is not this batch's: its
                    // arc field is never followed)
                    const bool reach = tq[q] >= 0 && tq[q] != src && dq[q] != INF_BITS;
                    const int pa = reach ? rq[q].arc : -1;
                    const int x = g.inCol[pa >= 0 ? pa & ~TIE_AMB : 0];
                    pq[q] = pa >= 0 ? x : -1;
                }
                if (g.oldId) {
#pragma unroll
                    for (int q = 0; q < WQ; ++q) {
                        const int x = g.oldId[pq[q] >= 0 ? pq[q] : 0];   // device id -> caller's id
                        pq[q] = pq[q] >= 0 ? x : -1;
                    }
                }
#pragma unroll
                for (int q = 0; q < WQ; ++q) {
                    const int t = tq[q];
                    double L = 0.0, Rl = 0.0;
                    int h = -1, pv = -1;
                    uint8_t f = 0;
                    if (t >= 0) {
                        if (t == src) {
                            if (srcSelf) {
                                L = selfL;
                                Rl = selfR;
                                h = 1;
                            } else {
                                f |= F_NOEDGE;
                            }
                        } else if (dq[q] == INF_BITS) {
                            f |= F_UNREACHABLE;
                        } else {
                            L = b2d(dq[q]);
                            h = rq[q].hops;
                            pv = pq[q];
                            if (srcVrel == 1.0 && vq[q] == 1.0)
                                Rl = rq[q].rel;
                            else
                                Rl = fold_rel_batch<LB>(g.vrel, g.inRel, g.inCol, LBL, l, src, t, h);
                            if (L == 0.0) {                 // topology.c:1848-1852
                                L = 1.0;
                                f |= F_ZEROLAT;
                            }
                        }
                    }
                    const int ti = l * BW + q * NG + gid;
                    tLat[ti] = L;
                    tRel[ti] = Rl;
                    tHop[ti] = h;
                    tPred[ti] = pv;
                    tFlg[ti] = f;
                }
                __syncthreads();
#pragma unroll
                for (int q = 0; q < WQ; ++q) {
                    const int c = j0 + q * NG + wc;
                    if (wrow >= 0 && c < T) {
                        const int ti2 = wl * BW + q * NG + wc;
                        const size_t o = wbase + (size_t)c;
                        __builtin_nontemporal_store(tLat[ti2], &tab.lat[o]);
                        __builtin_nontemporal_store(tRel[ti2], &tab.rel[o]);
                        __builtin_nontemporal_store(tHop[ti2], &tab.hops[o]);
                        __builtin_nontemporal_store(tFlg[ti2], &tab.flags[o]);
                        if (tab.pred) __builtin_nontemporal_store(tPred[ti2], &tab.pred[o]);
                    }
                }
                __syncthreads();
            }
        }
        if (relAmb) atomicOr(&ctl->ambMask, 1u << l);
        fence_wg();
        __syncthreads();
        // rows whose target paths meet an ambiguous entry (or that hit the
        // phase cap) go to k_exact_rows; their rows above are rewritten there
        needMask = failed ? LBMASK : ctl->ambMask;
        __syncthreads();
        if (tid == 0) ctl->ambMask = 0u;
        __syncthreads();
        // a tie row's export needs every vertex's parent: the full pass --
        // in line, or (the post kernel, with a deferred-export buffer) by
        // k_tie_export over the whole GPU after this kernel, so a tie batch
        // no longer runs a second full pass here (round 6: the c4q post
        // kernel was 43 vs 31 ms, a tie batch's in-line pass on its tail)
        const bool deferTie = PT == 2 && tieDesc != nullptr &&
                              __builtin_amdgcn_readfirstlane((int)(ld_wg(&tieDesc->req) != nullptr)) != 0;
        if (!fullPred && !failed && (retry || (needMask && !deferTie))) continue;
        lastFull = fullPred;
        break;
        }   // attempts
        if constexpr (PT == 1) {
            __syncthreads();
            if (dbg && tid == 0) {
                if (coMember == 0) {
                    dbg[16 * b + 0] = phases;
                    dbg[16 * b + 5] = (int)((ctl->t1 - ctl->t0) >> 10);
                    dbg[16 * b + 15] = repairs;
                }
                atomicAdd(&dbg[16 * b + 4], (int)ctl->dProcs);
                atomicAdd(&dbg[16 * b + 9], (int)(ctl->dArcs >> 4));
                atomicAdd(&dbg[16 * b + 10], (int)ctl->dLanes);
            }
            __syncthreads();
            continue;
        }
        if (dbg && tid == 0) ctl->t3 = (long long)clock64();

        // ---- tie export: hand k_exact_rows the final distances, the parents
        // and the ambiguous entries, so it emulates the heap only until the
        // last tied predecessor is popped (tie threshold) ----
        if (needMask && !failed && tieDesc) {
            // descriptor read from memory here only: as a kernel argument
            // it cost the hot loops registers (SGPR spills)
            const TieBuf tie = *tieDesc;
            // deferred (attempt 0 of the post kernel): the slot records the
            // request, k_tie_export fills it after this kernel
            const bool defer = PT == 2 && !lastFull;
            if (tid < LB) {
                int sl = -1;
                if ((needMask >> tid) & 1u) {
                    sl = atomicAdd(tie.count, 1);
                    if (sl >= tie.cap) sl = -1;
                }
                tieSlot[tid] = sl;
                tieThr[tid] = 0ull;
                if (defer && sl >= 0) {       // thread tid < LB is lane tid of group 0
                    tie.thr[sl] = 0.0;
                    tie.req[4 * sl + 0] = b;
                    tie.req[4 * sl + 1] = tid;
                    tie.req[4 * sl + 2] = src;
                    tie.req[4 * sl + 3] = *tie.round;
                }
            }
            __syncthreads();
            const int sl = defer ? -1 : tieSlot[l];
            unsigned long long thr = 0ull;
            for (int v = gid; v < n; v += NG) {
                if (sl < 0) continue;
                const size_t e = (size_t)v * LB + l;
                const int pe = lbl_arc(&LBL[e]);
                const bool am = pe >= 0 && (pe & TIE_AMB);
                const size_t o = (size_t)sl * (size_t)tie.n + v;
                tie.D[o] = b2d(dec(ld_wg(&D[(size_t)v * LB + l])));
                tie.P[o] = pe;
                if (am) {   // rare: re-derive the tied (minimum tight) predecessor distance
                    const unsigned long long dv = dec(ld_wg(&D[(size_t)v * LB + l]));
                    const int a0 = undirected ? g.rowPtr[v] : g.inPtr[v];
                    const int a1 = undirected ? g.rowPtr[v + 1] : g.inPtr[v + 1];
                    unsigned long long mt = INF_BITS;
                    for (int a = a0; a < a1; ++a) {
                        const int u = undirected ? g.col[a] : g.inCol[a];
                        const double w = undirected ? g.lat[a] : g.inLat[a];
                        const unsigned long long du = dec(ld_wg(&D[(size_t)u * LB + l]));
                        if (du <= dv && d2b(b2d(du) + w) == dv && du < mt) mt = du;
                    }
                    if (mt != INF_BITS) thr = mt > thr ? mt : thr;
                }
            }
            if (thr) atomicMax(&tieThr[l], thr);
            fence_wg();
            __syncthreads();
            if (!defer && gid == 0 && sl >= 0) tie.thr[sl] = b2d(tieThr[l]);
        } else if (tid < LB) {
            tieSlot[tid] = -1;
        }
        __syncthreads();
#ifdef SHDPE_DIAG_WHY
        if (failed) why |= 1u;
        if (why) atomicOr(&ctl->dWhy, why);
        __syncthreads();
#endif
        if (dbg && tid == 0) ctl->t4 = (long long)clock64();
        // 0 fast path, 1 full igraph-heap emulation, 2 + slot: early-stop
        // emulation with the exported tie data
        if (gid == 0 && row >= 0)
            rowAmbig[(size_t)b * LB + l] =
                ((needMask >> l) & 1u) ? (uint8_t)(tieSlot[l] >= 0 ? 2 + tieSlot[l] : 1) : (uint8_t)0;
        if (dbg && tid == 0) {
            if (PT == 0) {
                dbg[16 * b + 0] = phases;
                dbg[16 * b + 15] = repairs;
                dbg[16 * b + 5] = (int)((ctl->t1 - ctl->t0) >> 10);
                atomicAdd(&dbg[16 * b + 4], (int)ctl->dProcs);
                atomicAdd(&dbg[16 * b + 9], (int)(ctl->dArcs >> 4));
                atomicAdd(&dbg[16 * b + 10], (int)ctl->dLanes);
            }
            dbg[16 * b + 1] = (int)ctl->dWhy;
            dbg[16 * b + 3] = (int)needMask;
            dbg[16 * b + 6] = (int)((ctl->t2 - ctl->t1) >> 10);
            dbg[16 * b + 7] = (int)((ctl->t3 - ctl->t2) >> 10);
            dbg[16 * b + 11] = (int)((ctl->t4 - ctl->t3) >> 10);
        }
        fence_wg();
        __syncthreads();
        if (dbg && tid == 0) dbg[16 * b + 8] = (int)(((long long)clock64() - ctl->t4) >> 10);
    }
}

// k_tie_export: the deferred tie export of one round (launch_tie_export).
// One thread per (slot, vertex), grid-stride: the vertex's distance, and its
// parent exactly as the post kernel's full predecessor pass derives it (first
// in-arc, in incidence order, among the tight ones with minimum dist[u];
// TIE_AMB on equal minima or a zero-increment arc; -1 for the source and
// unreachable vertices), the threshold as the maximum tied-predecessor
// distance over the ambiguous entries (k_exact_rows' early stop), and the
// Bellman check over every in-arc (a violation sends the row to the full
// emulation, rowAmbig 1, as a failed batch would).  violSlot >= 0 (tests,
// SHDPE_TIE_CORRUPT=3): that slot's row is treated as violated.
template <int LB>
__global__ __launch_bounds__(256) void k_tie_export(DevGraph g0, BatchScratch bs, TieBuf tie, int round,
                                                    uint8_t* __restrict__ rowAmbig, int violSlot) {
    const DevGraph g = global_view(g0);
    const int n = g.n;
    const bool undirected = g.inCol == g.col;
    const int cnt = min(*as_global(tie.count), tie.cap);
    const size_t SE = (size_t)bs.nStride * LB;
    const size_t total = (size_t)cnt * (size_t)n;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (size_t)gridDim.x * 256) {
        const int sl = (int)(i / (size_t)n);
        const int v = (int)(i % (size_t)n);
        const int32_t* rq = as_global(tie.req) + 4 * sl;
        if (rq[3] != round) continue;
        const int b = rq[0], l = rq[1], src = rq[2];
        const unsigned long long* D = as_global(bs.D) + (size_t)b * SE;
        const unsigned long long dv = dec(D[(size_t)v * LB + l]);
        const size_t o = (size_t)sl * (size_t)tie.n + v;
        as_global(tie.D)[o] = b2d(dv);
        int pe = -1;
        if (v != src) {
            const int a0 = undirected ? g.rowPtr[v] : g.inPtr[v];
            const int a1 = undirected ? g.rowPtr[v + 1] : g.inPtr[v + 1];
            unsigned long long best = INF_BITS, mn = INF_BITS;
            int cnt2 = 0, ba = -1;
            for (int a = a0; a < a1; ++a) {
                const int u = undirected ? g.col[a] : g.inCol[a];
                const double w = undirected ? g.lat[a] : g.inLat[a];
                const unsigned long long du = dec(D[(size_t)u * LB + l]);
                const double cand = b2d(du) + w;
                const unsigned long long cb = d2b(cand);
                mn = cb < mn ? cb : mn;
                if (dv != INF_BITS && du <= dv && cand == b2d(dv)) {
                    if (du < best) {
                        best = du;
                        cnt2 = 1;
                        ba = a;
                    } else if (du == best) {
                        ++cnt2;
                    }
                }
            }
            if (mn < dv || sl == violSlot) rowAmbig[(size_t)b * LB + l] = 1;   // Bellman violation: full emulation
            if (dv != INF_BITS) {
                const bool ea = cnt2 != 1 || best == dv;
                pe = ea ? (TIE_AMB | (ba > 0 ? ba : 0)) : ba;
                if (ea && best != INF_BITS)
                    atomicMax(reinterpret_cast<unsigned long long*>(as_global(tie.thr) + sl), best);
            }
        }
        as_global(tie.P)[o] = pe;
    }
}

void launch_tie_export(const DevGraph& g, const BatchScratch& bs, int lb, const TieBuf& tie, int round,
                       uint8_t* dRowAmbig, int grid, int violSlot, void* stream) {
    if (tie.cap <= 0 || !tie.req) return;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    if (lb == 4)
        hipLaunchKernelGGL(k_tie_export<4>, dim3(grid), dim3(256), 0, st, g, bs, tie, round, dRowAmbig, violSlot);
    else if (lb == 8)
        hipLaunchKernelGGL(k_tie_export<8>, dim3(grid), dim3(256), 0, st, g, bs, tie, round, dRowAmbig, violSlot);
    else if (lb == 32)
        hipLaunchKernelGGL(k_tie_export<32>, dim3(grid), dim3(256), 0, st, g, bs, tie, round, dRowAmbig, violSlot);
    else
        hipLaunchKernelGGL(k_tie_export<16>, dim3(grid), dim3(256), 0, st, g, bs, tie, round, dRowAmbig, violSlot);
}

template <int LB, int WPE, bool GB, int PART>
static void launch_lb(const DevGraph& g, const DevTable& tab, const BatchScratch& bs,
                      const int32_t* dBatchRows, int32_t nBatches, uint8_t* dRowAmbig,
                      const BatchLaunch& cfg, int32_t* dDbg, const TieBuf* tie, hipStream_t st,
                      int grid) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_batch_rows<LB, WPE, GB, PART>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, cfg.ldsBytes);
    // (the kernel's NT is compile-time: the variant's own size, batch_threads)
    hipLaunchKernelGGL((k_batch_rows<LB, WPE, GB, PART>), dim3(grid), dim3(batch_threads(WPE)), cfg.ldsBytes,
                       st, g, tab, bs, dBatchRows, nBatches, dRowAmbig, cfg.delta, dDbg, tie);
}

// The cooperative relax (PART 3) exists for LB 8 and 16 with LDS bitmaps --
// the small-shard configurations it is for.  Launched cooperatively: the
// runtime refuses a grid that is not wholly resident (then the caller runs
// the plain relax).
template <int LB, int WPE>
static int launch_coop_lb(const DevGraph& g, const DevTable& tab, const BatchScratch& bs,
                          const int32_t* dBatchRows, int32_t nBatches, uint8_t* dRowAmbig,
                          const BatchLaunch& cfg, int32_t* dDbg, const TieBuf* tie, hipStream_t st,
                          int grid) {
    const void* fn = reinterpret_cast<const void*>(&k_batch_rows<LB, WPE, false, 3>);
    (void)hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, cfg.ldsBytes);
    DevGraph a0 = g;
    DevTable a1 = tab;
    BatchScratch a2 = bs;
    const int32_t* a3 = dBatchRows;
    int32_t a4 = nBatches;
    uint8_t* a5 = dRowAmbig;
    double a6 = cfg.delta;
    int32_t* a7 = dDbg;
    const TieBuf* a8 = tie;
    void* args[] = {&a0, &a1, &a2, &a3, &a4, &a5, &a6, &a7, &a8};
    return hipLaunchCooperativeKernel(fn, dim3(grid), dim3(batch_threads(WPE)), args, (unsigned)cfg.ldsBytes, st) ==
                   hipSuccess
               ? 0
               : -1;
}

template <int WPE>
static int launch_coop_w(const DevGraph& g, const DevTable& tab, const BatchScratch& bs,
                         const int32_t* dBatchRows, int32_t nBatches, uint8_t* dRowAmbig,
                         const BatchLaunch& cfg, int32_t* dDbg, const TieBuf* tie, hipStream_t st, int grid) {
    if (cfg.lb == 8)
        return launch_coop_lb<8, WPE>(g, tab, bs, dBatchRows, nBatches, dRowAmbig, cfg, dDbg, tie, st, grid);
    return launch_coop_lb<16, WPE>(g, tab, bs, dBatchRows, nBatches, dRowAmbig, cfg, dDbg, tie, st, grid);
}

int launch_batch_relax_coop(const DevGraph& g, const DevTable& tab, const BatchScratch& bs,
                            const int32_t* dBatchRows, int32_t nBatches, uint8_t* dRowAmbig,
                            const BatchLaunch& cfg, int32_t* dDbg, const TieBuf* tie, void* stream) {
    if (nBatches <= 0) return 0;
    if (cfg.gbits || (cfg.lb != 8 && cfg.lb != 16) || cfg.grid <= 0) return -1;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    if (cfg.wpe >= 8)
        return launch_coop_w<8>(g, tab, bs, dBatchRows, nBatches, dRowAmbig, cfg, dDbg, tie, st, cfg.grid);
    if (cfg.wpe == 6)
        return launch_coop_w<6>(g, tab, bs, dBatchRows, nBatches, dRowAmbig, cfg, dDbg, tie, st, cfg.grid);
    return launch_coop_w<4>(g, tab, bs, dBatchRows, nBatches, dRowAmbig, cfg, dDbg, tie, st, cfg.grid);
}

const void* batch_coop_kernel_ptr(int lb, int wpe) {
    if (lb == 8)
        return wpe >= 8 ? reinterpret_cast<const void*>(&k_batch_rows<8, 8, false, 3>)
             : wpe == 6 ? reinterpret_cast<const void*>(&k_batch_rows<8, 6, false, 3>)
                        : reinterpret_cast<const void*>(&k_batch_rows<8, 4, false, 3>);
    return wpe >= 8 ? reinterpret_cast<const void*>(&k_batch_rows<16, 8, false, 3>)
         : wpe == 6 ? reinterpret_cast<const void*>(&k_batch_rows<16, 6, false, 3>)
                    : reinterpret_cast<const void*>(&k_batch_rows<16, 4, false, 3>);
}

int batch_threads(int wpe) { return wpe == 6 ? 768 : BT_THREADS; }

int batch_lds_bytes(int n, int wpe, bool gbits) {
    const int nwp = (((n + 31) >> 5) + 3) & ~3;
    // label walks reuse the relax bitmaps' LDS for their stacks
    const int stack = batch_threads(wpe) * (wpe >= 6 ? BCfg<8>::SMAX : BCfg<4>::SMAX) * 8;
    const int bits = gbits ? 0 : 2 * 4 * nwp;
    return BCTRL_BYTES + (bits > stack ? bits : stack);
}

int64_t batch_bits_words(int n) { return 2 * (int64_t)((((n + 31) >> 5) + 3) & ~3); }

template <int WPE, int PART>
static const void* kptr(int lb, bool gb) {
    if (gb) return reinterpret_cast<const void*>(&k_batch_rows<16, WPE, true, PART>);
    if (lb == 4) return reinterpret_cast<const void*>(&k_batch_rows<4, WPE, false, PART>);
    if (lb == 8) return reinterpret_cast<const void*>(&k_batch_rows<8, WPE, false, PART>);
    if (lb == 32) return reinterpret_cast<const void*>(&k_batch_rows<32, WPE, false, PART>);
    return reinterpret_cast<const void*>(&k_batch_rows<16, WPE, false, PART>);
}

template <int WPE>
static const void* kptr_p(int lb, bool gb, int part) {
    return part == 1 ? kptr<WPE, 1>(lb, gb) : part == 2 ? kptr<WPE, 2>(lb, gb) : kptr<WPE, 0>(lb, gb);
}

const void* batch_kernel_ptr(int lb, int wpe, bool gbits, int part) {
    return wpe >= 8 ? kptr_p<8>(lb, gbits, part) : wpe == 6 ? kptr_p<6>(lb, gbits, part)
                                                             : kptr_p<4>(lb, gbits, part);
}

template <int WPE, int PART>
static void launch_w(const DevGraph& g, const DevTable& tab, const BatchScratch& bs,
                     const int32_t* dBatchRows, int32_t nBatches, uint8_t* dRowAmbig,
                     const BatchLaunch& cfg, int32_t* dDbg, const TieBuf* tie, hipStream_t st, int grid) {
    if (cfg.gbits)    // graphs whose bitmaps exceed LDS: LB 16 only (the engine forces it)
        launch_lb<16, WPE, true, PART>(g, tab, bs, dBatchRows, nBatches, dRowAmbig, cfg, dDbg, tie, st, grid);
    else if (cfg.lb == 4)
        launch_lb<4, WPE, false, PART>(g, tab, bs, dBatchRows, nBatches, dRowAmbig, cfg, dDbg, tie, st, grid);
    else if (cfg.lb == 8)
        launch_lb<8, WPE, false, PART>(g, tab, bs, dBatchRows, nBatches, dRowAmbig, cfg, dDbg, tie, st, grid);
    else if (cfg.lb == 32)
        launch_lb<32, WPE, false, PART>(g, tab, bs, dBatchRows, nBatches, dRowAmbig, cfg, dDbg, tie, st, grid);
    else
        launch_lb<16, WPE, false, PART>(g, tab, bs, dBatchRows, nBatches, dRowAmbig, cfg, dDbg, tie, st, grid);
}

template <int WPE>
static void launch_wp(const DevGraph& g, const DevTable& tab, const BatchScratch& bs,
                      const int32_t* dBatchRows, int32_t nBatches, uint8_t* dRowAmbig,
                      const BatchLaunch& cfg, int32_t* dDbg, const TieBuf* tie, hipStream_t st, int grid,
                      int part) {
    if (part == 1) launch_w<WPE, 1>(g, tab, bs, dBatchRows, nBatches, dRowAmbig, cfg, dDbg, tie, st, grid);
    else if (part == 2) launch_w<WPE, 2>(g, tab, bs, dBatchRows, nBatches, dRowAmbig, cfg, dDbg, tie, st, grid);
    else launch_w<WPE, 0>(g, tab, bs, dBatchRows, nBatches, dRowAmbig, cfg, dDbg, tie, st, grid);
}

void launch_batch_rows(const DevGraph& g, const DevTable& tab, const BatchScratch& bs,
                       const int32_t* dBatchRows, int32_t nBatches, uint8_t* dRowAmbig,
                       const BatchLaunch& cfg, int32_t* dDbg, const TieBuf* tie, void* stream, int part) {
    if (nBatches <= 0) return;
    const int grid = nBatches < cfg.grid ? nBatches : cfg.grid;
    if (grid <= 0) return;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    if (cfg.wpe >= 8)
        launch_wp<8>(g, tab, bs, dBatchRows, nBatches, dRowAmbig, cfg, dDbg, tie, st, grid, part);
    else if (cfg.wpe == 6)
        launch_wp<6>(g, tab, bs, dBatchRows, nBatches, dRowAmbig, cfg, dDbg, tie, st, grid, part);
    else
        launch_wp<4>(g, tab, bs, dBatchRows, nBatches, dRowAmbig, cfg, dDbg, tie, st, grid, part);
}

}  // namespace shdpe

// pe_engine.hip -- C-ABI implementation of the MI355X Shadow path engine.
//
// Replaces topology.c:1681-1866 (target collection + igraph Dijkstra +
// per-target fold) with device kernels; see include/shd_pathengine.h.
// No CPU compute fallback: every row comes from a gfx950 kernel, and create
// fails with SHD_PE_ENODEV when no device is usable.
//
// Multi-GPU: the T table rows are split into G contiguous
// row shards of (near-)equal kernel work units (shd_pe_plan_shards).  One
// engine owns one or more of them, one per device (nDevices); several
// engines in several processes own the rest (shardIndex / shardCount).  Each
// shard holds its own graph copy, stream and a shard-sized table
// (rows x T); compute runs all local shards concurrently (one host thread
// per device), never exchanging data.  shd_pe_gather assembles the whole
// table on every device with RCCL (a group of broadcasts = all-gather with
// per-shard sizes) over xGMI, or with device copies when several logical
// shards share a device.  The reference serialises every row on one core
// under graphLock (topology.c:1747-1781).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <sys/mman.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <memory>
#include <mutex>
#include <new>
#include <queue>
#include <chrono>
#include <thread>
#include <vector>

#include "pe_device.hpp"
#include "pe_graph.hpp"
#include "shd_pathengine.h"

using namespace shdpe;

namespace {

constexpr int LDS_BYTES = 160 * 1024;

struct Shard {
    int gindex = 0;                 // global shard index
    int device = 0;
    int numCUs = 256;
    int32_t rowStart = 0, rowCount = 0;   // table positions owned
    hipStream_t stream = nullptr;
    hipStream_t copyStream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr, evA = nullptr, evB = nullptr;
    hipEvent_t evP[3] = {nullptr, nullptr, nullptr};   // per-part timing (shd_pe_tune)
    std::vector<void*> allocs;
    DevGraph dg{};                  // path kernels (device ids, possibly relabelled)
    DevGraph dgAux{};               // caller's ids, rows sorted by id (aux kernels)
    DevTable tab{};                 // this shard's rows
    DevScratch sc{};
    bool tableReady = false;
    int32_t* dRows = nullptr;
    uint8_t* dRowAmbig = nullptr;
    int32_t* dDbg = nullptr;
    int32_t pathSrc = -1;           // source whose full parent array sits in exact slot 0
    int32_t* dPath = nullptr;       // path walk output (+ length), shd_pe_get_path
    int32_t rowsCap = 0;
    SparseLaunch cfg{};
    int exactGrid = 0, exactHc = 1;
    BatchLaunch bcfg{};
    BatchLaunch bcfgAlt{};          // the other kernel variant (grid 0: none), shd_pe_tune
    BatchLaunch bcfgAlt2{};         // a third variant (6 waves), shd_pe_tune
    BatchLaunch bcfgPost{};         // split kernels: post-kernel variant when the tune picked
                                    // another one than bcfg's (grid 0: bcfg)
    BatchLaunch bcfgCoop{};         // cooperative relax candidate (coop >= 2; grid 0: none)
    int64_t coopAborts = 0;         // cooperative relax launches aborted (round rerun plain)
    int32_t* dCoopAbort = nullptr;  // host-mapped copy target of the abort word
    bool tuned = false;
    bool timeParts = false;         // split kernels: time relax / post launches (tune)
    double msPart[2] = {0.0, 0.0};
    BatchScratch bsc{};
    bool batchReady = false;
    int32_t batchRound = 0;         // split kernels: batches per round (persisted dist arrays)
    int32_t batchSlots = 0;         // scratch slots allocated (no launch may exceed it)
    int32_t* dBatchRows = nullptr;
    uint8_t* dBatchAmb = nullptr;
    TieBuf tie{};                   // early-stop tie rows (batched path)
    int32_t* dSlots = nullptr;      // per exact row its tie slot, -1 full emulation
    TieBuf* dTie = nullptr;         // device copy of `tie` (k_batch_rows reads it)
    int32_t* dDenseIdx = nullptr;   // dense early-stop tie rows: their row of the D / P matrices
    long long* dXdbg = nullptr;     // exact-kernel counters (SHD_PE_DEBUG_COUNTERS)
    bool tieTried = false;
    double *dW = nullptr, *dRl = nullptr, *dD = nullptr;
    int32_t* dP = nullptr;
    uint8_t *dRowA = nullptr, *dRowB = nullptr, *dRowAmbD = nullptr, *dChunkEpoch = nullptr;
    void* dXList = nullptr;         // k_exact_dense: per slot its pushes / modifies of a pop
    int32_t* dAny = nullptr;
    int32_t denseRows = 0;
    DevTable full{};                // whole table on this device after gather
    bool fullOwner = false;         // first shard on its device owns `full`
    ncclComm_t comm = nullptr;      // in-process communicator (distinct devices)
    ShdPeStats stats{};
};

}  // namespace

struct ShdPe {
    HostGraph hg;
    std::vector<int32_t> attached;   // unique, first-occurrence order
    std::vector<int32_t> posOf;      // vertex -> table position or -1
    ShdPeOptions opt{};
    Tuning tu{};
    int mode = 1;
    bool batched = false;
    std::vector<int32_t> rank;       // table position -> batch order rank
    std::vector<double> rowOff;      // table position -> distance to its batch hub (order 1)
    std::vector<int32_t> devOf;      // caller vertex id -> device id (empty: identity)
    int G = 1;                       // global row shards
    std::vector<int32_t> bounds;     // G + 1 position bounds
    int firstShard = 0;              // global index of shards[0]
    std::vector<std::unique_ptr<Shard>> shards;
    std::unique_ptr<std::atomic<uint8_t>[]> rowDone;
    bool gathered = false;
    int64_t putRows = 0;             // distinct rows imported by shd_pe_put_rows (host transport)
    std::vector<uint8_t> putSeen;    // per table row: imported already (a repeated put counts once)
    bool putInit = false;            // own shard rows copied into the full table
    ncclComm_t xcomm = nullptr;      // cross-process communicator (shd_pe_comm_init)
    int32_t ownStart = 0, ownEnd = 0;
    unsigned char* stage[2] = {nullptr, nullptr};   // pinned host staging (portable)
    size_t stageBytes = 0;
    std::mutex mu;                   // compute / gather
    std::mutex copyMu;               // staging buffers
    double msGather = 0.0;
};

#define HIPCHK(x)                                   \
    do {                                            \
        if ((x) != hipSuccess) return SHD_PE_EHIP;  \
    } while (0)

static int dev_alloc(Shard* s, void** p, size_t bytes) {
    if (bytes == 0) bytes = 16;
    if (hipMalloc(p, bytes) != hipSuccess) { *p = nullptr; return SHD_PE_ENOMEM; }
    s->allocs.push_back(*p);
    return SHD_PE_OK;
}

template <class T, class A>
static int dev_upload(Shard* s, T** dst, const std::vector<T, A>& src) {
    int rc = dev_alloc(s, reinterpret_cast<void**>(dst), src.size() * sizeof(T));
    if (rc) return rc;
    if (!src.empty())
        HIPCHK(hipMemcpy(*dst, src.data(), src.size() * sizeof(T), hipMemcpyHostToDevice));
    return SHD_PE_OK;
}

// SHDPE_* tuning variables are read only under SHD_PE_DEBUG_ENV: a library
// linked into Shadow must not change behaviour with the environment.
static void read_tuning(Tuning& t, int32_t flags) {
    if (flags & SHD_PE_DEBUG_COUNTERS) t.debug = 1;
    if (!(flags & SHD_PE_DEBUG_ENV)) return;
    auto gi = [](const char* k, int& v) { const char* e = std::getenv(k); if (e && *e) v = std::atoi(e); };
    auto gd = [](const char* k, double& v) { const char* e = std::getenv(k); if (e && *e) v = std::atof(e); };
    gi("SHDPE_THREADS", t.spThreads);
    gi("SHDPE_HEAVY_DEG", t.heavyDeg);
    gi("SHDPE_LAYOUT", t.layout);
    gi("SHDPE_WG_PER_CU", t.wgPerCU);
    gi("SHDPE_KFLAGS", t.kflags);
    gd("SHDPE_DELTA_FACTOR", t.deltaFactor);
    gi("SHDPE_EXACT_HC", t.exactHc);
    gi("SHDPE_EXACT_PER_CU", t.exactPerCU);
    gi("SHDPE_BATCH", t.batch);
    gi("SHDPE_BATCH_LB", t.batchLB);
    gi("SHDPE_BATCH_GRID", t.batchGrid);
    gi("SHDPE_BATCH_ORDER", t.batchOrder);
    gi("SHDPE_BATCH_WPE", t.batchWpe);
    gi("SHDPE_RELABEL", t.relabel);
    gi("SHDPE_BATCH_SPLIT", t.batchSplit);
    gd("SHDPE_BATCH_DELTA_FACTOR", t.batchDeltaFactor);
    gd("SHDPE_BATCH_SCRATCH_GB", t.batchScratchGB);
    gd("SHDPE_DENSE_MIN", t.denseMin);
    gd("SHDPE_DENSE_BATCH_GB", t.denseBatchGB);
    gi("SHDPE_PRED_MI", t.densePredMi);
    gi("SHDPE_DENSE_EPOCHS", t.denseEpochs);
    gi("SHDPE_DEBUG", t.debug);
    gi("SHDPE_STREAM_WG_PER_CU", t.streamWgPerCU);
    gi("SHDPE_TIE_CORRUPT", t.tieCorrupt);
    gi("SHDPE_TUNE_FAIL_WPE", t.failWpe);
    gi("SHDPE_TUNE_LOG", t.tuneLog);
    gi("SHDPE_BATCH_COOP", t.batchCoop);
    gi("SHDPE_BATCH_COOP_WPE", t.batchCoopWpe);
    gi("SHDPE_COOP_SPIN", t.coopSpin);
}

extern "C" void shd_pe_default_options(ShdPeOptions* opt) {
    if (!opt) return;
    std::memset(opt, 0, sizeof(*opt));
    opt->device = 0;
    opt->delta = 0.0;
    opt->storePred = 1;
    opt->forceMode = 0;
    opt->nDevices = 1;
    opt->devices = nullptr;
    opt->shardIndex = 0;
    opt->shardCount = 1;
    opt->debugFlags = 0;
}

extern "C" const char* shd_pe_strerror(int code) {
    switch (code) {
        case SHD_PE_OK: return "ok";
        case SHD_PE_EINVAL: return "invalid argument or graph fails topology checks";
        case SHD_PE_ENOMEM: return "out of memory";
        case SHD_PE_ENODEV: return "no usable gfx950 device";
        case SHD_PE_EUNREACHABLE: return "target unreachable";
        case SHD_PE_ENOSELFLOOP: return "self-loop (s,s) missing";
        case SHD_PE_EMULTI: return "multigraph error (reserved: no longer returned)";
        case SHD_PE_EHIP: return "HIP runtime error";
        case SHD_PE_ENOTATTACHED: return "vertex is not attached";
        case SHD_PE_ENOEDGE: return "no edge between the vertices";
        case SHD_PE_ENOTOWNED: return "row belongs to another engine's shard (gather first)";
        case SHD_PE_ETOOBIG: return "graph exceeds the engine's vertex limit";
        case SHD_PE_ECOMM: return "RCCL communicator error";
        default: return "unknown error";
    }
}

static inline int a16(long x) { return (int)((x + 15) & ~15L); }

// Kernel configuration for one shard's device.  Returns SHD_PE_ETOOBIG when
// no kernel layout can hold the graph's per-row LDS state.
static int configure(ShdPe* pe, Shard* sh) {
    const HostGraph& g = pe->hg;
    const Tuning& tu = pe->tu;
    const long n = g.n;
    const long nw = (n + 31) / 32;
    const int LDS = LDS_BYTES;
    SparseLaunch c{};
    c.threads = std::min(tu.spThreads, sparse_max_threads());
    c.hcap = 256;
    c.heavyDeg = tu.heavyDeg;
    const int qmin = 2048;
    // LDS bytes per layout (queues are ping-pong pairs; LAYOUT 0/3 keep them in HBM)
    const int pend = a16(4 * nw), hbits = a16(4 * nw);
    const int hq2 = 2 * a16(4 * c.hcap);
    const long need2 = 64 + pend + hbits + hq2 + a16(8 * n) + a16(2 * n) + a16(4 * (n + 1));
    const long need1 = 64 + pend + hbits + hq2 + a16(8 * n);
    const long need3 = 64 + pend + a16(8 * n);
    const long need0 = 64 + pend + hbits;
    int layout = 0;
    long used = need0;
    if (need2 + 8 * qmin <= LDS) { layout = 2; used = need2; }
    else if (need1 + 8 * qmin <= LDS) { layout = 1; used = need1; }
    // LAYOUT 3 keeps only dist + pending bits in LDS: ~1.4x slower per row
    // than LAYOUT 2 (measured, C2) but fits more rows per CU; take it when it
    // at least doubles the resident rows.
    const int maxWgByThreads = 2048 / std::max(c.threads, 64);
    const long wg2 = layout == 2 ? std::min<long>(maxWgByThreads, LDS / (need2 + 8 * qmin)) : 0;
    const long wg3 = std::min<long>(maxWgByThreads, LDS / need3);
    if (need3 <= LDS && wg3 >= 2 * std::max<long>(wg2, 1)) { layout = 3; used = need3; }
    if (tu.layout == 3 && need3 <= LDS) { layout = 3; used = need3; }
    else if (tu.layout == 2 && need2 + 8 * qmin <= LDS) { layout = 2; used = need2; }
    else if (tu.layout == 1 && need1 + 8 * qmin <= LDS) { layout = 1; used = need1; }
    else if (tu.layout == 0) { layout = 0; used = need0; }
    c.layout = layout;
    if (layout == 1 || layout == 2) {
        c.qcap = (int)std::min<long>((LDS - used) / 8, std::max<long>(n, 1024)) & ~3;
        c.ldsBytes = (int)(used + 2 * a16(4 * c.qcap));
    } else {
        c.qcap = (int)((n + 63) & ~63L);
        c.ldsBytes = (int)used;
    }
    const int wgPerCU = std::max(1, std::min<int>({tu.wgPerCU, LDS / std::max(c.ldsBytes, 1),
                                                   2048 / c.threads}));
    c.grid = sh->numCUs * wgPerCU;
    c.delta = pe->opt.delta > 0 ? pe->opt.delta : g.meanArcLatency * tu.deltaFactor;
    if (!(c.delta > 0)) c.delta = 1.0;
    c.kflags = tu.kflags;
    sh->cfg = c;
    // exact kernels: n <= exact_soa_max_n() keeps heap + index2 wholly in
    // LDS (16 B per vertex, several rows per CU); larger graphs keep the top
    // of the heap in LDS (12 B per entry, up to the whole 160 KB) and the
    // tail in the global slot.
    const bool soa = n <= exact_soa_max_n() && tu.exactHc <= 0;
    const long perWG = soa ? 16L * n + 16 : std::min<long>(LDS, 12L * n + 16);
    // (512 B of the LDS stay free for the kernels' static shared variables;
    // k_exact_rows' preferred-child bits take their share when they fit in
    // half of it -- n <= ~650k)
    const long bitsB = !soa && exact_bits_bytes(n) <= LDS / 2 ? exact_bits_bytes(n) : 0;
    sh->exactHc = (int)std::max<long>(
        1, std::min<long>(n, (std::min<long>(LDS - 512 - bitsB, perWG) - 16) / 12));
    if (tu.exactHc > 0) sh->exactHc = std::min(sh->exactHc, tu.exactHc);   // tests: global heap tail
    const int exPerCU = (int)std::max<long>(1, std::min<long>(8, LDS / perWG));
    sh->exactGrid = sh->numCUs * (tu.exactPerCU > 0 ? tu.exactPerCU : exPerCU);
    // Batched multi-source kernel: the layout for graphs whose per-row state
    // does not fit LDS (LAYOUT 0), or on request (forceMode 5).
    pe->batched = pe->mode == 1 &&
                  (tu.batch == 1 || (tu.batch != 0 && layout == 0) || pe->opt.forceMode == 5);
    BatchLaunch b{};
    // LB = 16 sources per batch; 8 when a shard has too few rows to give
    // every CU a batch of 16.  C4 per-rank shard times, same box: round 5
    // (4-wave relax, one workgroup per CU; profiles/r05_ab_notes.txt r05w)
    // N=4 (4,096 rows) LB 16 28.8 ms vs LB 8 31.0, N=8 (2,048 rows) LB 8 17.2
    // vs LB 16 25.4; round 4 (two 8-wave workgroups per CU, r04_shard_times)
    // had N=4 at LB 8.  LB 4 (32-B line pieces) stays a SHDPE_BATCH_LB option.  (The
    // round-4 cooperative relax -- K workgroups per batch -- and the post
    // kernel over lane slices are patches under tools/variants/)
    b.lb = tu.batchLB;
    if (b.lb != 4 && b.lb != 8 && b.lb != 16 && b.lb != 32)
        b.lb = ((int64_t)sh->rowCount + 15) / 16 >= (int64_t)sh->numCUs ? 16 : 8;
    // (1024 threads, 768 for the 6-wave variant: compile-time in the kernel)
    b.threads = batch_threads(8);
    // pending bitmaps (2 x n/8 bytes) in LDS while they fit beside the
    // control block, else in each slot's global scratch (gbits, LB 16)
    b.gbits = pe->batched && batch_lds_bytes((int)n, 8, false) > LDS ? 1 : 0;
    if (b.gbits) b.lb = 16;
    auto occupancy = [&](int wpe, int threads) {
        const int lds = batch_lds_bytes((int)n, wpe, b.gbits != 0);
        int per = 0;
        if (lds > LDS ||
            hipFuncSetAttribute(batch_kernel_ptr(b.lb, wpe, b.gbits != 0),
                                hipFuncAttributeMaxDynamicSharedMemorySize, lds) != hipSuccess ||
            hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, batch_kernel_ptr(b.lb, wpe, b.gbits != 0),
                                                         threads, lds) != hipSuccess)
            per = 0;
        return per;
    };
    // Two kernel variants: 8 waves per SIMD (two 1024-thread workgroups per
    // CU, one vertex per group) and 4 (one workgroup per CU, two vertices
    // per group).  Which is faster differed from box to box of the same SKU
    // in rounds 3-4 (C4 same-box pairs: 172 vs 185 ms on some, 182 vs 142 ms
    // on others; profiles/r03_ab_notes.txt), so shd_pe_tune times them all;
    // SHDPE_BATCH_WPE forces one.  Since the round-5 loops the tune has
    // picked the 4-wave relax on every box (and the 6-wave post kernel for
    // batches of 16, the 4-wave one for 8), so an untuned engine -- the
    // drop-in computes once -- starts there.
    auto make = [&](int wpe) {
        BatchLaunch c = b;
        c.wpe = wpe;
        if (wpe == 6) c.threads = batch_threads(6);   // two 768-thread workgroups per CU
        c.ldsBytes = batch_lds_bytes((int)n, wpe, b.gbits != 0);
        const int per = c.ldsBytes <= LDS ? occupancy(wpe, c.threads) : 0;
        c.grid = sh->numCUs * std::max(per, 1);
        if (tu.batchGrid > 0 && tu.batchGrid < c.grid) c.grid = tu.batchGrid;
        c.delta = pe->opt.delta > 0 ? pe->opt.delta : g.meanArcLatency * tu.batchDeltaFactor;
        if (!(c.delta > 0)) c.delta = 1.0;
        return std::make_pair(c, per);
    };
    const int forced = tu.batchWpe == 4 || tu.batchWpe == 6 || tu.batchWpe == 8 ? tu.batchWpe : 0;
    auto v8 = make(8), v4 = make(4), v6 = make(6);
    const bool ok8 = v8.second >= 1, ok4 = v4.second >= 1, ok6 = v6.second >= 2 && b.threads == 1024;
    if (pe->batched && !ok8 && !ok4) return SHD_PE_ETOOBIG;
    if (!pe->batched && layout == 0 && need0 > LDS) return SHD_PE_ETOOBIG;
    const int first = forced == 6 && ok6 ? 6 : forced == 8 && ok8 ? 8 : ok4 ? 4 : 8;
    v8.first.split = v4.first.split = v6.first.split = tu.batchSplit ? 1 : 0;
    b = first == 8 ? v8.first : first == 6 ? v6.first : v4.first;
    sh->bcfgAlt = sh->bcfgAlt2 = BatchLaunch{};
    if (!forced && ok8 && ok4) sh->bcfgAlt = first == 8 ? v4.first : v8.first;
    // the 6-wave variant (768 threads: 80 VGPRs, fewer spills than 8 waves'
    // 64) joins the tune when two of its workgroups fit a CU
    if (!forced && ok6 && tu.batchSplit) sh->bcfgAlt2 = v6.first;
    (void)need0;
    sh->bcfg = b;
    sh->bcfgPost = BatchLaunch{};
    if (!forced && first == 4 && ok6 && b.split && b.lb >= 16) sh->bcfgPost = v6.first;
    // Cooperative relax (PART 3, K workgroups of one XCD per batch): for a
    // shard with fewer batches than the plain relax has workgroup slots --
    // the C4 8-GPU shard's 256 LB-8 batches leave one of the two 8-wave
    // slots of every CU idle -- the batch's listing rounds are shared by K
    // workgroups.  SHDPE_BATCH_COOP=K forces it, =1 makes it a candidate of
    // shd_pe_tune (off by default: slower than the plain relax wherever it
    // was measured).
    sh->bcfgCoop = BatchLaunch{};
    if (pe->batched && b.split && !b.gbits && (b.lb == 8 || b.lb == 16) && tu.batchCoop >= 1) {
        const int K = tu.batchCoop >= 2 ? std::min(tu.batchCoop, 8) : 2;
        const int wpeC = tu.batchCoopWpe == 4 || tu.batchCoopWpe == 6 || tu.batchCoopWpe == 8
                             ? tu.batchCoopWpe
                             : ok8 ? 8 : ok6 ? 6 : 4;
        BatchLaunch c2 = wpeC == 8 ? v8.first : wpeC == 6 ? v6.first : v4.first;
        c2.split = 1;
        const void* fn = batch_coop_kernel_ptr(b.lb, wpeC);
        int per = 0;
        if (c2.ldsBytes <= LDS &&
            hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, c2.ldsBytes) == hipSuccess &&
            hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, fn, c2.threads, c2.ldsBytes) == hipSuccess &&
            per >= 1) {
            c2.grid = sh->numCUs * per;
            c2.coop = K;
            const int64_t nB = ((int64_t)sh->rowCount + b.lb - 1) / b.lb;
            // a tune candidate only on request (SHDPE_BATCH_COOP=1): measured
            // slower than the plain relax at every shard size (round 6, C4
            // N=8: 17.1-22.6 vs 16.8 ms; profiles/r06_shard_times.txt)
            if (tu.batchCoop >= 2 || (tu.batchCoop == 1 && nB * K <= c2.grid && nB < b.grid))
                sh->bcfgCoop = c2;
        }
        if (tu.batchCoop >= 2 && sh->bcfgCoop.grid > 0) {
            sh->bcfg = sh->bcfgCoop;        // forced: the relax variant in use
            sh->bcfgPost = b;
            sh->bcfgAlt = sh->bcfgAlt2 = BatchLaunch{};
        }
    }
    sh->stats.deltaUsed = pe->batched ? b.delta : c.delta;
    sh->stats.batched = pe->batched ? 1 : 0;
    sh->stats.batchLanes = pe->batched ? b.lb : 0;
    sh->stats.batchWaves = pe->batched ? b.wpe : 0;
    sh->stats.batchPostWaves = pe->batched && b.split ? (sh->bcfgPost.grid > 0 ? sh->bcfgPost.wpe : b.wpe) : 0;
    return SHD_PE_OK;
}

// Batch order of the table positions: sources of one batch should have
// similar distance profiles so their delta-stepping frontiers coincide.
//   order 0: BFS visit rank (components in vertex order);
//   order 1 (default): nearest-hub cells -- a multi-source Dijkstra from
//            the K highest-degree vertices gives every vertex its closest
//            hub; sources sort by (hub, distance to it), so a batch holds
//            sources that reach the rest of the graph through one hub, and
//            the distance to the hub becomes the lane's bucket key offset
//            (k_batch_rows: a lane's key is dist + maxOff - off).
// Scheduling only: results never depend on it (tools/sim/ models the
// schedule: C4 arc visits 3.9 -> 2.2 x m per batch with offsets, dirty
// lanes and a far set at delta = mean arc latency).
static void compute_ranks(ShdPe* pe) {
    const HostGraph& g = pe->hg;
    std::vector<int32_t> order;
    order.reserve(g.n);
    if (pe->tu.batchOrder == 1) {
        const int32_t K = (int32_t)std::max<int64_t>(1, std::min<int64_t>(256, g.n / 400));
        std::vector<int32_t> byDeg(g.n);
        for (int32_t v = 0; v < g.n; ++v) byDeg[v] = v;
        std::stable_sort(byDeg.begin(), byDeg.end(), [&](int32_t a, int32_t b) {
            return g.rowPtr[a + 1] - g.rowPtr[a] > g.rowPtr[b + 1] - g.rowPtr[b];
        });
        std::vector<double> dist(g.n, INFINITY);
        std::vector<int32_t> owner(g.n, INT32_MAX);
        typedef std::pair<double, int32_t> QE;
        std::priority_queue<QE, std::vector<QE>, std::greater<QE>> q;
        for (int32_t k = 0; k < K; ++k) { dist[byDeg[k]] = 0.0; owner[byDeg[k]] = k; q.push({0.0, byDeg[k]}); }
        while (!q.empty()) {
            const QE top = q.top();
            q.pop();
            const int32_t u = top.second;
            if (top.first > dist[u]) continue;
            for (int32_t a = g.rowPtr[u]; a < g.rowPtr[u + 1]; ++a) {
                const int32_t v = g.col[a];
                const double nd = dist[u] + g.lat[a];
                if (nd < dist[v] || (nd == dist[v] && owner[u] < owner[v])) {
                    dist[v] = nd;
                    owner[v] = owner[u];
                    q.push({nd, v});
                }
            }
        }
        for (int32_t v = 0; v < g.n; ++v) order.push_back(v);
        std::stable_sort(order.begin(), order.end(), [&](int32_t a, int32_t b) {
            return owner[a] != owner[b] ? owner[a] < owner[b] : dist[a] < dist[b];
        });
        // bucket key offsets: a source's distance to its hub, so the lanes of
        // a batch reach the vertices behind the hub in the same bucket
        pe->rowOff.assign(pe->attached.size(), 0.0);
        for (size_t p = 0; p < pe->attached.size(); ++p) {
            const double d = dist[pe->attached[p]];
            pe->rowOff[p] = std::isfinite(d) ? d : 0.0;
        }
    } else {
        std::vector<uint8_t> seen(g.n, 0);
        for (int32_t r = 0; r < g.n; ++r) {
            if (seen[r]) continue;
            seen[r] = 1;
            size_t head = order.size();
            order.push_back(r);
            while (head < order.size()) {
                const int32_t u = order[head++];
                for (int32_t a = g.rowPtr[u]; a < g.rowPtr[u + 1]; ++a) {
                    const int32_t v = g.col[a];
                    if (!seen[v]) { seen[v] = 1; order.push_back(v); }
                }
                if (g.directed) {
                    for (int32_t a = g.inPtr[u]; a < g.inPtr[u + 1]; ++a) {
                        const int32_t v = g.inCol[a];
                        if (!seen[v]) { seen[v] = 1; order.push_back(v); }
                    }
                }
            }
        }
    }
    pe->rank.assign(pe->attached.size(), 0);
    int32_t k = 0;
    for (int32_t v : order)
        if (pe->posOf[v] >= 0) pe->rank[pe->posOf[v]] = k++;
}

// Row-shard plan: G contiguous position ranges with equal numbers of kernel
// work units (a unit = one batch of 16 rows in the batched sparse kernel,
// one row otherwise).  Per-unit cost is near-uniform for this path: every
// SSSP row settles all n vertices, every dense / direct row is n (T) wide
// (measured per-batch cycle spread in DESIGN.md §6), so equal units are the
// balanced split, and contiguous ranges let the all-gather land rows in
// place.  Host-only (no device), exported for the CPU tests.
extern "C" int shd_pe_plan_shards(int32_t T, int32_t G, int32_t unit, int32_t* bounds) {
    if (T < 0 || G < 1 || unit < 1 || !bounds) return SHD_PE_EINVAL;
    const int64_t units = ((int64_t)T + unit - 1) / unit;
    for (int g = 0; g < G; ++g)
        bounds[g] = (int32_t)std::min<int64_t>(T, (units * g / G) * unit);
    bounds[G] = T;
    return SHD_PE_OK;
}

static void plan_shards(ShdPe* pe) {
    pe->bounds.assign(pe->G + 1, 0);
    (void)shd_pe_plan_shards((int32_t)pe->attached.size(), pe->G, pe->batched ? 16 : 1,
                             pe->bounds.data());
}

static void destroy_shard(Shard* s) {
    if (!s) return;
    (void)hipSetDevice(s->device);
    if (s->stream) (void)hipStreamSynchronize(s->stream);
    if (s->comm) (void)ncclCommDestroy(s->comm);
    for (void* p : s->allocs) (void)hipFree(p);
    for (hipEvent_t e : {s->ev0, s->ev1, s->evA, s->evB, s->evP[0], s->evP[1], s->evP[2]})
        if (e) (void)hipEventDestroy(e);
    if (s->stream) (void)hipStreamDestroy(s->stream);
    if (s->copyStream) (void)hipStreamDestroy(s->copyStream);
    if (s->dCoopAbort) (void)hipHostFree(s->dCoopAbort);
}

// Upload the graph as a DevGraph.  oldOf == null: the caller's vertex ids.
// Otherwise device id k is the caller's vertex oldOf[k]: per-vertex arrays
// are permuted and arc targets renamed, but every row keeps its arcs in
// igraph incidence order (ascending CALLER id), so every pop / push order --
// and the tie-breaking that depends on it -- is unchanged; kernels map pred
// back through DevGraph::oldId.
static int upload_graph(ShdPe* pe, Shard* sh, DevGraph* out, const std::vector<int32_t>* oldOf) {
    const HostGraph& g0 = pe->hg;
    const int32_t n = g0.n;
    const int64_t m = g0.nArcs();
    int rc;
    // permuted host copies (only when relabelling)
    std::vector<int32_t> newOf, rp, ip;
    hvec<int32_t> col, o2i, icol;
    hvec<double> lat, rel, ilat, irel, flt, srl;
    std::vector<double> vrel, sl, sr, sml, smr;
    std::vector<uint8_t> hs;
    std::vector<int32_t> att;
    const bool perm = oldOf != nullptr;
    if (perm) {
        const std::vector<int32_t>& od = *oldOf;
        newOf.assign(n, 0);
        for (int32_t k = 0; k < n; ++k) newOf[od[k]] = k;
        rp.assign(n + 1, 0);
        for (int32_t k = 0; k < n; ++k) rp[k + 1] = rp[k] + (g0.rowPtr[od[k] + 1] - g0.rowPtr[od[k]]);
        std::vector<int32_t> arcNew(m);
        col.resize(m); lat.resize(m); rel.resize(m); o2i.resize(m);
        if (g0.latFold) { flt.resize(m); srl.resize(m); }
        for (int32_t k = 0; k < n; ++k) {
            const int32_t u = od[k];
            for (int32_t a = g0.rowPtr[u], j = rp[k]; a < g0.rowPtr[u + 1]; ++a, ++j) {
                arcNew[a] = j;
                col[j] = newOf[g0.col[a]];
                lat[j] = g0.lat[a];
                rel[j] = g0.rel[a];
                if (g0.latFold) { flt[j] = g0.foldLat[a]; srl[j] = g0.selfPathRel[a]; }
            }
        }
        if (g0.directed) {
            ip.assign(n + 1, 0);
            for (int32_t k = 0; k < n; ++k) ip[k + 1] = ip[k] + (g0.inPtr[od[k] + 1] - g0.inPtr[od[k]]);
            std::vector<int32_t> inNew(m);
            icol.resize(m); ilat.resize(m); irel.resize(m);
            for (int32_t k = 0; k < n; ++k) {
                const int32_t v = od[k];
                for (int32_t a = g0.inPtr[v], j = ip[k]; a < g0.inPtr[v + 1]; ++a, ++j) {
                    inNew[a] = j;
                    icol[j] = newOf[g0.inCol[a]];
                    ilat[j] = g0.inLat[a];
                    irel[j] = g0.inRel[a];
                }
            }
            for (int64_t a = 0; a < m; ++a) o2i[arcNew[a]] = inNew[g0.outToIn[a]];
        } else {
            for (int64_t a = 0; a < m; ++a) o2i[arcNew[a]] = arcNew[g0.outToIn[a]];
        }
        vrel.resize(n); sl.resize(n); sr.resize(n); hs.resize(n); sml.resize(n); smr.resize(n);
        for (int32_t k = 0; k < n; ++k) {
            vrel[k] = g0.vrel[od[k]]; sl[k] = g0.selfLat[od[k]];
            sr[k] = g0.selfRel[od[k]]; hs[k] = g0.hasSelf[od[k]];
            sml[k] = g0.selfMinLat[od[k]]; smr[k] = g0.selfMinRel[od[k]];
        }
        att.resize(pe->attached.size());
        for (size_t i = 0; i < att.size(); ++i) att[i] = newOf[pe->attached[i]];
    }
    const std::vector<int32_t>& RP = perm ? rp : g0.rowPtr;
    const hvec<int32_t>& COL = perm ? col : g0.col;
    const hvec<double>& LAT = perm ? lat : g0.lat;
    const hvec<double>& REL = perm ? rel : g0.rel;
    const std::vector<int32_t>& ATT = perm ? att : pe->attached;
    DevGraph d{};
    d.n = n;
    d.T = (int32_t)pe->attached.size();
    std::vector<uint8_t> isAtt(n, 0);
    for (int32_t v : ATT) isAtt[v] = 1;
    int32_t *rowPtr, *dcol, *outToIn, *datt;
    double *dlat, *drel, *dvrel, *dsl, *dsr, *dsml, *dsmr;
    uint8_t *dhs, *ia;
    if ((rc = dev_upload(sh, &rowPtr, RP)) || (rc = dev_upload(sh, &dcol, COL)) ||
        (rc = dev_upload(sh, &dlat, LAT)) || (rc = dev_upload(sh, &drel, REL)) ||
        (rc = dev_upload(sh, &outToIn, perm ? o2i : g0.outToIn)) ||
        (rc = dev_upload(sh, &dvrel, perm ? vrel : g0.vrel)) ||
        (rc = dev_upload(sh, &dsl, perm ? sl : g0.selfLat)) ||
        (rc = dev_upload(sh, &dsr, perm ? sr : g0.selfRel)) ||
        (rc = dev_upload(sh, &dsml, perm ? sml : g0.selfMinLat)) ||
        (rc = dev_upload(sh, &dsmr, perm ? smr : g0.selfMinRel)) ||
        (rc = dev_upload(sh, &dhs, perm ? hs : g0.hasSelf)) || (rc = dev_upload(sh, &datt, ATT)) ||
        (rc = dev_upload(sh, &ia, isAtt)))
        return rc;
    {
        std::vector<Arc> arcs(COL.size());
        for (size_t a = 0; a < arcs.size(); ++a) arcs[a] = Arc{LAT[a], COL[a], 0};
        Arc* da;
        if ((rc = dev_upload(sh, &da, arcs))) return rc;
        d.arcs = da;
        std::vector<Arc3> a3(COL.size());
        for (size_t a = 0; a < a3.size(); ++a) {
            uint64_t bits;
            std::memcpy(&bits, &LAT[a], 8);
            a3[a] = Arc3{COL[a], (uint32_t)bits, (uint32_t)(bits >> 32)};
        }
        Arc3* d3;
        if ((rc = dev_upload(sh, &d3, a3))) return rc;
        d.arc3 = d3;
    }
    d.rowPtr = rowPtr; d.col = dcol; d.lat = dlat; d.rel = drel; d.outToIn = outToIn;
    d.vrel = dvrel; d.selfLat = dsl; d.selfRel = dsr; d.hasSelf = dhs; d.attached = datt;
    d.selfMinLat = dsml; d.selfMinRel = dsmr;
    d.isAttached = ia;
    {
        const int hd = sh->cfg.heavyDeg;
        std::vector<uint32_t> hb((n + 31) / 32, 0u);
        for (int32_t v = 0; v < n; ++v)
            if (RP[v + 1] - RP[v] >= hd) hb[v >> 5] |= 1u << (v & 31);
        uint32_t* dhb;
        if ((rc = dev_upload(sh, &dhb, hb))) return rc;
        d.heavyBits = dhb;
    }
    if (g0.directed) {
        int32_t *dip, *dic;
        double *dil, *dir;
        if ((rc = dev_upload(sh, &dip, perm ? ip : g0.inPtr)) || (rc = dev_upload(sh, &dic, perm ? icol : g0.inCol)) ||
            (rc = dev_upload(sh, &dil, perm ? ilat : g0.inLat)) || (rc = dev_upload(sh, &dir, perm ? irel : g0.inRel)))
            return rc;
        d.inPtr = dip; d.inCol = dic; d.inLat = dil; d.inRel = dir;
    } else {
        d.inPtr = rowPtr; d.inCol = dcol; d.inLat = dlat; d.inRel = drel;
    }
    d.flat = d.srel = nullptr;
    if (g0.latFold) {
        double *dfl, *dsp;
        if ((rc = dev_upload(sh, &dfl, perm ? flt : g0.foldLat)) ||
            (rc = dev_upload(sh, &dsp, perm ? srl : g0.selfPathRel)))
            return rc;
        d.flat = dfl;
        d.srel = dsp;
    }
    d.oldId = nullptr;
    if (perm) {
        int32_t* dold;
        if ((rc = dev_upload(sh, &dold, *oldOf))) return rc;
        d.oldId = dold;
    }
    *out = d;
    return SHD_PE_OK;
}

// Device state of one shard: graph upload, stream, events, kernel config.
static int init_shard(ShdPe* pe, Shard* sh) {
    const HostGraph& g = pe->hg;
    if (hipSetDevice(sh->device) != hipSuccess) return SHD_PE_ENODEV;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, sh->device) != hipSuccess) return SHD_PE_ENODEV;
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) return SHD_PE_ENODEV;
    sh->numCUs = prop.multiProcessorCount;
    if (hipStreamCreateWithFlags(&sh->stream, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&sh->copyStream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreate(&sh->ev0) != hipSuccess || hipEventCreate(&sh->ev1) != hipSuccess ||
        hipEventCreate(&sh->evA) != hipSuccess || hipEventCreate(&sh->evB) != hipSuccess ||
        hipEventCreate(&sh->evP[0]) != hipSuccess || hipEventCreate(&sh->evP[1]) != hipSuccess ||
        hipEventCreate(&sh->evP[2]) != hipSuccess)
        return SHD_PE_ENODEV;
    int rc = configure(pe, sh);
    if (rc) return rc;
    const int32_t T = (int32_t)pe->attached.size();
    if ((rc = upload_graph(pe, sh, &sh->dgAux, nullptr))) return rc;
    sh->dg = sh->dgAux;
    if (pe->batched && pe->tu.relabel == 1) {
        // device ids by descending degree (stable): a wave's groups get
        // vertices of similar degree in the queue and predecessor pass (less
        // divergence), and the hubs' [v][LB] lines sit together
        const int32_t n = g.n;
        std::vector<int32_t> oldOf(n);
        for (int32_t v = 0; v < n; ++v) oldOf[v] = v;
        std::stable_sort(oldOf.begin(), oldOf.end(), [&](int32_t a, int32_t b) {
            return g.rowPtr[a + 1] - g.rowPtr[a] > g.rowPtr[b + 1] - g.rowPtr[b];
        });
        if ((rc = upload_graph(pe, sh, &sh->dg, &oldOf))) return rc;
        if (pe->devOf.empty()) {
            pe->devOf.assign(n, 0);
            for (int32_t k = 0; k < n; ++k) pe->devOf[oldOf[k]] = k;
        }
    }
    sh->stats.mode = pe->mode;
    sh->stats.isComplete = g.isComplete ? 1 : 0;
    sh->stats.nVertices = g.n;
    sh->stats.nArcs = g.nArcs();
    sh->stats.nAttached = T;
    return SHD_PE_OK;
}

static int select_mode(ShdPe* pe) {
    const HostGraph& g = pe->hg;
    int mode = (g.isComplete && pe->opt.forceMode != 1 && pe->opt.forceMode != 3) ? 2 : 1;
    if (pe->opt.forceMode == 2) mode = 2;
    // dense non-complete graphs: blocked min-plus (K2)
    const double density = (double)g.nArcs() / ((double)g.n * (double)g.n);
    const bool fitsDense = (int64_t)g.n <= 65536;
    if (mode == 1 && pe->opt.forceMode == 0 && fitsDense && density >= pe->tu.denseMin) mode = 3;
    if (pe->opt.forceMode == 4 && fitsDense) mode = 3;
    if (pe->opt.forceMode == 5) mode = 1;
    return mode;
}

extern "C" int shd_pe_create(const ShdPeGraphDesc* graph, const int32_t* attached,
                             int32_t nAttached, const ShdPeOptions* opt, ShdPe** out) {
    if (!out || !graph || nAttached <= 0 || !attached) return SHD_PE_EINVAL;
    *out = nullptr;
    std::unique_ptr<ShdPe> pe(new (std::nothrow) ShdPe());
    if (!pe) return SHD_PE_ENOMEM;
    if (opt) pe->opt = *opt; else shd_pe_default_options(&pe->opt);
    ShdPeOptions& o = pe->opt;
    if (o.nDevices <= 0) o.nDevices = 1;
    if (o.shardCount <= 0) o.shardCount = 1;
    if (o.shardIndex < 0 || o.shardIndex >= o.shardCount || o.nDevices > 64) return SHD_PE_EINVAL;
    read_tuning(pe->tu, o.debugFlags);
    int rc = build_host_graph(graph, &pe->hg);
    if (rc) return rc;
    const HostGraph& g = pe->hg;
    pe->posOf.assign(g.n, -1);
    for (int32_t i = 0; i < nAttached; ++i) {
        const int32_t v = attached[i];
        if (v < 0 || v >= g.n) return SHD_PE_EINVAL;
        if (pe->posOf[v] < 0) {
            pe->posOf[v] = (int32_t)pe->attached.size();
            pe->attached.push_back(v);
        }
    }
    const int32_t T = (int32_t)pe->attached.size();
    // ---- devices ----
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return SHD_PE_ENODEV;
    std::vector<int> devs(o.nDevices);
    for (int i = 0; i < o.nDevices; ++i) {
        devs[i] = o.devices ? o.devices[i] : o.device + i;
        if (devs[i] < 0 || devs[i] >= ndev) return SHD_PE_ENODEV;
    }
    pe->mode = select_mode(pe.get());
    pe->G = o.shardCount * o.nDevices;
    pe->firstShard = o.shardIndex * o.nDevices;
    // the batched-kernel decision (and so the shard unit) needs a configured
    // shard: configure a probe on the first device with the whole table
    {
        Shard probe;
        probe.device = devs[0];
        if (hipSetDevice(probe.device) != hipSuccess) return SHD_PE_ENODEV;
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, probe.device) != hipSuccess) return SHD_PE_ENODEV;
        if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) return SHD_PE_ENODEV;
        probe.numCUs = prop.multiProcessorCount;
        probe.rowCount = T;
        if ((rc = configure(pe.get(), &probe))) return rc;
    }
    plan_shards(pe.get());
    pe->ownStart = pe->bounds[pe->firstShard];
    pe->ownEnd = pe->bounds[pe->firstShard + o.nDevices];
    for (int i = 0; i < o.nDevices; ++i) {
        std::unique_ptr<Shard> sh(new (std::nothrow) Shard());
        if (!sh) return SHD_PE_ENOMEM;
        sh->gindex = pe->firstShard + i;
        sh->device = devs[i];
        sh->rowStart = pe->bounds[sh->gindex];
        sh->rowCount = pe->bounds[sh->gindex + 1] - sh->rowStart;
        sh->fullOwner = std::find(devs.begin(), devs.begin() + i, devs[i]) == devs.begin() + i;
        rc = init_shard(pe.get(), sh.get());
        pe->shards.push_back(std::move(sh));
        if (rc) { shd_pe_destroy(pe.release()); return rc; }
    }
    if (pe->mode == 1 && pe->batched) compute_ranks(pe.get());
    pe->rowDone.reset(new (std::nothrow) std::atomic<uint8_t>[T]);
    if (!pe->rowDone) { shd_pe_destroy(pe.release()); return SHD_PE_ENOMEM; }
    for (int32_t i = 0; i < T; ++i) pe->rowDone[i].store(0, std::memory_order_relaxed);
    *out = pe.release();
    return SHD_PE_OK;
}

static int ensure_table(ShdPe* pe, Shard* sh) {
    if (sh->tableReady) return SHD_PE_OK;
    const size_t T = pe->attached.size();
    const size_t cells = (size_t)sh->rowCount * T;
    int rc;
    void *lat, *rel, *hops, *flags, *pred = nullptr;
    if ((rc = dev_alloc(sh, &lat, cells * 8)) || (rc = dev_alloc(sh, &rel, cells * 8)) ||
        (rc = dev_alloc(sh, &hops, cells * 4)) || (rc = dev_alloc(sh, &flags, cells)))
        return rc;
    if (pe->opt.storePred && (rc = dev_alloc(sh, &pred, cells * 4))) return rc;
    sh->tab.lat = (double*)lat;
    sh->tab.rel = (double*)rel;
    sh->tab.hops = (int32_t*)hops;
    sh->tab.flags = (uint8_t*)flags;
    sh->tab.pred = (int32_t*)pred;
    sh->tab.T = (int64_t)T;
    sh->tab.rowStart = sh->rowStart;
    // scratch slots
    const int slots = pe->batched ? sh->exactGrid : std::max(sh->cfg.grid, sh->exactGrid);
    const size_t stride = ((size_t)pe->hg.n + 63) & ~(size_t)63;
    const size_t heapStride = std::max<size_t>(1, (size_t)pe->hg.n - (size_t)sh->exactHc);
    void *dist, *sho, *sr, *sp, *hk, *i2;
    if ((rc = dev_alloc(sh, &dist, slots * stride * 8)) ||
        (rc = dev_alloc(sh, &sho, slots * stride * 4)) ||
        (rc = dev_alloc(sh, &sr, slots * stride * 8)) ||
        (rc = dev_alloc(sh, &sp, slots * stride * 4)) ||
        (rc = dev_alloc(sh, &hk, (size_t)sh->exactGrid * heapStride * 16)) ||
        (rc = dev_alloc(sh, &i2, (size_t)sh->exactGrid * stride * 4)))
        return rc;
    sh->sc.dist = (double*)dist;
    sh->sc.hops = (int32_t*)sho;
    sh->sc.rel = (double*)sr;
    sh->sc.pred = (int32_t*)sp;
    sh->sc.heapTail = (double*)hk;
    sh->sc.heapStride = (int64_t)heapStride;
    sh->sc.index2 = (int32_t*)i2;
    sh->sc.stride = (int64_t)stride;
    sh->sc.lfold = nullptr;
    if (pe->hg.latFold) {
        void* lf;
        if ((rc = dev_alloc(sh, &lf, slots * stride * 8))) return rc;
        sh->sc.lfold = (double*)lf;
    }
    if (!pe->batched && (sh->cfg.layout == 3 || sh->cfg.layout == 0)) {
        void* q;
        const size_t per = 2 * ((size_t)sh->cfg.qcap + sh->cfg.hcap);
        if ((rc = dev_alloc(sh, &q, (size_t)sh->cfg.grid * per * 4))) return rc;
        sh->sc.queue = (int32_t*)q;
    }
    sh->rowsCap = (int32_t)std::max<size_t>(1, std::min<size_t>(sh->rowCount, 1 << 20));
    void *rows, *amb;
    if ((rc = dev_alloc(sh, &rows, (size_t)sh->rowsCap * 4)) ||
        (rc = dev_alloc(sh, &amb, (size_t)sh->rowsCap)))
        return rc;
    sh->dRows = (int32_t*)rows;
    sh->dRowAmbig = (uint8_t*)amb;
    if (pe->tu.debug) {
        void* dbg;
        if ((rc = dev_alloc(sh, &dbg, (size_t)sh->rowsCap * 64))) return rc;
        sh->dDbg = (int32_t*)dbg;
        void* xd;
        if ((rc = dev_alloc(sh, &xd, (size_t)sh->rowsCap * 64))) return rc;
        sh->dXdbg = (long long*)xd;
    }
    sh->tableReady = true;
    return SHD_PE_OK;
}

// Tie slots for the early-stop emulation (both sparse paths): D f64 + P i32
// + H i32 + R f64 per vertex, <= 2 GiB, <= 254 slots (rowAmbig stores
// 2 + slot in a byte); arc indices carry TIE_AMB in bit 30.
static int ensure_tie(ShdPe* pe, Shard* sh) {
    if (sh->dTie || sh->tieTried) return SHD_PE_OK;
    sh->tieTried = true;
    int rc;
    const size_t perTie = (size_t)pe->hg.n * 24;
    // (the dense path, mode 3, keeps slots out of rowAmbig's byte: more of them,
    // so its early-stop tie rows run in one launch)
    size_t cap = std::min<size_t>({pe->mode == 3 ? (size_t)4096 : (size_t)254, (size_t)sh->rowsCap,
                                   ((size_t)2 << 30) / perTie});
    if (pe->hg.nArcs() >= ((int64_t)1 << 30)) cap = 0;
    if (cap > 0) {
        void *td, *tp, *th, *tr, *tt, *tc, *sl, *dd, *rq;
        const size_t cn = cap * (size_t)pe->hg.n;
        if ((rc = dev_alloc(sh, &td, cn * 8)) || (rc = dev_alloc(sh, &tp, cn * 4)) ||
            (rc = dev_alloc(sh, &th, cn * 4)) || (rc = dev_alloc(sh, &tr, cn * 8)) ||
            (rc = dev_alloc(sh, &tt, cap * 8)) || (rc = dev_alloc(sh, &tc, 16)) ||
            (rc = dev_alloc(sh, &sl, (size_t)sh->rowsCap * 4)) ||
            (rc = dev_alloc(sh, &dd, sizeof(TieBuf))) || (rc = dev_alloc(sh, &rq, cap * 16)))
            return rc;
        // (tc: [0] slot counter, [1] the round word of the deferred export;
        // the batched path's post kernel defers its export to k_tie_export)
        sh->tie = TieBuf{(int32_t)cap, (int32_t*)tc, (double*)td, (int32_t*)tp, (double*)tt,
                         (int32_t*)th, (double*)tr, (int64_t)pe->hg.n,
                         pe->batched ? (int32_t*)rq : nullptr, (int32_t*)tc + 1};
        sh->dSlots = (int32_t*)sl;
        sh->dTie = (TieBuf*)dd;
        HIPCHK(hipMemcpy(sh->dTie, &sh->tie, sizeof(TieBuf), hipMemcpyHostToDevice));
    }
    return SHD_PE_OK;
}

static int ensure_batch(ShdPe* pe, Shard* sh) {
    if (sh->batchReady) return SHD_PE_OK;
    const size_t NS = ((size_t)pe->hg.n + 63) & ~(size_t)63;
    const size_t LB = (size_t)sh->bcfg.lb;
    const size_t bitBytes = sh->bcfg.gbits ? (size_t)batch_bits_words(pe->hg.n) * 4 : 0;
    const size_t perSlot = NS * LB * (8 + 16) + NS * 4 + bitBytes;   // D, L
    // scratch budget (default 64 GiB): fewer resident batches on huge graphs
    const double budget = pe->tu.batchScratchGB * (double)(1ull << 30);
    const size_t maxSlots = std::max<size_t>(1, (size_t)(budget / (double)perSlot));
    const size_t nBatchesAll = ((size_t)sh->rowCount + LB - 1) / LB;
    const size_t grid = (size_t)std::max({sh->bcfg.grid, sh->bcfgAlt.grid, sh->bcfgAlt2.grid});
    // (a cooperative launch needs one slot per resident workgroup: its grid
    // is the whole resident set, more workgroups than batches)
    const size_t coGrid = sh->bcfgCoop.grid > 0 ? (size_t)sh->bcfgCoop.grid : 0;
    const size_t slots = std::min<size_t>({std::max(grid, coGrid), maxSlots,
                                          std::max<size_t>({(size_t)1, nBatchesAll, coGrid})});
    if (coGrid > slots) {                          // scratch budget: no cooperative relax
        if (sh->bcfg.coop >= 2) { sh->bcfg = sh->bcfgPost.grid > 0 ? sh->bcfgPost : sh->bcfg; sh->bcfg.coop = 0; }
        sh->bcfgCoop = BatchLaunch{};
    }
    sh->bcfg.grid = (int32_t)std::min<size_t>(slots, (size_t)sh->bcfg.grid);
    if (sh->bcfgAlt.grid > 0) sh->bcfgAlt.grid = (int32_t)std::min<size_t>(slots, (size_t)sh->bcfgAlt.grid);
    if (sh->bcfgAlt2.grid > 0) sh->bcfgAlt2.grid = (int32_t)std::min<size_t>(slots, (size_t)sh->bcfgAlt2.grid);
    int rc;
    // split kernels: one persisted dist array per batch of a round (relax ->
    // post), the rest per resident workgroup; rounds sized by free memory
    // (at most 160 GiB of dist arrays: C4 one round of 13 GB, C5 one round
    // of 131 GB beside its 107 GB table -- 2 rounds under a 96 GiB cap were
    // 5% slower, profiles/r04_ab_notes.txt r04i)
    size_t roundB = slots;
    if (sh->bcfg.split) {
        size_t freeB = 0, totalB = 0;
        if (hipMemGetInfo(&freeB, &totalB) != hipSuccess) freeB = (size_t)16 << 30;
        const size_t perD = NS * LB * 8;
        const size_t rest = slots * (perSlot - NS * LB * 8);
        const size_t room = freeB > rest + ((size_t)12 << 30) ? freeB - rest - ((size_t)12 << 30) : perD;
        const size_t dBudget = std::min<size_t>(room, (size_t)160 << 30);
        roundB = std::max<size_t>(slots, std::min<size_t>(nBatchesAll, dBudget / perD));
    }
    sh->batchRound = (int32_t)roundB;
    sh->batchSlots = (int32_t)slots;
    void *D, *L, *q, *rows, *amb, *fl;
    if ((rc = dev_alloc(sh, &D, roundB * NS * LB * 8)) || (rc = dev_alloc(sh, &L, slots * NS * LB * 16)) ||
        (rc = dev_alloc(sh, &q, slots * NS * 4 + 64)) ||
        (rc = dev_alloc(sh, &rows, ((size_t)sh->rowsCap + 64) * 4)) ||
        (rc = dev_alloc(sh, &amb, (size_t)sh->rowsCap + 64)) || (rc = dev_alloc(sh, &fl, roundB * 4 + 64)))
        return rc;
    sh->bsc.flags = (int32_t*)fl;
    sh->bsc.D = (unsigned long long*)D;
    sh->bsc.L = (BLabel*)L;
    sh->bsc.queue = (int32_t*)q;
    sh->bsc.next = (int32_t*)q + slots * NS;
    sh->bsc.nStride = (int64_t)NS;
    sh->bsc.bits = nullptr;
    if (bitBytes) {
        void* bits;
        if ((rc = dev_alloc(sh, &bits, slots * bitBytes))) return rc;
        sh->bsc.bits = (uint32_t*)bits;
    }
    sh->bsc.rowOff = nullptr;
    if (!pe->rowOff.empty()) {
        double* ro;
        if ((rc = dev_upload(sh, &ro, pe->rowOff))) return rc;
        sh->bsc.rowOff = ro;
    }
    sh->dBatchRows = (int32_t*)rows;
    sh->dBatchAmb = (uint8_t*)amb;
    if (sh->bcfgCoop.grid > 0) {
        // cooperative relax state: control words, one barrier line per group,
        // two publication buffers of near bits + scalars per member per group
        const size_t maxGroups = (size_t)sh->bcfgCoop.grid;
        const size_t K = (size_t)sh->bcfgCoop.coop;
        const size_t nwp = (size_t)batch_bits_words(pe->hg.n) / 2;
        void *cc, *pub, *pubS;
        if ((rc = dev_alloc(sh, &cc, 128 + maxGroups * 128)) ||
            (rc = dev_alloc(sh, &pub, maxGroups * 2 * K * nwp * 4)) ||
            (rc = dev_alloc(sh, &pubS, maxGroups * 2 * K * 16)))
            return rc;
        sh->bsc.coCtl = (int32_t*)cc;
        sh->bsc.coBars = (int32_t*)cc + 32;
        sh->bsc.coPub = (uint32_t*)pub;
        sh->bsc.coPubS = (unsigned long long*)pubS;
        sh->bsc.coK = (int32_t)K;
        sh->bsc.coSpin = pe->tu.coopSpin;
        if (hipHostMalloc(reinterpret_cast<void**>(&sh->dCoopAbort), 4, hipHostMallocDefault) != hipSuccess)
            return SHD_PE_ENOMEM;
    }
    if ((rc = ensure_tie(pe, sh))) return rc;
    sh->batchReady = true;
    return SHD_PE_OK;
}

static int ensure_dense(ShdPe* pe, Shard* sh) {
    if (sh->dW) return SHD_PE_OK;
    const int64_t n = pe->hg.n;
    const int64_t R = std::max<int32_t>(1, sh->rowCount);
    int rc;
    void *w, *rl, *d, *p, *ra, *rb, *am, *any, *ce;
    // rows per batch: D (f64) + P (i32) per row
    const int64_t budget = (int64_t)(pe->tu.denseBatchGB * (double)(1LL << 30));
    int64_t rows = std::max<int64_t>(64, budget / (n * 12));
    rows = std::min<int64_t>(rows, R);
    if ((rc = dev_alloc(sh, &w, (size_t)(n * n * 8))) || (rc = dev_alloc(sh, &rl, (size_t)(n * n * 8))) ||
        (rc = dev_alloc(sh, &d, (size_t)(rows * n * 8))) || (rc = dev_alloc(sh, &p, (size_t)(rows * n * 4))) ||
        (rc = dev_alloc(sh, &ra, (size_t)rows)) || (rc = dev_alloc(sh, &rb, (size_t)rows)) ||
        (rc = dev_alloc(sh, &am, (size_t)rows)) || (rc = dev_alloc(sh, &any, 16)) ||
        (rc = dev_alloc(sh, &ce, (size_t)((rows / 16 + 1) * (n / 16 + 1)))))
        return rc;
    sh->dChunkEpoch = (uint8_t*)ce;
    sh->dW = (double*)w; sh->dRl = (double*)rl; sh->dD = (double*)d; sh->dP = (int32_t*)p;
    sh->dRowA = (uint8_t*)ra; sh->dRowB = (uint8_t*)rb; sh->dRowAmbD = (uint8_t*)am;
    sh->dAny = (int32_t*)any;
    sh->denseRows = (int32_t)rows;
    launch_dense_build(sh->dg, sh->dW, sh->dRl, n, pe->hg.nArcs(), sh->stream);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(sh->stream));
    return SHD_PE_OK;
}

static float elapsed(hipEvent_t a, hipEvent_t b) {
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, a, b);
    return ms;
}

// Kernel counters of k_batch_rows (SHD_PE_DEBUG_COUNTERS): phase cycles,
// re-visits, jump rounds, per-batch cost spread.
static void print_batch_debug(ShdPe* pe, Shard* sh, const int32_t* d0, int32_t nB) {
    double ph = 0, pr = 0, kc[5] = {0, 0, 0, 0, 0}, arcsP = 0, lanesP = 0, bmax = 0, bmean = 0, cand = 0,
           walks = 0;
    long ambB = 0, rep = 0;
    double tMin = 1e30, tMax = 0, tSum = 0, tSq = 0;
    for (int32_t i = 0; i < nB; ++i) {
        const int32_t* d = d0 + 16 * i;
        ph += d[0];
        ambB += d[3] != 0;
        rep += d[15];
        pr += d[4];
        double tb = 0;
        for (int k = 0; k < 3; ++k) { kc[k] += 1024.0 * d[5 + k]; tb += 1024.0 * d[5 + k]; }
        kc[3] += 1024.0 * d[11]; tb += 1024.0 * d[11];
        kc[4] += 1024.0 * d[8]; tb += 1024.0 * d[8];
        tMin = std::min(tMin, tb); tMax = std::max(tMax, tb); tSum += tb; tSq += tb * tb;
        arcsP += 16.0 * d[9];
        bmax += 1024.0 * d[12]; bmean += 1024.0 * d[13]; cand += d[14];
        lanesP += d[10];
        walks += 1024.0 * d[2];
    }
    const double mean = tSum / std::max(nB, 1);
    const double sd = std::sqrt(std::max(0.0, tSq / std::max(nB, 1) - mean * mean));
    std::fprintf(stderr, "[shdpe] shard %d batch relax Mcycles/batch: sum over phases of group-busy max=%.2f mean=%.2f | candidates/batch=%.0f\n",
                 sh->gindex, bmax / nB / 1e6, bmean / nB / 1e6, cand / nB);
    std::fprintf(stderr, "[shdpe] batch arc-visits/batch=%.0f (%.2f x nArcs) active lanes/proc=%.2f\n",
                 arcsP / nB, arcsP / nB / (double)pe->hg.nArcs(), lanesP / std::max(pr, 1.0));
    std::fprintf(stderr, "[shdpe] batch Mcycles/batch: relax=%.2f pred=%.2f labels+write=%.2f (walks %.2f) tie-export=%.2f tail=%.2f | "
                 "per-batch total min=%.2f mean=%.2f max=%.2f sd=%.2f\n", kc[0] / nB / 1e6, kc[1] / nB / 1e6,
                 kc[2] / nB / 1e6, walks / nB / 1e6, kc[3] / nB / 1e6, kc[4] / nB / 1e6, tMin / 1e6, mean / 1e6,
                 tMax / 1e6, sd / 1e6);
    // SHDPE_DIAG_WHY builds: per reason bit, the batches it fired in
    long why[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    bool anyWhy = false;
    for (int32_t i = 0; i < nB; ++i)
        for (int k = 0; k < 8; ++k)
            if ((d0[16 * i + 1] >> k) & 1) { ++why[k]; anyWhy = true; }
    if (anyWhy)
        std::fprintf(stderr, "[shdpe] batch why: failed=%ld viol-ondemand=%ld viol-full=%ld noparent=%ld "
                     "ambiguous=%ld deep=%ld fullpass=%ld relax-flag=%ld\n", why[0], why[1], why[2],
                     why[3], why[4], why[5], why[6], why[7]);
    std::fprintf(stderr, "[shdpe] batch LB=%d batches=%d grid=%d delta=%.3f | phases/batch=%.1f "
                 "vertex-procs/batch=%.0f (%.2f per vertex) | tie batches=%ld repairs=%ld\n",
                 sh->bcfg.lb, nB, sh->bcfg.grid, sh->bcfg.delta, ph / nB, pr / nB,
                 pr / nB / pe->hg.n, ambB, rep);
}

static void print_sparse_debug(ShdPe* pe, Shard* sh, const int32_t* dbg, int32_t cnt) {
    double ph = 0, cy[4] = {0, 0, 0, 0}, sub[4] = {0, 0, 0, 0};
    int phMax = 0, jMax = 0, mis = 0, am = 0;
    long jSum = 0;
    for (int32_t i = 0; i < cnt; ++i) {
        const int32_t* d = dbg + 16 * i;
        ph += d[0]; phMax = std::max(phMax, d[0]);
        jMax = std::max(jMax, d[1]); jSum += d[1];
        mis += d[2] != 0; am += d[3] != 0;
        for (int k = 0; k < 4; ++k) cy[k] += 16.0 * d[4 + k];
        for (int k = 0; k < 4; ++k) sub[k] += 16.0 * d[8 + k];
    }
    std::fprintf(stderr,
                 "[shdpe] shard %d sparse rows=%d phases mean=%.1f max=%d | mismatch rows=%d "
                 "jacobi rounds sum=%ld max=%d | ambiguous rows=%d | delta=%.3f | "
                 "kcycles/row scan=%.1f relax=%.1f final=%.1f write=%.1f | "
                 "cyc/phase bits=%.0f resv=%.0f light=%.0f heavy=%.0f\n",
                 sh->gindex, cnt, ph / cnt, phMax, mis, jSum, jMax, am, sh->cfg.delta,
                 cy[0] / cnt / 1e3, cy[1] / cnt / 1e3, cy[2] / cnt / 1e3, cy[3] / cnt / 1e3,
                 sub[0] / ph, sub[1] / ph, sub[2] / ph, sub[3] / ph);
    (void)pe;
}

// k_exact_rows counters: per row pops, pushes and cycles per pop segment.
static void print_exact_debug(Shard* sh, const std::vector<int32_t>& rows, int32_t nTie) {
    std::vector<long long> x(rows.size() * 8);
    if (hipMemcpy(x.data(), sh->dXdbg, x.size() * 8, hipMemcpyDeviceToHost) != hipSuccess) return;
    for (size_t i = 0; i < rows.size(); ++i) {
        const long long* c = &x[i * 8];
        const double p = (double)std::max<long long>(c[5], 1);
        std::fprintf(stderr, "[shdpe] exact row %d (%s): pops=%lld pushes+mods=%lld heap_end=%lld | "
                     "cyc/pop top=%.0f sink=%.0f arcs=%.0f push=%.0f fence=%.0f total=%.0f\n",
                     rows[i], (int32_t)i < nTie ? "early" : "full", c[5], c[6], c[7], c[0] / p,
                     c[1] / p, c[2] / p, c[3] / p, c[4] / p, (c[0] + c[1] + c[2] + c[3] + c[4]) / p);
    }
}

// SHDPE_TIE_CORRUPT (tests): after the relevance scan, halve the exported
// distances of the first early-stop slot that still needs the emulation --
// what a slot filled from another source's distance array would hold.  The
// exact kernel's consistency check must catch it (rowsTieRepaired).
static void corrupt_tie_slot(ShdPe* pe, Shard* sh, const std::vector<int32_t>& slots, int32_t nTie) {
    std::vector<double> thr((size_t)sh->tie.cap), d((size_t)pe->hg.n);
    if (hipStreamSynchronize(sh->stream) != hipSuccess ||
        hipMemcpy(thr.data(), sh->tie.thr, thr.size() * 8, hipMemcpyDeviceToHost) != hipSuccess)
        return;
    for (int32_t i = 0; i < nTie; ++i) {
        const int sl = slots[i];
        if (!(thr[(size_t)sl] > 0.0)) continue;
        double* dd = sh->tie.D + (size_t)sl * (size_t)sh->tie.n;
        if (hipMemcpy(d.data(), dd, d.size() * 8, hipMemcpyDeviceToHost) != hipSuccess) return;
        // 1: another source's array (halved distances); 2: an array whose
        // own source is not at 0 (every distance shifted)
        for (double& x : d) x = pe->tu.tieCorrupt == 2 ? x + 1.0 : x * 0.5;
        (void)hipMemcpy(dd, d.data(), d.size() * 8, hipMemcpyHostToDevice);
        return;
    }
}

// One round's relax by the cooperative kernel (K workgroups of one XCD per
// batch): its control state zeroed and the round's per-batch failure flags
// cleared by the host first.  If the runtime refuses the launch (the grid is
// not wholly resident) or a barrier wait aborted, the plain relax recomputes
// the round from scratch (it re-initialises every dist array it relaxes and
// writes every flag): the rows are never wrong and never missing.
// A cooperative launch takes every workgroup slot of its device: two of them
// at once (logical shards of one device, computed by concurrent host
// threads) could each hold part of the device while waiting for the rest of
// their own grid.  One at a time per device (the launch is synchronised
// before the lock is released, for the abort check anyway).
static std::mutex g_coopMu[64];

static int relax_coop(ShdPe* pe, Shard* sh, const BatchLaunch& relax, const int32_t* rows, int32_t rn,
                      uint8_t* amb, int32_t* dbg) {
    std::lock_guard<std::mutex> devLock(g_coopMu[sh->device & 63]);
    const size_t maxGroups = (size_t)sh->bcfgCoop.grid;
    HIPCHK(hipMemsetAsync(sh->bsc.coCtl, 0, 128 + maxGroups * 128, sh->stream));
    HIPCHK(hipMemsetAsync(sh->bsc.flags, 0, (size_t)rn * 4, sh->stream));
    BatchLaunch co = relax;
    co.grid = std::min(co.grid, sh->batchSlots);
    bool rerun = launch_batch_relax_coop(sh->dg, sh->tab, sh->bsc, rows, rn, amb, co, dbg, sh->dTie,
                                         sh->stream) != 0;
    if (rerun) {
        (void)hipGetLastError();                  // the refusal
    } else {
        HIPCHK(hipGetLastError());
        HIPCHK(hipMemcpyAsync(sh->dCoopAbort, sh->bsc.coCtl + 17, 4, hipMemcpyDeviceToHost, sh->stream));
        HIPCHK(hipStreamSynchronize(sh->stream));
        rerun = *sh->dCoopAbort != 0;
    }
    if (rerun) {
        ++sh->coopAborts;
        if (pe->tu.debug || pe->tu.tuneLog)
            std::fprintf(stderr, "[shdpe] shard %d: cooperative relax %s; round recomputed by the plain relax\n",
                         sh->gindex, *sh->dCoopAbort ? "aborted" : "refused");
        BatchLaunch plain = relax;
        plain.coop = 0;
        plain.grid = std::min(plain.grid, sh->batchSlots);
        HIPCHK(hipMemsetAsync(sh->bsc.next, 0, 4, sh->stream));
        launch_batch_rows(sh->dg, sh->tab, sh->bsc, rows, rn, amb, plain, dbg, sh->dTie, sh->stream, 1);
        HIPCHK(hipGetLastError());
    }
    return SHD_PE_OK;
}

// Compute the given table positions (all owned by `sh`), chunked.
static int compute_shard(ShdPe* pe, Shard* sh, const int32_t* pos, int32_t count) {
    if (count <= 0) return SHD_PE_OK;
    sh->pathSrc = -1;               // the exact kernels reuse slot 0
    if (hipSetDevice(sh->device) != hipSuccess) return SHD_PE_EHIP;
    int rc = ensure_table(pe, sh);
    if (rc) return rc;
    std::vector<uint8_t> amb;
    std::vector<int32_t> exactRows, exactSlots, fullRows;
    std::vector<int32_t> denseIdx;   // dense tie rows: their row of D / P (one dense chunk only)
    ShdPeStats& st = sh->stats;
    HIPCHK(hipEventRecord(sh->ev0, sh->stream));
    for (int32_t c0 = 0; c0 < count; c0 += sh->rowsCap) {
        const int32_t cnt = std::min(sh->rowsCap, count - c0);
        HIPCHK(hipMemcpyAsync(sh->dRows, pos + c0, (size_t)cnt * 4, hipMemcpyHostToDevice,
                              sh->stream));
        exactRows.clear();
        exactSlots.clear();
        denseIdx.clear();
        if (pe->mode == 2) {
            HIPCHK(hipEventRecord(sh->evA, sh->stream));
            launch_direct_rows(sh->dg, sh->tab, sh->dRows, cnt, sh->stream);
            HIPCHK(hipGetLastError());
            HIPCHK(hipEventRecord(sh->evB, sh->stream));
            HIPCHK(hipEventSynchronize(sh->evB));
            st.msDirectKernel += elapsed(sh->evA, sh->evB);
            st.launchesDirect++;
        } else if (pe->opt.forceMode == 3 || pe->hg.latFold) {
            // (latFold multigraphs: the reported latency is a fold of other
            // edges' latencies than the distance's -- the exact emulation
            // carries it as a label, so every row takes that path)
            exactRows.assign(pos + c0, pos + c0 + cnt);
        } else if (pe->mode == 3) {
            if ((rc = ensure_dense(pe, sh))) return rc;
            for (int32_t d0 = 0; d0 < cnt; d0 += sh->denseRows) {
                const int32_t dc = std::min(sh->denseRows, cnt - d0);
                HIPCHK(hipEventRecord(sh->evA, sh->stream));
                int sweeps = 0;
                double flops = 0.0;
                if (launch_dense_rows(sh->dg, sh->tab, sh->dW, sh->dRl, sh->dD, sh->dP, sh->dRowA,
                                      sh->dRowB, sh->dRowAmbD, sh->dAny, sh->dChunkEpoch,
                                      sh->dRows + d0, dc, pe->hg.n, pe->tu, sh->stream, &sweeps,
                                      &flops))
                    return SHD_PE_EHIP;
                HIPCHK(hipGetLastError());
                HIPCHK(hipEventRecord(sh->evB, sh->stream));
                amb.resize(dc);
                HIPCHK(hipMemcpyAsync(amb.data(), sh->dRowAmbD, dc, hipMemcpyDeviceToHost,
                                      sh->stream));
                HIPCHK(hipStreamSynchronize(sh->stream));
                st.msDenseKernel += elapsed(sh->evA, sh->evB);
                st.launchesDense++;
                st.denseSweeps += sweeps;
                st.denseFlops += flops;
                for (int32_t i = 0; i < dc; ++i)
                    if (amb[i]) {
                        exactRows.push_back(pos[c0 + d0 + i]);
                        if (dc == cnt) denseIdx.push_back(i);   // D / P still hold the row
                    }
            }
        } else if (pe->batched) {
            if ((rc = ensure_batch(pe, sh))) return rc;
            // batches of LB nearby sources (BFS rank order), -1 pads the last
            const int LB = sh->bcfg.lb;
            std::vector<int32_t> order(pos + c0, pos + c0 + cnt);
            std::stable_sort(order.begin(), order.end(),
                             [&](int32_t a, int32_t b) { return pe->rank[a] < pe->rank[b]; });
            const int32_t nB = (cnt + LB - 1) / LB;
            order.resize((size_t)nB * LB, -1);
            if (!pe->rowOff.empty() && nB > 1) {
                // longest batches first (workgroups take batches in order, so
                // the last round is made of short ones): a batch's cost grows
                // with its sources' mean distance to their hub (tools/sim/:
                // correlation 0.53 with arc visits at C4)
                std::vector<std::pair<double, int32_t>> key(nB);
                for (int32_t b = 0; b < nB; ++b) {
                    double s = 0.0;
                    int c = 0;
                    for (int l = 0; l < LB; ++l) {
                        const int32_t p = order[(size_t)b * LB + l];
                        if (p >= 0) { s += pe->rowOff[p]; ++c; }
                    }
                    key[b] = {c ? -s / c : 0.0, b};
                }
                std::stable_sort(key.begin(), key.end());
                std::vector<int32_t> re((size_t)nB * LB);
                for (int32_t i = 0; i < nB; ++i)
                    std::copy(order.begin() + (size_t)key[i].second * LB,
                              order.begin() + (size_t)(key[i].second + 1) * LB, re.begin() + (size_t)i * LB);
                order.swap(re);
            }
            HIPCHK(hipMemcpyAsync(sh->dBatchRows, order.data(), order.size() * 4,
                                  hipMemcpyHostToDevice, sh->stream));
            if (sh->dDbg) HIPCHK(hipMemsetAsync(sh->dDbg, 0, (size_t)nB * 64, sh->stream));
            if (sh->tie.cap > 0) HIPCHK(hipMemsetAsync(sh->tie.count, 0, 4, sh->stream));
            HIPCHK(hipMemsetAsync(sh->bsc.next, 0, 4, sh->stream));
            HIPCHK(hipEventRecord(sh->evA, sh->stream));
            // a workgroup indexes its scratch slot by blockIdx: never launch
            // more workgroups than ensure_batch allocated slots for
            BatchLaunch relax = sh->bcfg;
            relax.grid = std::min(relax.grid, sh->batchSlots);
            if (!sh->bcfg.split) {
                launch_batch_rows(sh->dg, sh->tab, sh->bsc, sh->dBatchRows, nB, sh->dBatchAmb, relax,
                                  sh->dDbg, sh->dTie, sh->stream, 0);
            } else {
                // rounds of batches: relax all of them, then the post kernel
                // over the same batches (their dist arrays persist in HBM)
                // (the post kernel may run another variant: bcfgPost)
                BatchLaunch post = sh->bcfgPost.grid > 0 ? sh->bcfgPost : sh->bcfg;
                post.grid = std::min(post.grid, sh->batchSlots);
                for (int32_t r0 = 0; r0 < nB; r0 += sh->batchRound) {
                    const int32_t rn = std::min(sh->batchRound, nB - r0);
                    const size_t ro = (size_t)r0 * LB;
                    if (sh->timeParts) HIPCHK(hipEventRecord(sh->evP[0], sh->stream));
                    for (int part = 1; part <= 2; ++part) {
                        int32_t* const dbgR = sh->dDbg ? sh->dDbg + 16 * r0 : nullptr;
                        if (part == 1 && relax.coop >= 2 && sh->bcfgCoop.grid > 0) {
                            if ((rc = relax_coop(pe, sh, relax, sh->dBatchRows + ro, rn, sh->dBatchAmb + ro,
                                                 dbgR)))
                                return rc;
                        } else {
                            HIPCHK(hipMemsetAsync(sh->bsc.next, 0, 4, sh->stream));
                            launch_batch_rows(sh->dg, sh->tab, sh->bsc, sh->dBatchRows + ro, rn,
                                              sh->dBatchAmb + ro, part == 1 ? relax : post, dbgR, sh->dTie,
                                              sh->stream, part);
                        }
                        // tests only (SHDPE_TUNE_FAIL_WPE): the relax variant of that wave
                        // count flags every batch failed, as a miscompiled variant would
                        if (part == 1 && pe->tu.failWpe && relax.wpe == pe->tu.failWpe)
                            HIPCHK(hipMemsetAsync(sh->bsc.flags, 1, (size_t)rn * 4, sh->stream));
                        if (sh->timeParts) HIPCHK(hipEventRecord(sh->evP[part], sh->stream));
                        // the post kernel's deferred tie export of this round
                        // (the round's dist arrays persist until the next
                        // round's relax)
                        if (part == 1 && sh->tie.req)
                            HIPCHK(hipMemsetD32Async((hipDeviceptr_t)sh->tie.round, r0 / sh->batchRound, 1,
                                                     sh->stream));
                        if (part == 2 && sh->tie.req)
                            launch_tie_export(sh->dg, sh->bsc, LB, sh->tie, r0 / sh->batchRound,
                                              sh->dBatchAmb + ro, sh->numCUs * 4,
                                              pe->tu.tieCorrupt == 3 ? 0 : -1, sh->stream);
                    }
                    if (sh->timeParts) {
                        HIPCHK(hipEventSynchronize(sh->evP[2]));
                        sh->msPart[0] += elapsed(sh->evP[0], sh->evP[1]);
                        sh->msPart[1] += elapsed(sh->evP[1], sh->evP[2]);
                    }
                }
            }
            HIPCHK(hipGetLastError());
            HIPCHK(hipEventRecord(sh->evB, sh->stream));
            amb.resize(order.size());
            HIPCHK(hipMemcpyAsync(amb.data(), sh->dBatchAmb, order.size(), hipMemcpyDeviceToHost,
                                  sh->stream));
            HIPCHK(hipStreamSynchronize(sh->stream));
            st.msSparseKernel += elapsed(sh->evA, sh->evB);
            st.launchesSparse++;
            // early-stop tie rows first (k_tie_write takes that prefix),
            // then rows needing the full emulation
            fullRows.clear();
            for (size_t i = 0; i < order.size(); ++i) {
                if (order[i] < 0 || !amb[i]) continue;
                if (amb[i] >= 2) {
                    exactRows.push_back(order[i]);
                    exactSlots.push_back(amb[i] - 2);
                } else {
                    fullRows.push_back(order[i]);
                }
            }
            if (!exactSlots.empty()) {
                exactRows.insert(exactRows.end(), fullRows.begin(), fullRows.end());
                exactSlots.resize(exactRows.size(), -1);
            } else {
                exactRows.swap(fullRows);
            }
            if (sh->dDbg) {
                std::vector<int32_t> dbg((size_t)nB * 16);
                HIPCHK(hipMemcpy(dbg.data(), sh->dDbg, dbg.size() * 4, hipMemcpyDeviceToHost));
                print_batch_debug(pe, sh, dbg.data(), nB);
                // SHDPE_DUMP_BATCHES=<file>: per batch its rows (table
                // positions, -1 pads), hub offsets and kernel counters, for
                // offline batch-cost models (tools/batch_cost.py)
                if (const char* f = std::getenv("SHDPE_DUMP_BATCHES")) {
                    if (FILE* fp = std::fopen(f, "wb")) {
                        const int32_t hdr[2] = {nB, LB};
                        std::fwrite(hdr, 4, 2, fp);
                        std::fwrite(order.data(), 4, order.size(), fp);
                        std::fwrite(dbg.data(), 4, dbg.size(), fp);
                        const int64_t nOff = (int64_t)pe->rowOff.size();
                        std::fwrite(&nOff, 8, 1, fp);
                        std::fwrite(pe->rowOff.data(), 8, pe->rowOff.size(), fp);
                        std::fclose(fp);
                    }
                }
            }
        } else {
            if ((rc = ensure_tie(pe, sh))) return rc;
            if (sh->dTie) HIPCHK(hipMemsetAsync(sh->tie.count, 0, 4, sh->stream));
            HIPCHK(hipEventRecord(sh->evA, sh->stream));
            launch_sparse_rows(sh->dg, sh->tab, sh->sc, sh->dRows, cnt, sh->dRowAmbig, sh->cfg,
                               sh->dDbg, sh->dTie, sh->stream);
            HIPCHK(hipGetLastError());
            HIPCHK(hipEventRecord(sh->evB, sh->stream));
            amb.resize(cnt);
            HIPCHK(hipMemcpyAsync(amb.data(), sh->dRowAmbig, cnt, hipMemcpyDeviceToHost,
                                  sh->stream));
            HIPCHK(hipStreamSynchronize(sh->stream));
            st.msSparseKernel += elapsed(sh->evA, sh->evB);
            st.launchesSparse++;
            fullRows.clear();
            for (int32_t i = 0; i < cnt; ++i) {
                if (!amb[i]) continue;
                if (amb[i] >= 2) {
                    exactRows.push_back(pos[c0 + i]);
                    exactSlots.push_back(amb[i] - 2);
                } else {
                    fullRows.push_back(pos[c0 + i]);
                }
            }
            if (!exactSlots.empty()) {
                exactRows.insert(exactRows.end(), fullRows.begin(), fullRows.end());
                exactSlots.resize(exactRows.size(), -1);
            } else {
                exactRows.swap(fullRows);
            }
            if (sh->dDbg) {
                std::vector<int32_t> dbg((size_t)cnt * 16);
                HIPCHK(hipMemcpy(dbg.data(), sh->dDbg, dbg.size() * 4, hipMemcpyDeviceToHost));
                print_sparse_debug(pe, sh, dbg.data(), cnt);
            }
        }
        // Dense tie rows with early stop (round 6; undirected graphs whose rows
        // fit one dense chunk, so D / P still hold them): in groups of the
        // tie slots, each row's slot filled from D / P (k_dense_tie_export),
        // the relevance scan, the emulation only until the row's tied
        // predecessors are popped (k_exact_dense) and k_tie_write.  A slot
        // failing the emulation's consistency check is redone in full.
        if (!exactRows.empty() && pe->mode == 3 && pe->opt.forceMode != 3 && !pe->hg.latFold &&
            !pe->hg.directed && denseIdx.size() == exactRows.size()) {
            if ((rc = ensure_tie(pe, sh))) return rc;
            if (sh->tie.cap > 0 && !sh->dDenseIdx) {
                void* di;
                if ((rc = dev_alloc(sh, &di, (size_t)sh->rowsCap * 4))) return rc;
                sh->dDenseIdx = (int32_t*)di;
            }
            if (sh->tie.cap > 0) {
                if (!sh->dXList &&
                    (rc = dev_alloc(sh, &sh->dXList, (size_t)sh->exactGrid * (size_t)sh->sc.stride *
                                                         (size_t)exact_dense_list_bytes())))
                    return rc;
                const int32_t cap = sh->tie.cap;
                std::vector<int32_t> slots(cap), redo;
                for (int32_t k = 0; k < cap; ++k) slots[k] = k;
                HIPCHK(hipMemcpyAsync(sh->dSlots, slots.data(), (size_t)cap * 4, hipMemcpyHostToDevice,
                                      sh->stream));
                HIPCHK(hipEventRecord(sh->evA, sh->stream));
                for (size_t g0 = 0; g0 < exactRows.size(); g0 += (size_t)cap) {
                    const int32_t k = (int32_t)std::min<size_t>(cap, exactRows.size() - g0);
                    HIPCHK(hipMemcpyAsync(sh->dRows, exactRows.data() + g0, (size_t)k * 4,
                                          hipMemcpyHostToDevice, sh->stream));
                    HIPCHK(hipMemcpyAsync(sh->dDenseIdx, denseIdx.data() + g0, (size_t)k * 4,
                                          hipMemcpyHostToDevice, sh->stream));
                    HIPCHK(hipMemsetAsync(sh->tie.thr, 0, (size_t)k * 8, sh->stream));
                    launch_dense_tie_export(sh->dg, sh->dD, sh->dP, pe->hg.n, sh->dDenseIdx, sh->dRows, sh->tie,
                                            k, sh->stream);
                    launch_tie_scan(sh->dg, sh->dRows, sh->dSlots, k, sh->tie, sh->stream);
                    // rows of unequal early-stop cost: taken from a counter
                    HIPCHK(hipMemsetAsync(sh->tie.count + 2, 0, 4, sh->stream));
                    launch_exact_dense(sh->dg, sh->tab, sh->sc, sh->dRows, k, sh->exactGrid, sh->exactHc,
                                       sh->dXList, sh->dSlots, sh->tie, sh->tie.count + 2, sh->stream);
                    launch_tie_write(sh->dg, sh->tab, sh->dRows, sh->dSlots, k, sh->tie, sh->stream);
                    HIPCHK(hipGetLastError());
                    std::vector<double> thr((size_t)k);
                    HIPCHK(hipMemcpyAsync(thr.data(), sh->tie.thr, (size_t)k * 8, hipMemcpyDeviceToHost,
                                          sh->stream));
                    HIPCHK(hipStreamSynchronize(sh->stream));
                    for (int32_t i = 0; i < k; ++i)
                        if (std::isnan(thr[(size_t)i])) redo.push_back(exactRows[g0 + (size_t)i]);
                    st.rowsTieEarly += k;
                }
                if (!redo.empty()) {
                    std::fprintf(stderr, "[shdpe] shard %d: %zu dense early-stop tie row(s) failed the slot "
                                 "consistency check; recomputed by the full emulation\n",
                                 sh->gindex, redo.size());
                    HIPCHK(hipMemcpyAsync(sh->dRows, redo.data(), redo.size() * 4, hipMemcpyHostToDevice,
                                          sh->stream));
                    launch_exact_dense(sh->dg, sh->tab, sh->sc, sh->dRows, (int32_t)redo.size(),
                                       sh->exactGrid, sh->exactHc, sh->dXList, nullptr, sh->tie, nullptr,
                                       sh->stream);
                    HIPCHK(hipGetLastError());
                    st.rowsTieRepaired += (int64_t)redo.size();
                }
                HIPCHK(hipEventRecord(sh->evB, sh->stream));
                HIPCHK(hipEventSynchronize(sh->evB));
                st.msExactKernel += elapsed(sh->evA, sh->evB);
                st.launchesExact++;
                st.rowsExact += (int64_t)exactRows.size();
                exactRows.clear();
            }
        }
        if (!exactRows.empty()) {
            HIPCHK(hipMemcpyAsync(sh->dRows, exactRows.data(), exactRows.size() * 4,
                                  hipMemcpyHostToDevice, sh->stream));
            const int32_t* dSl = nullptr;
            int32_t nTie = 0;
            if (!exactSlots.empty()) {
                HIPCHK(hipMemcpyAsync(sh->dSlots, exactSlots.data(), exactSlots.size() * 4,
                                      hipMemcpyHostToDevice, sh->stream));
                dSl = sh->dSlots;
                while (nTie < (int32_t)exactSlots.size() && exactSlots[nTie] >= 0) ++nTie;
            }
            const bool dense = pe->mode == 3 && pe->opt.forceMode != 3 && !pe->hg.latFold && !dSl;
            if (dense && !sh->dXList &&
                (rc = dev_alloc(sh, &sh->dXList, (size_t)sh->exactGrid * (size_t)sh->sc.stride *
                                                     (size_t)exact_dense_list_bytes())))
                return rc;
            HIPCHK(hipEventRecord(sh->evA, sh->stream));
            if (nTie > 0) launch_tie_scan(sh->dg, sh->dRows, sh->dSlots, nTie, sh->tie, sh->stream);
            if (nTie > 0 && (pe->tu.tieCorrupt == 1 || pe->tu.tieCorrupt == 2))
                corrupt_tie_slot(pe, sh, exactSlots, nTie);
            if (dense)      // ~n arcs per pop: the workgroup-wide scan
                launch_exact_dense(sh->dg, sh->tab, sh->sc, sh->dRows, (int32_t)exactRows.size(),
                                   sh->exactGrid, sh->exactHc, sh->dXList, nullptr, sh->tie, nullptr,
                                   sh->stream);
            else
                launch_exact_rows(sh->dg, sh->tab, sh->sc, sh->dRows, (int32_t)exactRows.size(),
                                  sh->exactGrid, sh->exactHc, pe->tu.exactHc > 0, dSl, sh->tie,
                                  sh->dXdbg, sh->stream);
            HIPCHK(hipGetLastError());
            if (nTie > 0) {
                launch_tie_write(sh->dg, sh->tab, sh->dRows, sh->dSlots, nTie, sh->tie, sh->stream);
                HIPCHK(hipGetLastError());
                st.rowsTieEarly += nTie;
            }
            HIPCHK(hipEventRecord(sh->evB, sh->stream));
            HIPCHK(hipEventSynchronize(sh->evB));
            st.msExactKernel += elapsed(sh->evA, sh->evB);
            st.launchesExact++;
            // early-stop rows whose slot failed the exact kernel's consistency
            // check (thr = NaN: the exported distances are not this row's):
            // k_tie_write skipped them; the full emulation recomputes them
            if (nTie > 0) {
                std::vector<double> thr((size_t)sh->tie.cap);
                HIPCHK(hipMemcpy(thr.data(), sh->tie.thr, thr.size() * 8, hipMemcpyDeviceToHost));
                std::vector<int32_t> redo;
                for (int32_t i = 0; i < nTie; ++i)
                    if (std::isnan(thr[(size_t)exactSlots[i]])) redo.push_back(exactRows[i]);
                if (!redo.empty()) {
                    std::fprintf(stderr, "[shdpe] shard %d: %zu early-stop tie row(s) failed the slot "
                                 "consistency check; recomputed by the full emulation\n",
                                 sh->gindex, redo.size());
                    HIPCHK(hipMemcpyAsync(sh->dRows, redo.data(), redo.size() * 4, hipMemcpyHostToDevice,
                                          sh->stream));
                    launch_exact_rows(sh->dg, sh->tab, sh->sc, sh->dRows, (int32_t)redo.size(), sh->exactGrid,
                                      sh->exactHc, pe->tu.exactHc > 0, nullptr, sh->tie, nullptr, sh->stream);
                    HIPCHK(hipGetLastError());
                    HIPCHK(hipStreamSynchronize(sh->stream));
                    st.rowsTieRepaired += (int64_t)redo.size();
                }
            }
            if (sh->dXdbg && pe->hg.n > 10240) print_exact_debug(sh, exactRows, nTie);
            st.rowsExact += (int64_t)exactRows.size();
        }
    }
    HIPCHK(hipEventRecord(sh->ev1, sh->stream));
    HIPCHK(hipEventSynchronize(sh->ev1));
    st.msTotal += elapsed(sh->ev0, sh->ev1);
    st.rowsComputed += count;
    st.arcsRelaxed += (int64_t)count * pe->hg.nArcs();
    for (int32_t i = 0; i < count; ++i) pe->rowDone[pos[i]].store(1, std::memory_order_release);
    return SHD_PE_OK;
}

static Shard* owner_of(ShdPe* pe, int32_t p) {
    for (auto& s : pe->shards)
        if (p >= s->rowStart && p < s->rowStart + s->rowCount) return s.get();
    return nullptr;
}

// Compute positions (caller holds pe->mu): split by shard, one host thread
// per shard when several shards have work (their devices run concurrently).
static int compute_positions_locked(ShdPe* pe, const int32_t* pos, int32_t count) {
    if (count <= 0) return SHD_PE_OK;
    std::vector<std::vector<int32_t>> per(pe->shards.size());
    for (int32_t i = 0; i < count; ++i) {
        Shard* s = owner_of(pe, pos[i]);
        if (!s) return SHD_PE_ENOTOWNED;
        per[s->gindex - pe->firstShard].push_back(pos[i]);
    }
    int busy = 0;
    for (auto& v : per) busy += !v.empty();
    if (busy <= 1) {
        for (size_t k = 0; k < per.size(); ++k)
            if (!per[k].empty()) return compute_shard(pe, pe->shards[k].get(), per[k].data(),
                                                      (int32_t)per[k].size());
        return SHD_PE_OK;
    }
    std::vector<int> rcs(per.size(), SHD_PE_OK);
    std::vector<std::thread> th;
    for (size_t k = 0; k < per.size(); ++k) {
        if (per[k].empty()) continue;
        th.emplace_back([&, k] {
            rcs[k] = compute_shard(pe, pe->shards[k].get(), per[k].data(), (int32_t)per[k].size());
        });
    }
    for (auto& t : th) t.join();
    for (int r : rcs)
        if (r) return r;
    return SHD_PE_OK;
}

static bool row_done(const ShdPe* pe, int32_t p) {
    return pe->rowDone[p].load(std::memory_order_acquire) != 0;
}

extern "C" int shd_pe_compute_positions(ShdPe* pe, int32_t start, int32_t count) {
    if (!pe || start < 0 || count < 0 || (int64_t)start + count > (int64_t)pe->attached.size())
        return SHD_PE_EINVAL;
    if (count && (start < pe->ownStart || start + count > pe->ownEnd)) return SHD_PE_ENOTOWNED;
    std::vector<int32_t> pos(count);
    for (int32_t i = 0; i < count; ++i) pos[i] = start + i;
    std::lock_guard<std::mutex> lk(pe->mu);
    return compute_positions_locked(pe, pos.data(), count);
}

extern "C" int shd_pe_compute_all(ShdPe* pe) {
    if (!pe) return SHD_PE_EINVAL;
    return shd_pe_compute_positions(pe, pe->ownStart, pe->ownEnd - pe->ownStart);
}

extern "C" int shd_pe_tune(ShdPe* pe) {
    if (!pe) return SHD_PE_EINVAL;
    if (!pe->batched) return SHD_PE_OK;
    std::lock_guard<std::mutex> lk(pe->mu);
    for (auto& sp : pe->shards) {
        Shard* sh = sp.get();
        if (sh->tuned || (sh->bcfgAlt.grid <= 0 && sh->bcfgAlt2.grid <= 0 && sh->bcfgCoop.grid <= 0) ||
            sh->rowCount <= 0)
            continue;
        // scratch first: ensure_batch sizes the slots and lowers the live
        // grids to them, and the candidates below are copies of those grids
        if (hipSetDevice(sh->device) != hipSuccess) return SHD_PE_EHIP;
        int rc0 = ensure_table(pe, sh);
        if (!rc0) rc0 = ensure_batch(pe, sh);
        if (rc0) return rc0;
        std::vector<int32_t> pos(sh->rowCount);
        for (int32_t i = 0; i < sh->rowCount; ++i) pos[i] = sh->rowStart + i;
        const ShdPeStats keep = sh->stats;
        double ms[4] = {0.0, 0.0, 0.0, 0.0}, part[4][2] = {{0.0, 0.0}, {0.0, 0.0}, {0.0, 0.0}, {0.0, 0.0}};
        int w[4] = {0, 0, 0, 0};
        int64_t ex[4] = {0, 0, 0, 0};   // rows each candidate sent to the exact path
        BatchLaunch cand[4] = {sh->bcfg, sh->bcfgAlt, sh->bcfgAlt2, sh->bcfgCoop};
        const BatchLaunch orig[3] = {sh->bcfg, sh->bcfgAlt, sh->bcfgAlt2};
        int nc = 1;
        if (sh->bcfgAlt.grid > 0) cand[nc++] = sh->bcfgAlt;
        if (sh->bcfgAlt2.grid > 0) cand[nc++] = sh->bcfgAlt2;
        // the cooperative relax (its post part runs the plain kernel of the
        // same variant, so it is timed as that variant's post)
        if (sh->bcfgCoop.grid > 0 && sh->bcfg.coop < 2 && sh->bcfg.split) cand[nc++] = sh->bcfgCoop;
        sh->bcfgPost = BatchLaunch{};
        for (int k = 0; k < nc; ++k) {
            sh->bcfg = cand[k];
            w[k] = sh->bcfg.wpe;
            // a first launch of each variant maps its code and scratch; the
            // second is timed (split kernels: relax and post separately)
            for (int rep = 0; rep < 2; ++rep) {
                const double m0 = sh->stats.msSparseKernel;
                const int64_t x0 = sh->stats.rowsExact;
                sh->msPart[0] = sh->msPart[1] = 0.0;
                sh->timeParts = rep == 1 && sh->bcfg.split;
                int rc = compute_shard(pe, sh, pos.data(), sh->rowCount);
                sh->timeParts = false;
                if (rc) {
                    sh->bcfg = orig[0]; sh->bcfgAlt = orig[1]; sh->bcfgAlt2 = orig[2];
                    sh->stats = keep;
                    return rc;
                }
                ms[k] = sh->stats.msSparseKernel - m0;
                part[k][0] = sh->msPart[0];
                part[k][1] = sh->msPart[1];
                ex[k] = sh->stats.rowsExact - x0;
            }
        }
        // Every variant computes the same rows, so they all send the same
        // rows to the exact path -- except one whose batches fail their
        // checks (a miscompiled instantiation: round 6 found one whose post
        // kernel failed every batch's Bellman check under one register
        // allocation).  Such a variant looks FASTER here (its
        // skipped phases are not in the batch-kernel time, the exact kernel
        // is), so it is never picked: only candidates at the fewest exact
        // rows compete.
        int64_t exMin = ex[0];
        for (int k = 1; k < nc; ++k) exMin = std::min(exMin, ex[k]);
        bool ok[4] = {false, false, false, false};
        for (int k = 0; k < nc; ++k) ok[k] = ex[k] == exMin;
        // whole launches, or per part when every variant ran split: the
        // relax kernel and the post kernel each take their fastest variant
        bool perPart = true;
        for (int k = 0; k < nc; ++k) perPart = perPart && cand[k].split && part[k][0] > 0.0;
        int rk = 0;
        while (!ok[rk]) ++rk;
        int pk = rk;
        for (int k = rk + 1; k < nc; ++k) {
            if (!ok[k]) continue;
            if (perPart ? part[k][0] < part[rk][0] : ms[k] < ms[rk]) rk = k;
            if (perPart ? part[k][1] < part[pk][1] : ms[k] < ms[pk]) pk = k;
        }
        if (!perPart) pk = rk;
        // bucket width: the chosen relax variant at delta and at 0.8 x delta,
        // timed alternately (A B A B, each width's best run), the narrower
        // width kept only if its relax kernel is faster by more than 1% on
        // this shard -- the gain is 1-2% where it exists (C4 same box: N=1
        // -1.2%, the N=8 shard's LB-8 batches -2%; C5 +1.2%, so not a fixed
        // default; profiles/r05_ab_notes.txt r05bg-bi), and a single run
        // against a measurement from another pass let noise pick the width.
        // The post kernel does not use delta.
        BatchLaunch relaxPick = cand[rk];
        double relaxAlt = 0.0, relaxBase = 0.0;
        if (perPart) {
            BatchLaunch alt = cand[rk];
            alt.delta = cand[rk].delta * 0.8;
            sh->bcfgPost = cand[pk];
            double best[2] = {0.0, 0.0};
            for (int rep = 0; rep < 4; ++rep) {
                sh->bcfg = (rep & 1) ? alt : cand[rk];
                sh->msPart[0] = sh->msPart[1] = 0.0;
                sh->timeParts = true;
                const int rc = compute_shard(pe, sh, pos.data(), sh->rowCount);
                sh->timeParts = false;
                if (rc) {
                    sh->bcfg = orig[0]; sh->bcfgAlt = orig[1]; sh->bcfgAlt2 = orig[2];
                    sh->bcfgPost = BatchLaunch{};
                    sh->stats = keep;
                    return rc;
                }
                double& b = best[rep & 1];
                if (sh->msPart[0] > 0.0 && (b == 0.0 || sh->msPart[0] < b)) b = sh->msPart[0];
            }
            relaxBase = best[0];
            relaxAlt = best[1];
            if (relaxAlt > 0.0 && relaxBase > 0.0 && relaxAlt < 0.99 * relaxBase) relaxPick = alt;
            sh->bcfgPost = BatchLaunch{};
        }
        sh->bcfg = relaxPick;
        if (pk != rk) sh->bcfgPost = cand[pk];
        sh->tuned = true;
        sh->stats = keep;
        sh->stats.deltaUsed = relaxPick.delta;
        sh->stats.batchWaves = sh->bcfg.wpe;
        sh->stats.batchPostWaves = sh->bcfg.split ? cand[pk].wpe : 0;
        if (pe->tu.debug || pe->tu.tuneLog)
            for (int k = 0; k < nc; ++k)
                std::fprintf(stderr, "[shdpe] shard %d tune: %d waves%s %.2f ms (relax %.2f post %.2f) exact rows %ld%s%s%s\n",
                             sh->gindex, w[k], cand[k].coop >= 2 ? " cooperative" : "", ms[k], part[k][0],
                             part[k][1], (long)ex[k], ok[k] ? "" : " (excluded)", k == rk ? " <relax" : "",
                             k == pk ? " <post" : "");
        if ((pe->tu.debug || pe->tu.tuneLog) && relaxAlt > 0.0)
            std::fprintf(stderr, "[shdpe] shard %d tune: relax at 0.8 x delta %.2f ms vs %.2f -> delta %.3f\n",
                         sh->gindex, relaxAlt, relaxBase, relaxPick.delta);
    }
    return SHD_PE_OK;
}

extern "C" int shd_pe_compute_rows(ShdPe* pe, const int32_t* src, int32_t count) {
    if (!pe || count < 0 || (count > 0 && !src)) return SHD_PE_EINVAL;
    std::vector<int32_t> pos(count);
    for (int32_t i = 0; i < count; ++i) {
        if (src[i] < 0 || src[i] >= pe->hg.n || pe->posOf[src[i]] < 0) return SHD_PE_ENOTATTACHED;
        pos[i] = pe->posOf[src[i]];
        if (pos[i] < pe->ownStart || pos[i] >= pe->ownEnd) return SHD_PE_ENOTOWNED;
    }
    std::lock_guard<std::mutex> lk(pe->mu);
    return compute_positions_locked(pe, pos.data(), count);
}

// Compute whatever rows of [start, start+count) are owned here and missing.
static int ensure_rows(ShdPe* pe, int32_t start, int32_t count) {
    bool all = true;
    for (int32_t i = start; i < start + count && all; ++i) all = row_done(pe, i);
    if (all) return SHD_PE_OK;
    std::lock_guard<std::mutex> lk(pe->mu);
    std::vector<int32_t> todo;
    for (int32_t i = start; i < start + count; ++i) {
        if (row_done(pe, i)) continue;
        if (i < pe->ownStart || i >= pe->ownEnd) return SHD_PE_ENOTOWNED;
        todo.push_back(i);
    }
    return compute_positions_locked(pe, todo.data(), (int32_t)todo.size());
}

// A contiguous run of table rows readable from one device table.
struct Piece {
    const DevTable* tab;
    hipStream_t stream;
    int device;
    int32_t start, count;   // table positions
};

static int table_pieces(ShdPe* pe, int32_t start, int32_t count, std::vector<Piece>& out) {
    out.clear();
    if (pe->gathered) {
        Shard* s = pe->shards[0].get();
        out.push_back(Piece{&s->full, s->copyStream, s->device, start, count});
        return SHD_PE_OK;
    }
    int32_t p = start;
    while (p < start + count) {
        Shard* s = owner_of(pe, p);
        if (!s || !s->tableReady) return SHD_PE_ENOTOWNED;
        const int32_t end = std::min(start + count, s->rowStart + s->rowCount);
        out.push_back(Piece{&s->tab, s->copyStream, s->device, p, end - p});
        p = end;
    }
    return SHD_PE_OK;
}

static int get_rows_staged(ShdPe* pe, int32_t start, int32_t count, double* lat, double* rel,
                           int32_t* hops, int32_t* pred, uint8_t* flags);

extern "C" int shd_pe_get_row(ShdPe* pe, int32_t srcVertex, double* lat, double* rel,
                              int32_t* hops, int32_t* pred, uint8_t* flags) {
    if (!pe || srcVertex < 0 || srcVertex >= pe->hg.n) return SHD_PE_EINVAL;
    const int32_t p = pe->posOf[srcVertex];
    if (p < 0) return SHD_PE_ENOTATTACHED;
    if (pred && !pe->opt.storePred) return SHD_PE_EINVAL;
    int rc = ensure_rows(pe, p, 1);
    if (rc) return rc;
    return get_rows_staged(pe, p, 1, lat, rel, hops, pred, flags);
}

// Host memcpy split over up to 8 threads: the drain of a staging block into
// caller (pageable, often freshly allocated) memory runs at one core's
// page-fault + copy rate otherwise.
static void par_memcpy(void* dst, const void* src, size_t bytes) {
    const size_t minChunk = (size_t)2 << 20;
    const unsigned hc = std::thread::hardware_concurrency();
    const int nt = (int)std::max<size_t>(1, std::min<size_t>({(size_t)8, hc ? hc : 1, bytes / minChunk}));
    if (nt <= 1) { std::memcpy(dst, src, bytes); return; }
    std::vector<std::thread> th;
    const size_t per = (bytes + nt - 1) / nt;
    for (int t = 1; t < nt; ++t) {
        const size_t o = per * t;
        if (o >= bytes) break;
        th.emplace_back([=]() { std::memcpy((char*)dst + o, (const char*)src + o, std::min(per, bytes - o)); });
    }
    std::memcpy(dst, src, std::min(per, bytes));
    for (auto& x : th) x.join();
}

// Page-locked host memory the device can DMA into (hipHostMalloc or
// hipHostRegister): such caller buffers skip the staging copy.
static bool is_pinned(const void* p) {
    if (!p) return true;
    hipPointerAttribute_t at;
    if (hipPointerGetAttributes(&at, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return at.type == hipMemoryTypeHost && at.hostPointer != nullptr;
}

// Rows [start, start+count) -> caller host buffers.  Pinned caller buffers
// take the DMA straight (five field copies per table piece); otherwise two
// pinned staging buffers: block b's field copies run on the copy stream
// while host threads copy block b-1 out of the other buffer.
static int get_rows_staged(ShdPe* pe, int32_t start, int32_t count, double* lat, double* rel,
                           int32_t* hops, int32_t* pred, uint8_t* flags) {
    const size_t T = pe->attached.size();
    const size_t perRow = T * (8 + 8 + 4 + 4 + 1);
    std::lock_guard<std::mutex> lk(pe->copyMu);
    std::vector<Piece> pieces;
    int rc = table_pieces(pe, start, count, pieces);
    if (rc) return rc;
    if (is_pinned(lat) && is_pinned(rel) && is_pinned(hops) && is_pinned(pred) && is_pinned(flags)) {
        for (const Piece& pc : pieces) {
            HIPCHK(hipSetDevice(pc.device));
            const DevTable& tb = *pc.tab;
            const size_t off = (size_t)(pc.start - tb.rowStart) * T, cells = (size_t)pc.count * T;
            const size_t o = (size_t)(pc.start - start) * T;
            if (lat) HIPCHK(hipMemcpyAsync(lat + o, tb.lat + off, cells * 8, hipMemcpyDeviceToHost, pc.stream));
            if (rel) HIPCHK(hipMemcpyAsync(rel + o, tb.rel + off, cells * 8, hipMemcpyDeviceToHost, pc.stream));
            if (hops) HIPCHK(hipMemcpyAsync(hops + o, tb.hops + off, cells * 4, hipMemcpyDeviceToHost, pc.stream));
            if (pred) HIPCHK(hipMemcpyAsync(pred + o, tb.pred + off, cells * 4, hipMemcpyDeviceToHost, pc.stream));
            if (flags) HIPCHK(hipMemcpyAsync(flags + o, tb.flags + off, cells, hipMemcpyDeviceToHost, pc.stream));
        }
        for (const Piece& pc : pieces) {
            HIPCHK(hipSetDevice(pc.device));
            HIPCHK(hipStreamSynchronize(pc.stream));
        }
        return SHD_PE_OK;
    }
    if (!pe->stage[0]) {
        const size_t want = std::max<size_t>(perRow, (size_t)64 << 20);
        for (auto& h : pe->stage)
            HIPCHK(hipHostMalloc(reinterpret_cast<void**>(&h), want, hipHostMallocPortable));
        pe->stageBytes = want;
    }
    const int32_t B = (int32_t)std::max<size_t>(1, pe->stageBytes / perRow);
    for (const Piece& pc : pieces) {
        HIPCHK(hipSetDevice(pc.device));
        const DevTable& tb = *pc.tab;
        struct Blk { int32_t r0, n; };   // r0 relative to pc.start
        auto issue = [&](int buf, Blk b) -> int {
            unsigned char* q = pe->stage[buf];
            const size_t off = ((size_t)(pc.start - tb.rowStart) + b.r0) * T, cells = (size_t)b.n * T;
            if (lat) { HIPCHK(hipMemcpyAsync(q, tb.lat + off, cells * 8, hipMemcpyDeviceToHost, pc.stream)); q += cells * 8; }
            if (rel) { HIPCHK(hipMemcpyAsync(q, tb.rel + off, cells * 8, hipMemcpyDeviceToHost, pc.stream)); q += cells * 8; }
            if (hops) { HIPCHK(hipMemcpyAsync(q, tb.hops + off, cells * 4, hipMemcpyDeviceToHost, pc.stream)); q += cells * 4; }
            if (pred) { HIPCHK(hipMemcpyAsync(q, tb.pred + off, cells * 4, hipMemcpyDeviceToHost, pc.stream)); q += cells * 4; }
            if (flags) { HIPCHK(hipMemcpyAsync(q, tb.flags + off, cells, hipMemcpyDeviceToHost, pc.stream)); }
            return SHD_PE_OK;
        };
        auto drain = [&](int buf, Blk b) {
            const unsigned char* q = pe->stage[buf];
            const size_t o = ((size_t)(pc.start - start) + b.r0) * T, cells = (size_t)b.n * T;
            if (lat) { par_memcpy(lat + o, q, cells * 8); q += cells * 8; }
            if (rel) { par_memcpy(rel + o, q, cells * 8); q += cells * 8; }
            if (hops) { par_memcpy(hops + o, q, cells * 4); q += cells * 4; }
            if (pred) { par_memcpy(pred + o, q, cells * 4); q += cells * 4; }
            if (flags) par_memcpy(flags + o, q, cells);
        };
        hipEvent_t done[2];
        HIPCHK(hipEventCreateWithFlags(&done[0], hipEventDisableTiming));
        if (hipEventCreateWithFlags(&done[1], hipEventDisableTiming) != hipSuccess) {
            (void)hipEventDestroy(done[0]);
            return SHD_PE_EHIP;
        }
        Blk prev{0, 0};
        int buf = 0;
        for (int32_t r0 = 0; r0 < pc.count && rc == SHD_PE_OK; r0 += B) {
            const Blk cur{r0, std::min(B, pc.count - r0)};
            if ((rc = issue(buf, cur)) == SHD_PE_OK &&
                hipEventRecord(done[buf], pc.stream) != hipSuccess)
                rc = SHD_PE_EHIP;
            if (rc == SHD_PE_OK && prev.n) {
                if (hipEventSynchronize(done[buf ^ 1]) != hipSuccess) rc = SHD_PE_EHIP;
                else drain(buf ^ 1, prev);
            }
            prev = cur;
            buf ^= 1;
        }
        if (rc == SHD_PE_OK && prev.n) {
            if (hipEventSynchronize(done[buf ^ 1]) != hipSuccess) rc = SHD_PE_EHIP;
            else drain(buf ^ 1, prev);
        }
        (void)hipStreamSynchronize(pc.stream);
        (void)hipEventDestroy(done[0]);
        (void)hipEventDestroy(done[1]);
        if (rc) return rc;
    }
    return rc;
}

extern "C" int shd_pe_get_rows(ShdPe* pe, int32_t start, int32_t count, double* lat, double* rel,
                               int32_t* hops, int32_t* pred, uint8_t* flags) {
    if (!pe || start < 0 || count < 0 || (int64_t)start + count > (int64_t)pe->attached.size())
        return SHD_PE_EINVAL;
    if (pred && !pe->opt.storePred) return SHD_PE_EINVAL;
    if (count == 0) return SHD_PE_OK;
    int rc = ensure_rows(pe, start, count);
    if (rc) return rc;
    return get_rows_staged(pe, start, count, lat, rel, hops, pred, flags);
}

extern "C" int shd_pe_get_path(ShdPe* pe, int32_t srcVertex, int32_t dstVertex, int32_t* verts,
                               int32_t cap, int32_t* len) {
    if (!pe || !verts || !len || cap < 1) return SHD_PE_EINVAL;
    *len = 0;
    const HostGraph& g = pe->hg;
    if (srcVertex < 0 || srcVertex >= g.n || dstVertex < 0 || dstVertex >= g.n) return SHD_PE_EINVAL;
    const int32_t ps = pe->posOf[srcVertex];
    if (ps < 0 || pe->posOf[dstVertex] < 0) return SHD_PE_ENOTATTACHED;
    if (srcVertex == dstVertex) {            // the 1-vertex igraph path [s] (:1469-1488)
        verts[0] = srcVertex;
        *len = 1;
        return SHD_PE_OK;
    }
    if (pe->mode == 2) {                     // complete graph: the direct edge (:1877-1927)
        if (cap < 2) return SHD_PE_EINVAL;
        if (g.findArc(srcVertex, dstVertex) < 0) return SHD_PE_ENOEDGE;
        verts[0] = srcVertex;
        verts[1] = dstVertex;
        *len = 2;
        return SHD_PE_OK;
    }
    std::lock_guard<std::mutex> lk(pe->mu);
    Shard* sh = owner_of(pe, ps);
    if (!sh) return SHD_PE_ENOTOWNED;
    HIPCHK(hipSetDevice(sh->device));
    int rc = ensure_table(pe, sh);
    if (rc) return rc;
    if (!sh->dPath) {
        void* p;
        if ((rc = dev_alloc(sh, &p, ((size_t)g.n + 64) * 4))) return rc;
        sh->dPath = (int32_t*)p;
    }
    if (sh->pathSrc != srcVertex) {
        // igraph's whole Dijkstra for this source (full 2-wheap emulation,
        // one wave): every vertex popped before the last target keeps its
        // chosen IN-arc in slot 0; the row it rewrites is the table's own
        HIPCHK(hipMemcpyAsync(sh->dRows, &ps, 4, hipMemcpyHostToDevice, sh->stream));
        launch_exact_rows(sh->dg, sh->tab, sh->sc, sh->dRows, 1, 1, sh->exactHc, pe->tu.exactHc > 0,
                          nullptr, sh->tie, nullptr, sh->stream);
        HIPCHK(hipGetLastError());
        sh->pathSrc = srcVertex;
    }
    int32_t* dLen = sh->dPath + g.n + 32;
    // reachability from the row the emulation just wrote: an unreached
    // target has no parent chain in slot 0 (its P entry is whatever an
    // earlier row left there), so it must not be walked
    {
        uint8_t f = 0;
        const size_t cell = (size_t)(ps - sh->tab.rowStart) * pe->attached.size() + pe->posOf[dstVertex];
        HIPCHK(hipMemcpyAsync(&f, sh->tab.flags + cell, 1, hipMemcpyDeviceToHost, sh->stream));
        HIPCHK(hipStreamSynchronize(sh->stream));
        if (f & F_UNREACHABLE) return SHD_PE_EUNREACHABLE;
    }
    // device ids of s and t (the batched path relabels vertices)
    int32_t sD = srcVertex, tD = dstVertex;
    if (!pe->devOf.empty()) { sD = pe->devOf[srcVertex]; tD = pe->devOf[dstVertex]; }
    launch_path_walk(sh->dg, sh->sc.pred, sD, tD, sh->dPath, std::min<int32_t>(cap, g.n + 1), dLen,
                     (int32_t)g.nArcs(), sh->stream);
    HIPCHK(hipGetLastError());
    int32_t n = 0;
    HIPCHK(hipMemcpyAsync(&n, dLen, 4, hipMemcpyDeviceToHost, sh->stream));
    HIPCHK(hipStreamSynchronize(sh->stream));
    if (n == -2) return SHD_PE_EINVAL;            // cap too small for the path
    if (n < 0) return SHD_PE_EUNREACHABLE;
    std::vector<int32_t> rev(n);
    HIPCHK(hipMemcpy(rev.data(), sh->dPath, (size_t)n * 4, hipMemcpyDeviceToHost));
    for (int32_t k = 0; k < n; ++k) verts[k] = rev[n - 1 - k];
    *len = n;
    return SHD_PE_OK;
}

extern "C" int shd_pe_host_alloc(int64_t bytes, void** out) {
    if (!out || bytes <= 0) return SHD_PE_EINVAL;
    *out = nullptr;
    if (hipHostMalloc(out, (size_t)bytes, hipHostMallocPortable) != hipSuccess) {
        *out = nullptr;
        return SHD_PE_ENOMEM;
    }
    return SHD_PE_OK;
}

extern "C" void shd_pe_host_free(void* p) {
    if (p) (void)hipHostFree(p);
}

extern "C" int shd_pe_copy_rows_device(ShdPe* pe, int32_t start, int32_t count, double* dLat,
                                       double* dRel, int32_t* dHops, uint8_t* dFlags) {
    if (!pe || start < 0 || count < 0 || (int64_t)start + count > (int64_t)pe->attached.size())
        return SHD_PE_EINVAL;
    if (count == 0) return SHD_PE_OK;
    int rc = ensure_rows(pe, start, count);       // same contract as shd_pe_get_rows
    if (rc) return rc;
    // table_pieces reads gathered / the full table, which shd_pe_gather
    // writes under copyMu
    std::lock_guard<std::mutex> lk(pe->copyMu);
    std::vector<Piece> pieces;
    if ((rc = table_pieces(pe, start, count, pieces))) return rc;
    const size_t T = pe->attached.size();
    for (const Piece& pc : pieces) {
        HIPCHK(hipSetDevice(pc.device));
        const DevTable& tb = *pc.tab;
        const size_t off = (size_t)(pc.start - tb.rowStart) * T, cells = (size_t)pc.count * T;
        const size_t o = (size_t)(pc.start - start) * T;
        if (dLat) HIPCHK(hipMemcpyAsync(dLat + o, tb.lat + off, cells * 8, hipMemcpyDeviceToDevice, pc.stream));
        if (dRel) HIPCHK(hipMemcpyAsync(dRel + o, tb.rel + off, cells * 8, hipMemcpyDeviceToDevice, pc.stream));
        if (dHops) HIPCHK(hipMemcpyAsync(dHops + o, tb.hops + off, cells * 4, hipMemcpyDeviceToDevice, pc.stream));
        if (dFlags) HIPCHK(hipMemcpyAsync(dFlags + o, tb.flags + off, cells, hipMemcpyDeviceToDevice, pc.stream));
        HIPCHK(hipStreamSynchronize(pc.stream));
    }
    return SHD_PE_OK;
}

extern "C" int shd_pe_row_checksums(ShdPe* pe, int32_t start, int32_t count, uint64_t* out) {
    if (!pe || !out || start < 0 || count < 0 || (int64_t)start + count > (int64_t)pe->attached.size())
        return SHD_PE_EINVAL;
    if (count == 0) return SHD_PE_OK;
    int rc = ensure_rows(pe, start, count);
    if (rc) return rc;
    std::lock_guard<std::mutex> lk(pe->copyMu);
    std::vector<Piece> pieces;
    if ((rc = table_pieces(pe, start, count, pieces))) return rc;
    for (const Piece& pc : pieces) {
        HIPCHK(hipSetDevice(pc.device));
        uint64_t* d = nullptr;
        if (hipMalloc(&d, (size_t)pc.count * 8) != hipSuccess) return SHD_PE_ENOMEM;
        launch_row_checksums(*pc.tab, (int64_t)pc.start - pc.tab->rowStart, pc.count, d, pc.stream);
        hipError_t e = hipGetLastError();
        if (e == hipSuccess)
            e = hipMemcpyAsync(out + (pc.start - start), d, (size_t)pc.count * 8, hipMemcpyDeviceToHost,
                               pc.stream);
        if (e == hipSuccess) e = hipStreamSynchronize(pc.stream);
        (void)hipFree(d);
        if (e != hipSuccess) return SHD_PE_EHIP;
    }
    return SHD_PE_OK;
}

// The whole-table path-cache fill (topology.c:1805-1864 for every row, in
// position order) as one device pass: k_pack_rowstore builds the row
// store's own image of its triangular rows (2.3 GB at C4 vs 7.8 GB of
// rows), one DMA lands it in page-locked host memory the store adopts.
//
// The host image (2.3 GB at C4) is anonymous memory with transparent huge
// pages, first-touched by 16 threads and then registered with the device
// (page-locked): hipHostMalloc of the same size took 430 ms, most of it
// faulting and zeroing 4-KB pages on one thread.  When the rows still have
// to be computed, that preparation runs on a host thread while the device
// computes them.
struct HostImage {
    void* p = nullptr;
    size_t bytes = 0;
    bool registered = false;
    double msTouch = 0.0, msRegister = 0.0;
    ~HostImage();
};

static void host_image_prepare(HostImage* im, size_t bytes) {
    const auto t0 = std::chrono::steady_clock::now();
    void* p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE, -1, 0);
    if (p == MAP_FAILED) return;
    (void)madvise(p, bytes, MADV_HUGEPAGE);
    const size_t nt = 16, chunk = ((bytes + nt - 1) / nt + 4095) & ~(size_t)4095;
    std::vector<std::thread> th;
    for (size_t t = 0; t < nt; ++t)
        th.emplace_back([=] {
            unsigned char* q = static_cast<unsigned char*>(p);
            for (size_t o = t * chunk; o < std::min(bytes, (t + 1) * chunk); o += 4096) q[o] = 0;
        });
    for (auto& x : th) x.join();
    im->p = p;
    im->bytes = bytes;
    const auto t1 = std::chrono::steady_clock::now();
    im->registered = hipHostRegister(p, bytes, hipHostRegisterDefault) == hipSuccess;
    const auto t2 = std::chrono::steady_clock::now();
    im->msTouch = std::chrono::duration<double, std::milli>(t1 - t0).count();
    im->msRegister = std::chrono::duration<double, std::milli>(t2 - t1).count();
}

static void host_image_release(HostImage* im) {
    if (!im->p) return;
    if (im->registered) (void)hipHostUnregister(im->p);
    (void)munmap(im->p, im->bytes);
    im->p = nullptr;
}

HostImage::~HostImage() { host_image_release(this); }   // every exit path of fill_rowstore

static void host_image_free_cb(void* ctx, void* p) {
    (void)p;
    delete static_cast<HostImage*>(ctx);
}

extern "C" int shd_pe_fill_rowstore(ShdPe* pe, ShdRowStore* st, int32_t* rowResult, double* msOut) {
    if (!pe || !st) return SHD_PE_EINVAL;
    if (shd_rowstore_size(st) != 0) return SHD_PE_EINVAL;   // (adopt_image re-checks under its lock)
    const int32_t T = (int32_t)pe->attached.size();
    auto now = [] { return std::chrono::steady_clock::now(); };
    auto ms = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
    std::vector<int64_t> off((size_t)T + 1);
    shd_rowstore_image_layout(T, off.data());
    const size_t bytes = (size_t)off[(size_t)T];
    const bool pack = !pe->hg.isComplete;    // a complete graph stores no non-direct path (:1321)
    const auto t0 = now();
    std::unique_ptr<HostImage> him(new HostImage);
    std::thread prep;
    if (pack) prep = std::thread(host_image_prepare, him.get(), bytes);   // beside the compute
    int rc = ensure_rows(pe, 0, T);
    const auto tc = now();
    if (prep.joinable()) prep.join();
    if (std::getenv("SHDPE_FILL_LOG"))
        std::fprintf(stderr, "[shdpe] fill_rowstore: compute %.1f ms, image %.2f GB touch %.1f ms + "
                     "register %.1f ms (%s), join wait %.1f ms\n", ms(t0, tc), bytes / 1e9, him->msTouch,
                     him->msRegister, him->registered ? "registered" : "NOT registered", ms(tc, now()));
    if (rc) return rc;
    if (pack && !him->p) return SHD_PE_ENOMEM;
    std::lock_guard<std::mutex> lk(pe->copyMu);
    const DevTable* tab = nullptr;
    Shard* s = pe->shards[0].get();
    if (pe->gathered) tab = &s->full;
    else if (pe->G == 1) tab = &s->tab;
    else return SHD_PE_ENOTOWNED;          // rows spread over shards: gather first
    if (hipSetDevice(s->device) != hipSuccess) return SHD_PE_EHIP;
    void *dImg = nullptr, *dOff = nullptr, *dAcc = nullptr, *dAll = nullptr;
    void* const hImg = him->p;
    struct Free {   // device temporaries, every exit path (the host image: ~HostImage)
        void** p[4];
        ~Free() {
            for (void** q : p) if (*q) (void)hipFree(*q);
        }
    } fr{{&dImg, &dOff, &dAcc, &dAll}};
    if ((pack && hipMalloc(&dImg, bytes) != hipSuccess) ||
        hipMalloc(&dOff, off.size() * 8) != hipSuccess || hipMalloc(&dAcc, 16) != hipSuccess ||
        hipMalloc(&dAll, (size_t)T * 4) != hipSuccess)
        return SHD_PE_ENOMEM;
    const auto t1 = now();
    const unsigned long long acc0[2] = {0ull, 0x7FF0000000000000ull};
    unsigned long long acc[2] = {0ull, 0ull};
    hipError_t e = hipMemcpyAsync(dOff, off.data(), off.size() * 8, hipMemcpyHostToDevice, s->copyStream);
    if (e == hipSuccess) e = hipMemcpyAsync(dAcc, acc0, 16, hipMemcpyHostToDevice, s->copyStream);
    if (e == hipSuccess) {
        if (pack)
            launch_pack_rowstore(*tab, (const int64_t*)dOff, (uint8_t*)dImg, (unsigned long long*)dAcc,
                                 s->copyStream);
        launch_rows_all_success(*tab, (int32_t*)dAll, s->copyStream);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipStreamSynchronize(s->copyStream);
    const auto t2 = now();
    if (e == hipSuccess && pack) e = hipMemcpyAsync(hImg, dImg, bytes, hipMemcpyDeviceToHost, s->copyStream);
    if (e == hipSuccess) e = hipMemcpyAsync(acc, dAcc, 16, hipMemcpyDeviceToHost, s->copyStream);
    if (e == hipSuccess && rowResult)
        e = hipMemcpyAsync(rowResult, dAll, (size_t)T * 4, hipMemcpyDeviceToHost, s->copyStream);
    if (e == hipSuccess) e = hipStreamSynchronize(s->copyStream);
    const auto t3 = now();
    if (e != hipSuccess) return SHD_PE_EHIP;
    if (pack) {
        double mn;
        std::memcpy(&mn, &acc[1], 8);
        rc = shd_rowstore_adopt_image(st, hImg, (int64_t)bytes, host_image_free_cb, him.get(),
                                      (int64_t)acc[0], mn);
        if (rc) return rc;
        him.release();   // the store owns it now
    }
    if (msOut) { msOut[0] = ms(t0, t1); msOut[1] = ms(t1, t2); msOut[2] = ms(t2, t3); }
    return SHD_PE_OK;
}

// ---------------------------------------------------------------------------
// Gather: the whole table on every device of this engine (and, with a
// cross-process communicator, of every engine).
// ---------------------------------------------------------------------------
static int ensure_full(ShdPe* pe, Shard* s, Shard* owner) {
    if (s != owner) { s->full = owner->full; return SHD_PE_OK; }
    if (s->full.lat) return SHD_PE_OK;
    const size_t T = pe->attached.size(), cells = T * T;
    if (pe->G == 1) { s->full = s->tab; return SHD_PE_OK; }   // the shard is the table
    HIPCHK(hipSetDevice(s->device));
    int rc;
    void *lat, *rel, *hops, *flags, *pred = nullptr;
    if ((rc = dev_alloc(s, &lat, cells * 8)) || (rc = dev_alloc(s, &rel, cells * 8)) ||
        (rc = dev_alloc(s, &hops, cells * 4)) || (rc = dev_alloc(s, &flags, cells)))
        return rc;
    if (pe->opt.storePred && (rc = dev_alloc(s, &pred, cells * 4))) return rc;
    s->full = DevTable{(double*)lat, (double*)rel, (int32_t*)hops, (int32_t*)pred, (uint8_t*)flags,
                       (int64_t)T, 0};
    return SHD_PE_OK;
}

struct Field { size_t off; size_t esize; ncclDataType_t type; };

static void table_fields(const ShdPe* pe, std::vector<Field>& f) {
    f = {{offsetof(DevTable, lat), 8, ncclUint64}, {offsetof(DevTable, rel), 8, ncclUint64},
         {offsetof(DevTable, hops), 4, ncclInt32}, {offsetof(DevTable, flags), 1, ncclUint8}};
    if (pe->opt.storePred) f.push_back({offsetof(DevTable, pred), 4, ncclInt32});
}

static void* field_ptr(const DevTable& t, const Field& f) {
    return *reinterpret_cast<void* const*>(reinterpret_cast<const char*>(&t) + f.off);
}

static int gather_locked(ShdPe* pe) {
    const int32_t T = (int32_t)pe->attached.size();
    std::vector<int32_t> all;
    for (int32_t p = pe->ownStart; p < pe->ownEnd; ++p)
        if (!row_done(pe, p)) all.push_back(p);
    int rc = compute_positions_locked(pe, all.data(), (int32_t)all.size());
    if (rc) return rc;
    for (auto& s : pe->shards) if ((rc = ensure_table(pe, s.get()))) return rc;
    // one full table per distinct device, owned by its first shard
    for (auto& s : pe->shards) {
        Shard* owner = nullptr;
        for (auto& o : pe->shards)
            if (o->device == s->device) { owner = o.get(); break; }
        if ((rc = ensure_full(pe, s.get(), owner))) return rc;
    }
    std::vector<Field> fields;
    table_fields(pe, fields);
    const size_t ts = (size_t)T;
    Shard* s0 = pe->shards[0].get();
    bool distinct = true;
    for (size_t i = 0; i < pe->shards.size(); ++i)
        for (size_t j = 0; j < i; ++j)
            if (pe->shards[i]->device == pe->shards[j]->device) distinct = false;
    // in-process RCCL over xGMI (distinct devices): one communicator per
    // device, created before the timed region
    if (pe->G > 1 && !pe->xcomm && distinct && !s0->comm) {
        std::vector<ncclComm_t> comms(pe->shards.size());
        std::vector<int> devs;
        for (auto& s : pe->shards) devs.push_back(s->device);
        if (ncclCommInitAll(comms.data(), (int)devs.size(), devs.data()) != ncclSuccess)
            return SHD_PE_ECOMM;
        for (size_t i = 0; i < comms.size(); ++i) pe->shards[i]->comm = comms[i];
    }
    struct Events {   // destroyed on every exit path
        hipEvent_t e[2] = {nullptr, nullptr};
        ~Events() { for (hipEvent_t x : e) if (x) (void)hipEventDestroy(x); }
    } ev;
    HIPCHK(hipSetDevice(s0->device));
    HIPCHK(hipEventCreate(&ev.e[0]));
    HIPCHK(hipEventCreate(&ev.e[1]));
    hipEvent_t e0 = ev.e[0], e1 = ev.e[1];
    HIPCHK(hipEventRecord(e0, s0->stream));
    if (pe->G == 1 && !pe->xcomm) {
        // nothing to exchange
    } else if (pe->xcomm) {
        // cross-process: every process owns one shard (nDevices == 1), rows
        // contiguous per shard.  Equal blocks (the plan's usual outcome, e.g.
        // C4 over 8 ranks: 2,048 rows each): one ncclAllGather per field
        // straight into the full table; otherwise a group of per-shard
        // broadcasts (an all-gather-v with blocks landing in place)
        Shard* s = s0;
        bool equal = true;
        for (int g = 1; g < pe->G; ++g)
            equal = equal && pe->bounds[g + 1] - pe->bounds[g] == pe->bounds[1] - pe->bounds[0];
        if (ncclGroupStart() != ncclSuccess) return SHD_PE_ECOMM;
        if (equal) {
            const size_t nr = (size_t)(pe->bounds[1] - pe->bounds[0]);
            for (const Field& f : fields)
                if (nr && ncclAllGather(field_ptr(s->tab, f), field_ptr(s->full, f), nr * ts, f.type, pe->xcomm,
                                        s->stream) != ncclSuccess)
                    rc = SHD_PE_ECOMM;
        } else {
            for (int g = 0; g < pe->G && rc == SHD_PE_OK; ++g) {
                const size_t r0 = (size_t)pe->bounds[g], nr = (size_t)(pe->bounds[g + 1] - pe->bounds[g]);
                if (!nr) continue;
                for (const Field& f : fields) {
                    char* dst = (char*)field_ptr(s->full, f) + r0 * ts * f.esize;
                    const void* src = g == s->gindex ? field_ptr(s->tab, f) : (const void*)dst;
                    if (ncclBroadcast(src, dst, nr * ts, f.type, g, pe->xcomm, s->stream) != ncclSuccess)
                        rc = SHD_PE_ECOMM;
                }
            }
        }
        if (ncclGroupEnd() != ncclSuccess) rc = SHD_PE_ECOMM;
        if (rc) return rc;
    } else {
        if (distinct) {
            // in-process RCCL over xGMI: a group of per-shard broadcasts
            if (ncclGroupStart() != ncclSuccess) return SHD_PE_ECOMM;
            for (size_t r = 0; r < pe->shards.size(); ++r) {
                Shard* root = pe->shards[r].get();
                const size_t r0 = (size_t)root->rowStart, nr = (size_t)root->rowCount;
                if (!nr) continue;
                for (auto& sp : pe->shards) {
                    Shard* s = sp.get();
                    for (const Field& f : fields) {
                        char* dst = (char*)field_ptr(s->full, f) + r0 * ts * f.esize;
                        const void* src = s == root ? field_ptr(root->tab, f) : (const void*)dst;
                        if (ncclBroadcast(src, dst, nr * ts, f.type, (int)r, s->comm, s->stream) !=
                            ncclSuccess)
                            rc = SHD_PE_ECOMM;
                    }
                }
            }
            if (ncclGroupEnd() != ncclSuccess) rc = SHD_PE_ECOMM;
            if (rc) return rc;
        } else {
            // logical shards sharing a device (tests): device / peer copies
            for (auto& src : pe->shards) {
                if (!src->rowCount) continue;
                for (auto& dstS : pe->shards) {
                    if (!dstS->fullOwner) continue;
                    HIPCHK(hipSetDevice(dstS->device));
                    for (const Field& f : fields) {
                        char* dst = (char*)field_ptr(dstS->full, f) + (size_t)src->rowStart * ts * f.esize;
                        HIPCHK(hipMemcpyAsync(dst, field_ptr(src->tab, f),
                                              (size_t)src->rowCount * ts * f.esize,
                                              hipMemcpyDeviceToDevice, dstS->stream));
                    }
                }
            }
        }
    }
    for (auto& s : pe->shards) {
        HIPCHK(hipSetDevice(s->device));
        HIPCHK(hipStreamSynchronize(s->stream));
    }
    HIPCHK(hipSetDevice(s0->device));
    HIPCHK(hipEventRecord(e1, s0->stream));
    HIPCHK(hipEventSynchronize(e1));
    pe->msGather += elapsed(e0, e1);
    for (int32_t p = 0; p < T; ++p) pe->rowDone[p].store(1, std::memory_order_release);
    pe->gathered = true;
    return SHD_PE_OK;
}

// Host-transport assembly (no RCCL): rows of other engines' shards arrive in
// host buffers (MPI, sockets, torch.distributed/gloo -- e.g. several ranks
// sharing one GPU, where RCCL refuses a communicator) and are written into
// the full table on every device of this engine; this engine's own rows are
// copied in on the first call.  Once all T rows are present the engine reads
// every row from the full table, as after shd_pe_gather.
extern "C" int shd_pe_put_rows(ShdPe* pe, int32_t start, int32_t count, const double* lat,
                               const double* rel, const int32_t* hops, const int32_t* pred,
                               const uint8_t* flags) {
    if (!pe || start < 0 || count < 0 || (int64_t)start + count > (int64_t)pe->attached.size())
        return SHD_PE_EINVAL;
    if (!lat || !rel || !hops || !flags || (pe->opt.storePred && !pred)) return SHD_PE_EINVAL;
    if (pe->opt.shardCount < 2 || pe->opt.nDevices != 1) return SHD_PE_EINVAL;
    if (start < pe->ownEnd && start + count > pe->ownStart) return SHD_PE_EINVAL;   // own rows
    if (count == 0) return SHD_PE_OK;
    std::lock_guard<std::mutex> lk(pe->mu);
    std::lock_guard<std::mutex> lk2(pe->copyMu);
    Shard* s = pe->shards[0].get();
    int rc = ensure_table(pe, s);
    if (rc) return rc;
    if (!pe->putInit) {
        std::vector<int32_t> all;
        for (int32_t p = pe->ownStart; p < pe->ownEnd; ++p)
            if (!row_done(pe, p)) all.push_back(p);
        if ((rc = compute_positions_locked(pe, all.data(), (int32_t)all.size()))) return rc;
        if ((rc = ensure_full(pe, s, s))) return rc;
        HIPCHK(hipSetDevice(s->device));
        std::vector<Field> fields;
        table_fields(pe, fields);
        const size_t ts = pe->attached.size();
        for (const Field& f : fields)
            HIPCHK(hipMemcpyAsync((char*)field_ptr(s->full, f) + (size_t)s->rowStart * ts * f.esize,
                                  field_ptr(s->tab, f), (size_t)s->rowCount * ts * f.esize,
                                  hipMemcpyDeviceToDevice, s->stream));
        HIPCHK(hipStreamSynchronize(s->stream));
        pe->putInit = true;
    }
    HIPCHK(hipSetDevice(s->device));
    const size_t ts = pe->attached.size(), o = (size_t)start * ts, cells = (size_t)count * ts;
    HIPCHK(hipMemcpyAsync(s->full.lat + o, lat, cells * 8, hipMemcpyHostToDevice, s->stream));
    HIPCHK(hipMemcpyAsync(s->full.rel + o, rel, cells * 8, hipMemcpyHostToDevice, s->stream));
    HIPCHK(hipMemcpyAsync(s->full.hops + o, hops, cells * 4, hipMemcpyHostToDevice, s->stream));
    HIPCHK(hipMemcpyAsync(s->full.flags + o, flags, cells, hipMemcpyHostToDevice, s->stream));
    if (pe->opt.storePred)
        HIPCHK(hipMemcpyAsync(s->full.pred + o, pred, cells * 4, hipMemcpyHostToDevice, s->stream));
    HIPCHK(hipStreamSynchronize(s->stream));
    if (pe->putSeen.empty()) pe->putSeen.assign(ts, 0);
    for (int32_t p = start; p < start + count; ++p)
        if (!pe->putSeen[(size_t)p]) { pe->putSeen[(size_t)p] = 1; ++pe->putRows; }
    if (pe->putRows + (pe->ownEnd - pe->ownStart) >= (int64_t)ts) {
        for (size_t p = 0; p < ts; ++p) pe->rowDone[p].store(1, std::memory_order_release);
        pe->gathered = true;
    }
    return SHD_PE_OK;
}

extern "C" int shd_pe_gather(ShdPe* pe) {
    if (!pe) return SHD_PE_EINVAL;
    std::lock_guard<std::mutex> lk(pe->mu);
    std::lock_guard<std::mutex> lk2(pe->copyMu);
    if (pe->G > 1 && pe->opt.shardCount > 1 && !pe->xcomm) return SHD_PE_ECOMM;
    return gather_locked(pe);
}

extern "C" int shd_pe_comm_unique_id(void* out, int32_t bytes) {
    if (!out || bytes < (int32_t)sizeof(ncclUniqueId)) return SHD_PE_EINVAL;
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) return SHD_PE_ECOMM;
    std::memcpy(out, &id, sizeof(id));
    return SHD_PE_OK;
}

extern "C" int shd_pe_comm_init(ShdPe* pe, const void* uniqueId, int32_t bytes) {
    if (!pe || !uniqueId || bytes < (int32_t)sizeof(ncclUniqueId)) return SHD_PE_EINVAL;
    // (shardCount 1: a one-rank communicator -- the gather then runs the same
    // RCCL calls as at N > 1, an in-place all-gather of the engine's own
    // rows: how the RCCL path is exercised on a one-GPU box)
    if (pe->opt.nDevices != 1 || pe->opt.shardCount < 1) return SHD_PE_EINVAL;
    std::lock_guard<std::mutex> lk(pe->mu);
    if (pe->xcomm) return SHD_PE_OK;
    ncclUniqueId id;
    std::memcpy(&id, uniqueId, sizeof(id));
    if (hipSetDevice(pe->shards[0]->device) != hipSuccess) return SHD_PE_EHIP;
    if (ncclCommInitRank(&pe->xcomm, pe->opt.shardCount, id, pe->opt.shardIndex) != ncclSuccess) {
        pe->xcomm = nullptr;
        return SHD_PE_ECOMM;
    }
    return SHD_PE_OK;
}

extern "C" int32_t shd_pe_num_shards(const ShdPe* pe) { return pe ? pe->G : 0; }

extern "C" int shd_pe_shard_bounds(const ShdPe* pe, int32_t* bounds) {
    if (!pe || !bounds) return SHD_PE_EINVAL;
    std::memcpy(bounds, pe->bounds.data(), pe->bounds.size() * sizeof(int32_t));
    return SHD_PE_OK;
}

extern "C" int shd_pe_owned_range(const ShdPe* pe, int32_t* start, int32_t* count) {
    if (!pe) return SHD_PE_EINVAL;
    if (start) *start = pe->ownStart;
    if (count) *count = pe->ownEnd - pe->ownStart;
    return SHD_PE_OK;
}

// Streaming copy for the achievable-HBM reference: 16-B
// loads and stores (float4-shaped), each thread moving UNR consecutive-stride
// elements per iteration so UNR loads are in flight before the first store,
// grid-stride over a footprint far past the 256 MiB Infinity Cache.  The
// reference is the best of a few shapes (cache policy x workgroups per CU):
// the figure is what this box's HBM delivers to a well-formed copy.
typedef unsigned int v4u __attribute__((ext_vector_type(4)));
template <bool NT, int UNR>
__global__ __launch_bounds__(256) void k_stream_copy(const v4u* __restrict__ a,
                                                      v4u* __restrict__ b, size_t n) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + (UNR - 1) * stride < n; i += UNR * stride) {
        v4u x[UNR];
#pragma unroll
        for (int k = 0; k < UNR; ++k) x[k] = NT ? __builtin_nontemporal_load(&a[i + k * stride]) : a[i + k * stride];
#pragma unroll
        for (int k = 0; k < UNR; ++k) {
            if (NT) __builtin_nontemporal_store(x[k], &b[i + k * stride]);
            else b[i + k * stride] = x[k];
        }
    }
    for (; i < n; i += stride) b[i] = a[i];
}

// one-pass shape: no grid-stride loop, one workgroup per 256 x UNR
// elements (a grid of ~10^5 workgroups), UNR coalesced 4-KiB wave spans per
// thread in flight before the stores
template <bool NT, int UNR>
__global__ __launch_bounds__(256) void k_stream_copy1(const v4u* __restrict__ a,
                                                       v4u* __restrict__ b, size_t n) {
    const size_t base = (size_t)blockIdx.x * 256 * UNR + threadIdx.x;
    v4u x[UNR];
#pragma unroll
    for (int k = 0; k < UNR; ++k) {
        const size_t i = base + (size_t)k * 256;
        if (i < n) x[k] = NT ? __builtin_nontemporal_load(&a[i]) : a[i];
    }
#pragma unroll
    for (int k = 0; k < UNR; ++k) {
        const size_t i = base + (size_t)k * 256;
        if (i < n) {
            if (NT) __builtin_nontemporal_store(x[k], &b[i]);
            else b[i] = x[k];
        }
    }
}

extern "C" int shd_pe_stream_bandwidth(ShdPe* pe, int64_t bytes, int32_t iters, double* gbps) {
    if (!pe || !gbps || bytes < (1 << 20) || iters < 1) return SHD_PE_EINVAL;
    Shard* sh = pe->shards[0].get();
    HIPCHK(hipSetDevice(sh->device));
    const size_t n = (size_t)bytes / 16;
    void *a = nullptr, *b = nullptr;
    if (hipMalloc(&a, n * 16) != hipSuccess) return SHD_PE_ENOMEM;
    if (hipMalloc(&b, n * 16) != hipSuccess) { (void)hipFree(a); return SHD_PE_ENOMEM; }
    int rc = SHD_PE_OK;
    double best = 0.0;
    if (hipMemsetAsync(a, 0, n * 16, sh->stream) != hipSuccess) rc = SHD_PE_EHIP;
    // shapes: cache policy (plain / non-temporal) x 4 or 8 loads in flight per
    // thread x workgroups per CU (SHDPE_STREAM_WG_PER_CU adds one more)
    // plus the one-pass shape (shapes 12..19: policy x 4 / 8 / 2 / 1 per
    // thread; nt with 4 per thread is the best on the boxes seen, ~6.1 TB/s)
    const int wgs[3] = {4, 8, pe->tu.streamWgPerCU};
    for (int shape = 0; shape < 20 && !rc; ++shape) {
        const bool nt = shape & 1;
        const bool onePass = shape >= 12;
        const int unr = shape >= 18 ? 1 : shape >= 16 ? 2 : (shape >> 1) & 1 ? 8 : 4;
        const int grid = onePass ? (int)((n + 256 * (size_t)unr - 1) / (256 * (size_t)unr))
                                 : sh->numCUs * wgs[shape >> 2];
        auto launch = [&]() {
            const v4u* pa = (const v4u*)a;
            v4u* pb = (v4u*)b;
            if (onePass) {
                if (unr == 2 && nt) hipLaunchKernelGGL((k_stream_copy1<true, 2>), dim3(grid), dim3(256), 0, sh->stream, pa, pb, n);
                else if (unr == 2) hipLaunchKernelGGL((k_stream_copy1<false, 2>), dim3(grid), dim3(256), 0, sh->stream, pa, pb, n);
                else if (unr == 1 && nt) hipLaunchKernelGGL((k_stream_copy1<true, 1>), dim3(grid), dim3(256), 0, sh->stream, pa, pb, n);
                else if (unr == 1) hipLaunchKernelGGL((k_stream_copy1<false, 1>), dim3(grid), dim3(256), 0, sh->stream, pa, pb, n);
                else if (nt && unr == 8) hipLaunchKernelGGL((k_stream_copy1<true, 8>), dim3(grid), dim3(256), 0, sh->stream, pa, pb, n);
                else if (nt) hipLaunchKernelGGL((k_stream_copy1<true, 4>), dim3(grid), dim3(256), 0, sh->stream, pa, pb, n);
                else if (unr == 8) hipLaunchKernelGGL((k_stream_copy1<false, 8>), dim3(grid), dim3(256), 0, sh->stream, pa, pb, n);
                else hipLaunchKernelGGL((k_stream_copy1<false, 4>), dim3(grid), dim3(256), 0, sh->stream, pa, pb, n);
            } else if (nt && unr == 8) hipLaunchKernelGGL((k_stream_copy<true, 8>), dim3(grid), dim3(256), 0, sh->stream, pa, pb, n);
            else if (nt) hipLaunchKernelGGL((k_stream_copy<true, 4>), dim3(grid), dim3(256), 0, sh->stream, pa, pb, n);
            else if (unr == 8) hipLaunchKernelGGL((k_stream_copy<false, 8>), dim3(grid), dim3(256), 0, sh->stream, pa, pb, n);
            else hipLaunchKernelGGL((k_stream_copy<false, 4>), dim3(grid), dim3(256), 0, sh->stream, pa, pb, n);
        };
        launch();   // warm-up
        (void)hipEventRecord(sh->evA, sh->stream);
        for (int i = 0; i < iters; ++i) launch();
        (void)hipEventRecord(sh->evB, sh->stream);
        if (hipGetLastError() != hipSuccess || hipStreamSynchronize(sh->stream) != hipSuccess) {
            rc = SHD_PE_EHIP;
            break;
        }
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, sh->evA, sh->evB);
        const double gb = ms > 0.f ? 2.0 * (double)n * 16.0 * iters / (ms * 1e-3) / 1e9 : 0.0;
        if (pe->tu.debug)
            std::fprintf(stderr, "[shdpe] stream shape %d (%s, %d per thread, grid %d): %.0f GB/s\n", shape,
                         nt ? "nt" : "plain", unr, grid, gb);
        best = std::max(best, gb);
    }
    if (!rc) *gbps = best;
    (void)hipFree(a);
    (void)hipFree(b);
    return rc;
}

extern "C" int shd_pe_synchronize(ShdPe* pe) {
    if (!pe) return SHD_PE_EINVAL;
    for (auto& s : pe->shards) {
        HIPCHK(hipSetDevice(s->device));
        HIPCHK(hipStreamSynchronize(s->stream));
    }
    return SHD_PE_OK;
}

extern "C" void shd_pe_destroy(ShdPe* pe) {
    if (!pe) return;
    for (auto& s : pe->shards) destroy_shard(s.get());
    if (pe->xcomm) (void)ncclCommDestroy(pe->xcomm);
    for (unsigned char* h : pe->stage)
        if (h) (void)hipHostFree(h);
    delete pe;
}

extern "C" int shd_pe_is_complete(const ShdPe* pe) { return pe && pe->hg.isComplete ? 1 : 0; }

extern "C" int32_t shd_pe_num_attached(const ShdPe* pe) {
    return pe ? (int32_t)pe->attached.size() : 0;
}

extern "C" int shd_pe_attached(const ShdPe* pe, int32_t* out) {
    if (!pe || !out) return SHD_PE_EINVAL;
    std::memcpy(out, pe->attached.data(), pe->attached.size() * sizeof(int32_t));
    return SHD_PE_OK;
}

extern "C" int shd_pe_get_stats(const ShdPe* pe, ShdPeStats* out) {
    if (!pe || !out) return SHD_PE_EINVAL;
    // compute updates the per-shard stats under mu: snapshot under it too
    // (a call during a compute returns once that compute is done)
    std::lock_guard<std::mutex> lk(const_cast<ShdPe*>(pe)->mu);
    for (auto& sp : pe->shards) {                // live per-shard counters into the stats
        sp->stats.relaxCoopAborts = sp->coopAborts;
        sp->stats.batchCoop = sp->bcfg.coop >= 2 ? sp->bcfg.coop : 0;
    }
    ShdPeStats t = pe->shards[0]->stats;
    for (size_t i = 1; i < pe->shards.size(); ++i) {
        const ShdPeStats& s = pe->shards[i]->stats;
        t.rowsComputed += s.rowsComputed;
        t.rowsExact += s.rowsExact;
        t.rowsTieEarly += s.rowsTieEarly;
        t.rowsTieRepaired += s.rowsTieRepaired;
        t.relaxCoopAborts += s.relaxCoopAborts;
        t.arcsRelaxed += s.arcsRelaxed;
        t.msSparseKernel += s.msSparseKernel;
        t.msExactKernel += s.msExactKernel;
        t.msDirectKernel += s.msDirectKernel;
        t.msTotal = std::max(t.msTotal, s.msTotal);   // shards run concurrently
        t.launchesSparse += s.launchesSparse;
        t.launchesExact += s.launchesExact;
        t.launchesDirect += s.launchesDirect;
        t.msDenseKernel += s.msDenseKernel;
        t.launchesDense += s.launchesDense;
        t.denseSweeps += s.denseSweeps;
        t.denseFlops += s.denseFlops;
    }
    t.nShards = (int32_t)pe->shards.size();
    t.msGather = pe->msGather;
    *out = t;
    return SHD_PE_OK;
}

extern "C" int64_t shd_pe_stats_size(void) { return (int64_t)sizeof(ShdPeStats); }

extern "C" int shd_pe_get_stats_sized(const ShdPe* pe, void* out, int64_t outBytes) {
    if (!pe || !out || outBytes <= 0) return SHD_PE_EINVAL;
    ShdPeStats t;
    const int rc = shd_pe_get_stats(pe, &t);
    if (rc) return rc;
    std::memcpy(out, &t, (size_t)std::min<int64_t>(outBytes, (int64_t)sizeof(ShdPeStats)));
    return SHD_PE_OK;
}

extern "C" int shd_pe_reset_stats(ShdPe* pe) {
    if (!pe) return SHD_PE_EINVAL;
    std::lock_guard<std::mutex> lk(pe->mu);
    for (auto& sp : pe->shards) {
        ShdPeStats& st = sp->stats;
        ShdPeStats keep = st;
        std::memset(&st, 0, sizeof(st));
        st.mode = keep.mode;
        st.isComplete = keep.isComplete;
        st.nVertices = keep.nVertices;
        st.nArcs = keep.nArcs;
        st.nAttached = keep.nAttached;
        st.deltaUsed = keep.deltaUsed;
        st.batched = keep.batched;
        st.batchLanes = keep.batchLanes;
        st.batchWaves = keep.batchWaves;
        st.batchPostWaves = keep.batchPostWaves;
        sp->coopAborts = 0;
    }
    pe->msGather = 0.0;
    return SHD_PE_OK;
}

extern "C" int shd_pe_direct_path(const ShdPe* pe, int32_t s, int32_t t, double* lat,
                                  double* rel) {
    if (!pe) return SHD_PE_EINVAL;
    return host_direct_path(pe->hg, s, t, lat, rel);
}

extern "C" int shd_pe_self_path(const ShdPe* pe, int32_t v, double* lat, double* rel) {
    if (!pe) return SHD_PE_EINVAL;
    return host_self_path(pe->hg, v, lat, rel);
}

extern "C" int shd_pe_adjacent(const ShdPe* pe, int32_t s, int32_t t) {
    if (!pe) return 0;
    return pe->hg.findArc(s, t) != -1 ? 1 : 0;
}

// ---- batched helpers (pe_aux.hip) ----------------------------------------
// Inputs / outputs are host arrays; chunks of up to 16M entries are staged
// through device buffers owned by the call, on shard 0's device and stream.
namespace {
struct AuxBufs {
    void* p[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
    ~AuxBufs() { for (void* x : p) if (x) (void)hipFree(x); }
};
constexpr int64_t AUX_CHUNK = (int64_t)1 << 24;
}  // namespace

extern "C" int shd_pe_self_paths(ShdPe* pe, const int32_t* vertices, int32_t count, double* lat,
                                 double* rel, uint8_t* flags) {
    if (!pe || count < 0 || (count > 0 && (!vertices || !lat || !rel || !flags))) return SHD_PE_EINVAL;
    if (count == 0) return SHD_PE_OK;
    std::lock_guard<std::mutex> lk(pe->mu);
    Shard* sh = pe->shards[0].get();
    HIPCHK(hipSetDevice(sh->device));
    const int64_t ch = std::min<int64_t>(count, AUX_CHUNK);
    AuxBufs b;
    if (hipMalloc(&b.p[0], ch * 4) || hipMalloc(&b.p[1], ch * 8) || hipMalloc(&b.p[2], ch * 8) ||
        hipMalloc(&b.p[3], ch))
        return SHD_PE_ENOMEM;
    for (int64_t c0 = 0; c0 < count; c0 += ch) {
        const int32_t c = (int32_t)std::min<int64_t>(ch, count - c0);
        HIPCHK(hipMemcpyAsync(b.p[0], vertices + c0, (size_t)c * 4, hipMemcpyHostToDevice, sh->stream));
        launch_self_paths(sh->dgAux, (const int32_t*)b.p[0], c, pe->hg.nEdges, (double*)b.p[1],
                          (double*)b.p[2], (uint8_t*)b.p[3], sh->stream);
        HIPCHK(hipGetLastError());
        HIPCHK(hipMemcpyAsync(lat + c0, b.p[1], (size_t)c * 8, hipMemcpyDeviceToHost, sh->stream));
        HIPCHK(hipMemcpyAsync(rel + c0, b.p[2], (size_t)c * 8, hipMemcpyDeviceToHost, sh->stream));
        HIPCHK(hipMemcpyAsync(flags + c0, b.p[3], (size_t)c, hipMemcpyDeviceToHost, sh->stream));
        HIPCHK(hipStreamSynchronize(sh->stream));
    }
    return SHD_PE_OK;
}

static int pairs_call(ShdPe* pe, const int32_t* src, const int32_t* dst, int64_t count, int mode,
                      double* lat, double* rel, uint8_t* flags) {
    if (!pe || count < 0 || (count > 0 && (!src || !dst || !flags || (mode == 0 && (!lat || !rel)))))
        return SHD_PE_EINVAL;
    if (count == 0) return SHD_PE_OK;
    std::lock_guard<std::mutex> lk(pe->mu);
    Shard* sh = pe->shards[0].get();
    HIPCHK(hipSetDevice(sh->device));
    const int64_t ch = std::min<int64_t>(count, AUX_CHUNK);
    AuxBufs b;
    if (hipMalloc(&b.p[0], ch * 4) || hipMalloc(&b.p[1], ch * 4) || hipMalloc(&b.p[4], ch) ||
        (mode == 0 && (hipMalloc(&b.p[2], ch * 8) || hipMalloc(&b.p[3], ch * 8))))
        return SHD_PE_ENOMEM;
    for (int64_t c0 = 0; c0 < count; c0 += ch) {
        const int64_t c = std::min<int64_t>(ch, count - c0);
        HIPCHK(hipMemcpyAsync(b.p[0], src + c0, (size_t)c * 4, hipMemcpyHostToDevice, sh->stream));
        HIPCHK(hipMemcpyAsync(b.p[1], dst + c0, (size_t)c * 4, hipMemcpyHostToDevice, sh->stream));
        launch_pairs(sh->dgAux, (const int32_t*)b.p[0], (const int32_t*)b.p[1], c, mode,
                     (double*)b.p[2], (double*)b.p[3], (uint8_t*)b.p[4], sh->stream);
        HIPCHK(hipGetLastError());
        if (mode == 0) {
            HIPCHK(hipMemcpyAsync(lat + c0, b.p[2], (size_t)c * 8, hipMemcpyDeviceToHost, sh->stream));
            HIPCHK(hipMemcpyAsync(rel + c0, b.p[3], (size_t)c * 8, hipMemcpyDeviceToHost, sh->stream));
        }
        HIPCHK(hipMemcpyAsync(flags + c0, b.p[4], (size_t)c, hipMemcpyDeviceToHost, sh->stream));
        HIPCHK(hipStreamSynchronize(sh->stream));
    }
    return SHD_PE_OK;
}

extern "C" int shd_pe_direct_paths(ShdPe* pe, const int32_t* src, const int32_t* dst, int64_t count,
                                   double* lat, double* rel, uint8_t* flags) {
    return pairs_call(pe, src, dst, count, 0, lat, rel, flags);
}

extern "C" int shd_pe_adjacent_pairs(ShdPe* pe, const int32_t* src, const int32_t* dst,
                                     int64_t count, uint8_t* out) {
    return pairs_call(pe, src, dst, count, 1, nullptr, nullptr, out);
}

extern "C" int shd_pe_is_complete_device(ShdPe* pe, int32_t* isComplete) {
    if (!pe || !isComplete) return SHD_PE_EINVAL;
    std::lock_guard<std::mutex> lk(pe->mu);
    Shard* sh = pe->shards[0].get();
    HIPCHK(hipSetDevice(sh->device));
    AuxBufs b;
    if (hipMalloc(&b.p[0], 4)) return SHD_PE_ENOMEM;
    const int32_t init = INT32_MAX;
    HIPCHK(hipMemcpyAsync(b.p[0], &init, 4, hipMemcpyHostToDevice, sh->stream));
    const std::vector<int32_t>& ec = pe->hg.edgeCount;    // multigraphs: edge counts
    if (!ec.empty()) {
        if (hipMalloc(&b.p[1], ec.size() * 4)) return SHD_PE_ENOMEM;
        HIPCHK(hipMemcpyAsync(b.p[1], ec.data(), ec.size() * 4, hipMemcpyHostToDevice, sh->stream));
    }
    launch_incident_min(sh->dgAux, ec.empty() ? nullptr : (const int32_t*)b.p[1], (int32_t*)b.p[0], sh->stream);
    HIPCHK(hipGetLastError());
    int32_t mn = 0;
    HIPCHK(hipMemcpyAsync(&mn, b.p[0], 4, hipMemcpyDeviceToHost, sh->stream));
    HIPCHK(hipStreamSynchronize(sh->stream));
    *isComplete = mn >= pe->hg.n ? 1 : 0;
    return SHD_PE_OK;
}

// exported for the host topology mirror (pe_topology.cpp)
const shdpe::HostGraph* shd_pe_host_graph(const ShdPe* pe) { return pe ? &pe->hg : nullptr; }
int32_t shd_pe_position(const ShdPe* pe, int32_t v) {
    return (pe && v >= 0 && v < pe->hg.n) ? pe->posOf[v] : -1;
}

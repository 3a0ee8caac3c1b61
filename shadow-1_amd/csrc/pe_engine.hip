// pe_engine.hip -- C-ABI implementation of the MI355X Shadow path engine.
//
// Replaces topology.c:1681-1866 (target collection + igraph Dijkstra +
// per-target fold) with device kernels; see include/shd_pathengine.h.
// No CPU compute fallback: every row comes from a gfx950 kernel, and create
// fails with SHD_PE_ENODEV when no device is usable.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <new>
#include <vector>

#include "pe_device.hpp"
#include "pe_graph.hpp"
#include "shd_pathengine.h"

using namespace shdpe;

struct ShdPe {
    HostGraph hg;
    std::vector<int32_t> attached;   // unique, first-occurrence order
    std::vector<int32_t> posOf;      // vertex -> table position or -1
    ShdPeOptions opt{};
    int device = 0;
    int numCUs = 256;
    hipStream_t stream = nullptr;
    hipStream_t copyStream = nullptr;     // D2H of rows (shd_pe_get_rows)
    unsigned char* stage[2] = {nullptr, nullptr};   // pinned host staging
    size_t stageBytes = 0;
    std::mutex copyMu;
    hipEvent_t ev0 = nullptr, ev1 = nullptr, evA = nullptr, evB = nullptr;
    std::vector<void*> allocs;
    DevGraph dg{};
    DevTable tab{};
    DevScratch sc{};
    bool tableReady = false;
    int32_t* dRows = nullptr;
    uint8_t* dRowAmbig = nullptr;
    int32_t* dDbg = nullptr;          // per-row kernel counters (SHDPE_DEBUG=1)
    int32_t rowsCap = 0;
    SparseLaunch cfg{};
    int exactGrid = 0;
    int exactHc = 1;
    bool exactLdsIdx = false;
    int mode = 1;
    std::vector<uint8_t> rowDone;
    // batched multi-source sparse path (pe_batch.hip)
    bool batched = false;
    BatchLaunch bcfg{};
    BatchScratch bsc{};
    bool batchReady = false;
    int32_t* dBatchRows = nullptr;
    uint8_t* dBatchAmb = nullptr;
    std::vector<int32_t> rank;        // table position -> BFS visit rank
    // dense path (mode 3)
    double* dW = nullptr;
    double* dRl = nullptr;
    double* dD = nullptr;
    int32_t* dP = nullptr;
    uint8_t* dRowA = nullptr;
    uint8_t* dRowB = nullptr;
    uint8_t* dRowAmbD = nullptr;
    uint8_t* dChunkEpoch = nullptr;   // dense: last sweep that changed (row tile, K chunk)
    int32_t* dAny = nullptr;
    int32_t denseRows = 0;
    ShdPeStats stats{};
    std::mutex mu;
};

#define HIPCHK(x)                                   \
    do {                                            \
        if ((x) != hipSuccess) return SHD_PE_EHIP;  \
    } while (0)

static int dev_alloc(ShdPe* pe, void** p, size_t bytes) {
    if (bytes == 0) bytes = 16;
    if (hipMalloc(p, bytes) != hipSuccess) { *p = nullptr; return SHD_PE_ENOMEM; }
    pe->allocs.push_back(*p);
    return SHD_PE_OK;
}

template <class T>
static int dev_upload(ShdPe* pe, T** dst, const std::vector<T>& src) {
    int rc = dev_alloc(pe, reinterpret_cast<void**>(dst), src.size() * sizeof(T));
    if (rc) return rc;
    if (!src.empty())
        HIPCHK(hipMemcpy(*dst, src.data(), src.size() * sizeof(T), hipMemcpyHostToDevice));
    return SHD_PE_OK;
}

static double env_double(const char* name, double dflt) {
    const char* v = std::getenv(name);
    return (v && *v) ? std::atof(v) : dflt;
}

static int env_int(const char* name, int dflt) {
    const char* v = std::getenv(name);
    return (v && *v) ? std::atoi(v) : dflt;
}

extern "C" void shd_pe_default_options(ShdPeOptions* opt) {
    if (!opt) return;
    std::memset(opt, 0, sizeof(*opt));
    opt->device = 0;
    opt->batchRows = 0;
    opt->delta = 0.0;
    opt->storePred = 1;
    opt->forceMode = 0;
}

extern "C" const char* shd_pe_strerror(int code) {
    switch (code) {
        case SHD_PE_OK: return "ok";
        case SHD_PE_EINVAL: return "invalid argument or graph fails topology checks";
        case SHD_PE_ENOMEM: return "out of memory";
        case SHD_PE_ENODEV: return "no usable gfx950 device";
        case SHD_PE_EUNREACHABLE: return "target unreachable";
        case SHD_PE_ENOSELFLOOP: return "self-loop (s,s) missing";
        case SHD_PE_EMULTI: return "parallel edges (multigraph) are not supported";
        case SHD_PE_EHIP: return "HIP runtime error";
        case SHD_PE_ENOTATTACHED: return "vertex is not attached";
        case SHD_PE_ENOEDGE: return "no edge between the vertices";
        default: return "unknown error";
    }
}

static inline int a16(long x) { return (int)((x + 15) & ~15L); }

static void configure(ShdPe* pe) {
    const HostGraph& g = pe->hg;
    const long n = g.n;
    const long nw = (n + 31) / 32;
    const int LDS = 160 * 1024;
    SparseLaunch c{};
    c.threads = env_int("SHDPE_THREADS", 512);
    if (c.threads > sparse_max_threads()) c.threads = sparse_max_threads();
    c.hcap = 256;
    c.heavyDeg = env_int("SHDPE_HEAVY_DEG", 64);
    const int qmin = 2048;
    // LDS bytes per layout (queues are ping-pong pairs; LAYOUT 0/3 keep them in HBM)
    const int pend = a16(4 * nw), hbits = a16(4 * nw);
    const int hq2 = 2 * a16(4 * c.hcap);
    const int need2 = 64 + pend + hbits + hq2 + a16(8 * n) + a16(2 * n) + a16(4 * (n + 1));
    const int need1 = 64 + pend + hbits + hq2 + a16(8 * n);
    const int need3 = 64 + pend + a16(8 * n);
    const int need0 = 64 + pend + hbits;
    int layout = 0, used = need0;
    if (need2 + 8 * qmin <= LDS) { layout = 2; used = need2; }
    else if (need1 + 8 * qmin <= LDS) { layout = 1; used = need1; }
    // LAYOUT 3 keeps only dist + pending bits in LDS: ~1.4x slower per row
    // than LAYOUT 2 (measured, C2) but fits more rows per CU; take it when it
    // at least doubles the resident rows.
    const int maxWgByThreads = 2048 / std::max(c.threads, 64);
    const int wg2 = layout == 2 ? std::min(maxWgByThreads, LDS / (need2 + 8 * qmin)) : 0;
    const int wg3 = std::min(maxWgByThreads, LDS / need3);
    if (need3 <= LDS && wg3 >= 2 * std::max(wg2, 1)) { layout = 3; used = need3; }
    const int forced = env_int("SHDPE_LAYOUT", -1);
    if (forced == 3 && need3 <= LDS) { layout = 3; used = need3; }
    else if (forced == 2 && need2 + 8 * qmin <= LDS) { layout = 2; used = need2; }
    else if (forced == 1 && need1 + 8 * qmin <= LDS) { layout = 1; used = need1; }
    else if (forced == 0) { layout = 0; used = need0; }
    c.layout = layout;
    if (layout == 1 || layout == 2) {
        c.qcap = (int)std::min<long>((LDS - used) / 8, std::max<long>(n, 1024)) & ~3;
        c.ldsBytes = used + 2 * a16(4 * c.qcap);
    } else {
        c.qcap = (int)((n + 63) & ~63L);
        c.ldsBytes = used;
    }
    const int maxWG = env_int("SHDPE_WG_PER_CU", 8);
    const int wgPerCU = std::max(1, std::min({maxWG, LDS / std::max(c.ldsBytes, 1),
                                              2048 / c.threads}));
    c.grid = pe->numCUs * wgPerCU;
    const double factor = env_double("SHDPE_DELTA_FACTOR", 16.0);
    c.delta = pe->opt.delta > 0 ? pe->opt.delta : g.meanArcLatency * factor;
    if (!(c.delta > 0)) c.delta = 1.0;
    c.kflags = env_int("SHDPE_KFLAGS", 0);
    pe->cfg = c;
    // k_exact_rows: index2 (4n) in LDS up to n = 24k, heap entries (24 B)
    // in LDS up to the budget, the tail of the heap in the global slot.  A
    // whole heap that fits leaves room for several rows per CU.
    pe->exactLdsIdx = (size_t)4 * n <= 96 * 1024;
    const long idxB = pe->exactLdsIdx ? 4 * n : 0;
    const long perWG = std::min<long>(LDS, idxB + 24 * n + 16);
    pe->exactHc = (int)std::max<long>(1, std::min<long>(n, (perWG - idxB - 16) / 24));
    const int hcCap = env_int("SHDPE_EXACT_HC", 0);   // testing: force the global heap tail
    if (hcCap > 0) pe->exactHc = std::min(pe->exactHc, hcCap);
    const int exPerCU = (int)std::max<long>(1, std::min<long>(8, LDS / perWG));
    pe->exactGrid = pe->numCUs * env_int("SHDPE_EXACT_PER_CU", exPerCU);
    pe->stats.deltaUsed = c.delta;
    // Batched multi-source kernel: the layout for graphs whose per-row state
    // does not fit LDS (LAYOUT 0), or on request (SHDPE_BATCH=1 / forceMode 5).
    const int wantBatch = env_int("SHDPE_BATCH", -1);
    pe->batched = wantBatch == 1 || (wantBatch != 0 && layout == 0) || pe->opt.forceMode == 5;
    BatchLaunch b{};
    b.lb = env_int("SHDPE_BATCH_LB", 16);
    if (b.lb != 8 && b.lb != 32) b.lb = 16;
    b.threads = env_int("SHDPE_BATCH_THREADS", 1024);
    if (b.threads != 256 && b.threads != 512) b.threads = 1024;
    b.ldsBytes = batch_lds_bytes((int)n);
    int bPerCU = 1;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&bPerCU, batch_kernel_ptr(b.lb), b.threads,
                                                     b.ldsBytes) != hipSuccess || bPerCU < 1)
        bPerCU = 1;
    b.grid = pe->numCUs * bPerCU;
    const int gcap = env_int("SHDPE_BATCH_GRID", 0);
    if (gcap > 0 && gcap < b.grid) b.grid = gcap;
    const double bf = env_double("SHDPE_BATCH_DELTA_FACTOR", 8.0);
    b.delta = pe->opt.delta > 0 ? pe->opt.delta : g.meanArcLatency * bf;
    if (!(b.delta > 0)) b.delta = 1.0;
    pe->bcfg = b;
    if (pe->batched) pe->stats.deltaUsed = b.delta;
    pe->stats.batched = pe->batched ? 1 : 0;
    pe->stats.batchLanes = pe->batched ? b.lb : 0;
}

// BFS visit rank of every table position (components in vertex order):
// batches of nearby sources share their delta-stepping frontiers.
static void compute_ranks(ShdPe* pe) {
    const HostGraph& g = pe->hg;
    std::vector<int32_t> order;
    order.reserve(g.n);
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
    pe->rank.assign(pe->attached.size(), 0);
    int32_t k = 0;
    for (int32_t v : order)
        if (pe->posOf[v] >= 0) pe->rank[pe->posOf[v]] = k++;
}

extern "C" int shd_pe_create(const ShdPeGraphDesc* graph, const int32_t* attached,
                             int32_t nAttached, const ShdPeOptions* opt, ShdPe** out) {
    if (!out || !graph || nAttached <= 0 || !attached) return SHD_PE_EINVAL;
    *out = nullptr;
    ShdPe* pe = new (std::nothrow) ShdPe();
    if (!pe) return SHD_PE_ENOMEM;
    if (opt) pe->opt = *opt; else shd_pe_default_options(&pe->opt);
    int rc = build_host_graph(graph, &pe->hg);
    if (rc) { delete pe; return rc; }
    const HostGraph& g = pe->hg;
    pe->posOf.assign(g.n, -1);
    for (int32_t i = 0; i < nAttached; ++i) {
        const int32_t v = attached[i];
        if (v < 0 || v >= g.n) { delete pe; return SHD_PE_EINVAL; }
        if (pe->posOf[v] < 0) {
            pe->posOf[v] = (int32_t)pe->attached.size();
            pe->attached.push_back(v);
        }
    }
    // ---- device ----
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0 || pe->opt.device < 0 ||
        pe->opt.device >= ndev) {
        delete pe;
        return SHD_PE_ENODEV;
    }
    pe->device = pe->opt.device;
    if (hipSetDevice(pe->device) != hipSuccess) { delete pe; return SHD_PE_ENODEV; }
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, pe->device) != hipSuccess) { delete pe; return SHD_PE_ENODEV; }
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) { delete pe; return SHD_PE_ENODEV; }
    pe->numCUs = prop.multiProcessorCount;
    if (hipStreamCreateWithFlags(&pe->stream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreate(&pe->ev0) != hipSuccess || hipEventCreate(&pe->ev1) != hipSuccess ||
        hipEventCreate(&pe->evA) != hipSuccess || hipEventCreate(&pe->evB) != hipSuccess) {
        shd_pe_destroy(pe);
        return SHD_PE_ENODEV;
    }
    configure(pe);
    const int32_t T = (int32_t)pe->attached.size();
    DevGraph& d = pe->dg;
    d.n = g.n;
    d.T = T;
    std::vector<uint8_t> isAtt(g.n, 0);
    for (int32_t v : pe->attached) isAtt[v] = 1;
    int32_t *rowPtr, *col, *outToIn, *att;
    double *lat, *rel, *vrel, *sl, *sr;
    uint8_t *hs, *ia;
    if ((rc = dev_upload(pe, &rowPtr, g.rowPtr)) || (rc = dev_upload(pe, &col, g.col)) ||
        (rc = dev_upload(pe, &lat, g.lat)) || (rc = dev_upload(pe, &rel, g.rel)) ||
        (rc = dev_upload(pe, &outToIn, g.outToIn)) || (rc = dev_upload(pe, &vrel, g.vrel)) ||
        (rc = dev_upload(pe, &sl, g.selfLat)) || (rc = dev_upload(pe, &sr, g.selfRel)) ||
        (rc = dev_upload(pe, &hs, g.hasSelf)) || (rc = dev_upload(pe, &att, pe->attached)) ||
        (rc = dev_upload(pe, &ia, isAtt))) {
        shd_pe_destroy(pe);
        return rc;
    }
    {
        std::vector<Arc> arcs(g.col.size());
        for (size_t a = 0; a < arcs.size(); ++a) arcs[a] = Arc{g.lat[a], g.col[a], 0};
        Arc* da;
        if ((rc = dev_upload(pe, &da, arcs))) { shd_pe_destroy(pe); return rc; }
        d.arcs = da;
        std::vector<Arc3> a3(g.col.size());
        for (size_t a = 0; a < a3.size(); ++a) {
            uint64_t bits;
            std::memcpy(&bits, &g.lat[a], 8);
            a3[a] = Arc3{g.col[a], (uint32_t)bits, (uint32_t)(bits >> 32)};
        }
        Arc3* d3;
        if ((rc = dev_upload(pe, &d3, a3))) { shd_pe_destroy(pe); return rc; }
        d.arc3 = d3;
    }
    d.rowPtr = rowPtr; d.col = col; d.lat = lat; d.rel = rel; d.outToIn = outToIn;
    d.vrel = vrel; d.selfLat = sl; d.selfRel = sr; d.hasSelf = hs; d.attached = att;
    d.isAttached = ia;
    {
        const int hd = pe->cfg.heavyDeg;
        std::vector<uint32_t> hb((g.n + 31) / 32, 0u);
        for (int32_t v = 0; v < g.n; ++v)
            if (g.rowPtr[v + 1] - g.rowPtr[v] >= hd) hb[v >> 5] |= 1u << (v & 31);
        uint32_t* dhb;
        if ((rc = dev_upload(pe, &dhb, hb))) { shd_pe_destroy(pe); return rc; }
        d.heavyBits = dhb;
    }
    if (g.directed) {
        int32_t *ip, *ic;
        double *il, *ir;
        if ((rc = dev_upload(pe, &ip, g.inPtr)) || (rc = dev_upload(pe, &ic, g.inCol)) ||
            (rc = dev_upload(pe, &il, g.inLat)) || (rc = dev_upload(pe, &ir, g.inRel))) {
            shd_pe_destroy(pe);
            return rc;
        }
        d.inPtr = ip; d.inCol = ic; d.inLat = il; d.inRel = ir;
    } else {
        d.inPtr = rowPtr; d.inCol = col; d.inLat = lat; d.inRel = rel;
    }
    pe->mode = (g.isComplete && pe->opt.forceMode != 1 && pe->opt.forceMode != 3) ? 2 : 1;
    if (pe->opt.forceMode == 2) pe->mode = 2;
    {
        // dense non-complete graphs: blocked min-plus (K2)
        const double density = (double)g.nArcs() / ((double)g.n * (double)g.n);
        const double dmin = env_double("SHDPE_DENSE_MIN", 0.25);
        const bool fitsDense = (int64_t)g.n <= 65536;
        if (pe->mode == 1 && pe->opt.forceMode == 0 && fitsDense && density >= dmin) pe->mode = 3;
        if (pe->opt.forceMode == 4 && fitsDense) pe->mode = 3;
    }
    pe->rowDone.assign(T, 0);
    if (pe->opt.forceMode == 5) pe->mode = 1;
    if (pe->mode == 1 && pe->batched) compute_ranks(pe);
    pe->stats.mode = pe->mode;
    pe->stats.isComplete = g.isComplete ? 1 : 0;
    pe->stats.nVertices = g.n;
    pe->stats.nArcs = g.nArcs();
    pe->stats.nAttached = T;
    *out = pe;
    return SHD_PE_OK;
}

static int ensure_table(ShdPe* pe) {
    if (pe->tableReady) return SHD_PE_OK;
    const size_t T = pe->attached.size();
    const size_t cells = T * T;
    int rc;
    void *lat, *rel, *hops, *flags, *pred = nullptr;
    if ((rc = dev_alloc(pe, &lat, cells * 8)) || (rc = dev_alloc(pe, &rel, cells * 8)) ||
        (rc = dev_alloc(pe, &hops, cells * 4)) || (rc = dev_alloc(pe, &flags, cells)))
        return rc;
    if (pe->opt.storePred && (rc = dev_alloc(pe, &pred, cells * 4))) return rc;
    pe->tab.lat = (double*)lat;
    pe->tab.rel = (double*)rel;
    pe->tab.hops = (int32_t*)hops;
    pe->tab.flags = (uint8_t*)flags;
    pe->tab.pred = (int32_t*)pred;
    pe->tab.T = (int64_t)T;
    // scratch slots
    const int slots = pe->batched ? pe->exactGrid : std::max(pe->cfg.grid, pe->exactGrid);
    const size_t stride = ((size_t)pe->hg.n + 63) & ~(size_t)63;
    const size_t heapStride = std::max<size_t>(1, (size_t)pe->hg.n - (size_t)pe->exactHc);
    void *dist, *sh, *sr, *sp, *hk, *i2;
    if ((rc = dev_alloc(pe, &dist, slots * stride * 8)) ||
        (rc = dev_alloc(pe, &sh, slots * stride * 4)) ||
        (rc = dev_alloc(pe, &sr, slots * stride * 8)) ||
        (rc = dev_alloc(pe, &sp, slots * stride * 4)) ||
        (rc = dev_alloc(pe, &hk, (size_t)pe->exactGrid * heapStride * sizeof(XEnt))) ||
        (rc = dev_alloc(pe, &i2, pe->exactLdsIdx ? 16 : (size_t)pe->exactGrid * stride * 4)))
        return rc;
    pe->sc.dist = (double*)dist;
    pe->sc.hops = (int32_t*)sh;
    pe->sc.rel = (double*)sr;
    pe->sc.pred = (int32_t*)sp;
    pe->sc.heapEnt = (XEnt*)hk;
    pe->sc.heapStride = (int64_t)heapStride;
    pe->sc.index2 = (int32_t*)i2;
    pe->sc.stride = (int64_t)stride;
    if (!pe->batched && (pe->cfg.layout == 3 || pe->cfg.layout == 0)) {
        void* q;
        const size_t per = 2 * ((size_t)pe->cfg.qcap + pe->cfg.hcap);
        if ((rc = dev_alloc(pe, &q, (size_t)pe->cfg.grid * per * 4))) return rc;
        pe->sc.queue = (int32_t*)q;
    }
    pe->rowsCap = (int32_t)std::min<size_t>(T, 1 << 20);
    void *rows, *amb;
    if ((rc = dev_alloc(pe, &rows, (size_t)pe->rowsCap * 4)) ||
        (rc = dev_alloc(pe, &amb, (size_t)pe->rowsCap)))
        return rc;
    pe->dRows = (int32_t*)rows;
    pe->dRowAmbig = (uint8_t*)amb;
    if (env_int("SHDPE_DEBUG", 0)) {
        void* dbg;
        if ((rc = dev_alloc(pe, &dbg, (size_t)pe->rowsCap * 64))) return rc;
        pe->dDbg = (int32_t*)dbg;
    }
    pe->tableReady = true;
    return SHD_PE_OK;
}

static int ensure_batch(ShdPe* pe) {
    if (pe->batchReady) return SHD_PE_OK;
    const size_t NS = ((size_t)pe->hg.n + 63) & ~(size_t)63;
    const size_t LB = (size_t)pe->bcfg.lb;
    const size_t perSlot = NS * LB * (8 + 8 + 4 + 4 + 16) + NS * 4 * 3;
    // scratch budget (default 64 GiB): fewer resident batches on huge graphs
    const double budget = env_double("SHDPE_BATCH_SCRATCH_GB", 64.0) * (double)(1ull << 30);
    const size_t maxSlots = std::max<size_t>(1, (size_t)(budget / (double)perSlot));
    const size_t nBatchesAll = (pe->attached.size() + LB - 1) / LB;
    size_t slots = std::min<size_t>({(size_t)pe->bcfg.grid, maxSlots, std::max<size_t>(1, nBatchesAll)});
    pe->bcfg.grid = (int32_t)slots;
    int rc;
    void *D, *R, *H, *P, *X, *pm, *q, *rows, *amb;
    if ((rc = dev_alloc(pe, &D, slots * NS * LB * 8)) || (rc = dev_alloc(pe, &R, slots * NS * LB * 8)) ||
        (rc = dev_alloc(pe, &X, slots * NS * LB * 16)) ||
        (rc = dev_alloc(pe, &H, slots * NS * LB * 4)) || (rc = dev_alloc(pe, &P, slots * NS * LB * 4)) ||
        (rc = dev_alloc(pe, &pm, slots * NS * 2 * 4)) || (rc = dev_alloc(pe, &q, slots * NS * 4)) ||
        (rc = dev_alloc(pe, &rows, ((size_t)pe->rowsCap + 64) * 4)) ||
        (rc = dev_alloc(pe, &amb, (size_t)pe->rowsCap + 64)))
        return rc;
    pe->bsc.D = (unsigned long long*)D;
    pe->bsc.R = (double*)R;
    pe->bsc.H = (int32_t*)H;
    pe->bsc.P = (int32_t*)P;
    pe->bsc.X = (int32_t*)X;
    pe->bsc.pm = (uint32_t*)pm;
    pe->bsc.queue = (int32_t*)q;
    pe->bsc.nStride = (int64_t)NS;
    pe->dBatchRows = (int32_t*)rows;
    pe->dBatchAmb = (uint8_t*)amb;
    pe->batchReady = true;
    return SHD_PE_OK;
}

static int ensure_dense(ShdPe* pe) {
    if (pe->dW) return SHD_PE_OK;
    const int64_t n = pe->hg.n;
    const int64_t T = (int64_t)pe->attached.size();
    int rc;
    void *w, *rl, *d, *p, *ra, *rb, *am, *any, *ce;
    // rows per batch: D (f64) + P (i32) per row
    const int64_t budget = (int64_t)env_double("SHDPE_DENSE_BATCH_GB", 24.0) * (1LL << 30);
    int64_t rows = std::max<int64_t>(64, budget / (n * 12));
    rows = std::min<int64_t>(rows, T);
    if ((rc = dev_alloc(pe, &w, (size_t)(n * n * 8))) || (rc = dev_alloc(pe, &rl, (size_t)(n * n * 8))) ||
        (rc = dev_alloc(pe, &d, (size_t)(rows * n * 8))) || (rc = dev_alloc(pe, &p, (size_t)(rows * n * 4))) ||
        (rc = dev_alloc(pe, &ra, (size_t)rows)) || (rc = dev_alloc(pe, &rb, (size_t)rows)) ||
        (rc = dev_alloc(pe, &am, (size_t)rows)) || (rc = dev_alloc(pe, &any, 16)) ||
        (rc = dev_alloc(pe, &ce, (size_t)((rows / 16 + 1) * (n / 16 + 1)))))
        return rc;
    pe->dChunkEpoch = (uint8_t*)ce;
    pe->dW = (double*)w; pe->dRl = (double*)rl; pe->dD = (double*)d; pe->dP = (int32_t*)p;
    pe->dRowA = (uint8_t*)ra; pe->dRowB = (uint8_t*)rb; pe->dRowAmbD = (uint8_t*)am;
    pe->dAny = (int32_t*)any;
    pe->denseRows = (int32_t)rows;
    launch_dense_build(pe->dg, pe->dW, pe->dRl, n, pe->hg.nArcs(), pe->stream);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(pe->stream));
    return SHD_PE_OK;
}

static float elapsed(hipEvent_t a, hipEvent_t b) {
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, a, b);
    return ms;
}

// Compute the given table positions (chunked); caller holds pe->mu.
static int compute_positions_locked(ShdPe* pe, const int32_t* pos, int32_t count) {
    if (count <= 0) return SHD_PE_OK;
    if (hipSetDevice(pe->device) != hipSuccess) return SHD_PE_EHIP;
    int rc = ensure_table(pe);
    if (rc) return rc;
    std::vector<uint8_t> amb;
    std::vector<int32_t> exactRows;
    HIPCHK(hipEventRecord(pe->ev0, pe->stream));
    for (int32_t c0 = 0; c0 < count; c0 += pe->rowsCap) {
        const int32_t cnt = std::min(pe->rowsCap, count - c0);
        HIPCHK(hipMemcpyAsync(pe->dRows, pos + c0, (size_t)cnt * 4, hipMemcpyHostToDevice,
                              pe->stream));
        exactRows.clear();
        if (pe->mode == 2) {
            HIPCHK(hipEventRecord(pe->evA, pe->stream));
            launch_direct_rows(pe->dg, pe->tab, pe->dRows, cnt, pe->stream);
            HIPCHK(hipGetLastError());
            HIPCHK(hipEventRecord(pe->evB, pe->stream));
            HIPCHK(hipEventSynchronize(pe->evB));
            pe->stats.msDirectKernel += elapsed(pe->evA, pe->evB);
            pe->stats.launchesDirect++;
        } else if (pe->opt.forceMode == 3) {
            exactRows.assign(pos + c0, pos + c0 + cnt);
        } else if (pe->mode == 3) {
            if ((rc = ensure_dense(pe))) return rc;
            for (int32_t d0 = 0; d0 < cnt; d0 += pe->denseRows) {
                const int32_t dc = std::min(pe->denseRows, cnt - d0);
                HIPCHK(hipEventRecord(pe->evA, pe->stream));
                int sweeps = 0;
                double flops = 0.0;
                if (launch_dense_rows(pe->dg, pe->tab, pe->dW, pe->dRl, pe->dD, pe->dP, pe->dRowA,
                                      pe->dRowB, pe->dRowAmbD, pe->dAny, pe->dChunkEpoch,
                                      pe->dRows + d0, dc,
                                      pe->hg.n, pe->stream, &sweeps, &flops))
                    return SHD_PE_EHIP;
                HIPCHK(hipGetLastError());
                HIPCHK(hipEventRecord(pe->evB, pe->stream));
                amb.resize(dc);
                HIPCHK(hipMemcpyAsync(amb.data(), pe->dRowAmbD, dc, hipMemcpyDeviceToHost,
                                      pe->stream));
                HIPCHK(hipStreamSynchronize(pe->stream));
                pe->stats.msDenseKernel += elapsed(pe->evA, pe->evB);
                pe->stats.launchesDense++;
                pe->stats.denseSweeps += sweeps;
                pe->stats.denseFlops += flops;
                for (int32_t i = 0; i < dc; ++i)
                    if (amb[i]) exactRows.push_back(pos[c0 + d0 + i]);
            }
        } else if (pe->batched) {
            if ((rc = ensure_batch(pe))) return rc;
            // batches of LB nearby sources (BFS rank order), -1 pads the last
            const int LB = pe->bcfg.lb;
            std::vector<int32_t> order(pos + c0, pos + c0 + cnt);
            std::stable_sort(order.begin(), order.end(),
                             [&](int32_t a, int32_t b) { return pe->rank[a] < pe->rank[b]; });
            const int32_t nB = (cnt + LB - 1) / LB;
            order.resize((size_t)nB * LB, -1);
            HIPCHK(hipMemcpyAsync(pe->dBatchRows, order.data(), order.size() * 4,
                                  hipMemcpyHostToDevice, pe->stream));
            if (pe->dDbg) HIPCHK(hipMemsetAsync(pe->dDbg, 0, (size_t)nB * 64, pe->stream));
            HIPCHK(hipEventRecord(pe->evA, pe->stream));
            launch_batch_rows(pe->dg, pe->tab, pe->bsc, pe->dBatchRows, nB, pe->dBatchAmb, pe->bcfg,
                              pe->dDbg, pe->stream);
            HIPCHK(hipGetLastError());
            HIPCHK(hipEventRecord(pe->evB, pe->stream));
            amb.resize(order.size());
            HIPCHK(hipMemcpyAsync(amb.data(), pe->dBatchAmb, order.size(), hipMemcpyDeviceToHost,
                                  pe->stream));
            HIPCHK(hipStreamSynchronize(pe->stream));
            pe->stats.msSparseKernel += elapsed(pe->evA, pe->evB);
            pe->stats.launchesSparse++;
            for (size_t i = 0; i < order.size(); ++i)
                if (order[i] >= 0 && amb[i]) exactRows.push_back(order[i]);
            if (pe->dDbg) {
                std::vector<int32_t> dbg((size_t)nB * 16);
                HIPCHK(hipMemcpy(dbg.data(), pe->dDbg, dbg.size() * 4, hipMemcpyDeviceToHost));
                double ph = 0, pr = 0, kc[5] = {0, 0, 0, 0, 0}, arcsP = 0, lanesP = 0, bmax = 0, bmean = 0, cand = 0;
                long rnd = 0, dmax = 0, ambB = 0, rep = 0;
                for (int32_t i = 0; i < nB; ++i) {
                    const int32_t* d = dbg.data() + 16 * i;
                    ph += d[0]; rnd += d[1]; dmax = std::max<long>(dmax, d[2]);
                    ambB += d[3] != 0;
                    rep += d[15];
                    pr += d[4];
                    for (int k = 0; k < 3; ++k) kc[k] += 1024.0 * d[5 + k];
                    kc[3] += 1024.0 * d[11];
                    kc[4] += 1024.0 * d[8];
                    arcsP += 16.0 * d[9];
                    bmax += 1024.0 * d[12]; bmean += 1024.0 * d[13]; cand += d[14];
                    lanesP += d[10];
                }
                std::fprintf(stderr, "[shdpe] batch relax Mcycles/batch: sum over phases of group-busy max=%.2f mean=%.2f | candidates/batch=%.0f\n",
                             bmax / nB / 1e6, bmean / nB / 1e6, cand / nB);
                std::fprintf(stderr, "[shdpe] batch arc-visits/batch=%.0f (%.2f x nArcs) active lanes/proc=%.2f\n",
                             arcsP / nB, arcsP / nB / (double)pe->hg.nArcs(), lanesP / std::max(pr, 1.0));
                std::fprintf(stderr, "[shdpe] batch Mcycles/batch: relax=%.2f pred=%.2f "
                             "depth=%.2f rel=%.2f write=%.2f\n", kc[0] / nB / 1e6, kc[1] / nB / 1e6,
                             kc[2] / nB / 1e6, kc[3] / nB / 1e6, kc[4] / nB / 1e6);
                std::fprintf(stderr, "[shdpe] batch LB=%d batches=%d grid=%d delta=%.3f | phases/batch=%.1f "
                             "vertex-procs/batch=%.0f (%.2f per vertex) | jump rounds/batch=%.1f max depth=%ld amb batches=%ld repairs=%ld\n",
                             LB, nB, pe->bcfg.grid, pe->bcfg.delta, ph / nB, pr / nB,
                             pr / nB / pe->hg.n, (double)rnd / nB, dmax, ambB, rep);
            }
        } else {
            HIPCHK(hipEventRecord(pe->evA, pe->stream));
            launch_sparse_rows(pe->dg, pe->tab, pe->sc, pe->dRows, cnt, pe->dRowAmbig, pe->cfg,
                               pe->dDbg, pe->stream);
            HIPCHK(hipGetLastError());
            HIPCHK(hipEventRecord(pe->evB, pe->stream));
            amb.resize(cnt);
            HIPCHK(hipMemcpyAsync(amb.data(), pe->dRowAmbig, cnt, hipMemcpyDeviceToHost,
                                  pe->stream));
            HIPCHK(hipStreamSynchronize(pe->stream));
            pe->stats.msSparseKernel += elapsed(pe->evA, pe->evB);
            pe->stats.launchesSparse++;
            for (int32_t i = 0; i < cnt; ++i)
                if (amb[i]) exactRows.push_back(pos[c0 + i]);
            if (pe->dDbg) {
                std::vector<int32_t> dbg((size_t)cnt * 16);
                HIPCHK(hipMemcpy(dbg.data(), pe->dDbg, dbg.size() * 4, hipMemcpyDeviceToHost));
                double ph = 0, cy[4] = {0, 0, 0, 0}, sub[4] = {0, 0, 0, 0};
                int phMax = 0, jMax = 0, mis = 0, am = 0; long jSum = 0;
                for (int32_t i = 0; i < cnt; ++i) {
                    const int32_t* d = dbg.data() + 16 * i;
                    ph += d[0]; phMax = std::max(phMax, d[0]);
                    jMax = std::max(jMax, d[1]); jSum += d[1];
                    mis += d[2] != 0; am += d[3] != 0;
                    for (int k = 0; k < 4; ++k) cy[k] += 16.0 * d[4 + k];
                    for (int k = 0; k < 4; ++k) sub[k] += 16.0 * d[8 + k];
                }
                {
                    double a0 = 0, a1 = 0, a2 = 0, calls = 0;
                    for (int32_t i = 0; i < cnt; ++i) {
                        a0 += 16.0 * dbg[16 * i + 12]; a1 += 16.0 * dbg[16 * i + 13];
                        a2 += 16.0 * dbg[16 * i + 14]; calls += dbg[16 * i + 15];
                    }
                    std::fprintf(stderr, "[shdpe] group call (wave0): calls/row=%.1f cyc arcs=%.0f "
                                 "reduce=%.0f label=%.0f\n", calls / cnt, a0 / calls, a1 / calls,
                                 a2 / calls);
                }
                std::fprintf(stderr,
                             "[shdpe] sparse rows=%d phases mean=%.1f max=%d | mismatch rows=%d "
                             "jacobi rounds sum=%ld max=%d | ambiguous rows=%d | delta=%.3f | "
                             "kcycles/row scan=%.1f relax=%.1f final=%.1f write=%.1f | "
                             "cyc/phase bits=%.0f resv=%.0f light=%.0f heavy=%.0f\n",
                             cnt, ph / cnt, phMax, mis, jSum, jMax, am, pe->cfg.delta,
                             cy[0] / cnt / 1e3, cy[1] / cnt / 1e3, cy[2] / cnt / 1e3,
                             cy[3] / cnt / 1e3, sub[0] / ph, sub[1] / ph, sub[2] / ph,
                             sub[3] / ph);
            }
        }
        if (!exactRows.empty()) {
            HIPCHK(hipMemcpyAsync(pe->dRows, exactRows.data(), exactRows.size() * 4,
                                  hipMemcpyHostToDevice, pe->stream));
            HIPCHK(hipEventRecord(pe->evA, pe->stream));
            launch_exact_rows(pe->dg, pe->tab, pe->sc, pe->dRows, (int32_t)exactRows.size(),
                              pe->exactGrid, pe->exactHc, pe->exactLdsIdx, pe->stream);
            HIPCHK(hipGetLastError());
            HIPCHK(hipEventRecord(pe->evB, pe->stream));
            HIPCHK(hipEventSynchronize(pe->evB));
            pe->stats.msExactKernel += elapsed(pe->evA, pe->evB);
            pe->stats.launchesExact++;
            pe->stats.rowsExact += (int64_t)exactRows.size();
        }
    }
    HIPCHK(hipEventRecord(pe->ev1, pe->stream));
    HIPCHK(hipEventSynchronize(pe->ev1));
    pe->stats.msTotal += elapsed(pe->ev0, pe->ev1);
    pe->stats.rowsComputed += count;
    pe->stats.arcsRelaxed += (int64_t)count * pe->hg.nArcs();
    for (int32_t i = 0; i < count; ++i) pe->rowDone[pos[i]] = 1;
    return SHD_PE_OK;
}

extern "C" int shd_pe_compute_positions(ShdPe* pe, int32_t start, int32_t count) {
    if (!pe || start < 0 || count < 0 || (int64_t)start + count > (int64_t)pe->attached.size())
        return SHD_PE_EINVAL;
    std::vector<int32_t> pos(count);
    for (int32_t i = 0; i < count; ++i) pos[i] = start + i;
    std::lock_guard<std::mutex> lk(pe->mu);
    return compute_positions_locked(pe, pos.data(), count);
}

extern "C" int shd_pe_compute_all(ShdPe* pe) {
    if (!pe) return SHD_PE_EINVAL;
    return shd_pe_compute_positions(pe, 0, (int32_t)pe->attached.size());
}

extern "C" int shd_pe_compute_rows(ShdPe* pe, const int32_t* src, int32_t count) {
    if (!pe || count < 0 || (count > 0 && !src)) return SHD_PE_EINVAL;
    std::vector<int32_t> pos(count);
    for (int32_t i = 0; i < count; ++i) {
        if (src[i] < 0 || src[i] >= pe->hg.n || pe->posOf[src[i]] < 0) return SHD_PE_ENOTATTACHED;
        pos[i] = pe->posOf[src[i]];
    }
    std::lock_guard<std::mutex> lk(pe->mu);
    return compute_positions_locked(pe, pos.data(), count);
}

static int get_rows_staged(ShdPe* pe, int32_t start, int32_t count, double* lat, double* rel,
                           int32_t* hops, int32_t* pred, uint8_t* flags);

extern "C" int shd_pe_get_row(ShdPe* pe, int32_t srcVertex, double* lat, double* rel,
                              int32_t* hops, int32_t* pred, uint8_t* flags) {
    if (!pe || srcVertex < 0 || srcVertex >= pe->hg.n) return SHD_PE_EINVAL;
    const int32_t p = pe->posOf[srcVertex];
    if (p < 0) return SHD_PE_ENOTATTACHED;
    if (pred && !pe->opt.storePred) return SHD_PE_EINVAL;
    if (!pe->rowDone[p]) {
        std::lock_guard<std::mutex> lk(pe->mu);
        if (!pe->rowDone[p]) {
            int rc = compute_positions_locked(pe, &p, 1);
            if (rc) return rc;
        }
    }
    return get_rows_staged(pe, p, 1, lat, rel, hops, pred, flags);
}

// Rows [start, start+count) -> caller host buffers through two pinned
// staging buffers: block b's five field copies run on copyStream while the
// host copies block b-1 out of the other buffer.
static int get_rows_staged(ShdPe* pe, int32_t start, int32_t count, double* lat, double* rel,
                           int32_t* hops, int32_t* pred, uint8_t* flags) {
    const size_t T = pe->attached.size();
    const size_t perRow = T * (8 + 8 + 4 + 4 + 1);
    std::lock_guard<std::mutex> lk(pe->copyMu);
    HIPCHK(hipSetDevice(pe->device));
    if (!pe->copyStream) HIPCHK(hipStreamCreateWithFlags(&pe->copyStream, hipStreamNonBlocking));
    if (!pe->stage[0]) {
        const size_t want = std::max<size_t>(perRow, (size_t)32 << 20);
        for (auto& h : pe->stage) HIPCHK(hipHostMalloc(reinterpret_cast<void**>(&h), want));
        pe->stageBytes = want;
    }
    const int32_t B = (int32_t)std::max<size_t>(1, pe->stageBytes / perRow);
    struct Blk { int32_t r0, n; };
    auto issue = [&](int buf, Blk b) -> int {
        unsigned char* h = pe->stage[buf];
        const size_t off = ((size_t)start + b.r0) * T, cells = (size_t)b.n * T;
        unsigned char* q = h;
        if (lat) { HIPCHK(hipMemcpyAsync(q, pe->tab.lat + off, cells * 8, hipMemcpyDeviceToHost, pe->copyStream)); q += cells * 8; }
        if (rel) { HIPCHK(hipMemcpyAsync(q, pe->tab.rel + off, cells * 8, hipMemcpyDeviceToHost, pe->copyStream)); q += cells * 8; }
        if (hops) { HIPCHK(hipMemcpyAsync(q, pe->tab.hops + off, cells * 4, hipMemcpyDeviceToHost, pe->copyStream)); q += cells * 4; }
        if (pred) { HIPCHK(hipMemcpyAsync(q, pe->tab.pred + off, cells * 4, hipMemcpyDeviceToHost, pe->copyStream)); q += cells * 4; }
        if (flags) { HIPCHK(hipMemcpyAsync(q, pe->tab.flags + off, cells, hipMemcpyDeviceToHost, pe->copyStream)); }
        return SHD_PE_OK;
    };
    auto drain = [&](int buf, Blk b) {
        const unsigned char* q = pe->stage[buf];
        const size_t o = (size_t)b.r0 * T, cells = (size_t)b.n * T;
        if (lat) { std::memcpy(lat + o, q, cells * 8); q += cells * 8; }
        if (rel) { std::memcpy(rel + o, q, cells * 8); q += cells * 8; }
        if (hops) { std::memcpy(hops + o, q, cells * 4); q += cells * 4; }
        if (pred) { std::memcpy(pred + o, q, cells * 4); q += cells * 4; }
        if (flags) std::memcpy(flags + o, q, cells);
    };
    hipEvent_t done[2];
    HIPCHK(hipEventCreateWithFlags(&done[0], hipEventDisableTiming));
    if (hipEventCreateWithFlags(&done[1], hipEventDisableTiming) != hipSuccess) {
        (void)hipEventDestroy(done[0]);
        return SHD_PE_EHIP;
    }
    int rc = SHD_PE_OK;
    Blk prev{0, 0};
    int buf = 0;
    for (int32_t r0 = 0; r0 < count && rc == SHD_PE_OK; r0 += B) {
        const Blk cur{r0, std::min(B, count - r0)};
        if ((rc = issue(buf, cur)) == SHD_PE_OK &&
            hipEventRecord(done[buf], pe->copyStream) != hipSuccess)
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
    (void)hipStreamSynchronize(pe->copyStream);
    (void)hipEventDestroy(done[0]);
    (void)hipEventDestroy(done[1]);
    return rc;
}

extern "C" int shd_pe_get_rows(ShdPe* pe, int32_t start, int32_t count, double* lat, double* rel,
                               int32_t* hops, int32_t* pred, uint8_t* flags) {
    if (!pe || start < 0 || count < 0 || (int64_t)start + count > (int64_t)pe->attached.size())
        return SHD_PE_EINVAL;
    if (pred && !pe->opt.storePred) return SHD_PE_EINVAL;
    if (count == 0) return SHD_PE_OK;
    bool all = true;
    for (int32_t i = start; i < start + count; ++i) all = all && pe->rowDone[i];
    if (!all) {
        std::lock_guard<std::mutex> lk(pe->mu);
        std::vector<int32_t> todo;
        for (int32_t i = start; i < start + count; ++i)
            if (!pe->rowDone[i]) todo.push_back(i);
        if (!todo.empty()) {
            int rc = compute_positions_locked(pe, todo.data(), (int32_t)todo.size());
            if (rc) return rc;
        }
    }
    return get_rows_staged(pe, start, count, lat, rel, hops, pred, flags);
}

extern "C" int shd_pe_copy_rows_device(ShdPe* pe, int32_t start, int32_t count, double* dLat,
                                       double* dRel, int32_t* dHops, uint8_t* dFlags) {
    if (!pe || start < 0 || count < 0 || (int64_t)start + count > (int64_t)pe->attached.size())
        return SHD_PE_EINVAL;
    if (!pe->tableReady) return SHD_PE_EINVAL;
    const size_t T = pe->attached.size(), off = (size_t)start * T, cells = (size_t)count * T;
    HIPCHK(hipSetDevice(pe->device));
    if (dLat) HIPCHK(hipMemcpyAsync(dLat, pe->tab.lat + off, cells * 8, hipMemcpyDeviceToDevice, pe->stream));
    if (dRel) HIPCHK(hipMemcpyAsync(dRel, pe->tab.rel + off, cells * 8, hipMemcpyDeviceToDevice, pe->stream));
    if (dHops) HIPCHK(hipMemcpyAsync(dHops, pe->tab.hops + off, cells * 4, hipMemcpyDeviceToDevice, pe->stream));
    if (dFlags) HIPCHK(hipMemcpyAsync(dFlags, pe->tab.flags + off, cells, hipMemcpyDeviceToDevice, pe->stream));
    HIPCHK(hipStreamSynchronize(pe->stream));
    return SHD_PE_OK;
}

// Streaming copy for the achievable-HBM reference: 16-B
// loads and stores, grid-stride, enough workgroups to fill all 8 XCDs.
typedef unsigned int v4u __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void k_stream_copy(const v4u* __restrict__ a,
                                                      v4u* __restrict__ b, size_t n) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + 3 * stride < n; i += 4 * stride) {
        // non-temporal: the copy streams through, nothing is re-read
        const v4u x0 = __builtin_nontemporal_load(&a[i]);
        const v4u x1 = __builtin_nontemporal_load(&a[i + stride]);
        const v4u x2 = __builtin_nontemporal_load(&a[i + 2 * stride]);
        const v4u x3 = __builtin_nontemporal_load(&a[i + 3 * stride]);
        __builtin_nontemporal_store(x0, &b[i]);
        __builtin_nontemporal_store(x1, &b[i + stride]);
        __builtin_nontemporal_store(x2, &b[i + 2 * stride]);
        __builtin_nontemporal_store(x3, &b[i + 3 * stride]);
    }
    for (; i < n; i += stride) b[i] = a[i];
}

extern "C" int shd_pe_stream_bandwidth(ShdPe* pe, int64_t bytes, int32_t iters, double* gbps) {
    if (!pe || !gbps || bytes < (1 << 20) || iters < 1) return SHD_PE_EINVAL;
    HIPCHK(hipSetDevice(pe->device));
    const size_t n = (size_t)bytes / 16;
    void *a = nullptr, *b = nullptr;
    if (hipMalloc(&a, n * 16) != hipSuccess) return SHD_PE_ENOMEM;
    if (hipMalloc(&b, n * 16) != hipSuccess) { (void)hipFree(a); return SHD_PE_ENOMEM; }
    int rc = SHD_PE_OK;
    const int grid = pe->numCUs * env_int("SHDPE_STREAM_WG_PER_CU", 4);
    if (hipMemsetAsync(a, 0, n * 16, pe->stream) != hipSuccess) rc = SHD_PE_EHIP;
    if (!rc) {
        hipLaunchKernelGGL(k_stream_copy, dim3(grid), dim3(256), 0, pe->stream, (const v4u*)a,
                           (v4u*)b, n);   // warm-up
        (void)hipEventRecord(pe->evA, pe->stream);
        for (int i = 0; i < iters; ++i)
            hipLaunchKernelGGL(k_stream_copy, dim3(grid), dim3(256), 0, pe->stream,
                               (const v4u*)a, (v4u*)b, n);
        (void)hipEventRecord(pe->evB, pe->stream);
        if (hipGetLastError() != hipSuccess || hipStreamSynchronize(pe->stream) != hipSuccess)
            rc = SHD_PE_EHIP;
    }
    if (!rc) {
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, pe->evA, pe->evB);
        *gbps = ms > 0.f ? 2.0 * (double)n * 16.0 * iters / (ms * 1e-3) / 1e9 : 0.0;
    }
    (void)hipFree(a);
    (void)hipFree(b);
    return rc;
}

extern "C" int shd_pe_synchronize(ShdPe* pe) {
    if (!pe) return SHD_PE_EINVAL;
    HIPCHK(hipSetDevice(pe->device));
    HIPCHK(hipStreamSynchronize(pe->stream));
    return SHD_PE_OK;
}

extern "C" void shd_pe_destroy(ShdPe* pe) {
    if (!pe) return;
    if (!pe->allocs.empty() || pe->stream) (void)hipSetDevice(pe->device);
    if (pe->stream) (void)hipStreamSynchronize(pe->stream);
    for (void* p : pe->allocs) (void)hipFree(p);
    if (pe->ev0) (void)hipEventDestroy(pe->ev0);
    if (pe->ev1) (void)hipEventDestroy(pe->ev1);
    if (pe->evA) (void)hipEventDestroy(pe->evA);
    if (pe->evB) (void)hipEventDestroy(pe->evB);
    if (pe->stream) (void)hipStreamDestroy(pe->stream);
    if (pe->copyStream) (void)hipStreamDestroy(pe->copyStream);
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
    *out = pe->stats;
    return SHD_PE_OK;
}

extern "C" int shd_pe_reset_stats(ShdPe* pe) {
    if (!pe) return SHD_PE_EINVAL;
    ShdPeStats keep = pe->stats;
    std::memset(&pe->stats, 0, sizeof(pe->stats));
    pe->stats.mode = keep.mode;
    pe->stats.isComplete = keep.isComplete;
    pe->stats.nVertices = keep.nVertices;
    pe->stats.nArcs = keep.nArcs;
    pe->stats.nAttached = keep.nAttached;
    pe->stats.deltaUsed = keep.deltaUsed;
    pe->stats.batched = keep.batched;
    pe->stats.batchLanes = keep.batchLanes;
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

// exported for the host topology mirror (pe_topology.cpp)
const shdpe::HostGraph* shd_pe_host_graph(const ShdPe* pe) { return pe ? &pe->hg : nullptr; }
int32_t shd_pe_position(const ShdPe* pe, int32_t v) {
    return (pe && v >= 0 && v < pe->hg.n) ? pe->posOf[v] : -1;
}

// pe_topology.cpp -- host mirror of the topology.c path API over the engine.
//
// Follows Shadow v1.14.0 src/main/routing/topology.c:
//   _topology_getPathFromCache      :1284-1305
//   _topology_shouldStorePath       :1307-1336
//   _topology_storePathInCache      :1338-1386
//   _topology_computeSourcePaths    :1655-1875 (rows from the GPU engine)
//   _topology_lookupDirectPath      :1877-1927
//   _topology_getPathEntry          :1969-2051
//   topology_getLatency/...         :2053-2092
// The first Dijkstra-row miss triggers one eager shd_pe_compute_all (all
// hosts are attached before the simulation starts, master.c:425 then :436);
// rows are then copied out per source.  Reference quirks kept on purpose:
// the first-computed direction is cached for both directions, the (s,s)
// value depends on query order (self path vs. self-loop row entry), and a
// row with any failed target makes the triggering lookup fail even if its
// own entry was stored.
#include <atomic>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <new>
#include <memory>
#include <vector>

#include "pe_graph.hpp"
#include "shd_pathengine.h"

const shdpe::HostGraph* shd_pe_host_graph(const ShdPe* pe);
int32_t shd_pe_position(const ShdPe* pe, int32_t v);

// The path cache is the triangular row store of pe_rowstore.cpp (SURVEY.md
// §8f rank 1; topology.c:1284-1386).  Cache hits never lock (the reference
// takes a reader lock per probe); a miss takes the topology mutex, probes
// again and computes -- the reference serialises the same work on
// graphLock / the cache writer lock.
struct ShdTopology {
    ShdPe* pe = nullptr;
    const shdpe::HostGraph* g = nullptr;
    int32_t prefersDirectPaths = 0;
    ShdRowStore* store = nullptr;
    std::atomic<int64_t> rowsComputed{0};
    bool allComputed = false;
    std::vector<double> rlat, rrel;
    std::vector<uint8_t> rflags, radj;
    std::vector<int32_t> attached;
    std::mutex mu;                      // misses: row computation + inserts
    ~ShdTopology() { shd_rowstore_free(store); }
};

namespace {
struct PathVal {
    bool ok = false;
    double lat = 0.0, rel = 0.0;
};
}  // namespace

static bool cache_has(const ShdTopology* t, int32_t s, int32_t d, PathVal* v) {
    return shd_rowstore_get(t->store, s, d, v ? &v->lat : nullptr, v ? &v->rel : nullptr,
                            nullptr, nullptr) == 1;
}

static void store_path(ShdTopology* t, bool isDirect, int32_t s, int32_t d, double lat,
                       double rel) {
    const int adjacentPref = t->prefersDirectPaths && !isDirect && t->g->findArc(s, d) != -1;
    (void)shd_rowstore_store(t->store, s, d, isDirect ? 1 : 0, t->g->isComplete ? 1 : 0,
                             adjacentPref, lat, rel);
}

static bool compute_source_paths(ShdTopology* t, int32_t s, int32_t d) {
    if (s == d) {
        double lat, rel;
        if (shdpe::host_self_path(*t->g, s, &lat, &rel)) return false;
        store_path(t, false, s, s, lat, rel);
        return true;
    }
    if (shd_pe_position(t->pe, d) < 0) return false;
    if (!t->allComputed) {
        if (shd_pe_compute_all(t->pe)) return false;
        t->allComputed = true;
    }
    const size_t T = t->attached.size();
    if (shd_pe_get_row(t->pe, s, t->rlat.data(), t->rrel.data(), nullptr, nullptr,
                       t->rflags.data()))
        return false;
    t->rowsComputed.fetch_add(1, std::memory_order_relaxed);
    const uint8_t* adj = nullptr;
    if (t->prefersDirectPaths) {
        for (size_t j = 0; j < T; ++j) t->radj[j] = t->g->findArc(s, t->attached[j]) != -1;
        adj = t->radj.data();
    }
    // topology.c:1815-1859: an empty igraph path (unreachable target) is
    // skipped WITHOUT clearing isAllSuccess; only a failed fold
    // (_topology_computePathProperties, e.g. a missing (s,s) self-loop) does
    return shd_rowstore_store_row(t->store, s, t->rlat.data(), t->rrel.data(), t->rflags.data(),
                                  t->g->isComplete ? 1 : 0, adj) == 1;
}

// _topology_getPathEntry (topology.c:1969-2051): (s,d), then (d,s) when
// undirected; a miss computes (direct path or source row) and re-reads both.
static PathVal get_path_entry(ShdTopology* t, int32_t s, int32_t d, int32_t* hitS,
                              int32_t* hitD) {
    const shdpe::HostGraph* g = t->g;
    PathVal p;
    if (s < 0 || s >= g->n || d < 0 || d >= g->n) return p;
    if (shd_pe_position(t->pe, s) < 0 || shd_pe_position(t->pe, d) < 0) return p;
    auto probe = [&](bool afterMiss) {
        if (cache_has(t, s, d, &p)) { *hitS = s; *hitD = d; return true; }
        if ((afterMiss || !g->directed) && cache_has(t, d, s, &p)) { *hitS = d; *hitD = s; return true; }
        return false;
    };
    if (probe(false)) { p.ok = true; return p; }
    std::lock_guard<std::mutex> lk(t->mu);
    if (probe(false)) { p.ok = true; return p; }     // filled while we waited
    bool success;
    const bool adjacent = g->findArc(s, d) != -1;
    if (g->isComplete || (t->prefersDirectPaths && adjacent)) {
        double lat, rel;
        success = shdpe::host_direct_path(*g, s, d, &lat, &rel) == SHD_PE_OK;
        if (success) store_path(t, true, s, d, lat, rel);
    } else {
        success = compute_source_paths(t, s, d);
    }
    if (success && probe(true)) p.ok = true;
    return p;
}

extern "C" int shd_topology_new(ShdPe* pe, int32_t prefersDirectPaths, ShdTopology** out) {
    if (!pe || !out) return SHD_PE_EINVAL;
    ShdTopology* t = new (std::nothrow) ShdTopology();
    if (!t) return SHD_PE_ENOMEM;
    t->pe = pe;
    t->g = shd_pe_host_graph(pe);
    t->prefersDirectPaths = prefersDirectPaths ? 1 : 0;
    const int32_t T = shd_pe_num_attached(pe);
    t->attached.resize(T);
    shd_pe_attached(pe, t->attached.data());
    const int rc = shd_rowstore_new(t->g->n, t->attached.data(), T, &t->store);
    if (rc) { delete t; return rc; }
    t->rlat.resize(T);
    t->rrel.resize(T);
    t->rflags.resize(T);
    t->radj.resize(T);
    *out = t;
    return SHD_PE_OK;
}

extern "C" void shd_topology_free(ShdTopology* t) { delete t; }

extern "C" double shd_topology_get_latency(ShdTopology* t, int32_t s, int32_t d) {
    if (!t) return -1.0;
    int32_t a, b;
    const PathVal p = get_path_entry(t, s, d, &a, &b);
    return p.ok ? p.lat : -1.0;
}

extern "C" double shd_topology_get_reliability(ShdTopology* t, int32_t s, int32_t d) {
    if (!t) return -1.0;
    int32_t a, b;
    const PathVal p = get_path_entry(t, s, d, &a, &b);
    return p.ok ? p.rel : -1.0;
}

extern "C" int shd_topology_is_routable(ShdTopology* t, int32_t s, int32_t d) {
    return shd_topology_get_latency(t, s, d) > -1 ? 1 : 0;
}

extern "C" int shd_topology_increment_path_packet_counter(ShdTopology* t, int32_t s, int32_t d) {
    if (!t) return -1;
    int32_t a = -1, b = -1;
    const PathVal p = get_path_entry(t, s, d, &a, &b);
    if (!p.ok) return -1;
    return shd_rowstore_increment(t->store, a, b);
}

extern "C" int shd_topology_cached(const ShdTopology* t, int32_t s, int32_t d, double* lat,
                                   double* rel, int32_t* isDirect, int64_t* packetCount) {
    if (!t) return 0;
    uint64_t pc = 0;
    if (!shd_rowstore_get(t->store, s, d, lat, rel, isDirect, &pc)) return 0;
    if (packetCount) *packetCount = (int64_t)pc;
    return 1;
}

extern "C" double shd_topology_min_latency(const ShdTopology* t) {
    return t ? shd_rowstore_min_latency(t->store) : 0.0;
}

extern "C" int64_t shd_topology_cache_size(const ShdTopology* t) {
    return t ? shd_rowstore_size(t->store) : 0;
}

extern "C" int64_t shd_topology_rows_computed(const ShdTopology* t) {
    return t ? t->rowsComputed.load(std::memory_order_relaxed) : 0;
}

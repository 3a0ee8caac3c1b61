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

// Dense host row store, replacing the reference's
// two-level GHashTable<src, GHashTable<dst, Path*>> (topology.c:1284-1386,
// path.c:13-38): one row per attached SOURCE ordinal, allocated on its first
// insert, with a state byte per attached DESTINATION ordinal (0 absent,
// 1 stored, 2 stored + isDirect) and the Path fields side by side.  Lookups
// and the should-store test are two array reads instead of two hash probes
// under rwlocks; a row insert is a sequential pass.  Semantics are the
// reference's, entry for entry.
namespace {
struct PathRow {
    std::vector<double> lat, rel;
    std::vector<int64_t> packets;
    std::vector<uint8_t> state;
    explicit PathRow(size_t T) : lat(T), rel(T), packets(T, 0), state(T, 0) {}
};
struct PathRef {                    // a cached Path: row + destination ordinal
    PathRow* row = nullptr;
    int32_t j = -1;
    explicit operator bool() const { return row != nullptr; }
};
}  // namespace

struct ShdTopology {
    ShdPe* pe = nullptr;
    const shdpe::HostGraph* g = nullptr;
    int32_t prefersDirectPaths = 0;
    std::vector<std::unique_ptr<PathRow>> rows;   // by attached ordinal of the source
    int64_t cacheSize = 0;
    double minimumPathLatency = 0.0;
    int64_t rowsComputed = 0;
    bool allComputed = false;
    std::vector<double> rlat, rrel;
    std::vector<uint8_t> rflags;
    std::vector<int32_t> attached;
    std::mutex mu;
};

static PathRef cache_get(const ShdTopology* t, int32_t s, int32_t d) {
    const int32_t ps = shd_pe_position(t->pe, s), pd = shd_pe_position(t->pe, d);
    if (ps < 0 || pd < 0) return PathRef{};
    PathRow* r = t->rows[ps].get();
    if (!r || !r->state[pd]) return PathRef{};
    return PathRef{r, pd};
}

static bool should_store(ShdTopology* t, bool isDirect, int32_t s, int32_t d) {
    if (cache_get(t, s, d) || cache_get(t, d, s)) return false;
    if (t->g->isComplete && !isDirect) return false;
    if (t->prefersDirectPaths && !isDirect && t->g->findArc(s, d) != -1) return false;
    return true;
}

static void store_path(ShdTopology* t, bool isDirect, int32_t s, int32_t d, double lat,
                       double rel) {
    if (!should_store(t, isDirect, s, d)) return;
    const int32_t ps = shd_pe_position(t->pe, s), pd = shd_pe_position(t->pe, d);
    auto& row = t->rows[ps];
    if (!row) row.reset(new PathRow(t->attached.size()));
    row->lat[pd] = lat;
    row->rel[pd] = rel;
    row->packets[pd] = 0;
    row->state[pd] = isDirect ? 2 : 1;
    t->cacheSize++;
    if (t->minimumPathLatency == 0 || lat < t->minimumPathLatency) t->minimumPathLatency = lat;
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
    t->rowsComputed++;
    // topology.c:1815-1859: an empty igraph path (unreachable target) is
    // skipped WITHOUT clearing isAllSuccess; only a failed fold
    // (_topology_computePathProperties, e.g. a missing (s,s) self-loop) does
    bool allSuccess = true;
    for (size_t j = 0; j < T; ++j) {
        if (t->rflags[j] & SHD_PE_F_UNREACHABLE) continue;
        if (t->rflags[j] & SHD_PE_F_NOEDGE) { allSuccess = false; continue; }
        store_path(t, false, s, t->attached[j], t->rlat[j], t->rrel[j]);
    }
    return allSuccess;
}

static PathRef get_path_entry(ShdTopology* t, int32_t s, int32_t d) {
    const shdpe::HostGraph* g = t->g;
    if (s < 0 || s >= g->n || d < 0 || d >= g->n) return PathRef{};
    if (shd_pe_position(t->pe, s) < 0 || shd_pe_position(t->pe, d) < 0) return PathRef{};
    PathRef p = cache_get(t, s, d);
    if (!p && !g->directed) p = cache_get(t, d, s);
    if (!p) {
        bool success;
        const bool adjacent = g->findArc(s, d) != -1;
        if (g->isComplete || (t->prefersDirectPaths && adjacent)) {
            double lat, rel;
            success = shdpe::host_direct_path(*g, s, d, &lat, &rel) == SHD_PE_OK;
            if (success) store_path(t, true, s, d, lat, rel);
        } else {
            success = compute_source_paths(t, s, d);
        }
        if (success) {
            p = cache_get(t, s, d);
            if (!p) p = cache_get(t, d, s);
        }
    }
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
    t->rlat.resize(T);
    t->rrel.resize(T);
    t->rflags.resize(T);
    t->rows.resize(T);
    *out = t;
    return SHD_PE_OK;
}

extern "C" void shd_topology_free(ShdTopology* t) { delete t; }

extern "C" double shd_topology_get_latency(ShdTopology* t, int32_t s, int32_t d) {
    if (!t) return -1.0;
    std::lock_guard<std::mutex> lk(t->mu);
    const PathRef p = get_path_entry(t, s, d);
    return p ? p.row->lat[p.j] : -1.0;
}

extern "C" double shd_topology_get_reliability(ShdTopology* t, int32_t s, int32_t d) {
    if (!t) return -1.0;
    std::lock_guard<std::mutex> lk(t->mu);
    const PathRef p = get_path_entry(t, s, d);
    return p ? p.row->rel[p.j] : -1.0;
}

extern "C" int shd_topology_is_routable(ShdTopology* t, int32_t s, int32_t d) {
    return shd_topology_get_latency(t, s, d) > -1 ? 1 : 0;
}

extern "C" int shd_topology_increment_path_packet_counter(ShdTopology* t, int32_t s, int32_t d) {
    if (!t) return -1;
    std::lock_guard<std::mutex> lk(t->mu);
    const PathRef p = get_path_entry(t, s, d);
    if (!p) return -1;
    p.row->packets[p.j]++;
    return 0;
}

extern "C" int shd_topology_cached(const ShdTopology* t, int32_t s, int32_t d, double* lat,
                                   double* rel, int32_t* isDirect, int64_t* packetCount) {
    if (!t) return 0;
    if (s < 0 || s >= t->g->n || d < 0 || d >= t->g->n) return 0;
    const PathRef p = cache_get(t, s, d);
    if (!p) return 0;
    if (lat) *lat = p.row->lat[p.j];
    if (rel) *rel = p.row->rel[p.j];
    if (isDirect) *isDirect = p.row->state[p.j] == 2 ? 1 : 0;
    if (packetCount) *packetCount = p.row->packets[p.j];
    return 1;
}

extern "C" double shd_topology_min_latency(const ShdTopology* t) {
    return t ? t->minimumPathLatency : 0.0;
}

extern "C" int64_t shd_topology_cache_size(const ShdTopology* t) {
    return t ? t->cacheSize : 0;
}

extern "C" int64_t shd_topology_rows_computed(const ShdTopology* t) {
    return t ? t->rowsComputed : 0;
}

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
#include <unordered_map>
#include <vector>

#include "pe_graph.hpp"
#include "shd_pathengine.h"

const shdpe::HostGraph* shd_pe_host_graph(const ShdPe* pe);
int32_t shd_pe_position(const ShdPe* pe, int32_t v);

namespace {
struct Path {                       // src/main/routing/path.c:13-21
    int32_t isDirect;
    int32_t src, dst;
    double latency, reliability;
    int64_t packetCount;
};
}  // namespace

struct ShdTopology {
    ShdPe* pe = nullptr;
    const shdpe::HostGraph* g = nullptr;
    int32_t prefersDirectPaths = 0;
    std::unordered_map<uint64_t, Path> cache;
    double minimumPathLatency = 0.0;
    int64_t rowsComputed = 0;
    bool allComputed = false;
    std::vector<double> rlat, rrel;
    std::vector<uint8_t> rflags;
    std::vector<int32_t> attached;
    std::mutex mu;
};

static inline uint64_t key(int32_t s, int32_t d) {
    return ((uint64_t)(uint32_t)s << 32) | (uint32_t)d;
}

static Path* cache_get(ShdTopology* t, int32_t s, int32_t d) {
    auto it = t->cache.find(key(s, d));
    return it == t->cache.end() ? nullptr : &it->second;
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
    t->cache[key(s, d)] = Path{isDirect ? 1 : 0, s, d, lat, rel, 0};
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
    bool allSuccess = true;
    for (size_t j = 0; j < T; ++j) {
        if (t->rflags[j] & SHD_PE_F_FAILED) { allSuccess = false; continue; }
        store_path(t, false, s, t->attached[j], t->rlat[j], t->rrel[j]);
    }
    return allSuccess;
}

static Path* get_path_entry(ShdTopology* t, int32_t s, int32_t d) {
    const shdpe::HostGraph* g = t->g;
    if (s < 0 || s >= g->n || d < 0 || d >= g->n) return nullptr;
    if (shd_pe_position(t->pe, s) < 0 || shd_pe_position(t->pe, d) < 0) return nullptr;
    Path* p = cache_get(t, s, d);
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
    *out = t;
    return SHD_PE_OK;
}

extern "C" void shd_topology_free(ShdTopology* t) { delete t; }

extern "C" double shd_topology_get_latency(ShdTopology* t, int32_t s, int32_t d) {
    if (!t) return -1.0;
    std::lock_guard<std::mutex> lk(t->mu);
    Path* p = get_path_entry(t, s, d);
    return p ? p->latency : -1.0;
}

extern "C" double shd_topology_get_reliability(ShdTopology* t, int32_t s, int32_t d) {
    if (!t) return -1.0;
    std::lock_guard<std::mutex> lk(t->mu);
    Path* p = get_path_entry(t, s, d);
    return p ? p->reliability : -1.0;
}

extern "C" int shd_topology_is_routable(ShdTopology* t, int32_t s, int32_t d) {
    return shd_topology_get_latency(t, s, d) > -1 ? 1 : 0;
}

extern "C" int shd_topology_increment_path_packet_counter(ShdTopology* t, int32_t s, int32_t d) {
    if (!t) return -1;
    std::lock_guard<std::mutex> lk(t->mu);
    Path* p = get_path_entry(t, s, d);
    if (!p) return -1;
    p->packetCount++;
    return 0;
}

extern "C" int shd_topology_cached(const ShdTopology* t, int32_t s, int32_t d, double* lat,
                                   double* rel, int32_t* isDirect, int64_t* packetCount) {
    if (!t) return 0;
    auto it = t->cache.find(key(s, d));
    if (it == t->cache.end()) return 0;
    if (lat) *lat = it->second.latency;
    if (rel) *rel = it->second.reliability;
    if (isDirect) *isDirect = it->second.isDirect;
    if (packetCount) *packetCount = it->second.packetCount;
    return 1;
}

extern "C" double shd_topology_min_latency(const ShdTopology* t) {
    return t ? t->minimumPathLatency : 0.0;
}

extern "C" int64_t shd_topology_cache_size(const ShdTopology* t) {
    return t ? (int64_t)t->cache.size() : 0;
}

extern "C" int64_t shd_topology_rows_computed(const ShdTopology* t) {
    return t ? t->rowsComputed : 0;
}

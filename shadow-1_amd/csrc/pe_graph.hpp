// pe_graph.hpp -- host-side graph model of the engine (no GPU types).
#pragma once
#include <stdint.h>

#include <memory>
#include <utility>
#include <vector>

#include "shd_pathengine.h"

namespace shdpe {

// std::vector whose elements are default-initialised: the arc arrays of a
// 2e8-edge topology are first touched by the (parallel) fill, not zeroed
// serially first.
template <class T>
struct DefaultInitAlloc : std::allocator<T> {
    template <class U> struct rebind { using other = DefaultInitAlloc<U>; };
    using std::allocator<T>::allocator;
    template <class U> void construct(U* p) noexcept { ::new (static_cast<void*>(p)) U; }
    template <class U, class... A> void construct(U* p, A&&... a) {
        ::new (static_cast<void*>(p)) U(std::forward<A>(a)...);
    }
};
template <class T>
using hvec = std::vector<T, DefaultInitAlloc<T>>;

// CSR in igraph incidence order (ascending neighbour id) with self-loops
// split out.  Built from the igraph edge list handed over the C-ABI.
struct HostGraph {
    int32_t n = 0;
    int32_t directed = 0;
    int64_t nEdges = 0;
    // OUT arcs without self-loops
    std::vector<int32_t> rowPtr;
    hvec<int32_t> col;
    hvec<double> lat, rel;
    // IN arcs (directed only; undirected uses the OUT arrays)
    std::vector<int32_t> inPtr;
    hvec<int32_t> inCol;
    hvec<double> inLat, inRel;
    hvec<int32_t> outToIn;
    // multigraphs whose newest parallel edge is not a fastest one (latFold):
    // per merged OUT arc the newest edge's latency (path folds, direct paths;
    // `lat` holds the group minimum) and the self path's reliability
    bool latFold = false;
    hvec<double> foldLat, selfPathRel;
    // vertex data
    std::vector<double> vrel;       // 1 - packetloss, 1.0 when absent/NaN
    std::vector<double> selfLat, selfRel;        // newest self-loop: igraph_get_eid(v, v)
    std::vector<double> selfMinLat, selfMinRel;  // several loops: the one the self path
                                                 // takes (first strict minimum, newest first)
    std::vector<uint8_t> hasSelf;
    bool isComplete = false;
    // multigraphs only (empty otherwise): per vertex the incident EDGE count
    // _topology_isComplete compares with vcount (parallel edges each, the
    // undirected self-loop correction applied) -- the merged rows undercount
    std::vector<int32_t> edgeCount;
    double meanArcLatency = 0.0;
    double minArcLatency = 0.0;     // smallest non-loop arc latency (0: no arcs)

    int64_t nArcs() const { return (int64_t)col.size(); }
    // igraph_get_eid(from,to): arc index into the OUT arrays (parallel edges
    // are merged into the arc of the newest one), -2 for the self-loop, -1
    // for none.
    int64_t findArc(int32_t from, int32_t to) const;
};

// Validate + build (topology.c:1041-1124 checks, igraph_add_edges order).
int build_host_graph(const ShdPeGraphDesc* d, HostGraph* g);

// _topology_lookupDirectPath (topology.c:1877-1927)
int host_direct_path(const HostGraph& g, int32_t s, int32_t t, double* lat, double* rel);
// _topology_computeShortestPathToSelf (topology.c:1545-1653)
int host_self_path(const HostGraph& g, int32_t v, double* lat, double* rel);

}  // namespace shdpe

/*
 * pe_oracle.h -- CPU ORACLE for the Shadow topology path engine.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product library (shadow-1_amd/)
 * links, loads or calls this code; only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg do, and there only as the checker.
 *
 * What it restates (all citations relative to /root/reference, Shadow v1.14.0):
 *   - _topology_computeSourcePaths        src/main/routing/topology.c:1655-1875
 *   - _topology_computePathProperties     topology.c:1407-1523  (fold order)
 *   - _topology_getEdgeHelper             topology.c:402-444    (rel = 1.0 - loss)
 *   - _topology_computeShortestPathToSelf topology.c:1545-1653
 *   - _topology_lookupDirectPath          topology.c:1877-1927
 *   - _topology_isComplete                topology.c:450-552
 *   - _topology_shouldStorePath / _topology_storePathInCache  topology.c:1307-1386
 *   - _topology_getPathEntry              topology.c:1969-2051
 *   - igraph 0.7.1 (external, NOT vendored in the reference; pinned by
 *     .github/workflows/build_shadow.yml:30 "libigraph0-dev" and
 *     .github/ISSUE_TEMPLATE/bug-report.md:24 "IGraph v0.7.1"):
 *       igraph_get_shortest_paths_dijkstra (structural_properties.c),
 *       igraph_2wheap_* (heap.c), igraph_add_edges/igraph_vector_order and
 *       igraph_incident / igraph_get_eid (type_indexededgelist.c).
 *     Restated from the published algorithm; igraph is
 *     absent from this container, so the tie-breaking order is
 *     "igraph-0.7.1-reconstructed" (parity pinning).
 */
#ifndef SHD_PE_ORACLE_H
#define SHD_PE_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* per-entry status bits (same meaning as the engine's SHD_PE_F_* flags) */
#define ORC_F_OK          0u
#define ORC_F_UNREACHABLE 1u   /* igraph could not reach the target            */
#define ORC_F_NOEDGE      2u   /* a hop (incl. the (s,s) self-loop) has no edge */
#define ORC_F_ZEROLAT     4u   /* latency 0 replaced by 1 (topology.c:1848)     */

typedef struct OrcGraph OrcGraph;

/* Build a graph from an edge list given in igraph edge-id order (GraphML
 * document order).  from/to are vertex indices as written in the file; for
 * undirected graphs they are normalised like igraph_add_edges (from=max,
 * to=min).  vertexLoss may be NULL (attribute absent); NaN entries mean
 * "attribute value absent" (topology.c:330-349).  Returns NULL on bad input. */
OrcGraph* orc_graph_new(int32_t nVertices, int64_t nEdges, int32_t directed,
                        const int32_t* from, const int32_t* to,
                        const double* latency, const double* packetLoss,
                        const double* vertexLoss);
void orc_graph_free(OrcGraph* g);

/* _topology_isComplete (topology.c:450-552) */
int32_t orc_is_complete(const OrcGraph* g);

/* igraph_get_eid(from,to,directed=isDirected,error=FALSE) (0.7.1 BINSEARCH):
 * returns the edge id or -1. */
int64_t orc_get_eid(const OrcGraph* g, int32_t from, int32_t to);

/* One source row with reference semantics (topology.c:1681-1866 with the
 * igraph 0.7.1 Dijkstra).  targets[0..T) are vertex ids (the attached set, in
 * the order the row is wanted).  Outputs per target j (any may be NULL):
 *   lat[j], rel[j]  -- exactly what _topology_computePathProperties returns
 *                      (after the latency==0 -> 1 rule);
 *   hops[j]         -- number of edges folded into lat (1 for t==s: the
 *                      self-loop, topology.c:1469-1488);
 *   pred[j]         -- vertex before t on the igraph path (-1 if t==s);
 *   flags[j]        -- ORC_F_* bits; a non-zero UNREACHABLE/NOEDGE entry is
 *                      not stored by the reference.
 * Returns 0, or -1 on invalid arguments. */
int32_t orc_dijkstra_row(const OrcGraph* g, int32_t src,
                         const int32_t* targets, int32_t nTargets,
                         double* lat, double* rel, int32_t* hops,
                         int32_t* pred, uint8_t* flags);

/* Raw igraph Dijkstra state for one source (for tests): dist (-1 = never
 * reached) and parent edge id + 1 (0 = none), and the pop order.  popped gets
 * the number of vertices popped before the early exit (all targets reached). */
int32_t orc_dijkstra_raw(const OrcGraph* g, int32_t src,
                         const int32_t* targets, int32_t nTargets,
                         double* dist, int64_t* parentEdgePlus1,
                         int32_t* popOrder, int32_t* popped);

/* _topology_lookupDirectPath (topology.c:1877-1927).  Returns 0 on success,
 * -1 if (s,t) has no edge. */
int32_t orc_direct_path(const OrcGraph* g, int32_t s, int32_t t,
                        double* lat, double* rel);

/* _topology_computeShortestPathToSelf (topology.c:1545-1653). 0 / -1. */
int32_t orc_self_path(const OrcGraph* g, int32_t v, double* lat, double* rel);

/* CPU baseline: rows for many sources with nThreads pthreads (one source per
 * task).  Output row-major [nSources][nTargets]. */
int32_t orc_rows_parallel(const OrcGraph* g, const int32_t* sources,
                          int32_t nSources, const int32_t* targets,
                          int32_t nTargets, int32_t nThreads,
                          double* lat, double* rel, int32_t* hops,
                          int32_t* pred, uint8_t* flags);

/* Checker: Bellman condition for R distance rows at once.  dT is [n][R]
 * (vertex-major: dT[v*R + r] = row r's distance to v, source 0, +inf
 * unreached); viol[r] = arcs (u,v) with dT[u] + w < dT[v].  0 / -1. */
int32_t orc_bellman_rows(const OrcGraph* g, const double* dT, int32_t R, int32_t nThreads,
                         int64_t* viol);

/* --------------------------------------------------------------------------
 * Path-cache / dispatcher restatement (topology.c:1284-1386, 1969-2092).
 * Queries are by vertex index (the Address->vertex map of topology.c:1388
 * stays in host C and is not part of the path).
 * ------------------------------------------------------------------------ */
typedef struct OrcTopology OrcTopology;

OrcTopology* orc_topology_new(const OrcGraph* g, const int32_t* attached,
                              int32_t nAttached, int32_t prefersDirectPaths);
void orc_topology_free(OrcTopology* t);
/* topology_getLatency / getReliability: -1.0 on failure (release build). */
double orc_topology_get_latency(OrcTopology* t, int32_t srcV, int32_t dstV);
double orc_topology_get_reliability(OrcTopology* t, int32_t srcV, int32_t dstV);
int32_t orc_topology_is_routable(OrcTopology* t, int32_t srcV, int32_t dstV);
int32_t orc_topology_increment_packet_counter(OrcTopology* t, int32_t srcV, int32_t dstV);
/* Inspect a cached entry exactly as stored under key (src,dst); returns 1 if
 * present.  isDirect/packetCount may be NULL. */
int32_t orc_topology_cached(const OrcTopology* t, int32_t srcV, int32_t dstV,
                            double* lat, double* rel, int32_t* isDirect,
                            int64_t* packetCount);
double orc_topology_min_latency(const OrcTopology* t);
int64_t orc_topology_rows_computed(const OrcTopology* t);
int64_t orc_topology_self_paths_computed(const OrcTopology* t);
int64_t orc_topology_cache_size(const OrcTopology* t);

/* Test hook: igraph's two-pass vector_order vs the counting-sort form on a
 * random multigraph edge list; 1 when identical. */
int32_t orc_selftest_vector_order(int64_t m, int32_t nodes, uint64_t seed);

#ifdef __cplusplus
}
#endif
#endif

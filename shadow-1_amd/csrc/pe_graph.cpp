// pe_graph.cpp -- host-side graph build for the engine (pure C++, no HIP).
//
// Input: the igraph edge list (edge ids = GraphML document order) that
// Shadow's host C already holds after _topology_loadGraph (topology.c:371).
// Output: CSR rows in igraph incidence order.  For a simple graph igraph's
// incidence list of v (igraph_incident, mode OUT; undirected -> ALL) is
// [oi: from==v sorted by to][ii: to==v sorted by from] with undirected edges
// stored from=max(a,b) -- i.e. ascending neighbour id, self-loop in place
// (SURVEY.md Appendix A.1-A.2).
//
// Multigraphs: igraph lists parallel edges to one neighbour consecutively
// (newest first), Dijkstra relaxes each of them, and the fold reads the edge
// igraph_get_eid returns -- the NEWEST (highest id) parallel edge
// (type_indexededgelist.c BINSEARCH over an index sorted with descending ids
// among equals; oracle/pe_oracle.c orc_get_eid).  Consecutive relaxations of
// one neighbour by w1, w2, ... leave the same distances, heap array and
// parent vertex as one relaxation by min(w) (a second shift_up continues the
// first over the same ancestor chain), so a group of parallel edges becomes
// ONE arc with the group's minimum latency and the newest edge's reliability.
// The path latency the reference reports is the fold of get_eid latencies
// (topology.c:1488-1498), which equals the Dijkstra distance when the newest
// edge of every group is a fastest one.  When some group's newest edge is
// slower (HostGraph::latFold), the merged arc keeps the group MINIMUM for the
// relaxations, `foldLat` the newest edge's latency for the path folds and
// direct paths, and `selfPathRel` the reliability of the edge the self path's
// strict-'<' scan of v's incident edges settles on (the newest of the
// group's fastest edges: igraph lists parallel edges newest first); the
// engine then computes such graphs' rows with the exact emulation, which
// folds the latency label along the path like the reference.
#include "pe_graph.hpp"

#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdint>
#include <thread>
#include <utility>
#include <vector>

namespace shdpe {

int64_t HostGraph::findArc(int32_t from, int32_t to) const {
    if (from < 0 || from >= n || to < 0 || to >= n) return -1;
    if (from == to) return hasSelf[from] ? -2 : -1;
    const int32_t* b = col.data() + rowPtr[from];
    const int32_t* e = col.data() + rowPtr[from + 1];
    const int32_t* p = std::lower_bound(b, e, to);
    if (p != e && *p == to) return (int64_t)(p - col.data());
    return -1;
}

// ---- deterministic parallel passes (results independent of thread count) --
static int host_threads() {
    const unsigned h = std::thread::hardware_concurrency();
    return (int)std::max(1u, std::min(16u, h ? h : 1u));
}

// f(chunk, lo, hi) over nChunks fixed chunks of [0, n), chunks dealt to
// threads; `work` (total element visits) below 2^20 runs inline
template <class F>
static void par_chunks(int64_t n, int nChunks, int64_t work, F f) {
    const int nt = std::min(host_threads(), nChunks);
    auto run = [&](int t) {
        for (int c = t; c < nChunks; c += nt) f(c, n * c / nChunks, n * (c + 1) / nChunks);
    };
    if (nt <= 1 || work < (1 << 20)) { run(0); if (nt > 1) for (int t = 1; t < nt; ++t) run(t); return; }
    std::vector<std::thread> th;
    for (int t = 1; t < nt; ++t) th.emplace_back(run, t);
    run(0);
    for (auto& x : th) x.join();
}

// Sort each row by neighbour id (igraph incidence order), parallel edges of
// one neighbour in edge-id order (the fill order); returns whether any row
// has a repeated neighbour (a multigraph).
static bool sort_rows(int32_t n, const std::vector<int32_t>& ptr, hvec<int32_t>& colv,
                      hvec<double>& latv, hvec<double>& relv) {
    const int nc = 64;
    std::vector<uint8_t> multi(nc, 0);
    par_chunks(n, nc, (int64_t)colv.size(), [&](int c, int64_t v0, int64_t v1) {
        std::vector<std::pair<int32_t, int32_t>> tmp;
        std::vector<double> l2, r2;
        for (int64_t v = v0; v < v1; ++v) {
            const int32_t b = ptr[v], e = ptr[v + 1];
            bool sorted = true;
            for (int32_t a = b + 1; a < e; ++a)
                if (colv[a - 1] >= colv[a]) { sorted = false; break; }
            if (sorted) continue;
            tmp.clear();
            for (int32_t a = b; a < e; ++a) tmp.emplace_back(colv[a], a);
            std::sort(tmp.begin(), tmp.end());
            for (size_t k = 1; k < tmp.size(); ++k)
                if (tmp[k].first == tmp[k - 1].first) multi[c] = 1;
            l2.resize(tmp.size());
            r2.resize(tmp.size());
            for (size_t k = 0; k < tmp.size(); ++k) {
                l2[k] = latv[tmp[k].second];
                r2[k] = relv[tmp[k].second];
            }
            for (size_t k = 0; k < tmp.size(); ++k) {
                colv[b + k] = tmp[k].first;
                latv[b + k] = l2[k];
                relv[b + k] = r2[k];
            }
        }
    });
    for (uint8_t x : multi)
        if (x) return true;
    return false;
}

// One arc per (vertex, neighbour): the group's minimum latency, the newest
// parallel edge's (the last of its group in edge-id order) reliability; for
// latFold graphs also the newest edge's latency and the self path's
// reliability (see the header); rows compacted in place.
static int merge_parallel(HostGraph* g) {
    const int32_t n = g->n;
    std::vector<int32_t>& ptr = g->rowPtr;
    hvec<int32_t>& colv = g->col;
    hvec<double>& latv = g->lat;
    hvec<double>& relv = g->rel;
    bool fold = false;
    for (int32_t v = 0; v < n && !fold; ++v)
        for (int32_t a = ptr[v]; a < ptr[v + 1];) {
            int32_t z = a + 1;
            double mn = latv[a];
            while (z < ptr[v + 1] && colv[z] == colv[a]) { mn = std::min(mn, latv[z]); ++z; }
            if (latv[z - 1] != mn) fold = true;
            a = z;
        }
    g->latFold = fold;
    if (fold) {
        g->foldLat.resize(colv.size());
        g->selfPathRel.resize(colv.size());
    }
    int32_t w = 0;
    for (int32_t v = 0; v < n; ++v) {
        const int32_t b = ptr[v], e = ptr[v + 1];
        ptr[v] = w;
        for (int32_t a = b; a < e;) {
            int32_t z = a + 1;
            double mn = latv[a];
            int32_t lastMin = a;
            while (z < e && colv[z] == colv[a]) {
                if (latv[z] <= mn) { mn = latv[z]; lastMin = z; }
                ++z;
            }
            const int32_t newest = z - 1;
            if (fold) {
                g->foldLat[w] = latv[newest];
                g->selfPathRel[w] = relv[lastMin];
            }
            colv[w] = colv[newest];
            latv[w] = mn;
            relv[w] = relv[newest];
            ++w;
            a = z;
        }
    }
    ptr[n] = w;
    colv.resize(w);
    latv.resize(w);
    relv.resize(w);
    if (fold) {
        g->foldLat.resize(w);
        g->selfPathRel.resize(w);
    }
    return SHD_PE_OK;
}

int build_host_graph(const ShdPeGraphDesc* d, HostGraph* g) {
    if (!d || !g || d->nVertices <= 0 || d->nEdges < 0) return SHD_PE_EINVAL;
    if (d->nEdges > 0 && (!d->edgeFrom || !d->edgeTo || !d->edgeLatency || !d->edgePacketLoss))
        return SHD_PE_EINVAL;
    const int32_t n = d->nVertices;
    const int64_t m = d->nEdges;
    g->n = n;
    g->directed = d->directed ? 1 : 0;
    g->nEdges = m;
    g->vrel.assign(n, 1.0);
    g->selfLat.assign(n, 0.0);
    g->selfRel.assign(n, 0.0);
    g->selfMinLat.assign(n, 0.0);
    g->selfMinRel.assign(n, 0.0);
    g->hasSelf.assign(n, 0);
    // topology.c:956-970 vertex packetloss range; NaN = absent (:330-349)
    if (d->vertexPacketLoss) {
        for (int32_t v = 0; v < n; ++v) {
            const double p = d->vertexPacketLoss[v];
            if (std::isnan(p)) continue;
            if (!(p >= 0.0 && p <= 1.0)) return SHD_PE_EINVAL;
            g->vrel[v] = 1.0 - p;                 // (1.0f - packetLoss), :1444
        }
    }
    // Pass 1 (chunks of the edge list): first invalid edge, self-loops in
    // edge order, and per-chunk arc counts per row.  The serial semantics --
    // the first bad edge in edge order decides the error -- are kept by
    // taking the minimum over chunks.
    const int NC = (int)std::max<int64_t>(1, std::min<int64_t>(64, m / 4096 + 1));
    std::vector<int64_t> firstBad(NC, INT64_MAX);
    std::vector<std::vector<int64_t>> loops(NC);
    std::vector<std::vector<int32_t>> cnt(NC);
    par_chunks(m, NC, m, [&](int c, int64_t e0, int64_t e1) {
        std::vector<int32_t>& k = cnt[c];
        k.assign(n, 0);
        for (int64_t e = e0; e < e1; ++e) {
            const int32_t a = d->edgeFrom[e], b = d->edgeTo[e];
            const double L = d->edgeLatency[e], p = d->edgePacketLoss[e];
            if (a < 0 || a >= n || b < 0 || b >= n || !(L > 0.0) ||   // :1070 (NaN fails too)
                !(p >= 0.0 && p <= 1.0)) {                            // :1090
                firstBad[c] = e;
                return;
            }
            if (a == b) { loops[c].push_back(e); continue; }
            k[a]++;
            if (!g->directed) k[b]++;
        }
    });
    int64_t bad = INT64_MAX;
    for (int64_t x : firstBad) bad = std::min(bad, x);
    // self-loops in edge order: the newest one of a vertex is its (v, v)
    // edge (the (s, s) path fold, direct paths, adjacency); nSelf counts them
    // for the completeness rule.  A self-loop never changes a distance, so
    // several loops need no merge rule: the self path
    // (_topology_computeShortestPathToSelf, topology.c:1582-1598) walks them
    // newest first and keeps the first strict minimum = the newest loop of
    // minimum latency (<= in edge order below)
    std::vector<int32_t> nSelf(n, 0);
    for (int c = 0; c < NC; ++c) {
        for (int64_t e : loops[c]) {
            if (e > bad) break;
            const int32_t a = d->edgeFrom[e];
            const double L = d->edgeLatency[e], R = 1.0 - d->edgePacketLoss[e];   // :437
            g->hasSelf[a] = 1;
            if (nSelf[a]++ == 0 || L <= g->selfMinLat[a]) { g->selfMinLat[a] = L; g->selfMinRel[a] = R; }
            g->selfLat[a] = L;
            g->selfRel[a] = R;
        }
    }
    if (bad != INT64_MAX) return SHD_PE_EINVAL;
    // row pointers; chunk c writes row v from offset rowPtr[v] + (arcs of v
    // in chunks < c): every row keeps edge-id order, as the serial fill
    g->rowPtr.assign(n + 1, 0);
    {
        int64_t acc = 0;
        for (int32_t v = 0; v < n; ++v) {
            g->rowPtr[v] = (int32_t)std::min<int64_t>(acc, INT32_MAX);
            for (int c = 0; c < NC; ++c) {
                const int32_t x = cnt[c][v];
                cnt[c][v] = (int32_t)std::min<int64_t>(acc, INT32_MAX);   // becomes the fill cursor
                acc += x;
            }
        }
        if (acc >= (int64_t)INT32_MAX) return SHD_PE_EINVAL;
        g->rowPtr[n] = (int32_t)acc;
    }
    const int64_t nArcs = g->rowPtr[n];
    g->col.resize(nArcs);
    g->lat.resize(nArcs);
    g->rel.resize(nArcs);
    par_chunks(m, NC, m, [&](int c, int64_t e0, int64_t e1) {
        std::vector<int32_t>& fill = cnt[c];
        for (int64_t e = e0; e < e1; ++e) {
            const int32_t a = d->edgeFrom[e], b = d->edgeTo[e];
            if (a == b) continue;
            const double L = d->edgeLatency[e], R = 1.0 - d->edgePacketLoss[e];
            int32_t k = fill[a]++;
            g->col[k] = b; g->lat[k] = L; g->rel[k] = R;
            if (!g->directed) {
                k = fill[b]++;
                g->col[k] = a; g->lat[k] = L; g->rel[k] = R;
            }
        }
    });
    cnt.clear();
    cnt.shrink_to_fit();
    // incident edge counts before parallel edges merge (_topology_isComplete
    // counts edges, not neighbours)
    std::vector<int32_t> rawDeg;
    if (sort_rows(n, g->rowPtr, g->col, g->lat, g->rel)) {
        rawDeg.resize(n);
        for (int32_t v = 0; v < n; ++v) rawDeg[v] = g->rowPtr[v + 1] - g->rowPtr[v];
        const int rc = merge_parallel(g);
        if (rc) return rc;
    }
    const int64_t nArcsM = g->rowPtr[n];

    g->outToIn.resize(nArcsM);
    if (g->directed) {
        // IN CSR sorted by source id
        std::vector<int32_t> cntIn(n + 1, 0);
        for (int64_t a = 0; a < nArcsM; ++a) cntIn[g->col[a] + 1]++;
        for (int32_t v = 0; v < n; ++v) cntIn[v + 1] += cntIn[v];
        g->inPtr = cntIn;
        g->inCol.resize(nArcsM);
        g->inLat.resize(nArcsM);
        g->inRel.resize(nArcsM);
        std::vector<int32_t> fill(cntIn.begin(), cntIn.end() - 1);
        for (int32_t u = 0; u < n; ++u) {               // rows visited in source order
            for (int32_t a = g->rowPtr[u]; a < g->rowPtr[u + 1]; ++a) {
                const int32_t v = g->col[a];
                const int32_t k = fill[v]++;
                g->inCol[k] = u; g->inLat[k] = g->lat[a]; g->inRel[k] = g->rel[a];
                g->outToIn[a] = k;
            }
        }
    } else {
        // reverse arc of u->v: position of u in v's sorted row
        std::vector<int> rcs(64, SHD_PE_OK);
        par_chunks(n, 64, nArcsM * 16, [&](int c, int64_t u0, int64_t u1) {
            for (int64_t u = u0; u < u1; ++u) {
                for (int32_t a = g->rowPtr[u]; a < g->rowPtr[u + 1]; ++a) {
                    const int64_t rev = g->findArc(g->col[a], (int32_t)u);
                    if (rev < 0) { rcs[c] = SHD_PE_EINVAL; return; }
                    g->outToIn[a] = (int32_t)rev;
                }
            }
        });
        for (int r : rcs)
            if (r) return r;
    }
    // _topology_isComplete (topology.c:450-552): incident EDGE count (parallel
    // edges each; an undirected self-loop counted twice, then one correction
    // when get_eid(v, v) exists) must reach vcount.
    bool complete = true;
    const bool multi = !rawDeg.empty() || *std::max_element(nSelf.begin(), nSelf.end()) > 1;
    if (multi) g->edgeCount.resize(n);
    for (int32_t v = 0; v < n; ++v) {
        int64_t c = rawDeg.empty() ? (int64_t)(g->rowPtr[v + 1] - g->rowPtr[v]) : rawDeg[v];
        c += g->directed ? nSelf[v] : 2 * (int64_t)nSelf[v];
        if (!g->directed && g->hasSelf[v]) c -= 1;
        if (c < n) complete = false;
        if (multi) g->edgeCount[v] = (int32_t)std::min<int64_t>(c, INT32_MAX);
        else if (!complete) break;
    }
    g->isComplete = complete;
    // mean arc latency (bucket width): fixed 64-chunk partial sums added in
    // order, so the value does not depend on the thread count
    std::vector<double> part(64, 0.0), pmin(64, INFINITY);
    par_chunks(nArcsM, 64, nArcsM, [&](int c, int64_t a0, int64_t a1) {
        double s = 0.0, mn = INFINITY;
        for (int64_t a = a0; a < a1; ++a) { s += g->lat[a]; mn = std::min(mn, g->lat[a]); }
        part[c] = s;
        pmin[c] = mn;
    });
    double sum = 0.0, mn = INFINITY;
    for (double x : part) sum += x;
    for (double x : pmin) mn = std::min(mn, x);
    g->minArcLatency = nArcsM ? mn : 0.0;
    g->meanArcLatency = nArcsM ? sum / (double)nArcsM : 1.0;
    return SHD_PE_OK;
}

int host_direct_path(const HostGraph& g, int32_t s, int32_t t, double* lat, double* rel) {
    if (s < 0 || s >= g.n || t < 0 || t >= g.n) return SHD_PE_EINVAL;
    double totalLatency = 0.0, totalReliability = 1.0;
    totalReliability *= g.vrel[s];                 // :1901-1903 (1.0 when absent)
    totalReliability *= g.vrel[t];                 // :1905-1907
    const int64_t a = g.findArc(s, t);
    double L, R;
    if (a == -2) { L = g.selfLat[s]; R = g.selfRel[s]; }
    else if (a >= 0) { L = g.latFold ? g.foldLat[a] : g.lat[a]; R = g.rel[a]; }   // get_eid: the newest
    else return SHD_PE_ENOEDGE;
    totalLatency += L;                              // :1920
    totalReliability *= R;                          // :1921
    if (lat) *lat = totalLatency;
    if (rel) *rel = totalReliability;
    return SHD_PE_OK;
}

int host_self_path(const HostGraph& g, int32_t v, double* lat, double* rel) {
    if (v < 0 || v >= g.n) return SHD_PE_EINVAL;
    // incident OUT edges in igraph order = ascending neighbour, self-loop in
    // place (twice for undirected -- harmless under the strict '<').
    double minLatency = 0.0, relMin = 0.0;
    bool any = false;
    auto visit = [&](double L, double R) {
        any = true;
        if (minLatency == 0 || L < minLatency) { minLatency = L; relMin = R; }   // :1592
    };
    const int32_t b = g.rowPtr[v], e = g.rowPtr[v + 1];
    int32_t a = b;
    const double* srel = g.latFold ? g.selfPathRel.data() : g.rel.data();
    for (; a < e && g.col[a] < v; ++a) visit(g.lat[a], srel[a]);
    if (g.hasSelf[v]) visit(g.selfMinLat[v], g.selfMinRel[v]);
    for (; a < e; ++a) visit(g.lat[a], srel[a]);
    if (!any && g.nEdges == 0) return SHD_PE_ENOEDGE;
    if (lat) *lat = 2.0 * minLatency;               // :1640
    if (rel) *rel = relMin * relMin;                // :1641
    return SHD_PE_OK;
}

}  // namespace shdpe

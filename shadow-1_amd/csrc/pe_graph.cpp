// pe_graph.cpp -- host-side graph build for the engine (pure C++, no HIP).
//
// Input: the igraph edge list (edge ids = GraphML document order) that
// Shadow's host C already holds after _topology_loadGraph (topology.c:371).
// Output: CSR rows in igraph incidence order.  For a simple graph igraph's
// incidence list of v (igraph_incident, mode OUT; undirected -> ALL) is
// [oi: from==v sorted by to][ii: to==v sorted by from] with undirected edges
// stored from=max(a,b) -- i.e. ascending neighbour id, self-loop in place
// (SURVEY.md Appendix A.1-A.2).  Multigraphs are rejected (SHD_PE_EMULTI).
#include "pe_graph.hpp"

#include <algorithm>
#include <cmath>
#include <utility>

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

static int sort_rows(int32_t n, std::vector<int32_t>& ptr, std::vector<int32_t>& colv,
                     std::vector<double>& latv, std::vector<double>& relv) {
    std::vector<std::pair<int32_t, int32_t>> tmp;
    std::vector<double> l2, r2;
    for (int32_t v = 0; v < n; ++v) {
        const int32_t b = ptr[v], e = ptr[v + 1];
        bool sorted = true;
        for (int32_t a = b + 1; a < e; ++a)
            if (colv[a - 1] >= colv[a]) { sorted = false; break; }
        if (sorted) continue;
        tmp.clear();
        for (int32_t a = b; a < e; ++a) tmp.emplace_back(colv[a], a);
        std::sort(tmp.begin(), tmp.end());
        for (size_t k = 1; k < tmp.size(); ++k)
            if (tmp[k].first == tmp[k - 1].first) return SHD_PE_EMULTI;
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
    int64_t nonLoop = 0;
    std::vector<int64_t> deg(n + 1, 0);
    for (int64_t e = 0; e < m; ++e) {
        const int32_t a = d->edgeFrom[e], b = d->edgeTo[e];
        if (a < 0 || a >= n || b < 0 || b >= n) return SHD_PE_EINVAL;
        const double L = d->edgeLatency[e], p = d->edgePacketLoss[e];
        if (!(L > 0.0)) return SHD_PE_EINVAL;                  // :1070 (NaN fails too)
        if (!(p >= 0.0 && p <= 1.0)) return SHD_PE_EINVAL;     // :1090
        if (a == b) {
            if (g->hasSelf[a]) return SHD_PE_EMULTI;
            g->hasSelf[a] = 1;
            g->selfLat[a] = L;
            g->selfRel[a] = 1.0 - p;                            // :437
            continue;
        }
        ++nonLoop;
        deg[a + 1]++;
        if (!g->directed) deg[b + 1]++;
    }
    const int64_t nArcs = g->directed ? nonLoop : 2 * nonLoop;
    if (nArcs >= (int64_t)INT32_MAX) return SHD_PE_EINVAL;
    for (int32_t v = 0; v < n; ++v) deg[v + 1] += deg[v];
    g->rowPtr.assign(n + 1, 0);
    for (int32_t v = 0; v <= n; ++v) g->rowPtr[v] = (int32_t)deg[v];
    g->col.assign(nArcs, 0);
    g->lat.assign(nArcs, 0.0);
    g->rel.assign(nArcs, 0.0);
    {
        std::vector<int32_t> fill(g->rowPtr.begin(), g->rowPtr.end() - 1);
        for (int64_t e = 0; e < m; ++e) {
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
    }
    int rc = sort_rows(n, g->rowPtr, g->col, g->lat, g->rel);
    if (rc) return rc;

    g->outToIn.assign(nArcs, -1);
    if (g->directed) {
        // IN CSR sorted by source id
        std::vector<int32_t> cnt(n + 1, 0);
        for (int64_t a = 0; a < nArcs; ++a) cnt[g->col[a] + 1]++;
        for (int32_t v = 0; v < n; ++v) cnt[v + 1] += cnt[v];
        g->inPtr = cnt;
        g->inCol.assign(nArcs, 0);
        g->inLat.assign(nArcs, 0.0);
        g->inRel.assign(nArcs, 0.0);
        std::vector<int32_t> fill(cnt.begin(), cnt.end() - 1);
        for (int32_t u = 0; u < n; ++u) {               // rows visited in source order
            for (int32_t a = g->rowPtr[u]; a < g->rowPtr[u + 1]; ++a) {
                const int32_t v = g->col[a];
                const int32_t k = fill[v]++;
                g->inCol[k] = u; g->inLat[k] = g->lat[a]; g->inRel[k] = g->rel[a];
                g->outToIn[a] = k;
            }
        }
    } else {
        for (int32_t u = 0; u < n; ++u) {
            for (int32_t a = g->rowPtr[u]; a < g->rowPtr[u + 1]; ++a) {
                const int64_t rev = g->findArc(g->col[a], u);
                if (rev < 0) return SHD_PE_EINVAL;
                g->outToIn[a] = (int32_t)rev;
            }
        }
    }
    // _topology_isComplete (topology.c:450-552): incident count (undirected
    // self-loop counted twice, then corrected by one) must reach vcount.
    bool complete = true;
    for (int32_t v = 0; v < n && complete; ++v) {
        int64_t c = (int64_t)(g->rowPtr[v + 1] - g->rowPtr[v]);
        c += g->hasSelf[v] ? (g->directed ? 1 : 2) : 0;
        if (!g->directed && g->hasSelf[v]) c -= 1;
        if (c < n) complete = false;
    }
    g->isComplete = complete;
    double sum = 0.0;
    for (int64_t a = 0; a < nArcs; ++a) sum += g->lat[a];
    g->meanArcLatency = nArcs ? sum / (double)nArcs : 1.0;
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
    else if (a >= 0) { L = g.lat[a]; R = g.rel[a]; }
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
    for (; a < e && g.col[a] < v; ++a) visit(g.lat[a], g.rel[a]);
    if (g.hasSelf[v]) visit(g.selfLat[v], g.selfRel[v]);
    for (; a < e; ++a) visit(g.lat[a], g.rel[a]);
    if (!any && g.nEdges == 0) return SHD_PE_ENOEDGE;
    if (lat) *lat = 2.0 * minLatency;               // :1640
    if (rel) *rel = relMin * relMin;                // :1641
    return SHD_PE_OK;
}

}  // namespace shdpe

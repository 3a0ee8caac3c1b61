/*
 * pe_oracle.c -- CPU ORACLE (test infrastructure only; see pe_oracle.h).
 *
 * A plain-C restatement of the reference path: Shadow v1.14.0
 * src/main/routing/topology.c (path-compute portion) on top of a restatement
 * of igraph 0.7.1's Dijkstra, 2-way heap, edge storage and incidence order.
 * Each function cites the reference code it follows.  Never linked into the
 * product library.
 */
#define _GNU_SOURCE
#include "pe_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------ */
/* Graph storage: igraph "indexed edge list" (type_indexededgelist.c).       */
/* ------------------------------------------------------------------------ */
struct OrcGraph {
    int32_t n;
    int64_t m;
    int32_t directed;
    int32_t* from;    /* normalised like igraph_add_edges: undirected from=max */
    int32_t* to;
    double* lat;      /* 'latency' attribute (EANV, topology.c:1237)          */
    double* loss;     /* 'packetloss' attribute                               */
    double* vloss;    /* vertex 'packetloss' or NULL when absent               */
    int64_t* oi;      /* edge ids ordered by (from, to), ties: descending id  */
    int64_t* ii;      /* edge ids ordered by (to, from), ties: descending id  */
    int64_t* os;      /* os[v]..os[v+1]: oi range with from == v               */
    int64_t* is;      /* is[v]..is[v+1]: ii range with to == v                 */
};

/* igraph_vector_order(v, v2, res, nodes): two bucket passes, the first on the
 * secondary key v2, the second (stable over the first) on v.  Inside one
 * bucket the first pass lists edges in DESCENDING id order (the linked list
 * is built by prepending), which the second pass preserves -- this is why
 * parallel edges come out newest-first. */
static int orc_vector_order(const int32_t* v, const int32_t* v2, int64_t m,
                            int32_t nodes, int64_t* res) {
    int64_t* ptr = calloc((size_t)nodes + 1, sizeof(int64_t));
    int64_t* rad = calloc((size_t)(m > 0 ? m : 1), sizeof(int64_t));
    if (!ptr || !rad) { free(ptr); free(rad); return -1; }
    for (int64_t i = 0; i < m; i++) {
        int32_t radix = v2[i];
        if (ptr[radix] != 0) rad[i] = ptr[radix];
        ptr[radix] = i + 1;
    }
    int64_t j = 0;
    for (int64_t i = 0; i < (int64_t)nodes + 1; i++) {
        if (ptr[i] != 0) {
            int64_t next = ptr[i] - 1;
            res[j++] = next;
            while (rad[next] != 0) { next = rad[next] - 1; res[j++] = next; }
        }
    }
    memset(ptr, 0, ((size_t)nodes + 1) * sizeof(int64_t));
    memset(rad, 0, (size_t)(m > 0 ? m : 1) * sizeof(int64_t));
    for (int64_t i = 0; i < m; i++) {
        int64_t edge = res[m - i - 1];
        int32_t radix = v[edge];
        if (ptr[radix] != 0) rad[edge] = ptr[radix];
        ptr[radix] = edge + 1;
    }
    j = 0;
    for (int64_t i = 0; i < (int64_t)nodes + 1; i++) {
        if (ptr[i] != 0) {
            int64_t next = ptr[i] - 1;
            res[j++] = next;
            while (rad[next] != 0) { next = rad[next] - 1; res[j++] = next; }
        }
    }
    free(ptr);
    free(rad);
    return 0;
}

/* The same permutation as orc_vector_order -- (v ascending, v2 ascending,
 * edge id DESCENDING) -- by two counting sorts with sequential reads, for
 * edge lists where the linked-list walk's random accesses dominate (the
 * 2e8-edge C3 graphs).  orc_selftest_vector_order pins the equivalence. */
static int orc_vector_order_counting(const int32_t* v, const int32_t* v2, int64_t m,
                                     int32_t nodes, int64_t* res) {
    int64_t* cnt = calloc((size_t)nodes + 1, sizeof(int64_t));
    int64_t* tmp = malloc((size_t)(m > 0 ? m : 1) * sizeof(int64_t));
    if (!cnt || !tmp) { free(cnt); free(tmp); return -1; }
    for (int64_t i = 0; i < m; i++) cnt[v2[i] + 1]++;
    for (int32_t k = 0; k < nodes; k++) cnt[k + 1] += cnt[k];
    for (int64_t i = m - 1; i >= 0; i--) tmp[cnt[v2[i]]++] = i;   /* ids descending per bucket */
    memset(cnt, 0, ((size_t)nodes + 1) * sizeof(int64_t));
    for (int64_t i = 0; i < m; i++) cnt[v[i] + 1]++;
    for (int32_t k = 0; k < nodes; k++) cnt[k + 1] += cnt[k];
    for (int64_t i = 0; i < m; i++) { int64_t e = tmp[i]; res[cnt[v[e]]++] = e; }   /* stable */
    free(cnt);
    free(tmp);
    return 0;
}

static int orc_order(const int32_t* v, const int32_t* v2, int64_t m, int32_t nodes, int64_t* res) {
    return m < ((int64_t)1 << 22) ? orc_vector_order(v, v2, m, nodes, res)
                                  : orc_vector_order_counting(v, v2, m, nodes, res);
}

int32_t orc_selftest_vector_order(int64_t m, int32_t nodes, uint64_t seed) {
    int32_t* a = malloc((size_t)m * sizeof(int32_t));
    int32_t* b = malloc((size_t)m * sizeof(int32_t));
    int64_t* r1 = malloc((size_t)m * sizeof(int64_t));
    int64_t* r2 = malloc((size_t)m * sizeof(int64_t));
    int32_t ok = a && b && r1 && r2;
    uint64_t x = seed | 1;
    for (int64_t i = 0; ok && i < m; i++) {   /* xorshift; few nodes -> many parallel edges */
        x ^= x << 13; x ^= x >> 7; x ^= x << 17; a[i] = (int32_t)(x % (uint64_t)nodes);
        x ^= x << 13; x ^= x >> 7; x ^= x << 17; b[i] = (int32_t)(x % (uint64_t)nodes);
    }
    if (ok) ok = !orc_vector_order(a, b, m, nodes, r1) && !orc_vector_order_counting(a, b, m, nodes, r2);
    for (int64_t i = 0; ok && i < m; i++) ok = r1[i] == r2[i];
    free(a); free(b); free(r1); free(r2);
    return ok;
}

void orc_graph_free(OrcGraph* g) {
    if (!g) return;
    free(g->from); free(g->to); free(g->lat); free(g->loss); free(g->vloss);
    free(g->oi); free(g->ii); free(g->os); free(g->is);
    free(g);
}

OrcGraph* orc_graph_new(int32_t n, int64_t m, int32_t directed,
                        const int32_t* from, const int32_t* to,
                        const double* latency, const double* packetLoss,
                        const double* vertexLoss) {
    if (n <= 0 || m < 0 || (m > 0 && (!from || !to || !latency || !packetLoss)))
        return NULL;
    OrcGraph* g = calloc(1, sizeof(OrcGraph));
    if (!g) return NULL;
    g->n = n; g->m = m; g->directed = directed ? 1 : 0;
    size_t mm = (size_t)(m > 0 ? m : 1);
    g->from = malloc(mm * sizeof(int32_t));
    g->to = malloc(mm * sizeof(int32_t));
    g->lat = malloc(mm * sizeof(double));
    g->loss = malloc(mm * sizeof(double));
    g->oi = malloc(mm * sizeof(int64_t));
    g->ii = malloc(mm * sizeof(int64_t));
    g->os = calloc((size_t)n + 1, sizeof(int64_t));
    g->is = calloc((size_t)n + 1, sizeof(int64_t));
    if (!g->from || !g->to || !g->lat || !g->loss || !g->oi || !g->ii || !g->os || !g->is) {
        orc_graph_free(g);
        return NULL;
    }
    /* igraph_add_edges: undirected edges are stored with from = max(a,b). */
    for (int64_t e = 0; e < m; e++) {
        int32_t a = from[e], b = to[e];
        if (a < 0 || a >= n || b < 0 || b >= n) { orc_graph_free(g); return NULL; }
        if (g->directed || a > b) { g->from[e] = a; g->to[e] = b; }
        else { g->from[e] = b; g->to[e] = a; }
        g->lat[e] = latency[e];
        g->loss[e] = packetLoss[e];
    }
    if (vertexLoss) {
        g->vloss = malloc((size_t)n * sizeof(double));
        if (!g->vloss) { orc_graph_free(g); return NULL; }
        memcpy(g->vloss, vertexLoss, (size_t)n * sizeof(double));
    }
    if (orc_order(g->from, g->to, m, n, g->oi) ||
        orc_order(g->to, g->from, m, n, g->ii)) {
        orc_graph_free(g);
        return NULL;
    }
    /* igraph_i_create_start: os/is = start offsets into oi/ii */
    for (int64_t e = 0; e < m; e++) { g->os[g->from[e] + 1]++; g->is[g->to[e] + 1]++; }
    for (int32_t v = 0; v < n; v++) { g->os[v + 1] += g->os[v]; g->is[v + 1] += g->is[v]; }
    return g;
}

/* Incidence list of v, mode OUT (igraph_incident / igraph_lazy_inclist_get):
 * undirected graphs use mode ALL = [oi part][ii part]; a self-loop therefore
 * appears twice.  Returns the count; writes up to cap ids into out. */
static int64_t orc_incident_count(const OrcGraph* g, int32_t v) {
    int64_t c = g->os[v + 1] - g->os[v];
    if (!g->directed) c += g->is[v + 1] - g->is[v];
    return c;
}

static inline int64_t orc_incident_at(const OrcGraph* g, int32_t v, int64_t k) {
    int64_t no = g->os[v + 1] - g->os[v];
    if (k < no) return g->oi[g->os[v] + k];
    return g->ii[g->is[v] + (k - no)];
}

static inline int32_t orc_other(const OrcGraph* g, int64_t e, int32_t v) {
    /* IGRAPH_OTHER */
    return g->to[e] == v ? g->from[e] : g->to[e];
}

/* BINSEARCH from type_indexededgelist.c: leftmost entry >= value in the
 * sorted sub-range; hit only if equal. */
static int64_t orc_binsearch(const OrcGraph* g, int64_t start, int64_t end,
                             int32_t value, const int64_t* iindex,
                             const int32_t* edgelist, int64_t N) {
    while (start < end) {
        int64_t mid = start + (end - start) / 2;
        int64_t e = iindex[mid];
        if (edgelist[e] < value) start = mid + 1; else end = mid;
    }
    if (start < N) {
        int64_t e = iindex[start];
        if (edgelist[e] == value) return e;
    }
    (void)g;
    return -1;
}

static int64_t orc_find_directed(const OrcGraph* g, int32_t xfrom, int32_t xto) {
    int64_t start = g->os[xfrom], end = g->os[xfrom + 1], N = end;
    int64_t start2 = g->is[xto], end2 = g->is[xto + 1], N2 = end2;
    if (end - start < end2 - start2)
        return orc_binsearch(g, start, end, xto, g->oi, g->to, N);
    return orc_binsearch(g, start2, end2, xfrom, g->ii, g->from, N2);
}

/* igraph_get_eid(graph, &eid, from, to, directed=isDirected, error=FALSE)
 * as called by _topology_getEdgeHelper (topology.c:402-444). */
int64_t orc_get_eid(const OrcGraph* g, int32_t from, int32_t to) {
    if (from < 0 || from >= g->n || to < 0 || to >= g->n) return -1;
    if (g->directed) return orc_find_directed(g, from, to);
    int32_t a = from > to ? from : to, b = from > to ? to : from;
    return orc_find_directed(g, a, b);
}

/* _topology_findVertexAttributeDouble(VERTEX_ATTR_PACKETLOSS)
 * (topology.c:330-349): present iff the attribute exists and is not NaN. */
static inline int orc_vertex_loss(const OrcGraph* g, int32_t v, double* out) {
    if (!g->vloss) return 0;
    double x = g->vloss[v];
    if (isnan(x)) return 0;
    *out = x;
    return 1;
}

/* _topology_isComplete (topology.c:450-552) */
int32_t orc_is_complete(const OrcGraph* g) {
    for (int32_t v = 0; v < g->n; v++) {
        int64_t ecount = orc_incident_count(g, v);
        if (!g->directed) {
            if (orc_get_eid(g, v, v) >= 0) ecount -= 1;  /* :508-521 */
        }
        if (ecount < g->n) return 0;                    /* :523-530 */
    }
    return 1;
}

/* ------------------------------------------------------------------------ */
/* igraph_2wheap_t (heap.c, 0.7.1): binary MAX-heap with an index.           */
/* index2[v]: 0 = not in heap, else position + 2.                            */
/* ------------------------------------------------------------------------ */
typedef struct {
    double* data;
    int32_t* index;
    int64_t* index2;
    int64_t size;
} OrcHeap;

#define H_PARENT(x) ((((x) + 1) / 2) - 1)
#define H_LEFT(x) (((x) + 1) * 2 - 1)
#define H_RIGHT(x) (((x) + 1) * 2)

static inline void heap_switch(OrcHeap* h, int64_t e1, int64_t e2) {
    if (e1 != e2) {
        double tmp3 = h->data[e1];
        h->data[e1] = h->data[e2];
        h->data[e2] = tmp3;
        int32_t tmp1 = h->index[e1], tmp2 = h->index[e2];
        h->index2[tmp1] = e2 + 2;
        h->index2[tmp2] = e1 + 2;
        h->index[e1] = tmp2;
        h->index[e2] = tmp1;
    }
}

static void heap_shift_up(OrcHeap* h, int64_t elem) {
    /* recursive in igraph; iterative here with identical comparisons */
    while (!(elem == 0 || h->data[elem] < h->data[H_PARENT(elem)])) {
        heap_switch(h, elem, H_PARENT(elem));
        elem = H_PARENT(elem);
    }
}

static void heap_sink(OrcHeap* h, int64_t head) {
    for (;;) {
        int64_t size = h->size;
        if (H_LEFT(head) >= size) return;                      /* no subtrees */
        if (H_RIGHT(head) == size || h->data[H_LEFT(head)] >= h->data[H_RIGHT(head)]) {
            if (h->data[head] < h->data[H_LEFT(head)]) {       /* sink left */
                heap_switch(h, head, H_LEFT(head));
                head = H_LEFT(head);
            } else return;
        } else {
            if (h->data[head] < h->data[H_RIGHT(head)]) {      /* sink right */
                heap_switch(h, head, H_RIGHT(head));
                head = H_RIGHT(head);
            } else return;
        }
    }
}

static void heap_push_with_index(OrcHeap* h, int32_t idx, double elem) {
    int64_t size = h->size;
    h->data[size] = elem;
    h->index[size] = idx;
    h->size = size + 1;
    h->index2[idx] = size + 2;
    heap_shift_up(h, size);
}

static double heap_delete_max(OrcHeap* h) {
    double tmp = h->data[0];
    int32_t tmpidx = h->index[0];
    heap_switch(h, 0, h->size - 1);
    h->size -= 1;
    h->index2[tmpidx] = 0;
    heap_sink(h, 0);
    return tmp;
}

static void heap_modify(OrcHeap* h, int32_t idx, double elem) {
    int64_t pos = h->index2[idx] - 2;
    h->data[pos] = elem;
    heap_sink(h, pos);
    heap_shift_up(h, pos);
}

/* ------------------------------------------------------------------------ */
/* igraph_get_shortest_paths_dijkstra (0.7.1, structural_properties.c) as     */
/* called at topology.c:1765 (mode IGRAPH_OUT, weights = latency).           */
/* ------------------------------------------------------------------------ */
typedef struct {
    double* dist;        /* -1 = infinity (igraph's "dirty trick") */
    int64_t* parent;     /* parent edge id + 1, 0 = none           */
    uint8_t* isTarget;
    OrcHeap heap;
} OrcWork;

static int work_init(OrcWork* w, int32_t n) {
    memset(w, 0, sizeof(*w));
    w->dist = malloc((size_t)n * sizeof(double));
    w->parent = malloc((size_t)n * sizeof(int64_t));
    w->isTarget = malloc((size_t)n);
    w->heap.data = malloc((size_t)n * sizeof(double));
    w->heap.index = malloc((size_t)n * sizeof(int32_t));
    w->heap.index2 = malloc((size_t)n * sizeof(int64_t));
    return (w->dist && w->parent && w->isTarget && w->heap.data && w->heap.index && w->heap.index2) ? 0 : -1;
}

static void work_free(OrcWork* w) {
    free(w->dist); free(w->parent); free(w->isTarget);
    free(w->heap.data); free(w->heap.index); free(w->heap.index2);
}

static int32_t run_dijkstra(const OrcGraph* g, int32_t from, const int32_t* targets,
                            int32_t nTargets, OrcWork* w, int32_t* popOrder) {
    int32_t n = g->n;
    for (int32_t v = 0; v < n; v++) { w->dist[v] = -1.0; w->parent[v] = 0; w->isTarget[v] = 0; w->heap.index2[v] = 0; }
    w->heap.size = 0;
    int64_t toReach = nTargets;
    for (int32_t j = 0; j < nTargets; j++) {
        if (!w->isTarget[targets[j]]) w->isTarget[targets[j]] = 1;
        else toReach--;                       /* node given multiple times */
    }
    w->dist[from] = 0.0;
    w->parent[from] = 0;
    heap_push_with_index(&w->heap, from, 0);
    int32_t popped = 0;
    while (w->heap.size > 0 && toReach > 0) {
        int32_t minnei = w->heap.index[0];
        double mindist = -heap_delete_max(&w->heap);
        if (popOrder) popOrder[popped] = minnei;
        popped++;
        if (w->isTarget[minnei]) { w->isTarget[minnei] = 0; toReach--; }
        int64_t nlen = orc_incident_count(g, minnei);
        for (int64_t i = 0; i < nlen; i++) {
            int64_t edge = orc_incident_at(g, minnei, i);
            int32_t tto = orc_other(g, edge, minnei);
            double altdist = mindist + g->lat[edge];
            double curdist = w->dist[tto];
            if (curdist < 0) {
                /* first finite distance */
                w->dist[tto] = altdist;
                w->parent[tto] = edge + 1;
                heap_push_with_index(&w->heap, tto, -altdist);
            } else if (altdist < curdist) {
                /* shorter path */
                w->dist[tto] = altdist;
                w->parent[tto] = edge + 1;
                heap_modify(&w->heap, tto, -altdist);
            }
        }
    }
    return popped;
}

int32_t orc_dijkstra_raw(const OrcGraph* g, int32_t src, const int32_t* targets,
                         int32_t nTargets, double* dist, int64_t* parentEdgePlus1,
                         int32_t* popOrder, int32_t* popped) {
    if (!g || src < 0 || src >= g->n || nTargets < 0 || (nTargets > 0 && !targets)) return -1;
    for (int32_t j = 0; j < nTargets; j++) if (targets[j] < 0 || targets[j] >= g->n) return -1;
    OrcWork w;
    if (work_init(&w, g->n)) { work_free(&w); return -1; }
    int32_t p = run_dijkstra(g, src, targets, nTargets, &w, popOrder);
    if (dist) memcpy(dist, w.dist, (size_t)g->n * sizeof(double));
    if (parentEdgePlus1) memcpy(parentEdgePlus1, w.parent, (size_t)g->n * sizeof(int64_t));
    if (popped) *popped = p;
    work_free(&w);
    return 0;
}

/* One target: igraph path reconstruction (walk parent edges) followed by
 * _topology_computePathProperties (topology.c:1407-1523) and the zero-latency
 * rule of topology.c:1848-1852. */
static void fold_target(const OrcGraph* g, int32_t s, int32_t t, const OrcWork* w,
                        int32_t* pathBuf, double* lat, double* rel, int32_t* hops,
                        int32_t* pred, uint8_t* flags) {
    double totalLatency = 0.0, totalReliability = 1.0;
    int32_t h = 0, pv = -1;
    uint8_t f = ORC_F_OK;
    if (t != s && w->parent[t] == 0) {
        /* igraph 0.7.1 leaves an unreachable target with no parent chain; the
         * graph is required to be strongly connected (topology.c:799-806). */
        f = ORC_F_UNREACHABLE;
        goto out;
    }
    /* reconstruct [s, ..., t] */
    int64_t size = 0;
    int32_t act = t;
    while (w->parent[act]) { size++; act = orc_other(g, w->parent[act] - 1, act); }
    int64_t nVertices = size + 1;
    pathBuf[size] = t;
    act = t;
    int64_t k = size;
    while (w->parent[act]) { act = orc_other(g, w->parent[act] - 1, act); pathBuf[--k] = act; }

    double ploss;
    if (orc_vertex_loss(g, s, &ploss)) totalReliability *= (1.0 - ploss);          /* :1443 */
    if ((s != t) || (s == t && nVertices > 2)) {                                    /* :1457 */
        if (orc_vertex_loss(g, t, &ploss)) totalReliability *= (1.0 - ploss);
    }
    int64_t start = nVertices == 1 ? 0 : 1;                                         /* :1471 */
    int32_t fromV = s;
    for (int64_t i = start; i < nVertices; i++) {
        int32_t toV = pathBuf[i];
        int64_t e = orc_get_eid(g, fromV, toV);                                     /* :1488 */
        if (e < 0) { f = ORC_F_NOEDGE; goto out; }                                  /* :1490 */
        double edgeLatency = g->lat[e];
        double edgeReliability = (1.0 - g->loss[e]);                                /* :437  */
        totalLatency += edgeLatency;                                                /* :1498 */
        totalReliability *= edgeReliability;                                        /* :1499 */
        h++;
        fromV = toV;
    }
    pv = nVertices >= 2 ? pathBuf[nVertices - 2] : -1;
    if (totalLatency == 0) { totalLatency = 1; f |= ORC_F_ZEROLAT; }               /* :1848 */
out:
    if (lat) *lat = totalLatency;
    if (rel) *rel = totalReliability;
    if (hops) *hops = h;
    if (pred) *pred = pv;
    if (flags) *flags = f;
}

static int32_t row_with_work(const OrcGraph* g, int32_t src, const int32_t* targets,
                             int32_t nTargets, OrcWork* w, int32_t* pathBuf,
                             double* lat, double* rel, int32_t* hops, int32_t* pred,
                             uint8_t* flags) {
    run_dijkstra(g, src, targets, nTargets, w, NULL);
    for (int32_t j = 0; j < nTargets; j++) {
        fold_target(g, src, targets[j], w, pathBuf,
                    lat ? lat + j : NULL, rel ? rel + j : NULL, hops ? hops + j : NULL,
                    pred ? pred + j : NULL, flags ? flags + j : NULL);
    }
    return 0;
}

int32_t orc_dijkstra_row(const OrcGraph* g, int32_t src, const int32_t* targets,
                         int32_t nTargets, double* lat, double* rel, int32_t* hops,
                         int32_t* pred, uint8_t* flags) {
    if (!g || src < 0 || src >= g->n || nTargets < 0 || (nTargets > 0 && !targets)) return -1;
    for (int32_t j = 0; j < nTargets; j++) if (targets[j] < 0 || targets[j] >= g->n) return -1;
    OrcWork w;
    int32_t* pathBuf = malloc((size_t)g->n * sizeof(int32_t) + sizeof(int32_t));
    if (work_init(&w, g->n) || !pathBuf) { work_free(&w); free(pathBuf); return -1; }
    row_with_work(g, src, targets, nTargets, &w, pathBuf, lat, rel, hops, pred, flags);
    work_free(&w);
    free(pathBuf);
    return 0;
}

/* ------------------------------------------------------------------------ */
/* CPU baseline helper: one source per task over nThreads pthreads.          */
/* ------------------------------------------------------------------------ */
typedef struct {
    const OrcGraph* g;
    const int32_t* sources; int32_t nSources;
    const int32_t* targets; int32_t nTargets;
    double* lat; double* rel; int32_t* hops; int32_t* pred; uint8_t* flags;
    int64_t next;     /* shared work counter */
    pthread_mutex_t mu;
} OrcPool;

static void* pool_worker(void* arg) {
    OrcPool* p = arg;
    OrcWork w;
    int32_t* pathBuf = malloc((size_t)p->g->n * sizeof(int32_t) + sizeof(int32_t));
    if (work_init(&w, p->g->n) || !pathBuf) { work_free(&w); free(pathBuf); return NULL; }
    for (;;) {
        pthread_mutex_lock(&p->mu);
        int64_t i = p->next++;
        pthread_mutex_unlock(&p->mu);
        if (i >= p->nSources) break;
        size_t off = (size_t)i * (size_t)p->nTargets;
        row_with_work(p->g, p->sources[i], p->targets, p->nTargets, &w, pathBuf,
                      p->lat ? p->lat + off : NULL, p->rel ? p->rel + off : NULL,
                      p->hops ? p->hops + off : NULL, p->pred ? p->pred + off : NULL,
                      p->flags ? p->flags + off : NULL);
    }
    work_free(&w);
    free(pathBuf);
    return NULL;
}

int32_t orc_rows_parallel(const OrcGraph* g, const int32_t* sources, int32_t nSources,
                          const int32_t* targets, int32_t nTargets, int32_t nThreads,
                          double* lat, double* rel, int32_t* hops, int32_t* pred,
                          uint8_t* flags) {
    if (!g || nSources < 0 || nTargets < 0 || nThreads < 1) return -1;
    for (int32_t i = 0; i < nSources; i++) if (sources[i] < 0 || sources[i] >= g->n) return -1;
    for (int32_t j = 0; j < nTargets; j++) if (targets[j] < 0 || targets[j] >= g->n) return -1;
    OrcPool p = {g, sources, nSources, targets, nTargets, lat, rel, hops, pred, flags, 0,
                 PTHREAD_MUTEX_INITIALIZER};
    if (nThreads == 1) { pool_worker(&p); return 0; }
    pthread_t* th = malloc(sizeof(pthread_t) * (size_t)nThreads);
    if (!th) return -1;
    for (int32_t i = 0; i < nThreads; i++) pthread_create(&th[i], NULL, pool_worker, &p);
    for (int32_t i = 0; i < nThreads; i++) pthread_join(th[i], NULL);
    free(th);
    return 0;
}

/* ------------------------------------------------------------------------ */
/* Checker (not a restatement): the Bellman condition of R rows at once.     */
/* dT[v * R + r] = row r's distance to vertex v (its source at 0, +inf for   */
/* unreached); viol[r] counts arcs (u, v) with dT[u] + w < dT[v] (the row is */
/* then not a shortest-path row).  Threads split the edge list; each edge is */
/* read once for all R rows.                                                  */
/* ------------------------------------------------------------------------ */
typedef struct {
    const OrcGraph* g; const double* dT; int32_t R;
    int64_t e0, e1; int64_t* viol;
} OrcBell;

static void* bell_worker(void* arg) {
    OrcBell* b = arg;
    const OrcGraph* g = b->g;
    const int32_t R = b->R;
    for (int64_t e = b->e0; e < b->e1; e++) {
        const int32_t u = g->from[e], v = g->to[e];
        if (u == v) continue;
        const double w = g->lat[e];
        const double* du = b->dT + (size_t)u * (size_t)R;
        const double* dv = b->dT + (size_t)v * (size_t)R;
        for (int32_t r = 0; r < R; r++) {
            b->viol[r] += (du[r] + w < dv[r]);
            if (!g->directed) b->viol[r] += (dv[r] + w < du[r]);
        }
    }
    return NULL;
}

int32_t orc_bellman_rows(const OrcGraph* g, const double* dT, int32_t R, int32_t nThreads,
                         int64_t* viol) {
    if (!g || !dT || R < 1 || nThreads < 1 || !viol) return -1;
    OrcBell* bs = calloc((size_t)nThreads, sizeof(OrcBell));
    int64_t* cnt = calloc((size_t)nThreads * (size_t)R, sizeof(int64_t));
    pthread_t* th = malloc(sizeof(pthread_t) * (size_t)nThreads);
    if (!bs || !cnt || !th) { free(bs); free(cnt); free(th); return -1; }
    for (int32_t t = 0; t < nThreads; t++) {
        bs[t] = (OrcBell){g, dT, R, g->m * t / nThreads, g->m * (t + 1) / nThreads,
                          cnt + (size_t)t * (size_t)R};
        pthread_create(&th[t], NULL, bell_worker, &bs[t]);
    }
    for (int32_t t = 0; t < nThreads; t++) pthread_join(th[t], NULL);
    for (int32_t r = 0; r < R; r++) {
        viol[r] = 0;
        for (int32_t t = 0; t < nThreads; t++) viol[r] += cnt[(size_t)t * (size_t)R + r];
    }
    free(bs); free(cnt); free(th);
    return 0;
}

/* _topology_lookupDirectPath (topology.c:1877-1927) */
int32_t orc_direct_path(const OrcGraph* g, int32_t s, int32_t t, double* lat, double* rel) {
    double totalLatency = 0.0, totalReliability = 1.0, ploss;
    if (!g || s < 0 || s >= g->n || t < 0 || t >= g->n) return -1;
    if (orc_vertex_loss(g, s, &ploss)) totalReliability *= (1.0 - ploss);           /* :1901 */
    if (orc_vertex_loss(g, t, &ploss)) totalReliability *= (1.0 - ploss);           /* :1905 */
    int64_t e = orc_get_eid(g, s, t);
    /* get_eid with error=FALSE returns success and eid=-1 for a missing edge;
     * the reference then asserts the attribute lookup -- treat as failure. */
    if (e < 0) return -1;
    totalLatency += g->lat[e];                                                      /* :1920 */
    totalReliability *= (1.0 - g->loss[e]);                                         /* :1921 */
    if (lat) *lat = totalLatency;
    if (rel) *rel = totalReliability;
    return 0;
}

/* _topology_computeShortestPathToSelf (topology.c:1545-1653) */
int32_t orc_self_path(const OrcGraph* g, int32_t v, double* lat, double* rel) {
    if (!g || v < 0 || v >= g->n) return -1;
    double minLatency = 0.0, relMin = 0.0;
    int64_t nlen = orc_incident_count(g, v);
    if (nlen == 0 && g->m == 0) return -1;   /* igraph_edge(0) would fail */
    for (int64_t i = 0; i < nlen; i++) {
        int64_t e = orc_incident_at(g, v, i);
        double edgeLatency = g->lat[e];
        if (minLatency == 0 || edgeLatency < minLatency) {                          /* :1592 */
            minLatency = edgeLatency;
            relMin = 1.0 - g->loss[e];                                              /* :1597 */
        }
    }
    if (lat) *lat = 2.0 * minLatency;                                               /* :1640 */
    if (rel) *rel = relMin * relMin;                                                /* :1641 */
    return 0;
}

/* ------------------------------------------------------------------------ */
/* Path cache + dispatcher (topology.c:1284-1386, 1969-2092).                */
/* ------------------------------------------------------------------------ */
typedef struct {
    uint64_t key;      /* (src << 32) | dst, UINT64_MAX = empty */
    double lat, rel;
    int32_t isDirect;
    int64_t packetCount;
} OrcPath;

struct OrcTopology {
    const OrcGraph* g;
    int32_t* attached; int32_t nAttached;
    uint8_t* isAttached;
    int32_t isComplete;
    int32_t prefersDirectPaths;
    OrcPath* slots; int64_t cap; int64_t count;
    double minimumPathLatency;
    int64_t rowsComputed, selfPathsComputed;
    /* row scratch */
    double* rlat; double* rrel; uint8_t* rflags;
};

#define ORC_EMPTY UINT64_MAX

static inline uint64_t orc_hash(uint64_t k) {
    k ^= k >> 33; k *= 0xff51afd7ed558ccdULL; k ^= k >> 33;
    k *= 0xc4ceb9fe1a85ec53ULL; k ^= k >> 33;
    return k;
}

static OrcPath* cache_find(const OrcTopology* t, int32_t s, int32_t d) {
    uint64_t key = ((uint64_t)(uint32_t)s << 32) | (uint32_t)d;
    uint64_t i = orc_hash(key) & (uint64_t)(t->cap - 1);
    for (;;) {
        OrcPath* p = &t->slots[i];
        if (p->key == ORC_EMPTY) return NULL;
        if (p->key == key) return p;
        i = (i + 1) & (uint64_t)(t->cap - 1);
    }
}

static int cache_grow(OrcTopology* t) {
    int64_t ncap = t->cap * 2;
    OrcPath* ns = malloc((size_t)ncap * sizeof(OrcPath));
    if (!ns) return -1;
    for (int64_t i = 0; i < ncap; i++) ns[i].key = ORC_EMPTY;
    for (int64_t i = 0; i < t->cap; i++) {
        if (t->slots[i].key == ORC_EMPTY) continue;
        uint64_t j = orc_hash(t->slots[i].key) & (uint64_t)(ncap - 1);
        while (ns[j].key != ORC_EMPTY) j = (j + 1) & (uint64_t)(ncap - 1);
        ns[j] = t->slots[i];
    }
    free(t->slots);
    t->slots = ns;
    t->cap = ncap;
    return 0;
}

static OrcPath* cache_insert(OrcTopology* t, int32_t s, int32_t d) {
    if ((t->count + 1) * 2 > t->cap && cache_grow(t)) return NULL;
    uint64_t key = ((uint64_t)(uint32_t)s << 32) | (uint32_t)d;
    uint64_t i = orc_hash(key) & (uint64_t)(t->cap - 1);
    while (t->slots[i].key != ORC_EMPTY && t->slots[i].key != key)
        i = (i + 1) & (uint64_t)(t->cap - 1);
    if (t->slots[i].key == ORC_EMPTY) t->count++;
    t->slots[i].key = key;
    return &t->slots[i];
}

OrcTopology* orc_topology_new(const OrcGraph* g, const int32_t* attached, int32_t nAttached,
                              int32_t prefersDirectPaths) {
    if (!g || nAttached < 0) return NULL;
    OrcTopology* t = calloc(1, sizeof(OrcTopology));
    if (!t) return NULL;
    t->g = g;
    t->isAttached = calloc((size_t)g->n, 1);
    t->attached = malloc(sizeof(int32_t) * (size_t)(nAttached > 0 ? nAttached : 1));
    t->cap = 1024;
    t->slots = malloc((size_t)t->cap * sizeof(OrcPath));
    t->rlat = malloc(sizeof(double) * (size_t)(nAttached > 0 ? nAttached : 1));
    t->rrel = malloc(sizeof(double) * (size_t)(nAttached > 0 ? nAttached : 1));
    t->rflags = malloc((size_t)(nAttached > 0 ? nAttached : 1));
    if (!t->isAttached || !t->attached || !t->slots || !t->rlat || !t->rrel || !t->rflags) {
        orc_topology_free(t);
        return NULL;
    }
    for (int64_t i = 0; i < t->cap; i++) t->slots[i].key = ORC_EMPTY;
    /* _topology_getUniqueVertexTargets: the unique attached vertices */
    for (int32_t i = 0; i < nAttached; i++) {
        int32_t v = attached[i];
        if (v < 0 || v >= g->n) { orc_topology_free(t); return NULL; }
        if (!t->isAttached[v]) { t->isAttached[v] = 1; t->attached[t->nAttached++] = v; }
    }
    t->isComplete = orc_is_complete(g);
    t->prefersDirectPaths = prefersDirectPaths ? 1 : 0;
    return t;
}

void orc_topology_free(OrcTopology* t) {
    if (!t) return;
    free(t->isAttached); free(t->attached); free(t->slots);
    free(t->rlat); free(t->rrel); free(t->rflags);
    free(t);
}

static int orc_adjacent(const OrcTopology* t, int32_t s, int32_t d) {
    return orc_get_eid(t->g, s, d) >= 0;                  /* topology.c:1248-1264 */
}

/* _topology_shouldStorePath (topology.c:1307-1336) */
static int should_store(const OrcTopology* t, int isDirect, int32_t s, int32_t d) {
    if (cache_find(t, s, d) || cache_find(t, d, s)) return 0;
    if (t->isComplete && !isDirect) return 0;
    if (t->prefersDirectPaths && !isDirect && orc_adjacent(t, s, d)) return 0;
    return 1;
}

/* _topology_storePathInCache (topology.c:1338-1386) */
static void store_path(OrcTopology* t, int isDirect, int32_t s, int32_t d, double lat, double rel) {
    if (!should_store(t, isDirect, s, d)) return;
    OrcPath* p = cache_insert(t, s, d);
    if (!p) return;
    p->lat = lat; p->rel = rel; p->isDirect = isDirect; p->packetCount = 0;
    if (t->minimumPathLatency == 0 || lat < t->minimumPathLatency) t->minimumPathLatency = lat;
}

/* _topology_computeSourcePaths (topology.c:1655-1875) */
static int compute_source_paths(OrcTopology* t, int32_t s, int32_t d) {
    if (s == d) {
        double lat, rel;
        t->selfPathsComputed++;
        if (orc_self_path(t->g, s, &lat, &rel)) return 0;
        store_path(t, 0, s, s, lat, rel);                  /* :1650 */
        return 1;
    }
    if (!t->isAttached[d]) return 0;                      /* utility_assert(:1742) */
    t->rowsComputed++;
    if (orc_dijkstra_row(t->g, s, t->attached, t->nAttached, t->rlat, t->rrel, NULL, NULL, t->rflags))
        return 0;
    int allSuccess = 1;
    for (int32_t j = 0; j < t->nAttached; j++) {
        /* nVertices == 0 (no igraph path): skipped, isAllSuccess untouched (:1815) */
        if (t->rflags[j] & ORC_F_UNREACHABLE) continue;
        /* _topology_computePathProperties failed: isAllSuccess = FALSE (:1857) */
        if (t->rflags[j] & ORC_F_NOEDGE) { allSuccess = 0; continue; }
        store_path(t, 0, s, t->attached[j], t->rlat[j], t->rrel[j]);   /* :1855 */
    }
    return allSuccess;
}

/* _topology_getPathEntry (topology.c:1969-2051) */
static OrcPath* get_path_entry(OrcTopology* t, int32_t s, int32_t d) {
    const OrcGraph* g = t->g;
    if (s < 0 || s >= g->n || d < 0 || d >= g->n) return NULL;
    if (!t->isAttached[s] || !t->isAttached[d]) return NULL;  /* not connected (:1973-1984) */
    OrcPath* p = cache_find(t, s, d);
    if (!p && !g->directed) p = cache_find(t, d, s);
    if (!p) {
        int success;
        int adjacent = orc_adjacent(t, s, d);
        if (t->isComplete || (t->prefersDirectPaths && adjacent)) {
            double lat, rel;
            success = orc_direct_path(g, s, d, &lat, &rel) == 0;
            if (success) store_path(t, 1, s, d, lat, rel);
        } else {
            success = compute_source_paths(t, s, d);
        }
        if (success) {
            p = cache_find(t, s, d);
            if (!p) p = cache_find(t, d, s);               /* :2034-2037 even if directed */
        }
    }
    return p;                                             /* NULL -> error() (:2040) */
}

double orc_topology_get_latency(OrcTopology* t, int32_t s, int32_t d) {
    OrcPath* p = get_path_entry(t, s, d);
    return p ? p->lat : -1.0;
}

double orc_topology_get_reliability(OrcTopology* t, int32_t s, int32_t d) {
    OrcPath* p = get_path_entry(t, s, d);
    return p ? p->rel : -1.0;
}

int32_t orc_topology_is_routable(OrcTopology* t, int32_t s, int32_t d) {
    return orc_topology_get_latency(t, s, d) > -1 ? 1 : 0;
}

int32_t orc_topology_increment_packet_counter(OrcTopology* t, int32_t s, int32_t d) {
    OrcPath* p = get_path_entry(t, s, d);
    if (!p) return -1;
    p->packetCount++;
    return 0;
}

int32_t orc_topology_cached(const OrcTopology* t, int32_t s, int32_t d, double* lat,
                            double* rel, int32_t* isDirect, int64_t* packetCount) {
    OrcPath* p = cache_find(t, s, d);
    if (!p) return 0;
    if (lat) *lat = p->lat;
    if (rel) *rel = p->rel;
    if (isDirect) *isDirect = p->isDirect;
    if (packetCount) *packetCount = p->packetCount;
    return 1;
}

double orc_topology_min_latency(const OrcTopology* t) { return t->minimumPathLatency; }
int64_t orc_topology_rows_computed(const OrcTopology* t) { return t->rowsComputed; }
int64_t orc_topology_self_paths_computed(const OrcTopology* t) { return t->selfPathsComputed; }
int64_t orc_topology_cache_size(const OrcTopology* t) { return t->count; }

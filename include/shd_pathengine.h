/*
 * shd_pathengine.h -- C-ABI of the MI355X-native Shadow path engine.
 *
 * Drop-in boundary for Shadow v1.14.0 src/main/routing/topology.c.  The
 * engine replaces the region topology.c:1681-1866 inside
 * _topology_computeSourcePaths (target collection, the igraph Dijkstra call at
 * :1765 and the per-target _topology_computePathProperties fold at :1805-1864):
 * one call returns the dense row for a source, and host C keeps calling
 * _topology_storePathInCache (:1855) per target, so the cache rules, the
 * min-latency/lookahead update (:1375-1385) and logging are unchanged.
 *
 * Plain C types only (no HIP/torch types).  All functions return 0 on success
 * or a negative SHD_PE_E* code; shd_pe_strerror() names it.  Caller-owned
 * input arrays are only borrowed for the duration of the call.  The engine
 * owns its device memory and stream; nothing it returns outlives
 * shd_pe_destroy().  The engine never calls back into topology.c.
 *
 * Threading: compute / gather calls serialise on an engine mutex (the
 * reference holds graphLock around the igraph call, topology.c:1747-1781);
 * shd_pe_get_row / get_rows may be called from any number of threads at any
 * time (a row not yet computed is computed under that mutex first; the
 * computed-row flags are acquire/release atomics).
 *
 * Multi-GPU: the T table rows are split into G contiguous
 * row shards.  One engine owns nDevices of them (one per device, computed
 * concurrently); with shardCount > 1 several engines -- one per process --
 * own the rest.  shd_pe_gather assembles the whole table on every device
 * with RCCL over xGMI (shd_pe_comm_init joins the processes).
 */
#ifndef SHD_PATHENGINE_H
#define SHD_PATHENGINE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SHD_PE_ABI_VERSION 3

/* ---- error codes ------------------------------------------------------ */
#define SHD_PE_OK            0
#define SHD_PE_EINVAL       -1   /* bad argument / graph fails topology.c checks  */
#define SHD_PE_ENOMEM       -2   /* host or device allocation failed              */
#define SHD_PE_ENODEV       -3   /* no usable gfx950 device / HIP init failed     */
#define SHD_PE_EUNREACHABLE -4   /* (per entry, see flags) target not reachable    */
#define SHD_PE_ENOSELFLOOP  -5   /* (per entry, see flags) (s,s) self-loop missing */
#define SHD_PE_EMULTI       -6   /* reserved (before round 5: a multigraph whose newest parallel edge is not a fastest one; every multigraph is supported now) */
#define SHD_PE_EHIP         -7   /* HIP runtime error during compute               */
#define SHD_PE_ENOTATTACHED -8   /* vertex is not in the attached set              */
#define SHD_PE_ENOEDGE      -9   /* direct path requested but (s,t) has no edge    */
#define SHD_PE_ENOTOWNED   -10   /* row lives in another engine's shard (gather)   */
#define SHD_PE_ETOOBIG     -11   /* graph exceeds the engine's kernel limits (int32
                                    arc / entry indices; no vertex-count cap since
                                    the pending bitmaps spill to HBM past ~655k)   */
#define SHD_PE_ECOMM       -12   /* RCCL communicator missing or failed            */

/* ---- per-entry flags (uint8) ------------------------------------------ */
#define SHD_PE_F_UNREACHABLE 0x01u /* igraph could not reach t: not stored         */
#define SHD_PE_F_NOEDGE      0x02u /* a hop (t==s: the self-loop) has no edge,
                                      topology.c:1490-1495: not stored            */
#define SHD_PE_F_ZEROLAT     0x04u /* latency 0 replaced by 1 (topology.c:1848)    */
#define SHD_PE_F_DIRECT      0x08u /* entry is a direct edge (isDirect=TRUE)       */
#define SHD_PE_F_EXACT       0x10u /* row had equal-distance predecessor ties and
                                      was resolved by the on-GPU igraph-heap kernel */
#define SHD_PE_F_FAILED (SHD_PE_F_UNREACHABLE | SHD_PE_F_NOEDGE)
#define SHD_PE_F_INVALID     0x80u /* batched helpers: vertex id out of range      */

/* ---- graph description (built once by host C from igraph) ------------- */
/* Edges in igraph edge-id order (GraphML document order), endpoints as
 * returned by igraph_edge(); latency/packetLoss are the 'latency' and
 * 'packetloss' edge attributes (EANV).  vertexPacketLoss is the optional
 * vertex 'packetloss' attribute (VANV) or NULL when the attribute is absent;
 * NaN entries mean "value absent" (topology.c:330-349). */
typedef struct ShdPeGraphDesc {
    int32_t nVertices;
    int64_t nEdges;
    int32_t directed;
    const int32_t* edgeFrom;
    const int32_t* edgeTo;
    const double* edgeLatency;
    const double* edgePacketLoss;
    const double* vertexPacketLoss;
} ShdPeGraphDesc;

/* ---- engine options ---------------------------------------------------- */
#define SHD_PE_DEBUG_ENV      0x1  /* read SHDPE_* tuning variables (never in Shadow) */
#define SHD_PE_DEBUG_COUNTERS 0x2  /* per-launch kernel counters on stderr          */

typedef struct ShdPeOptions {
    int32_t device;          /* first HIP device ordinal                          */
    int32_t batchRows;       /* reserved, 0                                       */
    double delta;            /* delta-stepping bucket width (ms); 0 = auto        */
    int32_t storePred;       /* keep a predecessor-vertex column in the table      */
    int32_t forceMode;       /* 0 auto, 1 sparse delta-stepping, 2 direct gather,
                                3 exact igraph-heap kernel for every row (tests),
                                4 dense blocked min-plus,
                                5 batched multi-source delta-stepping             */
    int32_t nDevices;        /* row shards in this engine, one per device; 0 = 1 */
    const int32_t* devices;  /* NULL: device, device+1, ...; else nDevices ordinals
                                (a repeated ordinal = several logical shards on
                                one device, e.g. to test sharding on one GPU)    */
    int32_t shardIndex;      /* multi-process: this engine's index ...            */
    int32_t shardCount;      /* ... among shardCount engines (0 or 1: all rows)   */
    int32_t debugFlags;      /* SHD_PE_DEBUG_*                                    */
} ShdPeOptions;

typedef struct ShdPe ShdPe;

/* Engine statistics (cumulative since create / reset). */
typedef struct ShdPeStats {
    int64_t rowsComputed;
    int64_t rowsExact;         /* rows resolved by the exact igraph-heap kernel   */
    int64_t arcsRelaxed;       /* sum over rows of m_arcs (frozen metric formula) */
    double msSparseKernel;     /* device time of the delta-stepping kernel        */
    double msExactKernel;      /* device time of the exact (tie) kernel           */
    double msDirectKernel;     /* device time of the direct-gather kernel         */
    double msTotal;            /* device time of whole compute calls              */
    int64_t launchesSparse, launchesExact, launchesDirect;
    int32_t mode;              /* 1 sparse, 2 direct (complete graph), 3 dense     */
    int32_t isComplete;        /* _topology_isComplete() of the graph              */
    int32_t nVertices;
    int64_t nArcs;             /* non-loop arcs (undirected edge = 2 arcs)         */
    int32_t nAttached;
    double deltaUsed;
    double msDenseKernel;      /* device time of the dense min-plus path           */
    int64_t launchesDense;
    int64_t denseSweeps;       /* min-plus sweeps (incl. the confirming one)       */
    double denseFlops;         /* executed min-plus work: 2 per (s,u,v) visited,
                                  sweeps (skipped K chunks excluded) + pred pass */
    int32_t batched;           /* mode 1 runs k_batch_rows (multi-source batches)  */
    int32_t batchLanes;        /* sources per batch (LB) when batched              */
    int32_t nShards;           /* row shards (devices) in this engine              */
    double msGather;           /* device time of shd_pe_gather                     */
    int64_t rowsTieEarly;      /* of rowsExact: early-stop emulation (distances,
                                  parents and the tie threshold exported by the
                                  sparse / batch kernels or, dense path,
                                  k_dense_tie_export; k_tie_write wrote the row) */
    int32_t batchWaves;        /* k_batch_rows variant in use: waves per SIMD (4,
                                  6 or 8; shd_pe_tune picks the faster); with the
                                  split kernels, the relaxation kernel's          */
    int32_t batchPostWaves;    /* split kernels: the post kernel's variant (the
                                  tune times relax and post separately)           */
    int64_t rowsTieRepaired;   /* early-stop tie rows whose exported slot failed the
                                  exact kernel's distance cross-check and were
                                  recomputed by the full emulation (0 when correct) */
    int32_t batchCoop;         /* relax kernel in use: workgroups per batch (>= 2:
                                  the cooperative relax of small shards; 0 plain) */
    int64_t relaxCoopAborts;   /* cooperative relax launches refused or aborted (a
                                  barrier wait ran too long); each round was
                                  recomputed by the plain relax */
} ShdPeStats;

/* Defaults for ShdPeOptions. */
void shd_pe_default_options(ShdPeOptions* opt);

/* Build the engine: validates the graph like _topology_checkGraphEdges
 * (latency > 0, packetloss in [0,1]; topology.c:1041-1124), builds the
 * CSR in igraph incidence order, uploads it, and fixes the target set =
 * attached[] (verticesWithAttachedHosts, topology.c:1525-1543; duplicates
 * removed, first occurrence order kept).  Row/column order of the table is
 * the order of the unique attached vertices. */
int shd_pe_create(const ShdPeGraphDesc* graph, const int32_t* attached,
                  int32_t nAttached, const ShdPeOptions* opt, ShdPe** out);

void shd_pe_destroy(ShdPe* pe);

const char* shd_pe_strerror(int code);

/* _topology_isComplete (topology.c:450-552) on the uploaded graph. */
int shd_pe_is_complete(const ShdPe* pe);

/* Number of unique attached vertices (T) and their order. */
int32_t shd_pe_num_attached(const ShdPe* pe);
int shd_pe_attached(const ShdPe* pe, int32_t* outVertices);

/* Compute all rows this engine owns (eager batch, e.g. on the first cache
 * miss); every local shard on its own device, concurrently. */
int shd_pe_compute_all(ShdPe* pe);

/* Optional, once, before timed or production use: computes the engine's
 * own rows with each k_batch_rows variant (8 / 6 / 4 waves per SIMD; the
 * relax and post kernels are timed separately and each keeps its faster
 * variant; the chosen relax is also timed at 0.8 x the bucket width and
 * keeps the faster width -- stats.deltaUsed) for later calls (the ranking
 * differs between boxes of the same SKU and between shard sizes).  The
 * table is left fully computed; no-op on other paths. */
int shd_pe_tune(ShdPe* pe);

/* Compute rows for the given sources (vertex ids, must be attached). */
int shd_pe_compute_rows(ShdPe* pe, const int32_t* srcVertices, int32_t count);

/* Compute rows by table position (0..T-1), e.g. a shard [start, start+count). */
int shd_pe_compute_positions(ShdPe* pe, int32_t start, int32_t count);

/* Copy the row of source srcVertex (computing it if needed) into caller
 * buffers of T entries in attached order.  Any pointer may be NULL.
 * lat/rel follow _topology_computePathProperties exactly; hops = edges folded
 * (1 for t == s: the self-loop); pred = vertex before t (-1 for t == s,
 * needs storePred); flags = SHD_PE_F_*.  For a complete graph the row holds
 * the direct-edge values (_topology_lookupDirectPath, topology.c:1877-1927). */
int shd_pe_get_row(ShdPe* pe, int32_t srcVertex, double* lat, double* rel,
                   int32_t* hops, int32_t* pred, uint8_t* flags);

/* Bulk copy of table rows by position [start, start+count) into caller
 * buffers laid out row-major (count x T, attached order), same fields and
 * values as shd_pe_get_row; any pointer may be NULL.  Rows not yet computed
 * are computed first.  Buffers from shd_pe_host_alloc (or otherwise
 * page-locked) receive the DMA directly; pageable buffers are filled through
 * the engine's pinned staging buffers (DMA of the next block overlaps the
 * multi-threaded host copy of the current one).  Either way a host row store
 * filled after shd_pe_compute_all (topology.c's cache inserts, :1805-1864)
 * pays one pass at PCIe rate instead of one synchronous transfer per field
 * per row. */
int shd_pe_get_rows(ShdPe* pe, int32_t start, int32_t count, double* lat, double* rel,
                    int32_t* hops, int32_t* pred, uint8_t* flags);

/* The igraph shortest path from srcVertex to dstVertex (both attached) as
 * the vertex sequence [src, ..., dst] in verts (cap entries), *len = its
 * length: what topology.c builds hop by hop into its path string
 * (_topology_computePathProperties :1449, :1502-1503, logged by
 * _topology_computeSourcePaths :1831-1841).  The table keeps only each
 * target's predecessor, so the first call for a source re-runs igraph's
 * Dijkstra for it on the device (the exact 2-wheap emulation, one wave:
 * milliseconds to ~1 s at 10^5 vertices); later calls for the same source
 * are a device walk until the next compute.  src == dst -> [src]; complete
 * graphs -> [src, dst] (_topology_lookupDirectPath).  SHD_PE_ENOTOWNED for a
 * source outside this engine's shard, SHD_PE_EUNREACHABLE, SHD_PE_EINVAL when
 * the path needs more than cap entries. */
int shd_pe_get_path(ShdPe* pe, int32_t srcVertex, int32_t dstVertex, int32_t* verts,
                    int32_t cap, int32_t* len);

/* Page-locked host memory for shd_pe_get_rows destinations (DMA target, no
 * staging copy).  No reference counterpart: Shadow's row buffers are plain
 * g_new allocations (topology.c:1805-1864). */
int shd_pe_host_alloc(int64_t bytes, void** out);
void shd_pe_host_free(void* p);

/* Copy rows [start, start+count) (table positions) of the device table into
 * caller DEVICE buffers (e.g. an RCCL all-gather staging area).  Row-major,
 * T entries per row.  Any pointer may be NULL.  Rows not yet computed are
 * computed first (as shd_pe_get_rows); rows of another engine's shard need
 * shd_pe_gather first (SHD_PE_ENOTOWNED). */
int shd_pe_copy_rows_device(ShdPe* pe, int32_t start, int32_t count,
                            double* dLat, double* dRel, int32_t* dHops,
                            uint8_t* dFlags);

/* ---- multi-GPU ----------------------------------------- */
/* Global row shards G = shardCount * nDevices and their position bounds
 * (G + 1 entries: shard g owns rows [bounds[g], bounds[g+1])). */
int32_t shd_pe_num_shards(const ShdPe* pe);
int shd_pe_shard_bounds(const ShdPe* pe, int32_t* bounds);
/* The plan itself (host only, no GPU): G contiguous blocks of T rows with
 * equal numbers of `unit`-row work units (16 = one k_batch_rows batch). */
int shd_pe_plan_shards(int32_t T, int32_t G, int32_t unit, int32_t* bounds);
/* Rows this engine owns (the union of its shards, contiguous). */
int shd_pe_owned_range(const ShdPe* pe, int32_t* start, int32_t* count);
/* Assemble the whole T x T table on every device of this engine (computing
 * missing owned rows first): RCCL broadcasts (all-gather with per-shard
 * blocks) over xGMI between distinct devices / processes, device copies
 * between logical shards of one device.  Afterwards every row is readable
 * here.  Multi-process engines need shd_pe_comm_init first. */
int shd_pe_gather(ShdPe* pe);
/* Cross-process RCCL communicator, one rank per engine (nDevices == 1,
 * rank = shardIndex, nranks = shardCount): one process makes the id, the
 * host's own channel (MPI, a socket, torch.distributed) hands its bytes to
 * every process, each calls shd_pe_comm_init.  shardCount 1 is accepted (a
 * one-rank communicator: the gather issues the same RCCL calls, an in-place
 * all-gather of the engine's own rows). */
int shd_pe_comm_unique_id(void* out, int32_t bytes);   /* bytes >= 128 */
int shd_pe_comm_init(ShdPe* pe, const void* uniqueId, int32_t bytes);
/* Host-transport assembly, the alternative to shd_pe_gather where RCCL has no
 * communicator (several ranks on one GPU, a host-only channel between nodes):
 * rows [start, start+count) of ANOTHER engine's shard, received in host
 * buffers (T entries per row, attached order; pred needed iff storePred), are
 * written into this engine's full table.  Multi-process engines only
 * (shardCount > 1, nDevices == 1); own rows -> SHD_PE_EINVAL.  Once every
 * foreign row has arrived, all rows read from the full table as after
 * shd_pe_gather. */
int shd_pe_put_rows(ShdPe* pe, int32_t start, int32_t count, const double* lat, const double* rel,
                    const int32_t* hops, const int32_t* pred, const uint8_t* flags);
/* 64-bit fingerprint of each table row [start, start+count) (computed on the
 * device; own rows, or any row after a gather / put_rows): the wrapping sum
 * over entries j and fields f (lat, rel, hops, flags, pred if stored) of
 * splitmix64(bits ^ (j * 0x9e3779b97f4a7c15 + f * 0xd1b54a32d192ed03)), f =
 * 1..5.  Owners fingerprint their rows before an exchange and every rank the
 * assembled table after it.  No reference counterpart. */
int shd_pe_row_checksums(ShdPe* pe, int32_t start, int32_t count, uint64_t* out);

/* The whole-table path-cache fill in one pass: rows 0..T-1 (computed first
 * if needed -- then the host image is prepared on a host thread while the
 * device computes, so the drop-in's cheapest call is this one alone; a
 * sharded engine must be gathered) into an EMPTY row store, with
 * exactly the result of shd_rowstore_store_rows over every row in position
 * order (isComplete from the graph, no prefersDirectPaths adjacency --
 * topology.c:1805-1864 per row).  The device packs the store's triangular
 * row image (shd_rowstore_image_layout: 17 B per unordered pair instead of
 * 34 B of two rows) and one DMA lands it in page-locked memory the store
 * adopts.  rowResult (optional, T entries): each row's store_row result.
 * msOut (optional, 3 entries): ms of compute (if any) overlapped with the
 * host image preparation, device pack, DMA. */
struct ShdRowStore;
int shd_pe_fill_rowstore(ShdPe* pe, struct ShdRowStore* st, int32_t* rowResult, double* msOut);

/* Wait for outstanding device work of this engine. */
int shd_pe_synchronize(ShdPe* pe);

/* Measurement helper (not on the path): achievable HBM bandwidth of this
 * engine's device, a 16-B streaming copy of `bytes` (read + write counted),
 * averaged over `iters` launches on the engine's stream; the best of several
 * copy shapes (cache policy, loads in flight, workgroups per CU).  SURVEY.md §8(d)
 * asks for it beside the spec peak; no reference counterpart. */
int shd_pe_stream_bandwidth(ShdPe* pe, int64_t bytes, int32_t iters, double* gbps);

/* Counters of this engine (all its shards).  Both calls take the engine's
 * compute lock: during a running compute they return once it is done.
 * ShdPeStats only grows at its end (ABI 3 added rowsTieRepaired, batchCoop,
 * relaxCoopAborts): a caller
 * built against another header than the library's passes its own
 * sizeof(ShdPeStats) to shd_pe_get_stats_sized, which copies at most that
 * many bytes (the fields both sides know); shd_pe_stats_size() is the
 * library's size.  shd_pe_get_stats writes the library's whole struct. */
int shd_pe_get_stats(const ShdPe* pe, ShdPeStats* out);
int shd_pe_get_stats_sized(const ShdPe* pe, void* out, int64_t outBytes);
int64_t shd_pe_stats_size(void);
int shd_pe_reset_stats(ShdPe* pe);

/* ---- batched helpers on the device ------------
 * The per-query lookups below, for many queries in one call: inputs and
 * outputs are host arrays of `count` entries (staged through the engine's
 * device in chunks).  Results are bit-identical to the one-query helpers. */

/* _topology_computeShortestPathToSelf (topology.c:1545-1653) per vertex:
 * lat = 2 * w_min, rel = (1 - loss_min)^2 over v's OUT-incident edges (the
 * first strict minimum in igraph incidence order).  flags[i]:
 * 0, SHD_PE_F_NOEDGE (graph has no edges), SHD_PE_F_INVALID (bad id). */
int shd_pe_self_paths(ShdPe* pe, const int32_t* vertices, int32_t count, double* lat,
                      double* rel, uint8_t* flags);
/* _topology_lookupDirectPath (topology.c:1877-1927) per pair (src[i],dst[i]):
 * flags[i] = SHD_PE_F_DIRECT with lat/rel, SHD_PE_F_NOEDGE (lat = rel = 0),
 * or SHD_PE_F_INVALID. */
int shd_pe_direct_paths(ShdPe* pe, const int32_t* src, const int32_t* dst, int64_t count,
                        double* lat, double* rel, uint8_t* flags);
/* _topology_verticesAreAdjacent (topology.c:1248-1264) per pair: out[i] 1 / 0
 * (0 for an invalid id; s == t is adjacent iff s has a self-loop). */
int shd_pe_adjacent_pairs(ShdPe* pe, const int32_t* src, const int32_t* dst, int64_t count,
                          uint8_t* out);
/* _topology_isComplete (topology.c:450-552) evaluated on the device from the
 * resident CSR: *isComplete = 1 / 0 (agrees with shd_pe_is_complete). */
int shd_pe_is_complete_device(ShdPe* pe, int32_t* isComplete);

/* ---- host-side helpers Shadow keeps in C (no GPU work) ----------------- */
/* _topology_lookupDirectPath (topology.c:1877-1927) for one pair. */
int shd_pe_direct_path(const ShdPe* pe, int32_t s, int32_t t, double* lat, double* rel);
/* _topology_computeShortestPathToSelf (topology.c:1545-1653). */
int shd_pe_self_path(const ShdPe* pe, int32_t v, double* lat, double* rel);
/* _topology_verticesAreAdjacent (topology.c:1248-1264): 1, 0. */
int shd_pe_adjacent(const ShdPe* pe, int32_t s, int32_t t);

/* ------------------------------------------------------------------------
 * Path cache as a dense triangular row store,
 * replacing topology.c's GHashTable<src, GHashTable<dst, Path*>>
 * (_topology_getPathFromCache :1284-1305, _topology_shouldStorePath
 * :1307-1336, _topology_storePathInCache :1338-1386, Path path.c:13-38).
 * Keys are vertex indices of attached vertices; one 25-B slot per unordered
 * pair (the store rule never keeps both directions), remembering the
 * direction it was stored under.  Thread safety: get / increment never lock
 * and may run concurrently with each other and with stores; stores
 * serialise internally.  No GPU work; usable without an engine.
 * ---------------------------------------------------------------------- */
typedef struct ShdRowStore ShdRowStore;

int shd_rowstore_new(int32_t nVertices, const int32_t* attached, int32_t nAttached,
                     ShdRowStore** out);
void shd_rowstore_free(ShdRowStore* st);
/* _topology_getPathFromCache(s, d): 1 and the Path fields if an entry was
 * stored under exactly (s, d), else 0. */
int shd_rowstore_get(const ShdRowStore* st, int32_t s, int32_t d, double* lat, double* rel,
                     int32_t* isDirect, uint64_t* packetCount);
/* _topology_storePathInCache: 1 stored, 0 refused by _topology_shouldStorePath
 * (either direction cached; a non-direct path on a complete graph; a
 * non-direct path for an adjacent pair under prefersDirectPaths -- the caller
 * passes isComplete and preferDirectAndAdjacent), < 0 error. */
int shd_rowstore_store(ShdRowStore* st, int32_t s, int32_t d, int32_t isDirect,
                       int32_t isComplete, int32_t preferDirectAndAdjacent, double lat,
                       double rel);
/* One engine row of source s (T entries in attached order, as shd_pe_get_row
 * returns them) through the per-target loop of topology.c:1815-1859.
 * adjacent (optional): adjacent[j] = prefersDirectPaths && (s, attached[j])
 * is an edge.  Returns 1 if every target succeeded, 0 if not, < 0 error. */
int shd_rowstore_store_row(ShdRowStore* st, int32_t s, const double* lat, const double* rel,
                           const uint8_t* flags, int32_t isComplete, const uint8_t* adjacent);
/* The whole-table fill: `count` engine rows at once (row i of source srcs[i]
 * at lat/rel/flags/adjacent + i * ld, ld >= nAttached -- e.g. a block of
 * shd_pe_get_rows output in shd_pe_host_alloc buffers), with exactly the
 * result of shd_rowstore_store_row on srcs[0], srcs[1], ... in order
 * (topology.c:1805-1864 once per row, in the order Shadow's first misses
 * would have asked for them).  Spread over nThreads host threads (<= 0: up
 * to 16) by slot rows, so no two threads touch one row.  rowResult
 * (optional) receives each row's store_row result (1 all success / 0).
 * Returns 0, or < 0 on error. */
int shd_rowstore_store_rows(ShdRowStore* st, const int32_t* srcs, int32_t count,
                            const double* lat, const double* rel, const uint8_t* flags,
                            int64_t ld, int32_t isComplete, const uint8_t* adjacent,
                            int32_t nThreads, int32_t* rowResult);
/* Bulk fill from a row IMAGE (the engine builds it on the device,
 * shd_pe_fill_rowstore): the store's own row layout, every triangular row a
 * (attached ordinal, len T - a) at offsets[a] from shd_rowstore_image_layout
 * (T + 1 entries, 64-B aligned): SHD_ROWSTORE_IMAGE_HEADER bytes the store
 * fills, lat f64[len], rel f64[len], state u8[len] (SHD_ROWSTORE_S_* bits).
 * Slot k of row a is the unordered pair (a, a + k).  adopt_image hands an
 * image to an EMPTY store (SHD_PE_EINVAL otherwise) with its entry count and
 * minimum stored latency; release(ctx, image) frees it with the store. */
#define SHD_ROWSTORE_IMAGE_HEADER 64
#define SHD_ROWSTORE_S_STORED   0x1u
#define SHD_ROWSTORE_S_DIRECT   0x2u
#define SHD_ROWSTORE_S_REVERSED 0x4u   /* stored under (larger, smaller) ordinal */
int shd_rowstore_image_layout(int32_t T, int64_t* offsets);
int shd_rowstore_adopt_image(ShdRowStore* st, void* image, int64_t bytes,
                             void (*release)(void* ctx, void* image), void* ctx, int64_t stored,
                             double minLatency);
/* topology_incrementPathPacketCounter on a cached entry: 0, or -1 if absent. */
int shd_rowstore_increment(ShdRowStore* st, int32_t s, int32_t d);
int64_t shd_rowstore_size(const ShdRowStore* st);
double shd_rowstore_min_latency(const ShdRowStore* st);
int64_t shd_rowstore_memory_bytes(const ShdRowStore* st);

/* Every cached entry, as stored (src, dst in the stored direction), for the
 * teardown dump (_topology_logAllCachedPaths, topology.c:1929-1967, which
 * walks the two-level GHashTable in hash order; here by smaller attached
 * ordinal).  Not safe against concurrent inserts.  Returns the number of
 * entries visited. */
typedef void (*ShdRowStoreVisit)(int32_t src, int32_t dst, double latency, double reliability,
                                 int32_t isDirect, uint64_t packetCount, void* user);
int64_t shd_rowstore_foreach(const ShdRowStore* st, ShdRowStoreVisit visit, void* user);

/* ------------------------------------------------------------------------
 * Host mirror of the topology.c path API (the drop-in seen by worker.c,
 * tcp.c, host.c): _topology_getPathEntry + the two-level path cache, with
 * rows coming from the engine.  Queries are by vertex index; Shadow's
 * Address -> vertex map (topology.c:1388-1405) stays where it is.
 * ---------------------------------------------------------------------- */
typedef struct ShdTopology ShdTopology;

int shd_topology_new(ShdPe* pe, int32_t prefersDirectPaths, ShdTopology** out);
void shd_topology_free(ShdTopology* top);
/* topology_getLatency / getReliability (topology.c:2065-2087): -1 on error. */
double shd_topology_get_latency(ShdTopology* top, int32_t srcV, int32_t dstV);
double shd_topology_get_reliability(ShdTopology* top, int32_t srcV, int32_t dstV);
/* topology_isRoutable (topology.c:2089-2092). */
int shd_topology_is_routable(ShdTopology* top, int32_t srcV, int32_t dstV);
/* topology_incrementPathPacketCounter (topology.c:2053-2063): 0 / -1. */
int shd_topology_increment_path_packet_counter(ShdTopology* top, int32_t srcV, int32_t dstV);
/* Inspect the cache entry stored under (src,dst): 1 present, 0 absent. */
int shd_topology_cached(const ShdTopology* top, int32_t srcV, int32_t dstV,
                        double* lat, double* rel, int32_t* isDirect, int64_t* packetCount);
double shd_topology_min_latency(const ShdTopology* top);
int64_t shd_topology_cache_size(const ShdTopology* top);
int64_t shd_topology_rows_computed(const ShdTopology* top);

/* ------------------------------------------------------------------------
 * GraphML ingestion (host only, no GPU work).  Replaces
 * igraph_read_graph_graphml in _topology_loadGraph (topology.c:371-399) plus
 * the attribute reads the path needs: edge 'latency' (EANV,
 * _topology_extractEdgeWeights topology.c:1212-1246), edge / vertex
 * 'packetloss' (topology.c:402-444, :1442-1462) and the graph string
 * 'preferdirectpaths' (topology.c:769-790, case-insensitive prefix
 * true/yes/1).  `buf` is the (decompressed) GraphML text.  Vertex ids follow
 * <node> order and edge ids <edge> order, as igraph assigns them; a missing or
 * unparsable number is NaN.  Duplicate node ids or an edge naming an unknown
 * node -> SHD_PE_EINVAL. */
typedef struct ShdGraphml ShdGraphml;
int shd_graphml_parse(const char* buf, int64_t len, ShdGraphml** out);
/* Fill a ShdPeGraphDesc whose arrays point into `g` (valid until
 * shd_graphml_free); vertexPacketLoss is NULL when no node 'packetloss' key
 * exists.  Pass it straight to shd_pe_create. */
int shd_graphml_describe(const ShdGraphml* g, ShdPeGraphDesc* desc, int32_t* prefersDirectPaths);
/* The GraphML id string of vertex v (NULL if out of range). */
const char* shd_graphml_vertex_id(const ShdGraphml* g, int32_t v);
void shd_graphml_free(ShdGraphml* g);

#ifdef __cplusplus
}
#endif
#endif

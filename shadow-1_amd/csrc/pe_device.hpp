// pe_device.hpp -- device-side data layout shared by the engine and kernels.
//
// HBM layout (one engine = one device):
//   graph  : CSR of OUT arcs without self-loops, rows sorted by neighbour id
//            (= igraph incidence order); SoA arrays
//            col[i32] lat[f64] rel[f64] (rel = 1.0 - packetloss, topology.c:437).
//            For directed graphs an IN-arc CSR (inCol/inLat/inRel) is kept for
//            the predecessor pass; undirected graphs alias it to the OUT CSR.
//   vertex : vrel[f64] (1 - vertex packetloss, 1.0 when absent/NaN),
//            self-loop latency/rel + hasSelf (the (s,s) hop, topology.c:1469).
//   table  : row-major [T rows][T cols] lat f64 | rel f64 | hops i32 |
//            flags u8 (| pred i32 optional), row/col order = attached[].
//   scratch: one slot per resident workgroup: dist f64, hops i32, rel f64,
//            pred i32 (+ heap key/idx, index2 for the exact kernel).
#pragma once
#include <stdint.h>

namespace shdpe {

// One out-arc, 16 bytes: a single global_load_dwordx4 per arc.
struct alignas(16) Arc {
    double lat;
    int32_t col;
    int32_t pad;
};

// 12-byte packed arc (col, lat as two dwords): one global_load_dwordx3 per
// arc and a single 12-B-per-arc copy of the graph for the sparse kernel's
// relax loop and predecessor pass (smaller L2 footprint than AoS 16 B + SoA).
struct alignas(4) Arc3 {
    int32_t col;
    uint32_t latLo, latHi;
};

struct DevGraph {
    int32_t n;
    int32_t T;                 // unique attached vertices (= targets)
    const int32_t* rowPtr;     // [n+1]
    const int32_t* col;        // [nArcs]
    const double* lat;
    const Arc* arcs;           // [nArcs] AoS copy of (lat, col) (batch kernel)
    const Arc3* arc3;          // [nArcs] packed 12-B (col, lat) for k_sparse_rows
    const double* rel;
    const int32_t* inPtr;      // [n+1] (aliases rowPtr when undirected)
    const int32_t* inCol;
    const double* inLat;
    const double* inRel;
    const int32_t* outToIn;    // out arc u->v  ->  index of that edge in v's IN list
    const double* vrel;        // [n]
    const double* selfLat;     // [n]
    const double* selfRel;     // [n]
    const uint8_t* hasSelf;    // [n]
    const double* selfMinLat;  // [n] the self path's loop (several loops: newest of min latency)
    const double* selfMinRel;  // [n]
    const int32_t* attached;   // [T]
    const uint8_t* isAttached; // [n]
    const uint32_t* heavyBits; // [ceil(n/32)] vertices with degree >= heavyDeg
    const double* flat;        // [nArcs] multigraphs with a slower newest parallel edge
                               // (latFold) only, else null: the newest edge's latency
                               // (path folds, direct paths; `lat` = group minimum)
    const double* srel;        // [nArcs] latFold only: the self path's reliability
    const int32_t* oldId;      // [n] device id -> caller's vertex id (null: identity).
                               // The batched path relabels vertices by degree (rows
                               // keep igraph's incidence order); pred is mapped back
};

// A table holds the contiguous block of rows [rowStart, rowStart + rows) of
// the T x T path table (one device shard, or the whole table); kernels write
// row position r at local row r - rowStart.
struct DevTable {
    double* lat;
    double* rel;
    int32_t* hops;
    int32_t* pred;     // may be null
    uint8_t* flags;
    int64_t T;
    int64_t rowStart;
};

// Engine tuning (defaults in the engine; SHDPE_* environment overrides only
// with SHD_PE_DEBUG_ENV, never in a production build of Shadow).
struct Tuning {
    int spThreads = 512, heavyDeg = 64, layout = -1, wgPerCU = 8, kflags = 0;
    double deltaFactor = 16.0;
    int exactHc = 0, exactPerCU = 0;
    int batch = -1, batchLB = 0, batchGrid = 0, batchOrder = 1, batchWpe = 0;
    int relabel = 1;           // batched path: 1 = device ids by descending degree, 0 = as given
    int batchSplit = 1;        // batched path: relax / post as two kernels (predecessors on demand)
    double batchDeltaFactor = 0.75, batchScratchGB = 64.0;
    double denseMin = 0.25, denseBatchGB = 24.0;
    int densePredMi = 2, denseEpochs = 1;
    int debug = 0, streamWgPerCU = 16;
    int tuneLog = 0;           // print shd_pe_tune's per-variant times (no kernel counters)
    int tieCorrupt = 0;        // tests only: 1 / 2 scale one early-stop slot's exported
                               // distances after the relevance scan (exercises the tie-slot
                               // repair); 3 = k_tie_export treats its first slot as violated
    int batchCoop = 0;         // cooperative relax: K workgroups per batch (>= 2 forces it,
                               // 1 = a shd_pe_tune candidate, 0 = off)
    int batchCoopWpe = 0;      // its variant (8 / 6 / 4 waves; 0 = the one with two
                               // workgroups per CU)
    int coopSpin = 1 << 22;    // its barrier poll limit (tests shrink it to force aborts)
    int failWpe = 0;           // tests only: the relax variant of this wave count flags
                               // every batch failed (a miscompiled variant; shd_pe_tune
                               // must not pick it)
};

struct DevScratch {
    double* dist;      // exact kernel: final distance at pop
    int32_t* hops;
    double* rel;
    int32_t* pred;     // IN-arc index of the chosen predecessor edge, -1 none
    double* heapTail;  // exact kernel: heap positions >= hc, per slot heapStride keys (f64)
                       // then heapStride vertex ids (i32) -- 16 B per entry of stride
    int64_t heapStride;  // heap tail entries per slot
    int32_t* index2;   // exact kernel: 0 never reached, 1 popped, >=2 heap pos+2
    int32_t* queue;    // sparse LAYOUT 3: frontier queues, (stride + hcap) per slot
    double* lfold;     // latFold graphs only (else null): the folded latency label
    int64_t stride;    // elements per slot (>= n)
};

// Batched multi-source kernel (pe_batch.hip): one slot per resident
// workgroup; every per-vertex array is [n][LB] (LB sources of the batch
// side by side, so one arc relaxation serves LB sources with one coalesced
// access).
// Per (vertex, lane) labels of the post kernel, one 16-B record: the label
// walks read a parent's reliability, hop count AND its own parent arc with
// one access instead of three (round 5).
struct alignas(16) BLabel {
    double rel;              // reliability product label (< 0 unresolved)
    unsigned long long ha;   // hop label (low 32 bits, -1 unresolved) | chosen IN-arc << 32
                             // (| TIE_AMB; -1 none)
};

struct BatchScratch {
    unsigned long long* D;   // [slot][nStride][LB] f64 bit patterns (dist)
    BLabel* L;               // [slot][nStride][LB] labels + chosen in-arc
    int32_t* queue;          // [slot][nStride] phase candidate list
    int32_t* next;           // next batch to take (device counter, zeroed per launch)
    int64_t nStride;         // >= n, multiple of 64
    uint32_t* bits;          // [slot][2 * words] pending bitmaps when they exceed LDS (gbits)
    int32_t* flags;          // split kernels: per batch of the round, 1 = phase cap hit
    const double* rowOff;    // [T] per table position: the source's distance to its
                             // batch hub (bucket key offset; null = no offsets)
    // cooperative relax (PART 3 of k_batch_rows): K workgroups of one XCD
    // share a batch; the group state below is zeroed by the host before
    // every launch
    int32_t* coCtl;          // [0..15] workgroups registered per XCD, [16] registered,
                             // [17] abort (a barrier wait ran past coSpin polls)
    int32_t* coBars;         // [group * 32]: one barrier counter per group (own line)
    uint32_t* coPub;         // [group][2][K][nwp] published near bits (two buffers)
    unsigned long long* coPubS;   // [group][2][K][2] published near count | far flag, far min
    int32_t coK;             // members per group (PART 3 only)
    int32_t coSpin;          // barrier poll limit (s_sleep 1 each)
};

struct BatchLaunch {
    int32_t lb;              // sources per batch (8, 16 or 32)
    int32_t threads;         // workgroup size
    int32_t grid;            // resident workgroups (= scratch slots)
    int32_t ldsBytes;
    int32_t wpe;             // waves per SIMD the kernel variant is built for (4 or 8)
    double delta;            // bucket width
    int32_t gbits;           // 1: pending bitmaps in global scratch (n > ~655k vertices)
    int32_t split;           // 1: relax and post as two kernels over rounds of batches
    int32_t coop;            // relax: K >= 2 workgroups (one XCD) per batch, PART 3 kernel
                             // launched cooperatively (all resident); 0 / 1: off
};

// Tie export (pe_batch.hip -> k_exact_rows early stop -> k_tie_write): per
// slot the final distances, the fast-path parents (IN-arc index) with
// TIE_AMB marking entries whose parent the igraph heap decides, and the
// largest tied predecessor distance (the emulation stops past it).
constexpr int32_t TIE_AMB = 1 << 30;
struct TieBuf {
    int32_t cap;             // slots (<= 254: rowAmbig holds 2 + slot)
    int32_t* count;          // device slot counter (reset per launch)
    double* D;               // [cap][n]
    int32_t* P;              // [cap][n]
    double* thr;             // [cap]
    int32_t* H;              // [cap][n] k_tie_write hop labels
    double* R;               // [cap][n] k_tie_write reliability labels
    int64_t n;
    // deferred export (k_batch_rows post kernel -> k_tie_export): per slot
    // {batch within its round, lane, source, round}; `round` = the device
    // word the host sets to the round whose post kernel runs (null: the
    // post kernel exports in line, after a full predecessor pass)
    int32_t* req;            // [cap][4]
    int32_t* round;
};

// per-entry flags (mirror SHD_PE_F_* in include/shd_pathengine.h)
constexpr uint8_t F_UNREACHABLE = 0x01;
constexpr uint8_t F_NOEDGE = 0x02;
constexpr uint8_t F_ZEROLAT = 0x04;
constexpr uint8_t F_DIRECT = 0x08;
constexpr uint8_t F_EXACT = 0x10;
constexpr uint8_t F_INVALID = 0x80;   // batched helpers: vertex id out of range

struct SparseLaunch {
    int32_t threads;     // workgroup size
    int32_t grid;        // persistent workgroups (= scratch slots)
    int32_t ldsBytes;    // dynamic LDS
    int32_t qcap;        // light frontier queue capacity
    int32_t hcap;        // heavy (wave-per-vertex) queue capacity
    int32_t heavyDeg;    // degree threshold for the heavy queue
    int32_t layout;      // 2: dist+hops+rowPtr in LDS, 1: dist in LDS, 0: HBM slot,
                         // 3: dist+pending in LDS only (2 rows/CU), queues in HBM
    double delta;        // bucket width
    int32_t kflags;      // kernel variant bits (tuning): 1 AoS arcs in relax, 2 AoS in pred pass
};

// kernels (pe_kernels.hip); all launched on `stream`.
// rowAmbig[i]: 0 fast path, 1 full heap emulation, 2 + k tie data in slot k
// of *dTie (device copy; null disables the export)
void launch_sparse_rows(const DevGraph& g, const DevTable& tab, const DevScratch& sc,
                        const int32_t* dRows, int32_t nRows, uint8_t* dRowAmbig,
                        const SparseLaunch& cfg, int32_t* dDbg, const TieBuf* dTie,
                        void* stream);
// dSlots (may be null): per exact row its tie slot (-1 = full emulation);
// rows with a slot stop at the slot's threshold and leave their final
// parents in tie.P for launch_tie_write
// hc: heap positions held in LDS (k_exact_rows, n > exact_soa_max_n());
// forceGlobalHeap: k_exact_rows even when the SoA all-LDS kernel would fit
int exact_bits_bytes(int n);
void launch_exact_rows(const DevGraph& g, const DevTable& tab, const DevScratch& sc,
                       const int32_t* dRows, int32_t nRows, int32_t grid, int32_t hc,
                       bool forceGlobalHeap, const int32_t* dSlots, const TieBuf& tie,
                       long long* dXdbg, void* stream);
int exact_soa_max_n();
// tie rows of dense graphs (mode 3): the same emulation with the popped
// vertex's ~n arcs scanned by a whole 1024-thread workgroup; dList: per grid
// slot `stride` entries of exact_dense_list_bytes()
void launch_exact_dense(const DevGraph& g, const DevTable& tab, const DevScratch& sc,
                        const int32_t* dRows, int32_t nRows, int32_t grid, int32_t hc, void* dList,
                        const int32_t* dSlots, const TieBuf& tie, int32_t* dTake, void* stream);
// early-stop tie slots 0 .. nSlots-1 of dense tie rows (undirected graphs):
// distances, in-arc parents (TIE_AMB where the heap decides) and thresholds
// from the min-plus D / P rows dIdx[k] of table positions dPos[k]
void launch_dense_tie_export(const DevGraph& g, const double* D, const int32_t* P, int64_t n,
                             const int32_t* dIdx, const int32_t* dPos, const TieBuf& tie, int32_t nSlots,
                             void* stream);
int exact_dense_list_bytes();
// tie rows whose ambiguous entries lie on no target's path: thr := -1 (the
// exact kernel then keeps the fast-path parents)
void launch_tie_scan(const DevGraph& g, const int32_t* dRows, const int32_t* dSlots,
                     int32_t nRows, const TieBuf& tie, void* stream);
// rows (dRows) with their tie slots (dSlots): hops / reliability along the
// final parents, row writer
void launch_tie_write(const DevGraph& g, const DevTable& tab, const int32_t* dRows,
                      const int32_t* dSlots, int32_t nRows, const TieBuf& tie, void* stream);
void launch_direct_rows(const DevGraph& g, const DevTable& tab, const int32_t* dRows,
                        int32_t nRows, void* stream);
int sparse_max_threads();
// batched multi-source sparse path (pe_batch.hip): batchRows = nBatches*lb
// table positions (-1 pads a short batch); rowAmbig[i] != 0 when entry i's
// row has equal-distance predecessor ties (-> k_exact_rows): 1 = full heap
// emulation, 2 + k = tie data exported to slot k of *dTie (device copy of
// the descriptor; null disables the export).
// igraph path of one row from k_exact_rows' per-vertex IN-arcs (pe_aux.hip)
void launch_path_walk(const DevGraph& g, const int32_t* dP, int32_t s, int32_t t, int32_t* dOut,
                      int32_t cap, int32_t* dLen, int32_t nInArcs, void* stream);
void launch_batch_rows(const DevGraph& g, const DevTable& tab, const BatchScratch& bs,
                       const int32_t* dBatchRows, int32_t nBatches, uint8_t* dRowAmbig,
                       const BatchLaunch& cfg, int32_t* dDbg, const TieBuf* dTie, void* stream,
                       int part = 0);
const void* batch_kernel_ptr(int lb, int wpe, bool gbits, int part = 0);
// cooperative relax (PART 3; LB 8 / 16, LDS bitmaps): 0 launched, -1 refused
// (grid not resident / unsupported shape: run launch_batch_rows part 1)
int launch_batch_relax_coop(const DevGraph& g, const DevTable& tab, const BatchScratch& bs,
                            const int32_t* dBatchRows, int32_t nBatches, uint8_t* dRowAmbig,
                            const BatchLaunch& cfg, int32_t* dDbg, const TieBuf* tie, void* stream);
const void* batch_coop_kernel_ptr(int lb, int wpe);
int batch_lds_bytes(int n, int wpe, bool gbits);
// Deferred tie export of one round (after its post kernel): for every slot
// the post kernel requested in round `round`, the tie data of the lane's row
// -- every vertex's distance, its igraph parent (first tight in-arc of
// minimum dist[u], TIE_AMB on equal minima or a zero-increment arc) and the
// tie threshold -- from the round's persisted distance array, over the whole
// GPU; a Bellman violation sends the row to the full emulation (rowAmbig 1;
// violSlot >= 0: tests, that slot's row is treated as violated).
void launch_tie_export(const DevGraph& g, const BatchScratch& bs, int lb, const TieBuf& tie,
                       int round, uint8_t* dRowAmbig, int grid, int violSlot, void* stream);
int batch_threads(int wpe);    // workgroup size of a variant (6 waves: 768, else 1024)
int64_t batch_bits_words(int n);   // per slot, both bitmaps
// batched helpers (pe_aux.hip), all on `stream`
void launch_self_paths(const DevGraph& g, const int32_t* dVerts, int32_t count, int64_t nEdges,
                       double* dLat, double* dRel, uint8_t* dFlags, void* stream);
// mode 0 direct paths (lat, rel, flags), mode 1 adjacency (flags = 0 / 1)
void launch_pairs(const DevGraph& g, const int32_t* dSrc, const int32_t* dDst, int64_t count,
                  int mode, double* dLat, double* dRel, uint8_t* dFlags, void* stream);
void launch_incident_min(const DevGraph& g, const int32_t* dEdgeCount, int32_t* dOut, void* stream);
// path-cache image of the whole table (rows 0..T-1 of `tab`, rowStart 0) in
// the row store's layout (dOff: shd_rowstore_image_layout); dAcc[0] += stored
// entries, dAcc[1] = min stored latency bits (init INF_BITS)
void launch_pack_rowstore(const DevTable& tab, const int64_t* dOff, uint8_t* dImg,
                          unsigned long long* dAcc, void* stream);
// per table row: 1 = no F_NOEDGE target (isAllSuccess of topology.c:1815-1859)
void launch_rows_all_success(const DevTable& tab, int32_t* dOut, void* stream);
// 64-bit fingerprint per table row (local rows firstLocal .. + rows), pe_aux.hip
void launch_row_checksums(const DevTable& tab, int64_t firstLocal, int32_t rows, uint64_t* dOut,
                          void* stream);
// dense path (pe_dense.hip)
void launch_dense_build(const DevGraph& g, double* W, double* Rl, int64_t n, int64_t nArcs,
                        void* stream);
int launch_dense_rows(const DevGraph& g, const DevTable& tab, const double* W, const double* Rl,
                      double* D, int32_t* P, uint8_t* rowActive, uint8_t* rowChanged,
                      uint8_t* rowAmb, int32_t* dAny, uint8_t* chunkEpoch, const int32_t* dRows,
                      int32_t nRows, int64_t n, const Tuning& tu, void* stream, int* sweepsOut,
                      double* flopsOut);

}  // namespace shdpe

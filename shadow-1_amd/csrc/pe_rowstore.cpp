// pe_rowstore.cpp -- the path cache of topology.c as a dense triangular row
// store.
//
// Reference: _topology_getPathFromCache :1284-1305, _topology_shouldStorePath
// :1307-1336, _topology_storePathInCache :1338-1386, Path (path.c:13-38): a
// GHashTable<src, GHashTable<dst, Path*>> under one rwlock, ~100 B and two
// hash probes per entry.
//
// The store rule never keeps both (s,d) and (d,s) (shouldStorePath checks both
// directions), so one slot per UNORDERED pair of attached ordinals suffices:
// row a (the smaller ordinal) holds pairs {a, b >= a}, T - a slots, allocated
// on first insert.  A slot is lat f64 | rel f64 | packets u64 | state u8 with
// state bits STORED, DIRECT and REVERSED (stored under (larger, smaller)), so
// a lookup of (s,d) hits only the direction that was stored, exactly like
// the reference's two-level table.  25 B per unordered pair: C4 (T = 16k)
// 3.4 GB, C5 (T = 64k) 54 GB of host RAM at most, versus ~100 B per ordered
// pair in GHashTables.
//
// Concurrency: readers never lock.  A slot is published by a release store
// of its state byte after lat/rel are written, rows by a release store of
// the row pointer; readers load both with acquire.  Inserts serialise on one
// mutex (the reference's writer lock); packet counters are relaxed atomic
// increments.
#include <atomic>
#include <cstdint>
#include <cstring>
#include <memory>
#include <mutex>
#include <new>
#include <vector>

#include "shd_pathengine.h"

namespace {

constexpr uint8_t S_STORED = 1, S_DIRECT = 2, S_REVERSED = 4;

struct TriRow {
    std::unique_ptr<double[]> lat, rel;
    std::unique_ptr<std::atomic<uint64_t>[]> packets;
    std::unique_ptr<std::atomic<uint8_t>[]> state;
    explicit TriRow(size_t len)
        : lat(new double[len]), rel(new double[len]), packets(new std::atomic<uint64_t>[len]),
          state(new std::atomic<uint8_t>[len]) {
        for (size_t i = 0; i < len; ++i) {
            packets[i].store(0, std::memory_order_relaxed);
            state[i].store(0, std::memory_order_relaxed);
        }
    }
};

}  // namespace

struct ShdRowStore {
    int32_t n = 0, T = 0;
    std::vector<int32_t> posOf;                          // vertex -> attached ordinal or -1
    std::vector<int32_t> attached;                       // ordinal -> vertex
    std::unique_ptr<std::atomic<TriRow*>[]> rows;        // by smaller ordinal
    std::atomic<int64_t> size{0};
    std::atomic<double> minLatency{0.0};
    std::atomic<int64_t> bytes{0};
    std::mutex writer;
    ~ShdRowStore() {
        if (rows)
            for (int32_t a = 0; a < T; ++a) delete rows[a].load(std::memory_order_relaxed);
    }
};

namespace {

struct Slot {
    TriRow* row;
    int32_t k;
    uint8_t dirBit;      // S_REVERSED when the looked-up key is (larger, smaller)
};

inline bool slot_of(const ShdRowStore* st, int32_t s, int32_t d, Slot* out) {
    if (s < 0 || s >= st->n || d < 0 || d >= st->n) return false;
    const int32_t ps = st->posOf[s], pd = st->posOf[d];
    if (ps < 0 || pd < 0) return false;
    const int32_t a = ps < pd ? ps : pd, b = ps < pd ? pd : ps;
    out->row = st->rows[a].load(std::memory_order_acquire);
    out->k = b - a;
    out->dirBit = ps > pd ? S_REVERSED : 0;
    return true;
}

// _topology_getPathFromCache(s, d): the entry stored under exactly (s, d)
inline bool lookup(const ShdRowStore* st, int32_t s, int32_t d, TriRow** row, int32_t* k) {
    Slot sl;
    if (!slot_of(st, s, d, &sl) || !sl.row) return false;
    const uint8_t x = sl.row->state[sl.k].load(std::memory_order_acquire);
    if (!(x & S_STORED)) return false;
    if (s != d && (x & S_REVERSED) != sl.dirBit) return false;
    *row = sl.row;
    *k = sl.k;
    return true;
}

}  // namespace

extern "C" int shd_rowstore_new(int32_t nVertices, const int32_t* attached, int32_t T,
                                ShdRowStore** out) {
    if (!out || nVertices <= 0 || T < 0 || (T > 0 && !attached)) return SHD_PE_EINVAL;
    ShdRowStore* st = new (std::nothrow) ShdRowStore();
    if (!st) return SHD_PE_ENOMEM;
    st->n = nVertices;
    st->T = T;
    st->posOf.assign(nVertices, -1);
    st->attached.assign(attached, attached + T);
    for (int32_t j = 0; j < T; ++j) {
        const int32_t v = attached[j];
        if (v < 0 || v >= nVertices || st->posOf[v] >= 0) { delete st; return SHD_PE_EINVAL; }
        st->posOf[v] = j;
    }
    st->rows.reset(new (std::nothrow) std::atomic<TriRow*>[T > 0 ? T : 1]);
    if (!st->rows) { delete st; return SHD_PE_ENOMEM; }
    for (int32_t a = 0; a < T; ++a) st->rows[a].store(nullptr, std::memory_order_relaxed);
    *out = st;
    return SHD_PE_OK;
}

extern "C" void shd_rowstore_free(ShdRowStore* st) { delete st; }

extern "C" int shd_rowstore_get(const ShdRowStore* st, int32_t s, int32_t d, double* lat,
                                double* rel, int32_t* isDirect, uint64_t* packetCount) {
    if (!st) return 0;
    TriRow* r;
    int32_t k;
    if (!lookup(st, s, d, &r, &k)) return 0;
    if (lat) *lat = r->lat[k];
    if (rel) *rel = r->rel[k];
    if (isDirect) *isDirect = (r->state[k].load(std::memory_order_relaxed) & S_DIRECT) ? 1 : 0;
    if (packetCount) *packetCount = r->packets[k].load(std::memory_order_relaxed);
    return 1;
}

extern "C" int shd_rowstore_increment(ShdRowStore* st, int32_t s, int32_t d) {
    if (!st) return -1;
    TriRow* r;
    int32_t k;
    if (!lookup(st, s, d, &r, &k)) return -1;
    r->packets[k].fetch_add(1, std::memory_order_relaxed);
    return 0;
}

// _topology_shouldStorePath + _topology_storePathInCache; the caller passes
// the graph facts the rule needs.  Caller holds st->writer.
static int store_locked(ShdRowStore* st, int32_t s, int32_t d, int32_t isDirect,
                        int32_t isComplete, int32_t preferDirectAndAdjacent, double lat,
                        double rel) {
    Slot sl;
    if (!slot_of(st, s, d, &sl)) return SHD_PE_ENOTATTACHED;
    if (sl.row) {
        const uint8_t x = sl.row->state[sl.k].load(std::memory_order_relaxed);
        if (x & S_STORED) return 0;            // (s,d) or (d,s) already cached (:1312-1318)
    }
    if (isComplete && !isDirect) return 0;     // :1321-1323
    if (preferDirectAndAdjacent && !isDirect) return 0;   // :1325-1332
    if (!sl.row) {
        const int32_t ps = st->posOf[s], pd = st->posOf[d];
        const int32_t a = ps < pd ? ps : pd;
        TriRow* r = new (std::nothrow) TriRow((size_t)(st->T - a));
        if (!r) return SHD_PE_ENOMEM;
        st->rows[a].store(r, std::memory_order_release);
        st->bytes.fetch_add((int64_t)(st->T - a) * 25, std::memory_order_relaxed);
        sl.row = r;
    }
    sl.row->lat[sl.k] = lat;
    sl.row->rel[sl.k] = rel;
    sl.row->packets[sl.k].store(0, std::memory_order_relaxed);
    sl.row->state[sl.k].store((uint8_t)(S_STORED | (isDirect ? S_DIRECT : 0) |
                                        (s != d ? sl.dirBit : 0)),
                              std::memory_order_release);
    st->size.fetch_add(1, std::memory_order_relaxed);
    const double m = st->minLatency.load(std::memory_order_relaxed);
    if (m == 0 || lat < m) st->minLatency.store(lat, std::memory_order_relaxed);   // :1375-1378
    return 1;
}

extern "C" int shd_rowstore_store(ShdRowStore* st, int32_t s, int32_t d, int32_t isDirect,
                                  int32_t isComplete, int32_t preferDirectAndAdjacent,
                                  double lat, double rel) {
    if (!st) return SHD_PE_EINVAL;
    std::lock_guard<std::mutex> lk(st->writer);
    return store_locked(st, s, d, isDirect, isComplete, preferDirectAndAdjacent, lat, rel);
}

// One engine row of source s (attached order), the per-target loop of
// topology.c:1815-1859: unreachable targets skipped (isAllSuccess kept),
// failed folds (SHD_PE_F_NOEDGE) skipped and clear it, the rest stored
// non-direct.  adjacent[j] (optional, with prefersDirectPaths) = (s,
// attached[j]) is an edge.  Returns 1 all success, 0 not, < 0 error.
extern "C" int shd_rowstore_store_row(ShdRowStore* st, int32_t s, const double* lat,
                                      const double* rel, const uint8_t* flags, int32_t isComplete,
                                      const uint8_t* adjacent) {
    if (!st || !lat || !rel || !flags) return SHD_PE_EINVAL;
    if (s < 0 || s >= st->n || st->posOf[s] < 0) return SHD_PE_ENOTATTACHED;
    std::lock_guard<std::mutex> lk(st->writer);
    int all = 1;
    const int32_t* att = st->attached.data();
    for (int32_t j = 0; j < st->T; ++j) {
        if (flags[j] & SHD_PE_F_UNREACHABLE) continue;
        if (flags[j] & SHD_PE_F_NOEDGE) { all = 0; continue; }
        const int rc = store_locked(st, s, att[j], 0, isComplete, adjacent ? adjacent[j] : 0,
                                    lat[j], rel[j]);
        if (rc < 0) return rc;
    }
    return all;
}

extern "C" int64_t shd_rowstore_size(const ShdRowStore* st) {
    return st ? st->size.load(std::memory_order_relaxed) : 0;
}

extern "C" double shd_rowstore_min_latency(const ShdRowStore* st) {
    return st ? st->minLatency.load(std::memory_order_relaxed) : 0.0;
}

extern "C" int64_t shd_rowstore_memory_bytes(const ShdRowStore* st) {
    return st ? st->bytes.load(std::memory_order_relaxed) + (int64_t)st->T * 8 +
                    (int64_t)st->n * 4
              : 0;
}

extern "C" int64_t shd_rowstore_foreach(const ShdRowStore* st, ShdRowStoreVisit visit, void* user) {
    if (!st || !visit) return 0;
    int64_t cnt = 0;
    for (int32_t a = 0; a < st->T; ++a) {
        const TriRow* r = st->rows[a].load(std::memory_order_acquire);
        if (!r) continue;
        for (int32_t k = 0; a + k < st->T; ++k) {
            const uint8_t x = r->state[k].load(std::memory_order_acquire);
            if (!(x & S_STORED)) continue;
            const int32_t va = st->attached[a], vb = st->attached[a + k];
            const bool rev = (x & S_REVERSED) != 0;     // stored under (larger, smaller)
            visit(rev ? vb : va, rev ? va : vb, r->lat[k], r->rel[k], (x & S_DIRECT) ? 1 : 0,
                  r->packets[k].load(std::memory_order_relaxed), user);
            ++cnt;
        }
    }
    return cnt;
}

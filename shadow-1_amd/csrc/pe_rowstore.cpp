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
// on first insert.  A slot is lat f64 | rel f64 | state u8 with state bits
// STORED, DIRECT and REVERSED (stored under (larger, smaller)), so a lookup
// of (s,d) hits only the direction that was stored, exactly like the
// reference's two-level table; a row's u64 packet counters appear with its
// first increment.  17 B per unordered pair (+ 8 once counted): C4 (T = 16k)
// 2.3 GB, C5 (T = 64k) 37 GB of host RAM at most, versus ~100 B per ordered
// pair in GHashTables.  Rows come from huge-page arenas.
//
// Concurrency: readers never lock.  A slot is published by a release store
// of its state byte after lat/rel are written, rows (and a row's counter
// array) by a release store / CAS of the pointer; readers load them with
// acquire.  Inserts serialise on one mutex (the reference's writer lock), a
// bulk fill (shd_rowstore_store_rows) splits the rows among its threads
// under it; packet counters are relaxed atomic increments.
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdlib>
#include <cstdint>
#include <cstring>
#include <memory>
#include <mutex>
#include <new>
#include <sys/mman.h>
#include <thread>
#include <vector>

#include "shd_pathengine.h"

namespace {

constexpr uint8_t S_STORED = SHD_ROWSTORE_S_STORED, S_DIRECT = SHD_ROWSTORE_S_DIRECT,
                  S_REVERSED = SHD_ROWSTORE_S_REVERSED;

// One triangular row: lat | rel | state, carved from an arena; the packet
// counters (u64 per slot) are allocated on the row's first increment -- the
// table fill never touches them.
struct TriRow {
    double* lat;
    double* rel;
    std::atomic<uint8_t>* state;
    std::atomic<std::atomic<uint64_t>*> packets;
    size_t len;
};

// Row memory: zero-filled anonymous mappings of >= 64 MiB with transparent
// huge pages requested (a C4 table is 3.4 GB of rows: 4-KiB page faults
// alone cost seconds), rows carved in order and released with the store.
// One arena per writer (the insert mutex, or one per thread of a bulk fill).
struct Arena {
    std::vector<std::pair<char*, size_t>> maps;
    char* cur = nullptr;
    size_t left = 0;
    void* take(size_t bytes) {
        bytes = (bytes + 63) & ~(size_t)63;
        if (bytes > left) {
            const size_t sz = std::max<size_t>((size_t)64 << 20, (bytes + ((2u << 20) - 1)) & ~(((size_t)2 << 20) - 1));
            void* m = mmap(nullptr, sz, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
            if (m == MAP_FAILED) return nullptr;
            (void)madvise(m, sz, MADV_HUGEPAGE);
            maps.emplace_back(static_cast<char*>(m), sz);
            cur = static_cast<char*>(m);
            left = sz;
        }
        void* r = cur;
        cur += bytes;
        left -= bytes;
        return r;
    }
    void absorb(Arena& o) {
        maps.insert(maps.end(), o.maps.begin(), o.maps.end());
        o.maps.clear();
        o.cur = nullptr;
        o.left = 0;
    }
    ~Arena() { for (auto& m : maps) munmap(m.first, m.second); }
};

TriRow* make_row(Arena& ar, size_t len) {
    static_assert(sizeof(std::atomic<uint64_t>) == 8 && sizeof(std::atomic<uint8_t>) == 1, "");
    static_assert(sizeof(TriRow) <= 64, "");
    char* p = static_cast<char*>(ar.take(64 + len * 17));
    if (!p) return nullptr;
    TriRow* r = new (p) TriRow();
    p += 64;
    r->lat = reinterpret_cast<double*>(p);
    r->rel = reinterpret_cast<double*>(p + len * 8);
    r->state = reinterpret_cast<std::atomic<uint8_t>*>(p + len * 16);
    r->packets.store(nullptr, std::memory_order_relaxed);
    r->len = len;
    return r;
}

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
    Arena arena;                                         // rows (freed with the store)
    // adopted row images (shd_rowstore_adopt_image), released with the store
    std::vector<std::pair<void*, std::pair<void (*)(void*, void*), void*>>> images;
    ~ShdRowStore() {
        if (rows)
            for (int32_t a = 0; a < T; ++a)
                if (TriRow* r = rows[a].load(std::memory_order_relaxed))
                    std::free(r->packets.load(std::memory_order_relaxed));
        for (auto& im : images) im.second.first(im.second.second, im.first);
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
    if (packetCount) {
        const std::atomic<uint64_t>* pk = r->packets.load(std::memory_order_acquire);
        *packetCount = pk ? pk[k].load(std::memory_order_relaxed) : 0;
    }
    return 1;
}

extern "C" int shd_rowstore_increment(ShdRowStore* st, int32_t s, int32_t d) {
    if (!st) return -1;
    TriRow* r;
    int32_t k;
    if (!lookup(st, s, d, &r, &k)) return -1;
    std::atomic<uint64_t>* pk = r->packets.load(std::memory_order_acquire);
    if (!pk) {   // first increment in this row: publish a zeroed counter array
        auto* fresh = static_cast<std::atomic<uint64_t>*>(std::calloc(r->len, 8));
        if (!fresh) return -1;
        if (r->packets.compare_exchange_strong(pk, fresh, std::memory_order_acq_rel,
                                               std::memory_order_acquire)) {
            pk = fresh;
            st->bytes.fetch_add((int64_t)r->len * 8, std::memory_order_relaxed);
        } else {
            std::free(fresh);     // another thread published first: pk holds its array
        }
    }
    pk[k].fetch_add(1, std::memory_order_relaxed);
    return 0;
}

// _topology_shouldStorePath + _topology_storePathInCache for the pair of
// attached ordinals (ps, pd), source first.  The caller owns row min(ps, pd)
// for writing (the writer mutex, or the row's thread in a bulk store) and
// accounts size / minLatency itself.  1 stored, 0 refused, < 0 error.
static inline int store_ord(ShdRowStore* st, Arena& ar, int32_t ps, int32_t pd, int32_t isDirect,
                            int32_t isComplete, int32_t preferDirectAndAdjacent, double lat,
                            double rel) {
    const int32_t a = ps < pd ? ps : pd, k = (ps < pd ? pd : ps) - a;
    TriRow* row = st->rows[a].load(std::memory_order_relaxed);
    if (row && (row->state[k].load(std::memory_order_relaxed) & S_STORED))
        return 0;                              // (s,d) or (d,s) already cached (:1312-1318)
    if (isComplete && !isDirect) return 0;     // :1321-1323
    if (preferDirectAndAdjacent && !isDirect) return 0;   // :1325-1332
    if (!row) {
        row = make_row(ar, (size_t)(st->T - a));
        if (!row) return SHD_PE_ENOMEM;
        st->rows[a].store(row, std::memory_order_release);
        st->bytes.fetch_add((int64_t)(st->T - a) * 17, std::memory_order_relaxed);
    }
    row->lat[k] = lat;
    row->rel[k] = rel;
    row->state[k].store((uint8_t)(S_STORED | (isDirect ? S_DIRECT : 0) | (ps > pd ? S_REVERSED : 0)),
                        std::memory_order_release);
    return 1;
}

// the minimum-latency tracker of :1375-1378, one stored latency at a time
static inline void track_min(ShdRowStore* st, double lat) {
    const double m = st->minLatency.load(std::memory_order_relaxed);
    if (m == 0 || lat < m) st->minLatency.store(lat, std::memory_order_relaxed);
}

extern "C" int shd_rowstore_store(ShdRowStore* st, int32_t s, int32_t d, int32_t isDirect,
                                  int32_t isComplete, int32_t preferDirectAndAdjacent,
                                  double lat, double rel) {
    if (!st) return SHD_PE_EINVAL;
    if (s < 0 || s >= st->n || d < 0 || d >= st->n) return SHD_PE_ENOTATTACHED;
    const int32_t ps = st->posOf[s], pd = st->posOf[d];
    if (ps < 0 || pd < 0) return SHD_PE_ENOTATTACHED;
    std::lock_guard<std::mutex> lk(st->writer);
    const int rc = store_ord(st, st->arena, ps, pd, isDirect, isComplete, preferDirectAndAdjacent, lat, rel);
    if (rc == 1) {
        st->size.fetch_add(1, std::memory_order_relaxed);
        track_min(st, lat);
    }
    return rc;
}

// One engine row of source s (attached order), the per-target loop of
// topology.c:1815-1859: unreachable targets skipped (isAllSuccess kept),
// failed folds (SHD_PE_F_NOEDGE) skipped and clear it, the rest stored
// non-direct.  adjacent[j] (optional, with prefersDirectPaths) = (s,
// attached[j]) is an edge.  Returns 1 all success, 0 not, < 0 error.
// Target j of the row IS attached ordinal j, so no vertex lookups.
static int store_row_locked(ShdRowStore* st, int32_t ps, const double* lat, const double* rel,
                            const uint8_t* flags, int32_t isComplete, const uint8_t* adjacent) {
    int all = 1;
    int64_t added = 0;
    int rc = 0;
    for (int32_t j = 0; j < st->T; ++j) {
        if (flags[j] & SHD_PE_F_UNREACHABLE) continue;
        if (flags[j] & SHD_PE_F_NOEDGE) { all = 0; continue; }
        rc = store_ord(st, st->arena, ps, j, 0, isComplete, adjacent ? adjacent[j] : 0, lat[j], rel[j]);
        if (rc < 0) break;
        if (rc == 1) { ++added; track_min(st, lat[j]); }
    }
    st->size.fetch_add(added, std::memory_order_relaxed);
    return rc < 0 ? rc : all;
}

extern "C" int shd_rowstore_store_row(ShdRowStore* st, int32_t s, const double* lat,
                                      const double* rel, const uint8_t* flags, int32_t isComplete,
                                      const uint8_t* adjacent) {
    if (!st || !lat || !rel || !flags) return SHD_PE_EINVAL;
    if (s < 0 || s >= st->n || st->posOf[s] < 0) return SHD_PE_ENOTATTACHED;
    std::lock_guard<std::mutex> lk(st->writer);
    return store_row_locked(st, st->posOf[s], lat, rel, flags, isComplete, adjacent);
}

// Many rows at once (the whole-table fill after shd_pe_compute_all), with the
// exact result of calling shd_rowstore_store_row on srcs[0], srcs[1], ... in
// that order.  The triangular rows are split among the threads by equal slot
// counts; every thread walks all the source rows in order and applies only
// the pairs whose slot row it owns, so each slot sees its candidates in the
// sequential order and no two threads write one row.  The minimum latency
// is order-dependent only through its 0 sentinel (:1375): inputs that would
// store a latency <= 0 (never an engine row: latencies are > 0 and a 0 sum
// becomes 1, :1848) take the sequential path.
extern "C" int shd_rowstore_store_rows(ShdRowStore* st, const int32_t* srcs, int32_t count,
                                       const double* lat, const double* rel, const uint8_t* flags,
                                       int64_t ld, int32_t isComplete, const uint8_t* adjacent,
                                       int32_t nThreads, int32_t* rowResult) {
    if (!st || count < 0 || (count > 0 && (!srcs || !lat || !rel || !flags)) || ld < st->T)
        return SHD_PE_EINVAL;
    const int32_t T = st->T;
    std::vector<int32_t> ps(count);
    for (int32_t i = 0; i < count; ++i) {
        if (srcs[i] < 0 || srcs[i] >= st->n || st->posOf[srcs[i]] < 0) return SHD_PE_ENOTATTACHED;
        ps[i] = st->posOf[srcs[i]];
    }
    const unsigned hc = std::thread::hardware_concurrency();
    // default: up to 16 threads (the GPU box's CPU share), none for tiny tables
    int nt = nThreads > 0 ? std::min(nThreads, std::max(1, T))
                          : std::max(1, std::min<int>({16, hc ? (int)hc : 1, std::max(1, T / 256)}));
    std::lock_guard<std::mutex> lk(st->writer);
    // row results + the latency check, by source row
    std::vector<uint8_t> zero(nt, 0);
    auto scan = [&](int t) {
        for (int32_t i = t; i < count; i += nt) {
            const double* L = lat + (size_t)i * ld;
            const uint8_t* F = flags + (size_t)i * ld;
            int all = 1;
            for (int32_t j = 0; j < T; ++j) {
                if (F[j] & SHD_PE_F_UNREACHABLE) continue;
                if (F[j] & SHD_PE_F_NOEDGE) { all = 0; continue; }
                if (!(L[j] > 0.0)) zero[t] = 1;
            }
            if (rowResult) rowResult[i] = all;
        }
    };
    {
        std::vector<std::thread> th;
        for (int t = 1; t < nt; ++t) th.emplace_back(scan, t);
        scan(0);
        for (auto& x : th) x.join();
    }
    bool seq = false;
    for (uint8_t z : zero) seq = seq || z;
    if (seq || nt == 1) {
        for (int32_t i = 0; i < count; ++i) {
            const size_t o = (size_t)i * ld;
            const int rc = store_row_locked(st, ps[i], lat + o, rel + o, flags + o, isComplete,
                                            adjacent ? adjacent + o : nullptr);
            if (rc < 0) return rc;
        }
        return SHD_PE_OK;
    }
    // slot-row ownership, balanced for THIS call's work: row r gets one put
    // per source p > r (target r, slot p - r) plus the T - r puts of its own
    // row when r is a source itself
    std::vector<int32_t> rb(nt + 1, T);
    {
        std::vector<int64_t> w(T + 1, 0);
        for (int32_t i = 0; i < count; ++i) w[ps[i]] += T - ps[i];   // own row segment
        std::vector<int32_t> atLeast(T + 1, 0);   // sources with ordinal p, suffix-summed below
        for (int32_t i = 0; i < count; ++i) atLeast[ps[i]]++;
        int64_t greater = 0, total = 0;
        for (int32_t r = T - 1; r >= 0; --r) {     // sources with p > r
            w[r] += greater;
            greater += atLeast[r];
            total += w[r];
        }
        int64_t cum = 0;
        int t = 1;
        rb[0] = 0;
        for (int32_t r = 0; r < T && t < nt; ++r) {
            cum += w[r];
            while (t < nt && (double)cum >= (double)total * t / nt) rb[t++] = r + 1;
        }
    }
    struct Acc { int64_t added = 0; double mn = INFINITY; int err = 0; Arena ar; };
    std::vector<Acc> acc(nt);
    // Each slot row a is one thread's.  A thread takes its rows in tiles of
    // RT; per tile the sources go in order, a source p offering slot p - r of
    // every tile row r < p (target r: RT consecutive input columns) and, when
    // p is in the tile, its own row segment.  Every slot sees its candidates
    // in the sequential order; inputs are read along their rows (a column
    // walk over a block of rows costs a TLB miss per element).
    constexpr int32_t RT = 64;
    auto work = [&](int t) {
        const int32_t lo = rb[t], hi = rb[t + 1];
        Acc& A = acc[t];
        auto put = [&](int32_t p, int32_t j, size_t o) {
            if (flags[o + j] & (SHD_PE_F_UNREACHABLE | SHD_PE_F_NOEDGE)) return true;
            const int rc = store_ord(st, A.ar, p, j, 0, isComplete, adjacent ? adjacent[o + j] : 0,
                                     lat[o + j], rel[o + j]);
            if (rc < 0) { A.err = rc; return false; }
            if (rc == 1) { ++A.added; A.mn = lat[o + j] < A.mn ? lat[o + j] : A.mn; }
            return true;
        };
        for (int32_t r0 = lo; r0 < hi && !A.err; r0 += RT) {
            const int32_t r1 = std::min(hi, r0 + RT);
            for (int32_t i = 0; i < count && !A.err; ++i) {
                const int32_t p = ps[i];
                const size_t o = (size_t)i * ld;
                const int32_t re = std::min(r1, p);
                for (int32_t r = r0; r < re; ++r)
                    if (!put(p, r, o)) break;
                if (p >= r0 && p < r1)
                    for (int32_t j = p; j < T; ++j)
                        if (!put(p, j, o)) break;
            }
        }
    };
    {
        std::vector<std::thread> th;
        for (int t = 1; t < nt; ++t) th.emplace_back(work, t);
        work(0);
        for (auto& x : th) x.join();
    }
    for (Acc& A : acc) st->arena.absorb(A.ar);
    int64_t added = 0;
    double mn = INFINITY;
    int err = 0;
    for (const Acc& A : acc) {
        added += A.added;
        mn = std::min(mn, A.mn);
        if (A.err && !err) err = A.err;
    }
    st->size.fetch_add(added, std::memory_order_relaxed);
    if (added) track_min(st, mn);          // every stored latency is > 0 here
    return err ? err : SHD_PE_OK;
}

// Row image (SHD_ROWSTORE_IMAGE_*): every triangular row a (len T - a) at
// offsets[a], 64-B aligned: a 64-B header the store fills (the TriRow),
// lat f64[len], rel f64[len], state u8[len] -- the layout make_row carves
// from an arena, so an adopted image IS the store's rows.
extern "C" int shd_rowstore_image_layout(int32_t T, int64_t* offsets) {
    static_assert(sizeof(TriRow) <= SHD_ROWSTORE_IMAGE_HEADER, "");
    if (T < 0 || !offsets) return SHD_PE_EINVAL;
    int64_t o = 0;
    for (int32_t a = 0; a < T; ++a) {
        offsets[a] = o;
        o += (SHD_ROWSTORE_IMAGE_HEADER + 17 * (int64_t)(T - a) + 63) & ~(int64_t)63;
    }
    offsets[T] = o;
    return SHD_PE_OK;
}

extern "C" int shd_rowstore_adopt_image(ShdRowStore* st, void* image, int64_t bytes,
                                        void (*release)(void* ctx, void* image), void* ctx,
                                        int64_t stored, double minLatency) {
    if (!st || !image || !release || stored < 0) return SHD_PE_EINVAL;
    std::lock_guard<std::mutex> lk(st->writer);
    if (st->size.load(std::memory_order_relaxed) != 0) return SHD_PE_EINVAL;
    for (int32_t a = 0; a < st->T; ++a)
        if (st->rows[a].load(std::memory_order_relaxed)) return SHD_PE_EINVAL;
    std::vector<int64_t> off((size_t)st->T + 1);
    shd_rowstore_image_layout(st->T, off.data());
    if (bytes < off[st->T]) return SHD_PE_EINVAL;
    char* base = static_cast<char*>(image);
    for (int32_t a = 0; a < st->T; ++a) {
        char* p = base + off[a];
        const size_t len = (size_t)(st->T - a);
        TriRow* r = new (p) TriRow();
        p += SHD_ROWSTORE_IMAGE_HEADER;
        r->lat = reinterpret_cast<double*>(p);
        r->rel = reinterpret_cast<double*>(p + len * 8);
        r->state = reinterpret_cast<std::atomic<uint8_t>*>(p + len * 16);
        r->packets.store(nullptr, std::memory_order_relaxed);
        r->len = len;
        st->rows[a].store(r, std::memory_order_release);
    }
    st->images.push_back({image, {release, ctx}});
    st->bytes.fetch_add(off[st->T], std::memory_order_relaxed);
    st->size.store(stored, std::memory_order_relaxed);
    if (stored) track_min(st, minLatency);
    return SHD_PE_OK;
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
        const std::atomic<uint64_t>* pk = r->packets.load(std::memory_order_acquire);
        for (int32_t k = 0; a + k < st->T; ++k) {
            const uint8_t x = r->state[k].load(std::memory_order_acquire);
            if (!(x & S_STORED)) continue;
            const int32_t va = st->attached[a], vb = st->attached[a + k];
            const bool rev = (x & S_REVERSED) != 0;     // stored under (larger, smaller)
            visit(rev ? vb : va, rev ? va : vb, r->lat[k], r->rel[k], (x & S_DIRECT) ? 1 : 0,
                  pk ? pk[k].load(std::memory_order_relaxed) : 0, user);
            ++cnt;
        }
    }
    return cnt;
}

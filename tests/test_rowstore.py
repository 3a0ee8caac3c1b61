"""shd_rowstore_* (pe_rowstore.cpp): topology.c's two-level path cache
(_topology_getPathFromCache :1284-1305, _topology_shouldStorePath
:1307-1336, _topology_storePathInCache :1338-1386) as a triangular dense
store.  Checked here (CPU, no device) against a literal dict model of the
reference's GHashTable<src, GHashTable<dst, Path*>>, and under concurrent
readers."""
import threading

import numpy as np
import pytest

from shdpe.engine import RowStore, F_NOEDGE, F_UNREACHABLE


class RefCache:
    """The reference cache, restated with dicts (topology.c:1284-1386)."""

    def __init__(self):
        self.c = {}
        self.min_lat = 0.0

    def get(self, s, d):
        return self.c.get(s, {}).get(d)

    def should_store(self, is_direct, s, d, is_complete, adjacent_pref):
        if self.get(s, d) is not None or self.get(d, s) is not None:
            return False
        if is_complete and not is_direct:
            return False
        if adjacent_pref and not is_direct:
            return False
        return True

    def store(self, s, d, is_direct, is_complete, adjacent_pref, lat, rel):
        if not self.should_store(is_direct, s, d, is_complete, adjacent_pref):
            return 0
        self.c.setdefault(s, {})[d] = [lat, rel, bool(is_direct), 0]
        if self.min_lat == 0 or lat < self.min_lat:
            self.min_lat = lat
        return 1


def _attached(n, k, seed):
    rng = np.random.default_rng(seed)
    return np.sort(rng.choice(n, size=k, replace=False)).astype(np.int32)


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_store_get_semantics_match_reference_cache(seed):
    n, k = 300, 120
    att = _attached(n, k, seed)
    st, ref = RowStore(n, att), RefCache()
    rng = np.random.default_rng(seed)
    for _ in range(6000):
        s, d = (int(x) for x in rng.choice(att, 2))
        if rng.random() < 0.1:
            d = s
        is_direct = bool(rng.random() < 0.2)
        is_complete = bool(rng.random() < 0.05)
        adj = bool(rng.random() < 0.1)
        lat, rel = float(rng.uniform(1, 100)), float(rng.uniform(0.9, 1))
        assert st.store(s, d, is_direct, is_complete, adj, lat, rel) == \
            ref.store(s, d, is_direct, is_complete, adj, lat, rel)
        if rng.random() < 0.3:
            a, b = (int(x) for x in rng.choice(att, 2))
            e = ref.get(a, b)
            if e is not None:
                e[3] += 1
            assert st.increment(a, b) == (0 if e is not None else -1)
    for s in att:
        for d in att:
            e, g = ref.get(int(s), int(d)), st.get(s, d)
            assert (e is None) == (g is None), (s, d)
            if e is not None:
                assert g == tuple(e)
    assert st.size() == sum(len(v) for v in ref.c.values())
    assert st.min_latency() == ref.min_lat
    # the teardown dump (_topology_logAllCachedPaths, topology.c:1929-1967):
    # every cached entry once, under the direction it was stored in
    items = st.items()
    assert len(items) == st.size()
    want = {(s, d): tuple(e) for s, row in ref.c.items() for d, e in row.items()}
    got = {(s, d): (lat, rel, bool(isd), pc) for s, d, lat, rel, isd, pc in items}
    assert got == want
    # one slot per unordered pair at most, allocated per touched row
    assert st.memory_bytes() <= (k * (k + 1) // 2) * 25 + k * 8 + n * 4


def test_unattached_and_invalid_ids():
    st = RowStore(10, np.array([1, 3, 5], np.int32))
    assert st.get(0, 1) is None and st.get(-1, 3) is None and st.get(3, 99) is None
    assert st.increment(1, 2) == -1
    with pytest.raises(Exception):
        st.store(1, 2, 0, 0, 0, 1.0, 1.0)
    assert st.store(1, 3, 0, 0, 0, 2.0, 0.5) == 1
    assert st.get(1, 3) == (2.0, 0.5, False, 0) and st.get(3, 1) is None
    assert st.store(3, 1, 1, 0, 0, 9.0, 0.1) == 0          # reverse direction cached
    with pytest.raises(Exception):
        RowStore(10, np.array([1, 1], np.int32))            # duplicate attached vertex


def test_store_row_follows_row_loop():
    """topology.c:1815-1859 over one engine row: unreachable skipped, failed
    fold skipped + isAllSuccess cleared, adjacency under prefersDirectPaths."""
    att = np.array([2, 4, 6, 8], np.int32)
    st, ref = RowStore(10, att), RefCache()
    lat = np.array([1.0, 2.0, 3.0, 4.0])
    rel = np.array([0.9, 0.8, 0.7, 0.6])
    flags = np.array([0, F_UNREACHABLE, 0, 0], np.uint8)
    adj = np.array([0, 0, 1, 0], np.uint8)
    assert st.store_row(4, lat, rel, flags, False, adj) is True
    for j, t in enumerate(att):
        if not flags[j]:
            ref.store(4, int(t), False, False, bool(adj[j]), lat[j], rel[j])
    for t in att:
        e, g = ref.get(4, int(t)), st.get(4, t)
        assert (e is None) == (g is None) and (e is None or g == tuple(e))
    flags2 = np.array([0, 0, F_NOEDGE, 0], np.uint8)
    assert st.store_row(8, lat, rel, flags2) is False
    assert st.store_row(2, lat, rel, np.zeros(4, np.uint8), True) is True   # complete: nothing
    assert st.get(2, 6) is None


def test_concurrent_readers_and_writer():
    """8 reader threads probe and count packets while a writer inserts rows;
    every value a reader sees is the one stored, counters add up."""
    n, k = 2000, 400
    att = _attached(n, k, 7)
    st = RowStore(n, att)
    rng = np.random.default_rng(7)
    lat = rng.uniform(1, 100, size=(k, k))
    rel = rng.uniform(0.5, 1, size=(k, k))
    stop = threading.Event()
    errors, incs = [], [0] * 8

    def reader(i):
        r = np.random.default_rng(100 + i)
        while not stop.is_set():
            a, b = (int(x) for x in r.integers(0, k, 2))
            g = st.get(att[a], att[b])
            if g is not None:
                if g[0] not in (lat[a, b], lat[b, a]) or g[1] not in (rel[a, b], rel[b, a]):
                    errors.append((a, b, g))
                if st.increment(att[a], att[b]) == 0:
                    incs[i] += 1

    th = [threading.Thread(target=reader, args=(i,)) for i in range(8)]
    for t in th:
        t.start()
    for a in range(k):
        st.store_row(att[a], lat[a], rel[a], np.zeros(k, np.uint8))
    stop.set()
    for t in th:
        t.join()
    assert not errors
    assert st.size() == k * (k + 1) // 2
    total = 0
    for a in range(k):
        for b in range(a, k):
            g = st.get(att[a], att[b])
            assert g is not None and g[0] == lat[a, b] and g[1] == rel[a, b]
            total += g[3]
    assert total == sum(incs)


def test_rowstore_under_thread_sanitizer(tmp_path):
    """pe_rowstore.cpp built with -fsanitize=thread (host code), readers racing
    a writer: no data race reported, counters and values consistent."""
    import os
    import shutil
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    gxx = shutil.which("g++")
    if gxx is None:
        pytest.skip("no g++")
    exe = str(tmp_path / "rowstore_race")
    cmd = [gxx, "-std=c++17", "-O1", "-g", "-fsanitize=thread", "-pthread",
           "-I", os.path.join(root, "include"),
           os.path.join(root, "tests", "native", "rowstore_race.cpp"),
           os.path.join(root, "shadow-1_amd", "csrc", "pe_rowstore.cpp"), "-o", exe]
    b = subprocess.run(cmd, capture_output=True, text=True)
    if b.returncode != 0 and "tsan" in (b.stderr or "").lower():
        pytest.skip("ThreadSanitizer runtime unavailable")
    assert b.returncode == 0, b.stderr[-2000:]
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 exitcode=66")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0 and "OK" in r.stdout, (r.stdout, r.stderr[-3000:])


@pytest.mark.parametrize("threads", [1, 3, 8])
def test_store_rows_equals_sequential_store_row(threads):
    """shd_rowstore_store_rows (the whole-table fill, threads by slot rows)
    leaves exactly what store_row over the same sources in the same order
    does: first stored direction wins, unreachable / failed targets, complete
    and prefersDirectPaths refusals, per-row isAllSuccess, min latency."""
    n, k = 500, 97
    att = _attached(n, k, 11)
    rng = np.random.default_rng(threads)
    order = rng.permutation(k)
    order = np.concatenate([order, order[:10]])         # repeated sources: nothing new
    srcs = att[order]
    lat = rng.uniform(1, 100, size=(srcs.shape[0], k + 3))   # ld > T
    rel = rng.uniform(0.5, 1, size=lat.shape)
    flags = np.zeros(lat.shape, np.uint8)
    flags[rng.random(lat.shape) < 0.03] = F_UNREACHABLE
    flags[rng.random(lat.shape) < 0.01] = F_NOEDGE
    adj = (rng.random(lat.shape) < 0.05).astype(np.uint8)
    for is_complete, use_adj in ((False, False), (False, True), (True, False)):
        a, b = RowStore(n, att), RowStore(n, att)
        a.store(int(att[5]), int(att[9]), 1, 0, 0, 0.5, 0.25)   # a prior direct entry
        b.store(int(att[5]), int(att[9]), 1, 0, 0, 0.5, 0.25)
        A = adj if use_adj else None
        want = [a.store_row(int(s), lat[i], rel[i], flags[i], is_complete,
                            None if A is None else A[i]) for i, s in enumerate(srcs)]
        got = b.store_rows(srcs, lat, rel, flags, is_complete, A, threads=threads)
        assert [bool(x) for x in got] == want
        assert a.size() == b.size() and a.min_latency() == b.min_latency()
        assert sorted(a.items()) == sorted(b.items())


def test_store_rows_rejects_bad_buffers():
    att = np.arange(0, 40, 2, dtype=np.int32)
    st = RowStore(40, att)
    lat = np.ones((3, 20)); rel = np.ones((3, 20)); fl = np.zeros((3, 20), np.uint8)
    with pytest.raises(ValueError):
        st.store_rows(att[:4], lat, rel, fl)                 # 4 rows, buffers hold 3
    with pytest.raises(ValueError):
        st.store_rows(att[:3], lat[:, :10], rel[:, :10], fl[:, :10])   # rows shorter than T
    with pytest.raises(ValueError):
        st.store_rows(att[:3], lat.astype(np.float32), rel, fl)
    with pytest.raises(Exception):
        st.store_rows(np.array([1, 2, 3], np.int32), lat, rel, fl)    # 1 is not attached


def pack_image_model(lat, rel, flags):
    """The row image shd_pe_fill_rowstore's k_pack_rowstore builds (pe_aux.hip),
    restated in numpy from the whole T x T table: slot (a, a+k) = row a's
    entry a+k if that fold succeeded, else row a+k's entry a stored under the
    reversed key, else empty -- shd_rowstore_store_rows over rows 0..T-1."""
    import ctypes as C
    from shdpe.engine import load_library
    T = lat.shape[0]
    off = np.empty(T + 1, np.int64)
    assert load_library().shd_rowstore_image_layout(T, off.ctypes.data_as(C.c_void_p)) == 0
    img = np.zeros(int(off[T]), np.uint8)
    ok = (flags & (F_UNREACHABLE | F_NOEDGE)) == 0
    stored, mn = 0, np.inf
    for a in range(T):
        n = T - a
        b = np.arange(a, T)
        fwd = ok[a, b]
        rev = ~fwd & (b > a) & ok[b, a]
        L = np.where(fwd, lat[a, b], np.where(rev, lat[b, a], 0.0))
        R = np.where(fwd, rel[a, b], np.where(rev, rel[b, a], 0.0))
        S = np.where(fwd, 1, np.where(rev, 1 | 4, 0)).astype(np.uint8)
        o = int(off[a]) + 64
        img[o:o + 8 * n] = L.view(np.uint8)
        img[o + 8 * n:o + 16 * n] = R.view(np.uint8)
        img[o + 16 * n:o + 17 * n] = S
        stored += int((S != 0).sum())
        if (S != 0).any():
            mn = min(mn, float(L[S != 0].min()))
    return img, stored, (0.0 if stored == 0 else mn)


def _random_table(T, seed, directed):
    rng = np.random.default_rng(seed)
    lat = rng.uniform(0.5, 50.0, (T, T))
    rel = rng.uniform(0.9, 1.0, (T, T))
    flags = np.zeros((T, T), np.uint8)
    flags[rng.random((T, T)) < 0.08] = F_UNREACHABLE
    if not directed:
        flags = np.maximum(flags, flags.T)
    d = rng.random(T) < 0.3
    flags[d, d] = F_NOEDGE                              # missing (s, s) self-loops
    return lat, rel, flags


@pytest.mark.parametrize("directed", [False, True])
def test_adopted_image_equals_store_rows(directed):
    """An image in the store's row layout (shd_rowstore_image_layout), built by
    the pack rule shd_pe_fill_rowstore's kernel implements, adopted by an
    empty store (shd_rowstore_adopt_image) answers every lookup, the size,
    the minimum latency and the entry walk exactly as shd_rowstore_store_rows
    over all rows in position order -- the layout and rule the GPU fill
    relies on, pinned on the CPU."""
    import ctypes as C
    T, n = 70, 90
    att = _attached(n, T, seed=3)
    lat, rel, flags = _random_table(T, 11 + int(directed), directed)
    ref = RowStore(n, att)
    ref.store_rows(att, lat, rel, flags)
    img, stored, mn = pack_image_model(lat, rel, flags)
    st = RowStore(n, att)
    lib = st._lib if hasattr(st, "_lib") else None
    from shdpe.engine import load_library
    lib = load_library()
    REL = C.CFUNCTYPE(None, C.c_void_p, C.c_void_p)
    keep = REL(lambda ctx, p: None)                     # the test owns the buffer
    rc = lib.shd_rowstore_adopt_image(st.h, img.ctypes.data_as(C.c_void_p), img.nbytes,
                                      C.cast(keep, C.c_void_p), None, stored, mn)
    assert rc == 0
    assert st.size() == ref.size() == stored
    assert st.min_latency() == ref.min_latency()
    assert sorted(st.items()) == sorted(ref.items())
    for s in att[::7]:
        for d in att[::5]:
            assert st.get(int(s), int(d)) == ref.get(int(s), int(d)), (s, d)
    # a second image, or one into a store with entries, is refused
    assert lib.shd_rowstore_adopt_image(st.h, img.ctypes.data_as(C.c_void_p), img.nbytes,
                                        C.cast(keep, C.c_void_p), None, stored, mn) != 0
    assert lib.shd_rowstore_adopt_image(ref.h, img.ctypes.data_as(C.c_void_p), img.nbytes,
                                        C.cast(keep, C.c_void_p), None, stored, mn) != 0
    # the adopted rows take packet counters like any other
    s, d = next((int(a), int(b)) for a in att for b in att if st.get(int(a), int(b)) is not None)
    assert st.increment(s, d) == 0 and st.get(s, d)[3] == 1
    st.close()
    ref.close()

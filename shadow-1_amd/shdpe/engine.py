"""ctypes binding of libshdpe.so (include/shd_pathengine.h).

This is plumbing for tests and bench.py: every entry point goes straight to
the C-ABI library built from shadow-1_amd/csrc (HIP kernels for gfx950).
There is no Python/CPU compute path -- if the library or a gfx950 device is
missing, loading / creating the engine raises.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))   # shadow-1_amd/
LIB_PATH = os.path.join(_PKG, "libshdpe.so")

OK, EINVAL, ENOMEM, ENODEV, EUNREACHABLE, ENOSELFLOOP, EMULTI, EHIP, ENOTATTACHED, ENOEDGE = (
    0, -1, -2, -3, -4, -5, -6, -7, -8, -9)
ENOTOWNED, ETOOBIG, ECOMM = -10, -11, -12
DEBUG_ENV, DEBUG_COUNTERS = 0x1, 0x2
F_UNREACHABLE, F_NOEDGE, F_ZEROLAT, F_DIRECT, F_EXACT = 0x01, 0x02, 0x04, 0x08, 0x10
F_FAILED = F_UNREACHABLE | F_NOEDGE
F_INVALID = 0x80

EXPORTS = [
    "shd_pe_default_options", "shd_pe_create", "shd_pe_destroy", "shd_pe_strerror",
    "shd_pe_is_complete", "shd_pe_num_attached", "shd_pe_attached", "shd_pe_compute_all",
    "shd_pe_compute_rows", "shd_pe_compute_positions", "shd_pe_get_row", "shd_pe_get_rows",
    "shd_pe_copy_rows_device", "shd_pe_synchronize", "shd_pe_get_stats", "shd_pe_reset_stats",
    "shd_pe_get_stats_sized", "shd_pe_stats_size",
    "shd_pe_stream_bandwidth", "shd_pe_num_shards", "shd_pe_shard_bounds", "shd_pe_plan_shards", "shd_pe_owned_range",
    "shd_pe_gather", "shd_pe_comm_unique_id", "shd_pe_comm_init",
    "shd_pe_direct_path", "shd_pe_self_path", "shd_pe_adjacent", "shd_pe_self_paths",
    "shd_pe_direct_paths", "shd_pe_adjacent_pairs", "shd_pe_is_complete_device", "shd_topology_new",
    "shd_topology_free", "shd_topology_get_latency", "shd_topology_get_reliability",
    "shd_topology_is_routable", "shd_topology_increment_path_packet_counter",
    "shd_topology_cached", "shd_topology_min_latency", "shd_topology_cache_size",
    "shd_topology_rows_computed", "shd_graphml_parse", "shd_graphml_describe",
    "shd_graphml_vertex_id", "shd_graphml_free", "shd_rowstore_new", "shd_rowstore_free",
    "shd_rowstore_get", "shd_rowstore_store", "shd_rowstore_store_row", "shd_rowstore_increment",
    "shd_rowstore_size", "shd_rowstore_min_latency", "shd_rowstore_memory_bytes",
    "shd_pe_host_alloc", "shd_pe_host_free", "shd_pe_tune", "shd_pe_get_path",
    "shd_rowstore_foreach", "shd_rowstore_store_rows", "shd_pe_put_rows", "shd_pe_row_checksums",
    "shd_rowstore_image_layout", "shd_rowstore_adopt_image", "shd_pe_fill_rowstore",
]


class GraphDesc(C.Structure):
    _fields_ = [("nVertices", C.c_int32), ("nEdges", C.c_int64), ("directed", C.c_int32),
                ("edgeFrom", C.c_void_p), ("edgeTo", C.c_void_p), ("edgeLatency", C.c_void_p),
                ("edgePacketLoss", C.c_void_p), ("vertexPacketLoss", C.c_void_p)]


class Options(C.Structure):
    _fields_ = [("device", C.c_int32), ("batchRows", C.c_int32), ("delta", C.c_double),
                ("storePred", C.c_int32), ("forceMode", C.c_int32), ("nDevices", C.c_int32),
                ("devices", C.c_void_p), ("shardIndex", C.c_int32), ("shardCount", C.c_int32),
                ("debugFlags", C.c_int32)]


class Stats(C.Structure):
    _fields_ = [("rowsComputed", C.c_int64), ("rowsExact", C.c_int64),
                ("arcsRelaxed", C.c_int64), ("msSparseKernel", C.c_double),
                ("msExactKernel", C.c_double), ("msDirectKernel", C.c_double),
                ("msTotal", C.c_double), ("launchesSparse", C.c_int64),
                ("launchesExact", C.c_int64), ("launchesDirect", C.c_int64),
                ("mode", C.c_int32), ("isComplete", C.c_int32), ("nVertices", C.c_int32),
                ("nArcs", C.c_int64), ("nAttached", C.c_int32), ("deltaUsed", C.c_double),
                ("msDenseKernel", C.c_double), ("launchesDense", C.c_int64),
                ("denseSweeps", C.c_int64), ("denseFlops", C.c_double),
                ("batched", C.c_int32), ("batchLanes", C.c_int32), ("nShards", C.c_int32),
                ("msGather", C.c_double), ("rowsTieEarly", C.c_int64), ("batchWaves", C.c_int32),
                ("batchPostWaves", C.c_int32), ("rowsTieRepaired", C.c_int64),
                ("batchCoop", C.c_int32), ("relaxCoopAborts", C.c_int64)]


class EngineError(RuntimeError):
    def __init__(self, code, what):
        super().__init__(f"{what}: {strerror(code)} ({code})")
        self.code = code


_lib = None


def load_library(path: str = LIB_PATH):
    """Load libshdpe.so; raises if it has not been built (no fallback).
    SHDPE_LIB names another build of the same library (same-box A/B runs)."""
    global _lib
    if _lib is not None:
        return _lib
    path = os.environ.get("SHDPE_LIB") or path
    if not os.path.exists(path):
        raise RuntimeError(f"libshdpe.so not built at {path}: run "
                           "`python -c 'import __graft_entry__ as g; g.build()'` (or make -C shadow-1_amd)")
    lib = C.CDLL(path)
    vp, i32, i64, f64 = C.c_void_p, C.c_int32, C.c_int64, C.c_double
    sig = {
        "shd_pe_default_options": (None, [vp]),
        "shd_pe_create": (C.c_int, [vp, vp, i32, vp, vp]),
        "shd_pe_destroy": (None, [vp]),
        "shd_pe_strerror": (C.c_char_p, [C.c_int]),
        "shd_pe_is_complete": (C.c_int, [vp]),
        "shd_pe_num_attached": (i32, [vp]),
        "shd_pe_attached": (C.c_int, [vp, vp]),
        "shd_pe_compute_all": (C.c_int, [vp]),
        "shd_pe_compute_rows": (C.c_int, [vp, vp, i32]),
        "shd_pe_compute_positions": (C.c_int, [vp, i32, i32]),
        "shd_pe_get_row": (C.c_int, [vp, i32, vp, vp, vp, vp, vp]),
        "shd_pe_get_rows": (C.c_int, [vp, i32, i32, vp, vp, vp, vp, vp]),
        "shd_pe_copy_rows_device": (C.c_int, [vp, i32, i32, vp, vp, vp, vp]),
        "shd_pe_synchronize": (C.c_int, [vp]),
        "shd_pe_get_stats": (C.c_int, [vp, vp]),
        "shd_pe_get_stats_sized": (C.c_int, [vp, vp, C.c_int64]),
        "shd_pe_stats_size": (C.c_int64, []),
        "shd_pe_reset_stats": (C.c_int, [vp]),
        "shd_pe_stream_bandwidth": (C.c_int, [vp, i64, i32, vp]),
        "shd_pe_num_shards": (i32, [vp]),
        "shd_pe_shard_bounds": (C.c_int, [vp, vp]),
        "shd_pe_plan_shards": (C.c_int, [i32, i32, i32, vp]),
        "shd_pe_owned_range": (C.c_int, [vp, vp, vp]),
        "shd_pe_gather": (C.c_int, [vp]),
        "shd_pe_comm_unique_id": (C.c_int, [vp, i32]),
        "shd_pe_comm_init": (C.c_int, [vp, vp, i32]),
        "shd_pe_direct_path": (C.c_int, [vp, i32, i32, vp, vp]),
        "shd_pe_self_path": (C.c_int, [vp, i32, vp, vp]),
        "shd_pe_adjacent": (C.c_int, [vp, i32, i32]),
        "shd_pe_self_paths": (C.c_int, [vp, vp, i32, vp, vp, vp]),
        "shd_pe_direct_paths": (C.c_int, [vp, vp, vp, i64, vp, vp, vp]),
        "shd_pe_adjacent_pairs": (C.c_int, [vp, vp, vp, i64, vp]),
        "shd_pe_is_complete_device": (C.c_int, [vp, vp]),
        "shd_topology_new": (C.c_int, [vp, i32, vp]),
        "shd_topology_free": (None, [vp]),
        "shd_topology_get_latency": (f64, [vp, i32, i32]),
        "shd_topology_get_reliability": (f64, [vp, i32, i32]),
        "shd_topology_is_routable": (C.c_int, [vp, i32, i32]),
        "shd_topology_increment_path_packet_counter": (C.c_int, [vp, i32, i32]),
        "shd_topology_cached": (C.c_int, [vp, i32, i32, vp, vp, vp, vp]),
        "shd_topology_min_latency": (f64, [vp]),
        "shd_topology_cache_size": (i64, [vp]),
        "shd_topology_rows_computed": (i64, [vp]),
        "shd_graphml_parse": (C.c_int, [C.c_char_p, i64, vp]),
        "shd_graphml_describe": (C.c_int, [vp, vp, vp]),
        "shd_graphml_vertex_id": (C.c_char_p, [vp, i32]),
        "shd_graphml_free": (None, [vp]),
        "shd_rowstore_new": (C.c_int, [i32, vp, i32, vp]),
        "shd_rowstore_free": (None, [vp]),
        "shd_rowstore_get": (C.c_int, [vp, i32, i32, vp, vp, vp, vp]),
        "shd_rowstore_store": (C.c_int, [vp, i32, i32, i32, i32, i32, f64, f64]),
        "shd_rowstore_store_row": (C.c_int, [vp, i32, vp, vp, vp, i32, vp]),
        "shd_rowstore_increment": (C.c_int, [vp, i32, i32]),
        "shd_rowstore_size": (i64, [vp]),
        "shd_rowstore_min_latency": (f64, [vp]),
        "shd_rowstore_memory_bytes": (i64, [vp]),
        "shd_pe_host_alloc": (C.c_int, [i64, vp]),
        "shd_pe_host_free": (None, [vp]),
        "shd_pe_tune": (C.c_int, [vp]),
        "shd_pe_get_path": (C.c_int, [vp, i32, i32, vp, i32, vp]),
        "shd_rowstore_foreach": (i64, [vp, vp, vp]),
        "shd_rowstore_store_rows": (C.c_int, [vp, vp, i32, vp, vp, vp, i64, i32, vp, i32, vp]),
        "shd_pe_put_rows": (C.c_int, [vp, i32, i32, vp, vp, vp, vp, vp]),
        "shd_pe_row_checksums": (C.c_int, [vp, i32, i32, vp]),
        "shd_rowstore_image_layout": (C.c_int, [i32, vp]),
        "shd_rowstore_adopt_image": (C.c_int, [vp, vp, i64, vp, vp, i64, f64]),
        "shd_pe_fill_rowstore": (C.c_int, [vp, vp, vp, vp]),
    }
    # ABI-3 additions: an older build loaded through SHDPE_LIB (same-box A/B)
    # lacks them; the in-tree library must have every symbol
    optional = {"shd_pe_get_stats_sized", "shd_pe_stats_size"} if os.environ.get("SHDPE_LIB") else set()
    for name, (res, args) in sig.items():
        if name in optional and not hasattr(lib, name):
            continue
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def plan_shards(T: int, G: int, unit: int = 1) -> np.ndarray:
    """shd_pe_plan_shards: the engine's row-shard bounds (host only)."""
    b = np.empty(G + 1, np.int32)
    rc = load_library().shd_pe_plan_shards(int(T), int(G), int(unit), _p(b))
    if rc:
        raise EngineError(rc, "shd_pe_plan_shards")
    return b


class _PinnedBuf:
    """Owner of one shd_pe_host_alloc block (freed with the last array view)."""

    def __init__(self, lib, nbytes):
        self.lib, self.p = lib, C.c_void_p()
        rc = lib.shd_pe_host_alloc(int(nbytes), C.byref(self.p))
        if rc:
            raise EngineError(rc, "shd_pe_host_alloc")

    def __del__(self):
        if self.p:
            self.lib.shd_pe_host_free(self.p)
            self.p = C.c_void_p()


def _pinned_array(shape, dtype, lib):
    nbytes = int(np.prod(shape)) * np.dtype(dtype).itemsize
    buf = _PinnedBuf(lib, max(1, nbytes))
    raw = (C.c_char * max(1, nbytes)).from_address(buf.p.value)
    raw._owner = buf                         # keep the block alive with the array
    return np.frombuffer(raw, dtype=dtype, count=int(np.prod(shape))).reshape(shape)


def kernel_source_hash() -> str:
    """sha256 (first 16 hex digits) of the device-code sources libshdpe.so is
    built from (csrc/*.hip, *.hpp): identifies the measured kernels in
    profiles/traffic_<wl>.json so bench.py drops a stale traffic figure."""
    import glob
    import hashlib
    h = hashlib.sha256()
    csrc = os.path.join(_PKG, "csrc")
    for f in sorted(glob.glob(os.path.join(csrc, "*.hip")) + glob.glob(os.path.join(csrc, "*.hpp"))):
        h.update(os.path.basename(f).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


_CK_K, _CK_C = np.uint64(0x9E3779B97F4A7C15), np.uint64(0xD1B54A32D192ED03)


def _mix64(z):
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def row_checksums_host(rows: dict) -> np.ndarray:
    """numpy twin of shd_pe_row_checksums (k_row_checksums, pe_aux.hip) over
    rows as get_rows returns them (count x T per field): per row the wrapping
    sum over entries j and fields f of splitmix64(bits ^ (j*K + f*C))."""
    lat = np.atleast_2d(rows["lat"])
    count, T = lat.shape
    kj = np.arange(T, dtype=np.uint64) * _CK_K
    fields = [(rows["lat"], 1), (rows["rel"], 2), (rows["hops"], 3), (rows["flags"], 4)]
    if rows.get("pred") is not None:
        fields.append((rows["pred"], 5))
    out = np.zeros(count, np.uint64)
    with np.errstate(over="ignore"):
        for a, f in fields:
            a = np.atleast_2d(a)
            if a.dtype == np.float64:
                bits = a.view(np.uint64)
            else:       # i32 / u8 zero-extended, as the kernel does
                bits = a.view(np.uint32 if a.dtype.itemsize == 4 else np.uint8).astype(np.uint64)
            out += _mix64(bits ^ (kj + np.uint64(f) * _CK_C)[None, :]).sum(axis=1, dtype=np.uint64)
    return out


def strerror(code: int) -> str:
    return load_library().shd_pe_strerror(int(code)).decode()


def _p(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


class Engine:
    """One path engine on one gfx950 device (shd_pe_create)."""

    def __init__(self, top, attached, device: int = 0, delta: float = 0.0,
                 store_pred: bool = True, force_mode: int = 0, devices=None,
                 shard_index: int = 0, shard_count: int = 1, debug_flags: int = 0):
        """devices: list of HIP ordinals, one row shard each (repeats = logical
        shards on one device); shard_index/shard_count: this process's engine
        among several (multi-process row shards)."""
        lib = load_library()
        self._lib = lib
        self.top = top
        self._arrays = [top.src, top.dst, top.latency, top.loss, top.vloss]
        d = GraphDesc(top.n, top.m, int(top.directed), _p(top.src), _p(top.dst),
                      _p(top.latency), _p(top.loss), _p(top.vloss))
        o = Options()
        lib.shd_pe_default_options(C.byref(o))
        o.device, o.delta, o.storePred, o.forceMode = device, delta, int(store_pred), force_mode
        o.shardIndex, o.shardCount, o.debugFlags = shard_index, shard_count, debug_flags
        if devices is not None:
            self._devs = np.ascontiguousarray(devices, dtype=np.int32)
            o.nDevices, o.devices = int(self._devs.shape[0]), _p(self._devs)
        att = np.ascontiguousarray(attached, dtype=np.int32)
        h = C.c_void_p()
        rc = lib.shd_pe_create(C.byref(d), _p(att), att.shape[0], C.byref(o), C.byref(h))
        if rc:
            raise EngineError(rc, "shd_pe_create")
        self.h = h
        self.store_pred = store_pred
        T = lib.shd_pe_num_attached(h)
        self.attached = np.empty(T, np.int32)
        lib.shd_pe_attached(h, _p(self.attached))
        self.T = T
        st, cnt = C.c_int32(), C.c_int32()
        lib.shd_pe_owned_range(h, C.byref(st), C.byref(cnt))
        self.owned = (st.value, cnt.value)

    def shard_bounds(self):
        G = self._lib.shd_pe_num_shards(self.h)
        b = np.empty(G + 1, np.int32)
        self._chk(self._lib.shd_pe_shard_bounds(self.h, _p(b)), "shd_pe_shard_bounds")
        return b

    def gather(self):
        self._chk(self._lib.shd_pe_gather(self.h), "shd_pe_gather")

    @staticmethod
    def comm_unique_id() -> bytes:
        buf = C.create_string_buffer(128)
        rc = load_library().shd_pe_comm_unique_id(buf, 128)
        if rc:
            raise EngineError(rc, "shd_pe_comm_unique_id")
        return buf.raw

    def comm_init(self, uid: bytes):
        self._chk(self._lib.shd_pe_comm_init(self.h, uid, len(uid)), "shd_pe_comm_init")

    def row_checksums(self, start: int, count: int) -> np.ndarray:
        """shd_pe_row_checksums: 64-bit fingerprint of rows [start, start+count)
        computed on the device (same formula as row_checksums_host)."""
        out = np.empty(count, np.uint64)
        self._chk(self._lib.shd_pe_row_checksums(self.h, int(start), int(count), _p(out)),
                  "shd_pe_row_checksums")
        return out

    def put_rows(self, start: int, rows: dict):
        """shd_pe_put_rows: another shard's rows [start, start+count) from host
        buffers into this engine's full table (host-transport assembly)."""
        lat = np.ascontiguousarray(rows["lat"], np.float64)
        count = lat.shape[0]
        rel = np.ascontiguousarray(rows["rel"], np.float64)
        hops = np.ascontiguousarray(rows["hops"], np.int32)
        flags = np.ascontiguousarray(rows["flags"], np.uint8)
        pred = np.ascontiguousarray(rows["pred"], np.int32) if self.store_pred else None
        for a in (rel, hops, flags) + ((pred,) if pred is not None else ()):
            if a.shape != (count, self.T):
                raise ValueError(f"put_rows: field of shape {a.shape}, want {(count, self.T)}")
        self._chk(self._lib.shd_pe_put_rows(self.h, int(start), int(count), _p(lat), _p(rel), _p(hops),
                                            _p(pred), _p(flags)), "shd_pe_put_rows")

    def close(self):
        if getattr(self, "h", None):
            self._lib.shd_pe_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()

    def _chk(self, rc, what):
        if rc:
            raise EngineError(rc, what)

    @property
    def is_complete(self) -> bool:
        return bool(self._lib.shd_pe_is_complete(self.h))

    def compute_all(self):
        self._chk(self._lib.shd_pe_compute_all(self.h), "shd_pe_compute_all")

    def compute_rows(self, sources):
        s = np.ascontiguousarray(sources, dtype=np.int32)
        self._chk(self._lib.shd_pe_compute_rows(self.h, _p(s), s.shape[0]), "shd_pe_compute_rows")

    def compute_positions(self, start: int, count: int):
        self._chk(self._lib.shd_pe_compute_positions(self.h, int(start), int(count)),
                  "shd_pe_compute_positions")

    def synchronize(self):
        self._chk(self._lib.shd_pe_synchronize(self.h), "shd_pe_synchronize")

    def stream_bandwidth(self, nbytes: int = 2 << 30, iters: int = 10) -> float:
        """Achievable HBM GB/s of this engine's device (16-B streaming copy)."""
        out = C.c_double()
        self._chk(self._lib.shd_pe_stream_bandwidth(self.h, int(nbytes), int(iters),
                                                    C.byref(out)), "shd_pe_stream_bandwidth")
        return out.value

    def get_row(self, src: int):
        T = self.T
        lat = np.empty(T); rel = np.empty(T)
        hops = np.empty(T, np.int32); flags = np.empty(T, np.uint8)
        pred = np.empty(T, np.int32) if self.store_pred else None
        self._chk(self._lib.shd_pe_get_row(self.h, int(src), _p(lat), _p(rel), _p(hops),
                                           _p(pred), _p(flags)), "shd_pe_get_row")
        return dict(lat=lat, rel=rel, hops=hops, pred=pred, flags=flags)

    def get_rows(self, start: int, count: int, out: dict | None = None):
        """Rows [start, start+count) by table position, row-major (count x T).
        `out` (e.g. from pinned_rows) receives them in place."""
        T = self.T
        if out is not None:
            # the C side writes count * T elements per field: check every
            # buffer before handing it over (a short or mistyped one would be
            # overrun)
            want = {"lat": np.float64, "rel": np.float64, "hops": np.int32, "flags": np.uint8,
                    "pred": np.int32}
            for k, dt in want.items():
                a = out.get(k)
                if a is None:
                    continue
                if a.dtype != dt or a.ndim != 2 or a.shape[1] != T or a.shape[0] < count \
                        or not a.flags.c_contiguous:
                    raise ValueError(f"get_rows: out[{k!r}] must be C-contiguous {np.dtype(dt)} "
                                     f"of shape (>= {count}, {T}), got {a.dtype} {a.shape}")
            if out.get("pred") is not None and not self.store_pred:
                raise ValueError("get_rows: pred requested but the engine stores no predecessors")
            lat, rel, hops, flags, pred = (out[k][:count] if out.get(k) is not None else None
                                           for k in ("lat", "rel", "hops", "flags", "pred"))
        else:
            lat = np.empty((count, T)); rel = np.empty((count, T))
            hops = np.empty((count, T), np.int32); flags = np.empty((count, T), np.uint8)
            pred = np.empty((count, T), np.int32) if self.store_pred else None
        self._chk(self._lib.shd_pe_get_rows(self.h, int(start), int(count), _p(lat), _p(rel),
                                            _p(hops), _p(pred), _p(flags)), "shd_pe_get_rows")
        return dict(lat=lat, rel=rel, hops=hops, pred=pred, flags=flags)

    def pinned_rows(self, count: int, fields=("lat", "rel", "hops", "flags", "pred")) -> dict:
        """Row buffers for get_rows(out=...) in page-locked host memory
        (shd_pe_host_alloc): the DMA lands in them without a staging copy.
        Fields not listed are None (not copied).  Freed when the returned
        arrays are garbage collected."""
        T = self.T
        out = {}
        for k, dt in (("lat", np.float64), ("rel", np.float64), ("hops", np.int32),
                      ("flags", np.uint8), ("pred", np.int32)):
            if k not in fields or (k == "pred" and not self.store_pred):
                out[k] = None
                continue
            out[k] = _pinned_array((count, T), dt, self._lib)
        return out

    def copy_rows_device(self, start, count, d_lat=0, d_rel=0, d_hops=0, d_flags=0):
        self._chk(self._lib.shd_pe_copy_rows_device(
            self.h, int(start), int(count), d_lat or None, d_rel or None, d_hops or None,
            d_flags or None), "shd_pe_copy_rows_device")

    def get_path(self, src: int, dst: int, cap: int | None = None) -> list:
        """shd_pe_get_path: the igraph shortest path [src, ..., dst] (vertex ids)."""
        cap = cap or self.top.n + 1
        buf = np.empty(cap, np.int32)
        ln = C.c_int32(0)
        self._chk(self._lib.shd_pe_get_path(self.h, int(src), int(dst), _p(buf), int(cap), C.byref(ln)),
                  "shd_pe_get_path")
        return buf[:ln.value].tolist()

    def tune(self):
        """shd_pe_tune: time both k_batch_rows variants on this engine's rows,
        keep the faster (leaves the table computed)."""
        self._chk(self._lib.shd_pe_tune(self.h), "shd_pe_tune")

    def stats(self) -> dict:
        s = Stats()
        self._chk(self._lib.shd_pe_get_stats(self.h, C.byref(s)), "shd_pe_get_stats")
        return {f: getattr(s, f) for f, _ in Stats._fields_}

    def reset_stats(self):
        self._chk(self._lib.shd_pe_reset_stats(self.h), "shd_pe_reset_stats")

    def direct_path(self, s, t):
        lat, rel = C.c_double(), C.c_double()
        rc = self._lib.shd_pe_direct_path(self.h, int(s), int(t), C.byref(lat), C.byref(rel))
        return None if rc else (lat.value, rel.value)

    def self_path(self, v):
        lat, rel = C.c_double(), C.c_double()
        rc = self._lib.shd_pe_self_path(self.h, int(v), C.byref(lat), C.byref(rel))
        return None if rc else (lat.value, rel.value)

    # ---- batched helpers on the device (pe_aux.hip) ----
    def self_paths(self, vertices):
        v = np.ascontiguousarray(vertices, dtype=np.int32)
        n = v.shape[0]
        lat, rel, flags = np.empty(n), np.empty(n), np.empty(n, np.uint8)
        self._chk(self._lib.shd_pe_self_paths(self.h, _p(v), n, _p(lat), _p(rel), _p(flags)),
                  "shd_pe_self_paths")
        return lat, rel, flags

    def direct_paths(self, src, dst):
        s = np.ascontiguousarray(src, dtype=np.int32)
        d = np.ascontiguousarray(dst, dtype=np.int32)
        if s.shape != d.shape:
            raise ValueError("src/dst shapes differ")
        n = s.shape[0]
        lat, rel, flags = np.empty(n), np.empty(n), np.empty(n, np.uint8)
        self._chk(self._lib.shd_pe_direct_paths(self.h, _p(s), _p(d), n, _p(lat), _p(rel),
                                                _p(flags)), "shd_pe_direct_paths")
        return lat, rel, flags

    def adjacent_pairs(self, src, dst):
        s = np.ascontiguousarray(src, dtype=np.int32)
        d = np.ascontiguousarray(dst, dtype=np.int32)
        if s.shape != d.shape:
            raise ValueError("src/dst shapes differ")
        out = np.empty(s.shape[0], np.uint8)
        self._chk(self._lib.shd_pe_adjacent_pairs(self.h, _p(s), _p(d), s.shape[0], _p(out)),
                  "shd_pe_adjacent_pairs")
        return out

    def fill_rowstore(self, store) -> tuple:
        """shd_pe_fill_rowstore: the whole table (computed first if needed,
        the host image prepared meanwhile) into an empty RowStore in one
        device pack + DMA; returns (per-row store_row results, ms of
        compute-and-image-preparation ("alloc") / pack / DMA)."""
        res = np.empty(self.T, np.int32)
        ms = np.zeros(3)
        self._chk(self._lib.shd_pe_fill_rowstore(self.h, store.h, _p(res), _p(ms)), "shd_pe_fill_rowstore")
        return res, {"alloc": ms[0], "pack": ms[1], "dma": ms[2]}

    def is_complete_device(self) -> bool:
        x = C.c_int32(0)
        self._chk(self._lib.shd_pe_is_complete_device(self.h, C.byref(x)),
                  "shd_pe_is_complete_device")
        return bool(x.value)


class RowStore:
    """shd_rowstore_*: topology.c's path cache (:1284-1386) as a triangular
    dense store; host only (no device)."""

    def __init__(self, n_vertices: int, attached):
        self._lib = load_library()
        self._att = np.ascontiguousarray(attached, dtype=np.int32)
        h = C.c_void_p()
        rc = self._lib.shd_rowstore_new(int(n_vertices), _p(self._att), self._att.shape[0],
                                        C.byref(h))
        if rc:
            raise EngineError(rc, "shd_rowstore_new")
        self.h = h

    def close(self):
        if getattr(self, "h", None):
            self._lib.shd_rowstore_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    _VISIT = C.CFUNCTYPE(None, C.c_int32, C.c_int32, C.c_double, C.c_double, C.c_int32, C.c_uint64,
                         C.c_void_p)

    def items(self) -> list:
        """shd_rowstore_foreach: every stored entry as (src, dst, lat, rel,
        isDirect, packetCount) in the stored direction."""
        out = []
        cb = RowStore._VISIT(lambda s, d, lat, rel, isd, pc, u: out.append((s, d, lat, rel, isd, pc)))
        n = self._lib.shd_rowstore_foreach(self.h, cb, None)
        assert n == len(out)
        return out

    def get(self, s, d):
        """(lat, rel, isDirect, packetCount) stored under exactly (s, d), or None."""
        lat, rel = C.c_double(), C.c_double()
        isd, pc = C.c_int32(), C.c_uint64()
        if not self._lib.shd_rowstore_get(self.h, int(s), int(d), C.byref(lat), C.byref(rel),
                                          C.byref(isd), C.byref(pc)):
            return None
        return lat.value, rel.value, bool(isd.value), pc.value

    def store(self, s, d, is_direct, is_complete, prefer_direct_and_adjacent, lat, rel) -> int:
        rc = self._lib.shd_rowstore_store(self.h, int(s), int(d), int(is_direct),
                                          int(is_complete), int(prefer_direct_and_adjacent),
                                          float(lat), float(rel))
        if rc < 0:
            raise EngineError(rc, "shd_rowstore_store")
        return rc

    def store_row(self, s, lat, rel, flags, is_complete=False, adjacent=None) -> bool:
        lat = np.ascontiguousarray(lat, dtype=np.float64)
        rel = np.ascontiguousarray(rel, dtype=np.float64)
        flags = np.ascontiguousarray(flags, dtype=np.uint8)
        adj = None if adjacent is None else np.ascontiguousarray(adjacent, dtype=np.uint8)
        T = self._att.shape[0]           # the C side reads T entries of each array
        for name, arr in (("lat", lat), ("rel", rel), ("flags", flags), ("adjacent", adj)):
            if arr is not None and arr.shape[0] < T:
                raise ValueError(f"store_row: {name} has {arr.shape[0]} entries, need {T}")
        rc = self._lib.shd_rowstore_store_row(self.h, int(s), _p(lat), _p(rel), _p(flags),
                                              int(is_complete), _p(adj))
        if rc < 0:
            raise EngineError(rc, "shd_rowstore_store_row")
        return rc == 1

    def store_rows(self, srcs, lat, rel, flags, is_complete=False, adjacent=None,
                   threads: int = 0) -> np.ndarray:
        """shd_rowstore_store_rows: rows i = 0..count-1 of (count, >= T) arrays
        (e.g. Engine.pinned_rows blocks), as store_row on srcs in order; returns
        each row's all-success flag."""
        s = np.ascontiguousarray(srcs, dtype=np.int32)
        count, T = s.shape[0], self._att.shape[0]
        arrs = {"lat": (lat, np.float64), "rel": (rel, np.float64), "flags": (flags, np.uint8),
                "adjacent": (adjacent, np.uint8)}
        ld = None
        for name, (arr, dt) in arrs.items():
            if arr is None:
                continue
            if arr.dtype != dt or arr.ndim != 2 or not arr.flags.c_contiguous:
                raise ValueError(f"store_rows: {name} must be a C-contiguous 2-D {np.dtype(dt)} array")
            if arr.shape[0] < count or arr.shape[1] < T:
                raise ValueError(f"store_rows: {name} is {arr.shape}, need >= ({count}, {T})")
            if ld is not None and arr.shape[1] != ld:
                raise ValueError("store_rows: arrays differ in row length")
            ld = arr.shape[1]
        res = np.empty(count, np.int32)
        rc = self._lib.shd_rowstore_store_rows(self.h, _p(s), count, _p(lat), _p(rel), _p(flags),
                                               int(ld or T), int(is_complete), _p(adjacent),
                                               int(threads), _p(res))
        if rc < 0:
            raise EngineError(rc, "shd_rowstore_store_rows")
        return res

    def increment(self, s, d) -> int:
        return self._lib.shd_rowstore_increment(self.h, int(s), int(d))

    def size(self) -> int:
        return self._lib.shd_rowstore_size(self.h)

    def min_latency(self) -> float:
        return self._lib.shd_rowstore_min_latency(self.h)

    def memory_bytes(self) -> int:
        return self._lib.shd_rowstore_memory_bytes(self.h)


class TopologyShim:
    """topology_getLatency/getReliability/isRoutable/incrementPathPacketCounter
    (topology.c:2053-2092) over the engine (shd_topology_*)."""

    def __init__(self, engine: Engine, prefers_direct: bool = False):
        self.engine = engine
        self._lib = engine._lib
        h = C.c_void_p()
        rc = self._lib.shd_topology_new(engine.h, int(prefers_direct), C.byref(h))
        if rc:
            raise EngineError(rc, "shd_topology_new")
        self.h = h

    def close(self):
        if getattr(self, "h", None):
            self._lib.shd_topology_free(self.h)
            self.h = None

    def __del__(self):
        self.close()

    def get_latency(self, s, d):
        return self._lib.shd_topology_get_latency(self.h, int(s), int(d))

    def get_reliability(self, s, d):
        return self._lib.shd_topology_get_reliability(self.h, int(s), int(d))

    def is_routable(self, s, d):
        return bool(self._lib.shd_topology_is_routable(self.h, int(s), int(d)))

    def increment(self, s, d):
        return self._lib.shd_topology_increment_path_packet_counter(self.h, int(s), int(d))

    def cached(self, s, d):
        lat, rel = C.c_double(), C.c_double()
        isd, pc = C.c_int32(), C.c_int64()
        ok = self._lib.shd_topology_cached(self.h, int(s), int(d), C.byref(lat), C.byref(rel),
                                           C.byref(isd), C.byref(pc))
        return (lat.value, rel.value, bool(isd.value), pc.value) if ok else None

    @property
    def min_latency(self):
        return self._lib.shd_topology_min_latency(self.h)

    @property
    def cache_size(self):
        return self._lib.shd_topology_cache_size(self.h)

    @property
    def rows_computed(self):
        return self._lib.shd_topology_rows_computed(self.h)


def parse_graphml(data, name: str = "topology", with_ids: bool = True):
    """Native GraphML ingestion (shd_graphml_parse, pe_graphml.cpp): text or
    bytes (an ``.xz`` path is decompressed here) -> Topology.  Host-only, no
    GPU needed; the same result as igraph's import order (ids in document
    order)."""
    import lzma
    from .graph import Topology
    if isinstance(data, str) and not data.lstrip().startswith("<"):
        with open(data, "rb") as f:
            raw = f.read()
        data = lzma.decompress(raw) if str(data).endswith(".xz") else raw
    if isinstance(data, str):
        data = data.encode()
    lib = load_library()
    h = C.c_void_p()
    rc = lib.shd_graphml_parse(data, len(data), C.byref(h))
    if rc:
        raise EngineError(rc, "shd_graphml_parse")
    try:
        d = GraphDesc()
        pdp = C.c_int32()
        rc = lib.shd_graphml_describe(h, C.byref(d), C.byref(pdp))
        if rc:
            raise EngineError(rc, "shd_graphml_describe")
        n, m = int(d.nVertices), int(d.nEdges)

        def arr(ptr, ctype, count, dtype):
            if count == 0 or not ptr:
                return np.zeros(count, dtype)
            return np.ctypeslib.as_array(C.cast(ptr, C.POINTER(ctype)), shape=(count,)).astype(dtype)

        src = arr(d.edgeFrom, C.c_int32, m, np.int32)
        dst = arr(d.edgeTo, C.c_int32, m, np.int32)
        lat = arr(d.edgeLatency, C.c_double, m, np.float64)
        loss = arr(d.edgePacketLoss, C.c_double, m, np.float64)
        vloss = arr(d.vertexPacketLoss, C.c_double, n, np.float64) if d.vertexPacketLoss else None
        ids = [lib.shd_graphml_vertex_id(h, v).decode() for v in range(n)] if with_ids else None
        return Topology(n=n, directed=bool(d.directed), src=src, dst=dst, latency=lat, loss=loss,
                        vloss=vloss, ids=ids, prefers_direct=bool(pdp.value), name=name)
    finally:
        lib.shd_graphml_free(h)

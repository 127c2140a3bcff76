"""ctypes binding of libcep.so (include/cep.h) — the product path.

There is no fallback: if libcep.so is missing or no GPU is visible, the calls raise.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# $CEP_MEASURE set: the measurement build (libcep_measure.so, Makefile `measure`), the one that
# reads the $CEP_* tuning knobs; the release libcep.so runs the defaults
LIB_PATH = os.path.join(_HERE, "libcep_measure.so" if os.environ.get("CEP_MEASURE") else "libcep.so")
SYNTH_LIB_PATH = os.path.join(_HERE, "libcep_synth.so")  # bench/test generators (include/cep_synth.h)

CEP_MEM_HOST, CEP_MEM_DEVICE = 0, 1
CEP_KIND_NFA, CEP_KIND_STENCIL = 0, 1
CEP_TIER_JIT, CEP_TIER_INTERP = 0, 1
KEY_ERRORS = {0: None, 1: "NullPointerException", 2: "IllegalStateException",
              3: "ArithmeticException", 16: "capacity"}

# every symbol include/cep.h declares (tests check the library exports them all)
EXPORTS = [
    "cep_query_compile", "cep_query_info_get", "cep_query_stage_name", "cep_query_destroy",
    "cep_session_create", "cep_session_destroy", "cep_push_batch", "cep_sync", "cep_poll_matches",
    "cep_key_errors", "cep_match_digest", "cep_watermark", "cep_last_timing", "cep_last_error",
    "cep_alloc_pinned", "cep_free_pinned", "cep_device_alloc", "cep_device_free", "cep_memcpy",
    "cep_query_jit_source", "cep_jit_precompile", "cep_session_reset", "cep_live_floor",
    "cep_batch_layout", "cep_session_snapshot", "cep_session_restore",
    "cep_decode_stock_json", "cep_jit_precompile_group", "cep_query_group_plan",
    "cep_last_stats", "cep_gather_keys", "cep_timing_totals", "cep_symbol_keys", "cep_lane_balance",
]
# every symbol include/cep_synth.h declares (the generator library of the bench and tests)
SYNTH_EXPORTS = ["cep_synth_last_error", "cep_synth_count", "cep_synth_generate", "cep_synth_generate_arrival",
                 "cep_synth_ts", "cep_synth_stock_json"]


class QueryInfo(C.Structure):
    _fields_ = [("n_patterns", C.c_uint32), ("n_stages", C.c_uint32), ("n_names", C.c_uint32),
                ("n_fields", C.c_uint32), ("n_states", C.c_uint32), ("kind", C.c_uint32),
                ("arity", C.c_uint32), ("compile_error", C.c_int32)]


class Opts(C.Structure):
    _fields_ = [("device", C.c_int), ("force_nfa", C.c_int), ("tier", C.c_int), ("max_runs", C.c_uint32),
                ("pool_factor", C.c_double), ("streaming", C.c_int), ("no_groups", C.c_int)]


class BatchStats(C.Structure):
    _fields_ = [("group", C.c_uint32), ("group_queries", C.c_uint32), ("kernel_ms", C.c_double),
                ("main_ms", C.c_double), ("retry_ms", C.c_double), ("retried_jobs", C.c_uint64),
                ("nodes_used", C.c_uint64), ("preds_used", C.c_uint64), ("out_chunks_used", C.c_uint64),
                ("launches", C.c_uint32), ("allocs", C.c_uint32)]


class Batch(C.Structure):
    _fields_ = [("n_keys", C.c_uint64), ("n_events", C.c_uint64), ("key_off", C.c_void_p),
                ("cols", C.POINTER(C.c_void_p)), ("ts", C.c_void_p), ("memory", C.c_int),
                ("arrival_key", C.c_void_p)]


class Matches(C.Structure):
    _fields_ = [("n_matches", C.c_uint64), ("n_pairs", C.c_uint64), ("arity", C.c_uint32),
                ("arity_stage", C.POINTER(C.c_uint16)), ("key", C.POINTER(C.c_uint32)),
                ("emit_seq", C.POINTER(C.c_uint32)), ("pair_off", C.POINTER(C.c_uint64)),
                ("pair_seq", C.POINTER(C.c_uint32)), ("pair_stage", C.POINTER(C.c_uint16)),
                ("memory", C.c_int)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} is missing: run __graft_entry__.build() (no CPU fallback)")
        L = C.CDLL(LIB_PATH)
        vp, u64, u32, i32 = C.c_void_p, C.c_uint64, C.c_uint32, C.c_int32
        sig = {
            "cep_query_compile": ([C.c_char_p, C.c_size_t, C.POINTER(vp)], C.c_int),
            "cep_query_info_get": ([vp, C.POINTER(QueryInfo)], C.c_int),
            "cep_query_stage_name": ([vp, u32], C.c_char_p),
            "cep_query_destroy": ([vp], None),
            "cep_query_jit_source": ([vp], C.c_char_p),
            "cep_jit_precompile": ([vp, C.POINTER(C.c_double)], C.c_int),
            "cep_jit_precompile_group": ([C.POINTER(vp), C.c_int, C.POINTER(C.c_double)], C.c_int),
            "cep_query_group_plan": ([C.POINTER(vp), C.c_int, C.c_int, C.POINTER(C.c_char_p), C.POINTER(u32),
                                      C.POINTER(C.POINTER(i32)), C.POINTER(u32), C.POINTER(C.POINTER(C.c_int64))],
                                     C.c_int),
            "cep_session_create": ([C.POINTER(vp), C.c_int, C.POINTER(Opts), C.POINTER(vp)], C.c_int),
            "cep_session_destroy": ([vp], None),
            "cep_push_batch": ([vp, C.POINTER(Batch)], C.c_int),
            "cep_sync": ([vp], C.c_int),
            "cep_poll_matches": ([vp, C.c_int, C.c_int, C.POINTER(Matches)], C.c_int),
            "cep_key_errors": ([vp, C.c_int, C.POINTER(i32), C.POINTER(u32), u64], C.c_int),
            "cep_match_digest": ([vp, C.c_int, C.POINTER(u64), C.POINTER(u64)], C.c_int),
            "cep_watermark": ([vp, C.POINTER(C.c_int64)], C.c_int),
            "cep_last_timing": ([vp, C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_double), C.POINTER(u32)],
                                C.c_int),
            "cep_timing_totals": ([vp, C.c_int, C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_double), C.POINTER(u64)],
                                  C.c_int),
            "cep_last_error": ([], C.c_char_p),
            "cep_last_stats": ([vp, C.c_int, C.POINTER(BatchStats)], C.c_int),
            "cep_gather_keys": ([C.c_int, u64, vp, vp, vp, C.c_int, C.POINTER(u32), C.POINTER(vp), C.POINTER(vp),
                                 vp, vp], C.c_int),
            "cep_device_alloc": ([C.c_int, C.c_size_t, C.POINTER(vp)], C.c_int),
            "cep_device_free": ([vp], C.c_int),
            "cep_memcpy": ([vp, vp, C.c_size_t, C.c_int, C.c_int], C.c_int),
            "cep_batch_layout": ([vp, C.c_int, C.POINTER(vp), C.POINTER(vp), C.POINTER(C.c_double)], C.c_int),
            "cep_session_snapshot": ([vp, vp, C.c_size_t, C.POINTER(C.c_size_t)], C.c_int),
            "cep_session_restore": ([vp, vp, C.c_size_t], C.c_int),
            "cep_session_reset": ([vp], C.c_int),
            "cep_live_floor": ([vp, C.c_int, C.POINTER(u32), u64], C.c_int),
            "cep_decode_stock_json": ([C.c_int, vp, vp, u64, C.c_int, vp, vp, vp, vp, vp], C.c_int),
            "cep_symbol_keys": ([C.c_int, vp, vp, vp, vp, u64, u64, vp, C.POINTER(u64), vp], C.c_int),
            "cep_lane_balance": ([vp, C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_double)], C.c_int),
        }
        for name, (args, res) in sig.items():
            f = getattr(L, name)
            f.argtypes, f.restype = args, res
        _lib = L
    return _lib


_synth = None


def synth_lib():
    """libcep_synth.so: the synthetic generators (bench and tests only; the matcher never
    loads it)."""
    global _synth
    if _synth is None:
        if not os.path.exists(SYNTH_LIB_PATH):
            raise RuntimeError(f"{SYNTH_LIB_PATH} is missing: run __graft_entry__.build()")
        L = C.CDLL(SYNTH_LIB_PATH)
        vp, u64, u32 = C.c_void_p, C.c_uint64, C.c_uint32
        sig = {
            "cep_synth_last_error": ([], C.c_char_p),
            "cep_synth_ts": ([C.c_int, u64, C.c_int64, vp], C.c_int),
            "cep_synth_count": ([C.c_int, C.c_int, u64, u64, u64, u32, C.POINTER(u64)], C.c_int),
            "cep_synth_generate": ([C.c_int, C.c_int, u64, u64, u64, u32, vp, C.POINTER(vp)], C.c_int),
            "cep_synth_generate_arrival": ([C.c_int, C.c_int, u64, u64, u64, u32, vp, C.POINTER(vp)], C.c_int),
            "cep_synth_stock_json": ([C.c_int, vp, vp, u64, vp, u64, vp, C.POINTER(u64)], C.c_int),
        }
        for name, (args, res) in sig.items():
            f = getattr(L, name)
            f.argtypes, f.restype = args, res
        _synth = L
    return _synth


def _check_synth(rc):
    if rc != 0:
        raise CepError(f"libcep_synth error {rc}: {synth_lib().cep_synth_last_error().decode(errors='replace')}")


class CepError(RuntimeError):
    pass


def _check(rc):
    if rc != 0:
        raise CepError(f"libcep error {rc}: {lib().cep_last_error().decode(errors='replace')}")


class Query:
    """A compiled query (cep_query_compile ~ StatesFactory.make)."""

    def __init__(self, ir: bytes):
        self.ir = ir
        h = C.c_void_p()
        _check(lib().cep_query_compile(ir, len(ir), C.byref(h)))
        self.h = h
        self.info = QueryInfo()
        _check(lib().cep_query_info_get(self.h, C.byref(self.info)))
        self.stage_names = [lib().cep_query_stage_name(self.h, i).decode() for i in range(self.info.n_names)]

    @property
    def kind(self):
        return self.info.kind

    @property
    def jit_source(self) -> str:
        return lib().cep_query_jit_source(self.h).decode()

    def precompile(self) -> float:
        """Compile the JIT kernel into the code-object cache (no GPU needed); seconds spent."""
        t = C.c_double()
        _check(lib().cep_jit_precompile(self.h, C.byref(t)))
        return t.value

    def __del__(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.cep_query_destroy(self.h)
            self.h = None


def precompile_group(queries) -> float:
    """Compile the kernels a session over `queries` launches (one per group of queries that
    differ only in literals) into the code-object cache, without a GPU; seconds spent."""
    arr = (C.c_void_p * len(queries))(*[q.h.value for q in queries])
    t = C.c_double()
    _check(lib().cep_jit_precompile_group(arr, len(queries), C.byref(t)))
    return t.value


def group_plans(queries) -> list:
    """The kernel groups a session over `queries` launches: [{members, source, literals}],
    literals a (members x n) int64 table of the literals that differ (cep_query_group_plan)."""
    arr = (C.c_void_p * len(queries))(*[q.h.value for q in queries])
    out = []
    while True:
        src, nm, mem, nl, lits = C.c_char_p(), C.c_uint32(), C.POINTER(C.c_int32)(), C.c_uint32(), \
            C.POINTER(C.c_int64)()
        rc = lib().cep_query_group_plan(arr, len(queries), len(out), C.byref(src), C.byref(nm), C.byref(mem),
                                        C.byref(nl), C.byref(lits))
        if rc != 0:
            break
        members = [mem[i] for i in range(nm.value)]
        table = np.array([lits[i] for i in range(nm.value * nl.value)], np.int64).reshape(nm.value, nl.value)
        out.append({"members": members, "source": src.value.decode(), "literals": table})
    return out


class DeviceBuffer:
    def __init__(self, nbytes: int, device: int = 0):
        self.nbytes, self.device = int(nbytes), device
        p = C.c_void_p()
        _check(lib().cep_device_alloc(device, max(1, self.nbytes), C.byref(p)))
        self.ptr = p.value

    def upload(self, arr: np.ndarray):
        arr = np.ascontiguousarray(arr)
        assert arr.nbytes <= self.nbytes
        _check(lib().cep_memcpy(self.ptr, arr.ctypes.data, arr.nbytes, CEP_MEM_DEVICE, CEP_MEM_HOST))

    def download(self, dtype, count) -> np.ndarray:
        out = np.empty(count, dtype=dtype)
        if out.nbytes:
            _check(lib().cep_memcpy(out.ctypes.data, self.ptr, out.nbytes, CEP_MEM_HOST, CEP_MEM_DEVICE))
        return out

    def free(self):
        if self.ptr and _lib is not None:
            _lib.cep_device_free(self.ptr)
            self.ptr = None

    def __del__(self):
        self.free()


class DeviceStream:
    """A device-resident CSR batch (key_off u64 + int32 columns)."""

    def __init__(self, n_keys, n_events, key_off: DeviceBuffer, cols: list, device=0, keep=None):
        self.n_keys, self.n_events = int(n_keys), int(n_events)
        self.key_off, self.cols, self.device = key_off, cols, device
        self._keep = keep

    @classmethod
    def from_host(cls, key_off, cols, device=0):
        key_off = np.ascontiguousarray(key_off, dtype=np.uint64)
        kb = DeviceBuffer(key_off.nbytes, device)
        kb.upload(key_off)
        cbs = []
        for c in cols:
            c = np.ascontiguousarray(c)
            b = DeviceBuffer(c.nbytes, device)
            b.upload(c)
            cbs.append(b)
        return cls(len(key_off) - 1, int(key_off[-1]), kb, cbs, device)

    def download(self):
        off = self.key_off.download(np.uint64, self.n_keys + 1)
        cols = [c.download(np.int32, self.n_events) for c in self.cols]
        return off, cols


def synth_stream(kind: str, seed: int, n_keys: int, mean_events: int, key_base: int = 0,
                 device: int = 0) -> DeviceStream:
    """Generate workloads.SynthConfig data directly in HBM (csrc/synth_gen.hip, libcep_synth.so)."""
    k = {"abc": 0, "stock": 1}[kind]
    n = C.c_uint64()
    _check_synth(synth_lib().cep_synth_count(device, k, seed, n_keys, key_base, mean_events, C.byref(n)))
    off = DeviceBuffer(8 * (n_keys + 1), device)
    ncols = 1 if k == 0 else 2
    cols = [DeviceBuffer(4 * max(1, n.value), device) for _ in range(ncols)]
    ptrs = (C.c_void_p * ncols)(*[c.ptr for c in cols])
    _check_synth(synth_lib().cep_synth_generate(device, k, seed, n_keys, key_base, mean_events, off.ptr, ptrs))
    return DeviceStream(n_keys, n.value, off, cols, device)


def synth_ts(n_events: int, base: int = 1_600_000_000_000, device: int = 0) -> "DeviceBuffer":
    """Device timestamps base + CSR position for a synthetic stream (cep_synth_ts)."""
    b = DeviceBuffer(8 * max(1, n_events), device)
    _check_synth(synth_lib().cep_synth_ts(device, n_events, base, b.ptr))
    return b


def shard_stream(stream: "DeviceStream", keys: np.ndarray, local_off: np.ndarray, ts: "DeviceBuffer | None" = None):
    """The shard of a device-resident stream holding keys `keys` (shard.shard_layout), its
    events gathered on the device (cep_gather_keys).  Returns (DeviceStream, ts DeviceBuffer
    or None); the shard's key i is the stream's key keys[i]."""
    keys = np.ascontiguousarray(keys, np.uint32)
    local_off = np.ascontiguousarray(local_off, np.uint64)
    n = int(local_off[-1])
    sel = DeviceBuffer(max(4, keys.nbytes), stream.device)
    if keys.size:
        sel.upload(keys)
    off = DeviceBuffer(local_off.nbytes, stream.device)
    off.upload(local_off)
    cols = [DeviceBuffer(4 * max(1, n), stream.device) for _ in stream.cols]
    nc = len(cols)
    widths = (C.c_uint32 * nc)(*([4] * nc))
    src = (C.c_void_p * nc)(*[c.ptr for c in stream.cols])
    dst = (C.c_void_p * nc)(*[c.ptr for c in cols])
    dts = DeviceBuffer(8 * max(1, n), stream.device) if ts is not None else None
    _check(lib().cep_gather_keys(stream.device, len(keys), sel.ptr, stream.key_off.ptr, off.ptr, nc, widths, src, dst,
                                 ts.ptr if ts is not None else None, dts.ptr if dts is not None else None))
    return DeviceStream(len(keys), n, off, cols, stream.device), dts


def gather_ranges(stream: "DeviceStream", starts: np.ndarray, ends: np.ndarray) -> "DeviceStream":
    """A new CSR stream whose key k holds positions [starts[k], ends[k]) of `stream` (device
    gather, cep_gather_keys with a source-offset table of (start, end) pairs: key k reads
    src_off[2k] .. src_off[2k + 1]).  Used to cut a stream into consecutive per-key slices,
    the batches of a streaming session."""
    starts = np.ascontiguousarray(starts, np.uint64)
    ends = np.ascontiguousarray(ends, np.uint64)
    nk = len(starts)
    pairs = np.empty(2 * nk, np.uint64)
    pairs[0::2] = starts
    pairs[1::2] = ends
    local = np.zeros(nk + 1, np.uint64)
    np.cumsum(ends - starts, out=local[1:])
    n = int(local[-1])
    sel = DeviceBuffer(max(4, 4 * nk), stream.device)
    if nk:
        sel.upload((2 * np.arange(nk, dtype=np.uint64)).astype(np.uint32))
    src = DeviceBuffer(max(8, pairs.nbytes), stream.device)
    if nk:
        src.upload(pairs)
    off = DeviceBuffer(local.nbytes, stream.device)
    off.upload(local)
    cols = [DeviceBuffer(4 * max(1, n), stream.device) for _ in stream.cols]
    nc = len(cols)
    widths = (C.c_uint32 * nc)(*([4] * nc))
    sp = (C.c_void_p * nc)(*[c.ptr for c in stream.cols])
    dp = (C.c_void_p * nc)(*[c.ptr for c in cols])
    _check(lib().cep_gather_keys(stream.device, nk, sel.ptr, src.ptr, off.ptr, nc, widths, sp, dp, None, None))
    return DeviceStream(nk, n, off, cols, stream.device)


class ArrivalStream:
    """A device-resident arrival-order batch: the key of every event + int32 columns."""

    def __init__(self, n_keys, n_events, keys: DeviceBuffer, cols: list, device=0):
        self.n_keys, self.n_events = int(n_keys), int(n_events)
        self.keys, self.cols, self.device = keys, cols, device

    def download(self):
        return self.keys.download(np.uint32, self.n_events), [c.download(np.int32, self.n_events) for c in self.cols]


def synth_arrival_stream(kind: str, seed: int, n_keys: int, mean_events: int, key_base: int = 0,
                         device: int = 0) -> ArrivalStream:
    """workloads.generate_arrival's stream, generated in HBM (csrc/partition.hip)."""
    k = {"abc": 0, "stock": 1}[kind]
    n = C.c_uint64()
    _check_synth(synth_lib().cep_synth_count(device, k, seed, n_keys, key_base, mean_events, C.byref(n)))
    keys = DeviceBuffer(4 * max(1, n.value), device)
    cols = [DeviceBuffer(4 * max(1, n.value), device) for _ in range(1 if k == 0 else 2)]
    ptrs = (C.c_void_p * len(cols))(*[c.ptr for c in cols])
    _check_synth(synth_lib().cep_synth_generate_arrival(device, k, seed, n_keys, key_base, mean_events, keys.ptr, ptrs))
    return ArrivalStream(n_keys, n.value, keys, cols, device)


class StockJsonBatch:
    """Record values of the demo's StockEvents topic, back to back in HBM (bytes) with u64 offsets
    rec_off[n+1]: the input of StockEventSerDe's deserializer (test:demo/StockEventSerDe.java:58-72)
    for a whole batch."""

    def __init__(self, n, nbytes, data: DeviceBuffer, rec_off: DeviceBuffer, device=0):
        self.n, self.nbytes, self.data, self.rec_off, self.device = int(n), int(nbytes), data, rec_off, device

    @classmethod
    def from_records(cls, records, device=0):
        off = np.zeros(len(records) + 1, np.uint64)
        off[1:] = np.cumsum([len(r) for r in records], dtype=np.uint64) if records else []
        blob = np.frombuffer(b"".join(records), np.uint8)
        d = DeviceBuffer(max(1, blob.nbytes), device)
        if blob.nbytes:
            d.upload(blob)
        o = DeviceBuffer(off.nbytes, device)
        o.upload(off)
        return cls(len(records), blob.nbytes, d, o, device)

    @classmethod
    def synth(cls, price: DeviceBuffer, volume: DeviceBuffer, n: int, device=0):
        """json-simple's serialization of n StockEvents e1..en (csrc/ingest.hip), made in HBM."""
        o = DeviceBuffer(8 * (n + 1), device)
        tot = C.c_uint64()
        _check_synth(synth_lib().cep_synth_stock_json(device, price.ptr, volume.ptr, n, None, 0, o.ptr, C.byref(tot)))
        d = DeviceBuffer(max(1, tot.value), device)
        _check_synth(synth_lib().cep_synth_stock_json(device, price.ptr, volume.ptr, n, d.ptr, tot.value, o.ptr, C.byref(tot)))
        return cls(n, tot.value, d, o, device)

    def download(self):
        return bytes(self.data.download(np.uint8, self.nbytes)), self.rec_off.download(np.uint64, self.n + 1)


class DecodedStock:
    """Device columns of a decoded StockJsonBatch (price, volume, status, name spans)."""

    def __init__(self, n, col_width, device=0, name_spans=True):
        self.n, self.col_width = int(n), int(col_width)
        self.price = DeviceBuffer(col_width * max(1, n), device)
        self.volume = DeviceBuffer(col_width * max(1, n), device)
        self.status = DeviceBuffer(4 * max(1, n), device)
        self.name_span = DeviceBuffer(8 * max(1, n), device) if name_spans else None

    def download(self):
        dt = np.int32 if self.col_width == 4 else np.int64
        out = {"price": self.price.download(dt, self.n), "volume": self.volume.download(dt, self.n),
               "status": self.status.download(np.int32, self.n)}
        if self.name_span is not None:
            out["name_span"] = self.name_span.download(np.uint32, 2 * self.n).reshape(-1, 2)
        return out


def decode_stock_json(batch: StockJsonBatch, col_width: int = 8, out: DecodedStock | None = None,
                      stream=None, name_spans=True) -> DecodedStock:
    """cep_decode_stock_json: one launch over the batch (asynchronous on `stream`, a hipStream_t
    handle or None for the default stream)."""
    if out is None:
        out = DecodedStock(batch.n, col_width, batch.device, name_spans)
    assert out.n == batch.n and out.col_width == col_width
    _check(lib().cep_decode_stock_json(batch.device, batch.data.ptr, batch.rec_off.ptr, batch.n, col_width,
                                       out.price.ptr, out.volume.ptr, out.status.ptr,
                                       out.name_span.ptr if out.name_span is not None else None, stream))
    out._src = batch  # the launch is asynchronous: keep the input's device buffers alive with the output
    return out


def symbol_keys(batch: StockJsonBatch, decoded: DecodedStock, max_symbols: int = 0, stream=None):
    """cep_symbol_keys: the [symbol] key of every record (index of its name in order of first
    appearance; 0xFFFFFFFF for records whose deserialize() throws) -> (DeviceBuffer u32[n],
    n_symbols).  `decoded` must hold name spans."""
    assert decoded.name_span is not None and decoded.n == batch.n
    keys = DeviceBuffer(4 * max(1, batch.n), batch.device)
    ns = C.c_uint64()
    _check(lib().cep_symbol_keys(batch.device, batch.data.ptr, batch.rec_off.ptr, decoded.name_span.ptr,
                                 decoded.status.ptr, batch.n, max_symbols, keys.ptr, C.byref(ns), stream))
    return keys, ns.value


class Session:
    """cep_session: per-key NFA state for one or more queries on one GPU."""

    def __init__(self, queries, device: int = 0, force_nfa: bool = False, max_runs: int = 0,
                 pool_factor: float = 0.0, tier: int = CEP_TIER_JIT, streaming: bool = False,
                 groups: bool = True):
        if isinstance(queries, Query):
            queries = [queries]
        self.queries = list(queries)
        arr = (C.c_void_p * len(self.queries))(*[q.h.value for q in self.queries])
        opts = Opts(device, 1 if force_nfa else 0, tier, max_runs, pool_factor, 1 if streaming else 0,
                    0 if groups else 1)
        h = C.c_void_p()
        _check(lib().cep_session_create(arr, len(self.queries), C.byref(opts), C.byref(h)))
        self.h = h
        self.device = device
        self.n_keys = 0

    def close(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.cep_session_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()

    # -- input --
    def push(self, key_off, cols, ts=None):
        """Host numpy CSR batch."""
        key_off = np.ascontiguousarray(key_off, dtype=np.uint64)
        cols = [np.ascontiguousarray(c) for c in cols]
        ptrs = (C.c_void_p * max(1, len(cols)))(*[c.ctypes.data for c in cols])
        tsp = None
        if ts is not None:
            ts = np.ascontiguousarray(ts, dtype=np.int64)
            tsp = ts.ctypes.data
        b = Batch(len(key_off) - 1, int(key_off[-1]) if len(key_off) else 0, key_off.ctypes.data,
                  ptrs, tsp, CEP_MEM_HOST)
        _check(lib().cep_push_batch(self.h, C.byref(b)))
        self.n_keys = len(key_off) - 1

    def push_arrival(self, keys, cols, n_keys: int, ts=None):
        """Host batch in arrival order: keys[i] is the key of event i (partitioned on the GPU)."""
        keys = np.ascontiguousarray(keys, dtype=np.uint32)
        cols = [np.ascontiguousarray(c) for c in cols]
        ptrs = (C.c_void_p * max(1, len(cols)))(*[c.ctypes.data for c in cols])
        tsp = None
        if ts is not None:
            ts = np.ascontiguousarray(ts, dtype=np.int64)
            tsp = ts.ctypes.data
        b = Batch(n_keys, len(keys), None, ptrs, tsp, CEP_MEM_HOST, keys.ctypes.data)
        _check(lib().cep_push_batch(self.h, C.byref(b)))
        self.n_keys = n_keys

    def push_arrival_device(self, stream: ArrivalStream):
        ptrs = (C.c_void_p * len(stream.cols))(*[c.ptr for c in stream.cols])
        b = Batch(stream.n_keys, stream.n_events, None, ptrs, None, CEP_MEM_DEVICE, stream.keys.ptr)
        _check(lib().cep_push_batch(self.h, C.byref(b)))
        self.n_keys = stream.n_keys

    def layout(self):
        """(key_off, arrival_index or None, partition_ms) of the last batch (host copies)."""
        off, perm, ms = C.c_void_p(), C.c_void_p(), C.c_double()
        _check(lib().cep_batch_layout(self.h, CEP_MEM_HOST, C.byref(off), C.byref(perm), C.byref(ms)))
        ko = np.ctypeslib.as_array(C.cast(off, C.POINTER(C.c_uint64)), shape=(self.n_keys + 1,)).copy()
        ai = None
        if perm.value:
            ai = np.ctypeslib.as_array(C.cast(perm, C.POINTER(C.c_uint32)), shape=(int(ko[-1]),)).copy()
        return ko, ai, ms.value

    def push_device(self, stream: DeviceStream, ts_ptr=None):
        # the batch descriptor of a device-resident stream is built once and reused (pushing the
        # same buffers again is the bench's steady state; a stencil push is ~0.1 ms of GPU work,
        # so host-side microseconds per call show up between batches)
        key = (id(stream), ts_ptr)
        cached = getattr(self, "_dev_batch", None)
        if cached is None or cached[0] != key or cached[1] is not stream:
            ptrs = (C.c_void_p * len(stream.cols))(*[c.ptr for c in stream.cols])
            b = Batch(stream.n_keys, stream.n_events, stream.key_off.ptr, ptrs, ts_ptr, CEP_MEM_DEVICE)
            cached = (key, stream, ptrs, b, C.byref(b))
            self._dev_batch = cached
        _check(lib().cep_push_batch(self.h, cached[4]))
        self.n_keys = stream.n_keys

    # -- output --
    def matches(self, query: int = 0) -> dict:
        """Host copy of the last batch's matches, always in variable-length form."""
        m = Matches()
        _check(lib().cep_poll_matches(self.h, query, CEP_MEM_HOST, C.byref(m)))
        nm, npairs = m.n_matches, m.n_pairs

        def arr(p, n, dt):
            return np.ctypeslib.as_array(p, shape=(n,)).astype(dt, copy=True) if n else np.zeros(0, dt)

        key = arr(m.key, nm, np.uint32)
        seq = arr(m.pair_seq, npairs, np.uint32)
        if m.arity:
            a = m.arity
            stages = np.array([m.arity_stage[i] for i in range(a)], dtype=np.uint16)
            emit = seq[0::a].copy() if nm else np.zeros(0, np.uint32)
            off = (np.arange(nm + 1, dtype=np.uint64) * a)
            stage = np.tile(stages, nm)
        else:
            emit = arr(m.emit_seq, nm, np.uint32)
            off = arr(m.pair_off, nm + 1, np.uint64)
            stage = arr(m.pair_stage, npairs, np.uint16)
        return {"n_matches": nm, "n_pairs": npairs, "key": key, "emit_seq": emit, "pair_off": off,
                "pair_seq": seq, "pair_stage": stage, "arity": m.arity}

    def key_errors(self, query: int = 0, n_keys: int | None = None):
        n = self.n_keys if n_keys is None else n_keys
        code = np.zeros(n, np.int32)
        seq = np.zeros(n, np.uint32)
        _check(lib().cep_key_errors(self.h, query, code.ctypes.data_as(C.POINTER(C.c_int32)),
                                    seq.ctypes.data_as(C.POINTER(C.c_uint32)), n))
        return code, seq

    def digest(self, query: int = 0):
        n, d = C.c_uint64(), C.c_uint64()
        _check(lib().cep_match_digest(self.h, query, C.byref(n), C.byref(d)))
        return n.value, d.value

    def timing(self, query: int = 0):
        """(matching-kernel ms, setup/compaction ms, matching launches) of the last batch."""
        ms, aux, n = C.c_double(), C.c_double(), C.c_uint32()
        _check(lib().cep_last_timing(self.h, query, C.byref(ms), C.byref(aux), C.byref(n)))
        return ms.value, aux.value, n.value

    def timing_totals(self, query: int = 0, reset: bool = False):
        """(kernel ms, setup ms, batches) summed over the batches since the last reset."""
        ms, aux, n = C.c_double(), C.c_double(), C.c_uint64()
        _check(lib().cep_timing_totals(self.h, query, 1 if reset else 0, C.byref(ms), C.byref(aux), C.byref(n)))
        return ms.value, aux.value, n.value

    def lane_balance(self, query: int = 0):
        """cep_lane_balance: (longest-first lane order, key-index order) sum-over-waves of the
        busiest lane's work estimate / the mean lane's (1.0 = no lane idles)."""
        o, i = C.c_double(), C.c_double()
        _check(lib().cep_lane_balance(self.h, query, C.byref(o), C.byref(i)))
        return o.value, i.value

    def stats(self, query: int = 0) -> dict:
        """cep_last_stats: the last batch's NFA figures for the query's kernel group."""
        st = BatchStats()
        _check(lib().cep_last_stats(self.h, query, C.byref(st)))
        return {k: getattr(st, k) for k, _ in BatchStats._fields_}

    def live_floor(self, query: int = 0, n_keys: int | None = None) -> np.ndarray:
        """cep_live_floor: per key, the oldest sequence number a live buffer node still holds
        (0xFFFFFFFF: none) - a streaming session's only events a later match can contain."""
        n = self.n_keys if n_keys is None else n_keys
        out = np.zeros(n, np.uint32)
        _check(lib().cep_live_floor(self.h, query, out.ctypes.data_as(C.POINTER(C.c_uint32)), n))
        return out

    def reset(self) -> None:
        """cep_session_reset: every key of a streaming session back to the NFA's initial
        state (allocations kept)."""
        _check(lib().cep_session_reset(self.h))

    def snapshot(self) -> bytes:
        """The streaming session's complete per-key NFA state as a versioned blob
        (cep_session_snapshot; the reference's persistent run-queue/buffer stores)."""
        n = C.c_size_t()
        _check(lib().cep_session_snapshot(self.h, None, 0, C.byref(n)))
        buf = C.create_string_buffer(n.value)
        _check(lib().cep_session_snapshot(self.h, buf, n.value, C.byref(n)))
        return buf.raw[:n.value]

    def restore(self, blob: bytes) -> None:
        """Loads a snapshot into this (fresh, streaming) session over the same queries."""
        _check(lib().cep_session_restore(self.h, blob, len(blob)))

    def watermark(self) -> int:
        w = C.c_int64()
        _check(lib().cep_watermark(self.h, C.byref(w)))
        return w.value

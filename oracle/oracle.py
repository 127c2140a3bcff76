"""ctypes front-end of the CPU oracle — TEST INFRASTRUCTURE ONLY.

Loads oracle/_build/libcep_oracle.so (the literal restatement of the reference NFA,
cep_oracle.cpp).  Imported only by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg; the product package never imports this module.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "libcep_oracle.so")
_lib = None


class _Result(C.Structure):
    _fields_ = [
        ("n_keys", C.c_uint64), ("n_matches", C.c_uint64), ("n_pairs", C.c_uint64),
        ("key", C.POINTER(C.c_uint32)), ("emit_pos", C.POINTER(C.c_uint32)),
        ("pair_off", C.POINTER(C.c_uint64)), ("pair_pos", C.POINTER(C.c_uint32)),
        ("pair_stage", C.POINTER(C.c_uint16)),
        ("err_code", C.POINTER(C.c_int32)), ("err_pos", C.POINTER(C.c_uint32)),
        ("run_steps", C.c_uint64), ("max_live_runs", C.c_uint64), ("max_nodes_key", C.c_uint64),
        ("total_puts", C.c_uint64), ("max_puts_key", C.c_uint64),
        ("elapsed_s", C.c_double), ("threads", C.c_int),
    ]


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = C.CDLL(_LIB_PATH)
        L.oracle_run.argtypes = [C.c_char_p, C.c_size_t, C.c_uint64, C.POINTER(C.c_uint64),
                                 C.POINTER(C.c_void_p), C.POINTER(C.c_int64), C.c_int,
                                 C.POINTER(C.POINTER(_Result))]
        L.oracle_run.restype = C.c_int
        L.oracle_free.argtypes = [C.POINTER(_Result)]
        L.oracle_last_error.restype = C.c_char_p
        L.oracle_compile_check.argtypes = [C.c_char_p, C.c_size_t]
        L.oracle_dewey_apply.argtypes = [C.c_char_p, C.c_char_p, C.c_char_p, C.c_size_t]
        L.oracle_dewey_compatible.argtypes = [C.c_char_p, C.c_char_p]
        L.oracle_buffer_new.restype = C.c_void_p
        L.oracle_buffer_free.argtypes = [C.c_void_p]
        L.oracle_buffer_put_begin.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int64, C.c_char_p]
        L.oracle_buffer_put.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int64, C.c_int, C.c_int,
                                        C.c_int64, C.c_char_p]
        L.oracle_buffer_peek.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int64, C.c_char_p, C.c_int,
                                         C.POINTER(C.c_int32), C.POINTER(C.c_int64), C.c_int]
        _lib = L
    return _lib


def compile_check(ir: bytes) -> int:
    return lib().oracle_compile_check(ir, len(ir))


def run(ir: bytes, key_off, cols, ts=None, threads: int = 1) -> dict:
    """One reference NFA per key over a CSR batch.  Returns numpy arrays (copied)."""
    L = lib()
    key_off = np.ascontiguousarray(key_off, dtype=np.uint64)
    cols = [np.ascontiguousarray(c) for c in cols]
    ptrs = (C.c_void_p * max(1, len(cols)))(*[c.ctypes.data for c in cols])
    tsp = None
    if ts is not None:
        ts = np.ascontiguousarray(ts, dtype=np.int64)
        tsp = ts.ctypes.data_as(C.POINTER(C.c_int64))
    res = C.POINTER(_Result)()
    rc = L.oracle_run(ir, len(ir), len(key_off) - 1, key_off.ctypes.data_as(C.POINTER(C.c_uint64)),
                      ptrs, tsp, threads, C.byref(res))
    if rc != 0:
        raise RuntimeError(f"oracle_run failed ({rc}): {L.oracle_last_error().decode()}")
    r = res.contents
    nm, npairs, nk = r.n_matches, r.n_pairs, r.n_keys

    def arr(p, n, dt):
        return np.ctypeslib.as_array(p, shape=(n,)).astype(dt, copy=True) if n else np.zeros(0, dt)

    out = {
        "n_matches": nm, "n_pairs": npairs,
        "key": arr(r.key, nm, np.uint32), "emit_pos": arr(r.emit_pos, nm, np.uint32),
        "pair_off": arr(r.pair_off, nm + 1, np.uint64),
        "pair_pos": arr(r.pair_pos, npairs, np.uint32), "pair_stage": arr(r.pair_stage, npairs, np.uint16),
        "err_code": arr(r.err_code, nk, np.int32), "err_pos": arr(r.err_pos, nk, np.uint32),
        "run_steps": r.run_steps, "max_live_runs": r.max_live_runs, "max_nodes_key": r.max_nodes_key,
        "total_puts": r.total_puts, "max_puts_key": r.max_puts_key,
        "elapsed_s": r.elapsed_s, "threads": r.threads,
    }
    L.oracle_free(res)
    return out


def dewey(version: str, ops: str = "") -> str:
    buf = C.create_string_buffer(256)
    lib().oracle_dewey_apply(version.encode(), ops.encode(), buf, 256)
    return buf.value.decode()


def dewey_compatible(a: str, b: str) -> bool:
    return bool(lib().oracle_dewey_compatible(a.encode(), b.encode()))


class Buffer:
    """Scripted KVSharedVersionedBuffer for test:nfa/buffer/SharedVersionedBufferTest.java."""

    def __init__(self):
        self.h = lib().oracle_buffer_new()

    def __del__(self):
        if getattr(self, "h", None):
            lib().oracle_buffer_free(self.h)

    def put_begin(self, name, typ, off, ver):
        return lib().oracle_buffer_put_begin(self.h, name, typ, off, ver.encode())

    def put(self, name, typ, off, pname, ptyp, poff, ver):
        return lib().oracle_buffer_put(self.h, name, typ, off, pname, ptyp, poff, ver.encode())

    def peek(self, name, typ, off, ver, remove=False):
        cap = 4096
        ns = (C.c_int32 * cap)()
        os_ = (C.c_int64 * cap)()
        n = lib().oracle_buffer_peek(self.h, name, typ, off, ver.encode(), int(remove), ns, os_, cap)
        if n < 0:
            raise RuntimeError(f"java exception {-n}")
        return [(ns[i], os_[i]) for i in range(n)]

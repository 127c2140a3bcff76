"""CPU build of the GPU JSON decoder's per-record state machine (csrc/json_parser.h) — test
infrastructure: tests/json_cpu/json_cpu.cpp drives the exact parser the kernel runs, record by
record, so `-m "not gpu"` tests check it against oracle/json_oracle.py."""
import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(os.path.dirname(HERE), "kafkastreams-cep_amd", "csrc")
_lib = None


def lib():
    global _lib
    if _lib is None:
        out = os.path.join(os.environ.get("TMPDIR", "/tmp"), "cep_json_cpu.so")
        subprocess.check_call(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-Wno-unknown-pragmas",
                               f"-I{CSRC}", os.path.join(HERE, "json_cpu", "json_cpu.cpp"), "-o", out])
        _lib = C.CDLL(out)
    return _lib


def pack(records):
    """Record values back to back (+ 8 bytes of padding either side) and u64 offsets."""
    off = np.zeros(len(records) + 1, np.uint64)
    if records:
        off[1:] = np.cumsum([len(r) for r in records])
    buf = np.zeros(int(off[-1]) + 16, np.uint8)
    buf[8:8 + int(off[-1])] = np.frombuffer(b"".join(records), np.uint8)
    return buf, off


def decode(records, col_width=8):
    buf, off = pack(records)
    n = len(records)
    price, vol = np.zeros(n, np.int64), np.zeros(n, np.int64)
    st, span = np.zeros(n, np.int32), np.zeros(2 * n, np.uint32)
    p = lambda a: a.ctypes.data_as(C.c_void_p)  # noqa: E731
    lib().json_cpu_decode(C.c_void_p(buf.ctypes.data + 8), p(off), C.c_uint64(n), C.c_int(col_width),
                          p(price), p(vol), p(st), p(span))
    return st, price, vol, span.reshape(-1, 2)


def oracle_arrays(results):
    """oracle/json_oracle.py results -> the decoder's output arrays."""
    st = np.array([r[0] for r in results], np.int32)
    price = np.array([r[1] for r in results], np.int64)
    vol = np.array([r[2] for r in results], np.int64)
    span = np.array([(0, 0xFFFFFFFF) if r[3] is None else (r[3][0], r[3][1] | (r[3][2] << 31)) for r in results],
                    np.uint32).reshape(-1, 2)
    return st, price, vol, span


def fast_path(record: bytes):
    """(takes the fast path, fast and general paths agree) for one record."""
    buf, _ = pack([record])
    ok = C.c_int()
    f = lib().json_cpu_fast_agrees(C.c_void_p(buf.ctypes.data + 8), C.c_uint32(len(record)), C.byref(ok))
    return bool(f), bool(ok.value)

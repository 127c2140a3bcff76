"""CPU build of a query's generated NFA kernel (test infrastructure, no GPU).

The JIT source libcep generates for a query (compile.cpp generate_jit, on csrc/nfa_lane.h)
is compiled as host C++ against tests/lane_cpu/hip/hip_runtime.h (stubs: one lane per
wave, sequential atomics) and driven by tests/lane_cpu/driver.cpp, which mirrors
session.cpp's run_nfa (pools, deferred-walk queues, retries with walks in place).  It runs
the exact lane code the GPU runs, key by key, so the per-event logic and the deferred-walk
machinery are checked against the oracle by `-m "not gpu"` tests; the GPU tests remain the
parity tests proper.
"""
import ctypes as C
import hashlib
import os
import re
import subprocess

import numpy as np

from kafkastreams_cep_amd import native as N

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(os.path.dirname(HERE), "kafkastreams-cep_amd", "csrc")
CLANG = "/opt/rocm/lib/llvm/bin/clang++"
BUILD = os.path.join(os.environ.get("TMPDIR", "/tmp"), "cep_lane_cpu")
_libs = {}


# session.cpp's stream build (cep_internal.h jit_stream_source; the lane driver keeps its own
# persistent-lane setting)
STREAM_PREFIX = ("#define CEP_DEWEY_PAIRS 3\n#define CEP_LAYOUT_PAIRS 6\n#define CEP_PUT_LOG 1\n"
                 "#define CEP_STREAM_STOP 1\n#define CEP_WALK_IN_PLACE 0\n#define CEP_WAVES_EU 3\n")


def build(ir: bytes, source: str | None = None, narrow: bool = False, stream: bool = False):
    """Compile the query's kernel (or a group's `source`) for the host; returns the loaded
    library (cached).  The wide Dewey build (6 pairs) unless `narrow` or `stream`: the driver
    re-runs jobs in the same build, while libcep re-runs the narrow build's overflowing jobs in
    the wide one; `stream`: the build libcep's streams run, its stopped keys continued by the
    wide build (loaded alongside)."""
    # the occupancy attribute is for the GPU compile only (the host has no kernels)
    src = re.sub(r"__attribute__\(\(amdgpu_waves_per_eu\(\w+\)\)\)", "", source or N.Query(ir).jit_source)
    if stream:
        src = STREAM_PREFIX + src
    elif narrow:
        # (this driver re-runs a narrow job's walk conflicts in the same build with walks in
        # place; libcep re-runs them in the wide build, so its narrow build leaves that path out)
        src = "#define CEP_WALK_IN_PLACE 1\n" + src
    else:
        src = "#define CEP_DEWEY_PAIRS 6\n" + src
    # $CEP_LANE_DEFINES="A=1 B=2": tuning knobs of nfa_lane.h for this build (tests of the knobs)
    src = "".join(f"#define {d.replace('=', ' ', 1)}\n" for d in os.environ.get("CEP_LANE_DEFINES", "").split()) + src
    deps = "".join(open(os.path.join(CSRC, h)).read() for h in
                   ("cep_layout.h", "kernel_args.h", "dewey.h", "java.h", "nfa_lane.h"))
    deps += open(os.path.join(HERE, "lane_cpu", "driver.cpp")).read()
    deps += open(os.path.join(HERE, "lane_cpu", "hip", "hip_runtime.h")).read()
    deps += open(os.path.join(HERE, "lane_cpu", "wave_emu.h")).read()
    key = hashlib.sha1((src + deps).encode()).hexdigest()[:16]
    if key in _libs:
        return _libs[key]
    os.makedirs(BUILD, exist_ok=True)
    qsrc = os.path.join(BUILD, f"q_{key}.hip")
    so = os.path.join(BUILD, f"lane_{key}.so")
    if not os.path.exists(so):
        with open(qsrc, "w") as f:
            f.write(src)
        tmp = so + f".{os.getpid()}"
        subprocess.check_call([CLANG, "-x", "c++", "-std=c++17", "-O1", "-g", "-rdynamic", "-shared", "-fPIC",
                               "-ffp-contract=off", "-Wno-unused-value", "-w", "-DCEP_LANE_STATS", "-DCEP_PERSIST_LANES=1",
                               f"-I{os.path.join(HERE, 'lane_cpu')}", f"-I{CSRC}",
                               f'-DQUERY_SRC="{qsrc}"', os.path.join(HERE, "lane_cpu", "driver.cpp"),
                               "-o", tmp])
        os.replace(tmp, so)
    lib = C.CDLL(so)
    lib.lane_run.argtypes = [C.c_uint64, C.c_void_p, C.POINTER(C.c_void_p), C.c_int, C.c_void_p,
                             C.c_uint32, C.c_int, C.POINTER(C.c_uint32), C.c_int, C.c_int, C.c_uint32, C.c_void_p]
    lib.lane_n_matches.restype = C.c_uint64
    lib.lane_n_pairs.restype = C.c_uint64
    lib.lane_fetch.argtypes = [C.c_void_p] * 7
    lib.lane_widened.restype = C.c_uint64
    lib.lane_set_continuation.argtypes = [C.c_void_p]
    if stream:
        wide = build(ir, source)
        lib.lane_set_continuation(C.cast(wide.lane_continue, C.c_void_p).value)
        lib._wide = wide
    _libs[key] = lib
    return lib


def run(ir, key_off, cols, rcap=32, defer=True, streaming=False, reset=True, bits=True, _group=None, ts=None,
        narrow=False, wide_stream=False):
    """Same result dict as tests/gpu_helpers.gpu_run (minus the device digest).  streaming:
    the batch continues the keys' streams of the previous streaming call (reset=False), on the
    build libcep's streams run (the stream build when the query's versions fit it, unless
    wide_stream).  bits: quiet lanes use the begin-hit bitmap (as on the GPU) instead of the
    chunked scan."""
    stream = streaming and not narrow and not wide_stream and not _group
    lib = build(ir, _group["source"] if _group else None, narrow=narrow, stream=stream)
    n_q = len(_group["members"]) if _group else 1
    kc = np.ascontiguousarray(_group["literals"], np.int64) if _group else None
    if streaming and reset:
        lib.lane_stream_reset()
    key_off = np.ascontiguousarray(key_off, np.uint64)
    cols = [np.ascontiguousarray(c) for c in cols]
    ptrs = (C.c_void_p * max(1, len(cols)))(*[c.ctypes.data for c in cols])
    nk = len(key_off) - 1
    retried = C.c_uint32()
    ts = None if ts is None else np.ascontiguousarray(ts, np.int64)
    lib.lane_run(nk, key_off.ctypes.data, ptrs, len(cols), None if ts is None else ts.ctypes.data, rcap, 1 if defer else 0, C.byref(retried),
                 1 if streaming else 0, 1 if bits else 0, n_q, kc.ctypes.data if kc is not None and kc.size else None)
    nm, npairs = lib.lane_n_matches(), lib.lane_n_pairs()
    key = np.zeros(nm, np.uint32)
    emit = np.zeros(nm, np.uint32)
    off = np.zeros(nm + 1, np.uint64)
    seq = np.zeros(npairs, np.uint32)
    stage = np.zeros(npairs, np.uint16)
    err = np.zeros(nk * n_q, np.int32)
    err_seq = np.zeros(nk * n_q, np.uint32)
    lib.lane_fetch(*[a.ctypes.data for a in (key, emit, off, seq, stage, err, err_seq)])
    m = {"n_matches": nm, "n_pairs": npairs, "key": key, "emit_seq": emit, "pair_off": off,
         "pair_seq": seq, "pair_stage": stage, "err_code": err, "err_seq": err_seq,
         "retried": retried.value, "bits_used": bool(lib.lane_bits_used()), "widened": lib.lane_widened()}
    st = (C.c_uint64 * 10)()
    lib.lane_stats(st)
    m["stats"] = dict(zip(("events", "records", "walks", "walk_nodes", "pred_scans", "flushes", "chain_steps",
                           "flush_iters", "exact_conflicts", "twin_writes_saved"), list(st)))
    hops = (C.c_uint64 * 4)()
    lib.lane_hop_stats(hops)
    m["stats"].update(zip(("hops_branch", "hops_emit", "hops_emit_retrace", "hops_remove"), list(hops)))
    if _group:
        return m
    m["emit_pos"] = (key_off[key.astype(np.int64)] + emit).astype(np.uint64)
    pk = np.repeat(key.astype(np.int64), np.diff(off.astype(np.int64)))
    m["pair_pos"] = (key_off[pk] + seq).astype(np.uint64)
    return m


def run_group(irs, key_off, cols, **kw):
    """The kernel groups a session over `irs` would launch (cep_query_group_plan), each run as
    one job grid (query, key); returns one result dict per query, as run() would."""
    key_off = np.ascontiguousarray(key_off, np.uint64)
    nk = len(key_off) - 1
    res = [None] * len(irs)
    for g in N.group_plans([N.Query(ir) for ir in irs]):
        m = run(irs[g["members"][0]], key_off, cols, _group=g, **kw)
        job = m["key"].astype(np.int64)
        lens = np.diff(m["pair_off"].astype(np.int64))
        for qi, q in enumerate(g["members"]):
            sel = (job // nk) == qi
            psel = np.repeat(sel, lens)
            key = (job[sel] % nk).astype(np.uint32)
            off = np.zeros(int(sel.sum()) + 1, np.uint64)
            np.cumsum(lens[sel], out=off[1:])
            r = {"n_matches": int(sel.sum()), "n_pairs": int(psel.sum()), "key": key, "emit_seq": m["emit_seq"][sel],
                 "pair_off": off, "pair_seq": m["pair_seq"][psel], "pair_stage": m["pair_stage"][psel],
                 "err_code": m["err_code"][qi * nk:(qi + 1) * nk], "err_seq": m["err_seq"][qi * nk:(qi + 1) * nk],
                 "n_group": len(g["members"])}
            r["emit_pos"] = (key_off[key.astype(np.int64)] + r["emit_seq"]).astype(np.uint64)
            pk = np.repeat(key.astype(np.int64), lens[sel])
            r["pair_pos"] = (key_off[pk] + r["pair_seq"]).astype(np.uint64)
            res[q] = r
    return res


def assert_same(g, r, key_off):
    """lane result `g` equals oracle result `r` exactly (as gpu_helpers.assert_parity, no digest)."""
    assert g["n_matches"] == r["n_matches"], (g["n_matches"], r["n_matches"])
    assert g["n_pairs"] == r["n_pairs"]
    np.testing.assert_array_equal(g["key"], r["key"])
    np.testing.assert_array_equal(g["emit_pos"], r["emit_pos"].astype(np.uint64))
    np.testing.assert_array_equal(g["pair_off"], r["pair_off"])
    np.testing.assert_array_equal(g["pair_pos"], r["pair_pos"].astype(np.uint64))
    np.testing.assert_array_equal(g["pair_stage"], r["pair_stage"])
    np.testing.assert_array_equal(g["err_code"], r["err_code"])
    off = np.asarray(key_off, np.uint64)
    bad = r["err_code"] != 0
    np.testing.assert_array_equal(g["err_seq"][bad].astype(np.uint64) + off[:-1][bad],
                                  r["err_pos"][bad].astype(np.uint64))

"""CPU-side checks of the C-ABI boundary (no GPU calls): libcep.so loads, exports every
symbol include/cep.h declares, and its host query compiler agrees with the reference's
StatesFactory rules (stage counts, kernel choice, compile-time exceptions)."""
import os
import re

import pytest

import oracle
from kafkastreams_cep_amd import EventSchema, QueryBuilder
from kafkastreams_cep_amd import native as N
from kafkastreams_cep_amd import workloads as W

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions(header="cep.h"):
    src = open(os.path.join(ROOT, "include", header)).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(cep_[a-z_]+)\s*\(", src)))


def test_header_exports_match_binding():
    assert header_functions() == sorted(N.EXPORTS)
    assert header_functions("cep_synth.h") == sorted(N.SYNTH_EXPORTS)


def test_library_exports_every_declared_symbol():
    L = N.lib()
    for name in header_functions():
        assert hasattr(L, name), name
    G = N.synth_lib()
    for name in header_functions("cep_synth.h"):
        assert hasattr(G, name), name


def test_matcher_library_carries_no_generators():
    """the synthetic generators (and their hipCUB sorts/scans) live in libcep_synth.so only"""
    import subprocess
    syms = subprocess.run(["nm", "-D", "-C", N.LIB_PATH], capture_output=True, text=True, check=True).stdout
    assert "cep_synth" not in syms and "hipcub" not in syms.lower() and "rocprim" not in syms.lower()


def test_compile_kinds():
    q = N.Query(W.stock_query("readme").to_ir())
    assert q.kind == N.CEP_KIND_NFA
    # $final, R2, R1 (loop), W1 (wrapper), R0
    assert q.info.n_stages == 5 and q.info.n_patterns == 3 and q.info.n_states == 2
    assert q.stage_names == ["0", "1", "2", "$final"]
    q = N.Query(W.stock_query("test").to_ir())
    assert q.kind == N.CEP_KIND_NFA and q.info.n_stages == 4
    s = N.Query(W.strict_abc_query().to_ir())
    assert s.kind == N.CEP_KIND_STENCIL and s.info.arity == 3


def strict_chain(n):
    """SEQ(S0..S{n-1}) all ONE + strict, S_i: v % 4 == i % 4 (total, state-free)."""
    S = EventSchema({"v": "int"})
    b = QueryBuilder(S)
    for i in range(n):
        sel = b.select(f"S{i}").where(lambda k, v, ts, s, i=i: v.v % 4 == i % 4)
        b = sel.then() if i < n - 1 else sel
    return b.build()


@pytest.mark.parametrize("n,kind", [(8, N.CEP_KIND_STENCIL), (9, N.CEP_KIND_NFA), (12, N.CEP_KIND_NFA)])
def test_stencil_gate_stage_limit(n, kind):
    """The stencil kernels are instantiated for at most 8 stages: a longer strict chain is
    compiled for the NFA kernel (it would otherwise fail at every push)."""
    q = N.Query(strict_chain(n).to_ir())
    assert q.kind == kind and q.info.n_patterns == n


def _pred(k, v, ts, s):
    return v.price > 1


def test_compile_errors_match_reference():
    S = EventSchema({"price": "int"})
    # pattern ending in a Kleene stage: StatesFactory.java:102-104 -> NullPointerException
    q = QueryBuilder(S).select().where(_pred).then().select().oneOrMore().where(_pred).build()
    ir = q.to_ir()
    assert oracle.compile_check(ir) == 1
    assert N.Query(ir).info.compile_error == 1
    # a pattern without where(): Stage.java:159 -> IllegalArgumentException
    p = QueryBuilder(S).select().where(_pred).then()
    ir = p.to_ir()
    assert oracle.compile_check(ir) == 4
    assert N.Query(ir).info.compile_error == 4
    with pytest.raises(N.CepError):
        N.Session(N.Query(ir))


def test_bad_ir_is_rejected():
    with pytest.raises(N.CepError):
        N.Query(b"CEPQ\x02\x00\x00\x00")
    with pytest.raises(N.CepError):
        N.Query(W.stock_query().to_ir() + b"\x00")


def test_launch_path_reads_no_environment():
    """The measurement knobs ($CEP_*) are read in one place, tuning.cpp, when a session is
    created (and compile.cpp / jit.cpp at query compile); no source of the launch path (the
    session's push/run code, the kernels' host launchers) calls getenv."""
    csrc = os.path.join(ROOT, "kafkastreams-cep_amd", "csrc")
    allowed = {"tuning.cpp", "compile.cpp", "jit.cpp"}
    for f in sorted(os.listdir(csrc)):
        if f.endswith((".cpp", ".hip", ".h")) and f not in allowed:
            src = re.sub(r"//.*", "", open(os.path.join(csrc, f)).read())
            assert "getenv" not in src, f
    ses = open(os.path.join(csrc, "session.cpp")).read()
    assert "tuning_from_env()" in ses and ses.count("tuning_from_env") == 1


def _release_getenv_calls(src: str) -> list:
    """getenv("...") names outside `#ifdef CEP_MEASURE` regions (nested #if blocks tracked)"""
    names, stack = [], []
    for line in src.splitlines():
        t = line.strip()
        if t.startswith("#if"):
            stack.append(t == "#ifdef CEP_MEASURE")
        elif t.startswith("#else") and stack:
            stack[-1] = False if stack[-1] else stack[-1]
        elif t.startswith("#endif") and stack:
            stack.pop()
        elif not any(stack):
            code = re.sub(r"//.*", "", line)
            names += re.findall(r'getenv\(\s*("?[A-Za-z_]*"?)', code)
    return names


def test_release_build_reads_only_jit_cache():
    """ The release libcep.so reads one environment variable,
    $CEP_JIT_CACHE: every tuning knob is compiled in only under CEP_MEASURE (the measurement
    build, libcep_measure.so); and a knob set in the environment changes nothing the release
    build generates."""
    csrc = os.path.join(ROOT, "kafkastreams-cep_amd", "csrc")
    found = []
    for f in sorted(os.listdir(csrc)):
        if f.endswith((".cpp", ".hip", ".h")):
            found += [(f, n) for n in _release_getenv_calls(open(os.path.join(csrc, f)).read())]
    assert found == [("jit.cpp", '"CEP_JIT_CACHE"')], found
    ir = W.stock_query("readme").to_ir()
    base = N.Query(ir).jit_source
    env = {"CEP_WALK_FLUSH": "7", "CEP_PROF": "1", "CEP_DEWEY_PAIRS": "5", "CEP_JIT_WAVES": "4", "CEP_RING_LDS": "1"}
    saved = {k: os.environ.get(k) for k in env}
    try:
        os.environ.update(env)
        assert N.Query(ir).jit_source == base
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v

def test_no_stream_ordered_or_null_stream_allocation():
    """ The library allocates device memory with hipMalloc only - no
    stream-ordered pool (hipMallocAsync / hipFreeAsync) anywhere - and the session paths copy on
    the session's own stream (no null-stream hipMemcpy outside cep_memcpy, which waits for the
    device first)."""
    import subprocess
    so = os.path.join(ROOT, "kafkastreams-cep_amd", "libcep.so")
    syms = subprocess.run(["nm", "-D", "--undefined-only", so], capture_output=True, text=True, check=True).stdout
    for bad in ("hipMallocAsync", "hipFreeAsync", "hipMallocFromPoolAsync", "hipMemPool"):
        assert bad not in syms, bad
    csrc = os.path.join(ROOT, "kafkastreams-cep_amd", "csrc")
    ses = re.sub(r"//.*", "", open(os.path.join(csrc, "session.cpp")).read())
    assert len(re.findall(r"hipMemcpy\(", ses)) == 1  # cep_memcpy's, after hipDeviceSynchronize
    assert "hipDeviceSynchronize());\n    HIPCHECK(hipMemcpy(dst, src, bytes, k))" in ses

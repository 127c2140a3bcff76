"""Fills the JIT code-object cache for every NFA query the GPU tests, smoke() and bench.py
run (hipRTC needs no GPU), so a fresh GPU box loads them instead of compiling.
Usage: python tests/precompile_jit.py [--bench-only]"""
import os
import sys
import time
from concurrent.futures import ProcessPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]


def _irs(bench_only):
    import cepamd  # noqa: F401
    from kafkastreams_cep_amd import workloads as W

    irs = [W.stock_query(v).to_ir() for v in ("readme", "test", "demo")]
    irs += [W.strict_abc_query().to_ir(), W.any_kleene_query().to_ir(), W.any_kleene_query(carry_volume=True).to_ir()]
    irs += [p.to_ir() for p in W.multi_queries(64)]  # bench.py other_configs (cfg 5); tests use the first 8
    # semantic WITHIN (tests/test_semantic_within.py, bench.py semantic figure)
    irs += [q.to_ir(semantic_within=True) for q in (W.stock_query("readme"), W.stock_query("test"),
                                                     W.any_kleene_query())]
    if bench_only:
        return irs
    from fuzz_queries import random_query
    from ref_queries import STRING_KATS, build_case, kats

    for name, case in kats().items():
        if name in STRING_KATS:
            irs.append(build_case(name, case)[0].to_ir())
    from test_gpu_parity import FUZZ_JIT_SEEDS  # the interpreter-tier seeds need no JIT kernel
    from test_processor import arith_query
    irs.append(arith_query().to_ir())
    irs += [random_query(s).to_ir() for s in FUZZ_JIT_SEEDS]
    return irs


def _group_sets():
    """query sets whose kernel groups the tests and bench.py launch (cep_jit_precompile_group)"""
    import cepamd  # noqa: F401
    from kafkastreams_cep_amd import workloads as W

    mq = W.multi_queries(64)
    mixed = [W.stock_query("readme", begin_volume=1000), W.any_kleene_query(),
             W.stock_query("readme", begin_volume=1005), W.stock_query("test"), W.stock_query("readme", dip_num=90)]
    return [[p.to_ir() for p in mq], [p.to_ir() for p in mq[48:]], [p.to_ir() for p in mq[60:]],
            [p.to_ir() for p in mixed], [p.to_ir(semantic_within=True) for p in mq[:16]]]


def _compile_group(irs):
    import cepamd  # noqa: F401
    from kafkastreams_cep_amd import native as N

    return N.precompile_group([N.Query(ir) for ir in irs])


def _compile(ir):
    import cepamd  # noqa: F401
    from kafkastreams_cep_amd import native as N

    q = N.Query(ir)
    if q.info.compile_error:
        return 0.0
    return q.precompile()


def main(bench_only=False, workers=None):
    irs = _irs(bench_only)
    t = time.time()
    # (cep_jit_precompile*: a cache hit refreshes its entry's mtime, jit.cpp)
    with ProcessPoolExecutor(workers or min(8, os.cpu_count() or 1)) as ex:
        spent = list(ex.map(_compile, irs)) + list(ex.map(_compile_group, _group_sets()))
    pruned = 0
    if not bench_only:  # entries no current query maps to (an older kernel source): dropped
        cache = os.path.join(ROOT, "kafkastreams-cep_amd", "jit_cache")
        for f in os.listdir(cache) if os.path.isdir(cache) else []:
            p = os.path.join(cache, f)
            if f.endswith(".co") and os.path.getmtime(p) < t - 1:
                os.remove(p)
                pruned += 1
    print(f"jit cache: {len(irs)} queries, {sum(1 for s in spent if s > 0)} compiled, {pruned} stale entries "
          f"dropped, {time.time() - t:.1f}s")


if __name__ == "__main__":
    main("--bench-only" in sys.argv)

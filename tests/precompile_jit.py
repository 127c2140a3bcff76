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
    irs += [W.strict_abc_query().to_ir(), W.any_kleene_query().to_ir()]
    irs += [p.to_ir() for p in W.multi_queries(64)]  # bench.py other_configs (cfg 5); tests use the first 8
    if bench_only:
        return irs
    from fuzz_queries import random_query
    from ref_queries import STRING_KATS, build_case, kats

    for name, case in kats().items():
        if name in STRING_KATS:
            irs.append(build_case(name, case)[0].to_ir())
    irs += [random_query(s).to_ir() for s in range(0, 160)]
    return irs


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
    with ProcessPoolExecutor(workers or min(8, os.cpu_count() or 1)) as ex:
        spent = list(ex.map(_compile, irs))
    print(f"jit cache: {len(irs)} queries, {sum(1 for s in spent if s > 0)} compiled, {time.time() - t:.1f}s")


if __name__ == "__main__":
    main("--bench-only" in sys.argv)

import sys; sys.path[:0]=['.','oracle','tests']
import cepamd, numpy as np, oracle
from fuzz_queries import random_query, random_stream
from kafkastreams_cep_amd import native as N
seed=13; q=random_query(seed); ir=q.to_ir(); off, cols = random_stream(seed, 60, 14)
r=oracle.run(ir,off,cols)
for tier in (1, 0):
    for mr in (0, 4096):
        s=N.Session(N.Query(ir), tier=tier, max_runs=mr); s.push(off, cols)
        m=s.matches(0); code,_=s.key_errors(0)
        print('tier',tier,'max_runs',mr, m['n_matches'], r['n_matches'], 'errs', np.bincount(code), 'oracle errs', np.bincount(r['err_code']), s.stats(0))

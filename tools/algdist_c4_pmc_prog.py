"""Program profiled by the r04 alg-dist counter passes (rocprofv3 --pmc):
the random-row gather probe (64-B rows from a 610 MB table, 8 in flight:
a known byte pattern to calibrate FETCH_SIZE for random 16-B-per-lane
gathers) and 2 iterations of the C4 alg-dist relaxation with the shipped
64-B rows. `python tools/algdist_c4_pmc_prog.py`"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hypergraphembedding_amd import _hgx  # noqa: E402
from hypergraphembedding_amd.synthetic import powerlaw_hypergraph  # noqa: E402

inc = powerlaw_hypergraph()
ctx = _hgx.Context(0)
rate = ctx.probe_gather(610 << 20, 16, 8, 1)
print(f"probe {rate / 1e9:.2f} G rows/s; rows per launch {2**28}", flush=True)
ctx.upload(inc)
rs = np.random.RandomState(0)
ctx.alg_set(rs.random_sample((inc.N, 10)).astype(np.float32),
            rs.random_sample((inc.E, 10)).astype(np.float32))
ctx.alg_run(2)
ms, by = ctx.alg_stats()
print(f"alg-dist 2 it: {ms:.2f} ms, nnz {inc.nnz}", flush=True)
ctx.close()

"""Measurements of the widened rows, one MI355X:
  * native hypergraph.proto reader on the C4 graph (2e8 incidences, > 2 GiB,
    beyond Python protobuf) and, on a C3-size message, against Python
    protobuf + Incidence.from_hypergraph;
  * weighted-Jaccard sampling at C3 (UniformWeight, S=200, K=5) and its
    probability kernel against the CPU oracle on the same pairs.
Writes the JSON to argv[1] (default gpurun_out/widened.json)."""
import json, os, sys, time
import numpy as np
sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle")]
from hypergraphembedding_amd import _hgx, Hypergraph, Incidence
from hypergraphembedding_amd.proto_native import read_incidence
from hypergraphembedding_amd.synthetic import powerlaw_hypergraph, random_hypergraph
import oracle as O

out_path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/widened.json"
res = {}
# ---- proto reader, C4 ----
big = powerlaw_hypergraph(seed=0)
t = time.perf_counter()
buf = _hgx.write_hypergraph_bytes(big)
tw = time.perf_counter() - t
t = time.perf_counter()
inc = read_incidence(buf)
tr = time.perf_counter() - t
assert inc.nnz == big.nnz and np.array_equal(inc.col_n, big.col_n)
res["proto_c4"] = {"bytes": int(buf.size), "nnz": big.nnz, "write_s": round(tw, 2),
                   "parse_s": round(tr, 2),
                   "parse_mb_per_s": round(buf.size / tr / 1e6, 1),
                   "parse_incidences_per_s": round(big.nnz / tr, 1),
                   "cores": "min(16, hardware_concurrency) threads"}
del buf, inc, big
# ---- proto reader vs Python protobuf, C3 ----
c3 = random_hypergraph(seed=0)
buf = _hgx.write_hypergraph_bytes(c3).tobytes()
t = time.perf_counter()
hg = Hypergraph()
hg.ParseFromString(buf)
py_inc = Incidence.from_hypergraph(hg)
tp = time.perf_counter() - t
t = time.perf_counter()
nat = read_incidence(buf)
tn = time.perf_counter() - t
assert np.array_equal(nat.col_n, py_inc.col_n)
res["proto_c3"] = {"bytes": len(buf), "nnz": c3.nnz, "python_protobuf_s": round(tp, 3),
                   "native_s": round(tn, 3), "speedup": round(tp / tn, 1)}
# ---- weighted-Jaccard sampling, C3 ----
ctx = _hgx.Context(0)
ctx.upload(c3)
fn, fe = ctx.incidence_weights(_hgx.WEIGHT_UNIFORM, 0.0)
ctx.features_set(fn, fe)
q_n = np.full(c3.N, 200, np.int32)
q_e = np.full(c3.E, 200, np.int32)
ctx.sample_jaccard(1, 5, q_n, q_e)  # warm (builds the centroids)
ctx.features_set(fn, fe)  # drop the centroids: time them too
ctx.synchronize()
t = time.perf_counter()
n = ctx.sample_jaccard(2, 5, q_n, q_e)
ctx.synchronize()
ts = time.perf_counter() - t
idx, tgt = ctx.records_get()
ne = (idx[:, 0] > 0) & (idx[:, 3] > 0) & (idx[:, 2] == 0)
sel = np.flatnonzero(ne)[np.random.RandomState(0).permutation(int(ne.sum()))[:20000]]
v, e = idx[sel, 0] - 1, idx[sel, 3] - 1
ctx.jaccard_probs(2, v, e)  # warm
t = time.perf_counter()
pg = ctx.jaccard_probs(2, v, e)
tg = time.perf_counter() - t
t = time.perf_counter()
pc = O.jaccard_probs(2, v, e, c3, fn, fe)
tc = time.perf_counter() - t
assert np.array_equal(pg, pc)
res["jaccard_c3"] = {"records": n, "sampling_s_incl_centroids": round(ts, 3),
                     "records_per_s": round(n / ts, 1),
                     "ne_prob_pairs": int(sel.size),
                     "gpu_ne_probs_per_s_incl_pcie": round(sel.size / tg, 1),
                     "cpu_oracle_ne_probs_per_s": round(sel.size / tc, 1),
                     "cpu_oracle_note": "oracle/hgref.c, single thread, includes "
                                        "building both centroid matrices"}
json.dump(res, open(out_path, "w"), indent=1)
print(json.dumps(res, indent=1))

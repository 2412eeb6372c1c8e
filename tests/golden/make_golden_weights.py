#!/usr/bin/env python3
"""Golden fixtures for the hg2v_weighting distance / span weights, made by
RUNNING THE REFERENCE (build container only; needs /root/reference):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_weights.py

weights_dist.npz holds, per case, the scipy CSR (indptr, indices, data after
sort_indices) the reference returns:
  * WeightByDistance (hg2v_weighting.py:67-103): node2edge / edge2node, with
    norm = np.linalg.norm, on youtube_tiny with its 10-d alg-dist coordinates
    (algdist_tiny.npz x_20 / y_20, the reference's own float32 output) at
    alpha 0 and 0.3, and on a small random graph with a 40-d embedding
    (OpenBLAS sdot's vector kernel, n >= 32) at alpha 0;
  * WeightBySameTypeDistance (:34-64): node2node / edge2edge on the same
    cases;
  * ComputeSpans (:236-293) with a given embedding: node / edge spans;
  * WeightByAlgebraicSpan (:170-192) with ComputeSpans bound to that
    embedding (the default computes a random 5-d alg-dist first);
  * ComputeSpans with its default embedding under np.random.seed(9) on the
    small graph (tolerance fixture: the reference relaxes in float64).
Only data is written; nothing of the reference is copied.
"""

import functools
import hashlib
import os
import random
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import refload  # noqa: E402

ref = refload.load()
hu = ref.hypergraph_util
W = ref.hg2v_weighting
from hypergraphembedding_amd.proto import Hypergraph, HypergraphEmbedding  # noqa: E402


def emb_from(node_ids, X, edge_ids, Y):
  e = HypergraphEmbedding()
  e.dim = X.shape[1]
  for i, v in zip(node_ids.tolist(), X):
    e.node[int(i)].values.extend(v.tolist())
  for i, v in zip(edge_ids.tolist(), Y):
    e.edge[int(i)].values.extend(v.tolist())
  return e


def digest(*arrays):
  h = hashlib.sha256()
  for a in arrays:
    h.update(np.ascontiguousarray(a).tobytes())
  return h.hexdigest()


def put(out, key, m):
  """The CSR in full; past 200k entries (youtube_tiny's A A^T: 5.7M) its
  sha256 plus every entry of each 97th row instead."""
  m = m.tocsr()
  m.sort_indices()
  ip = m.indptr.astype(np.int64)
  ix = m.indices.astype(np.int32)
  dv = np.asarray(m.data, np.float32)
  out[f"{key}_shape"] = np.array(m.shape, np.int64)
  if ix.size <= 200_000:
    out[f"{key}_indptr"], out[f"{key}_indices"], out[f"{key}_data"] = ip, ix, dv
    return
  out[f"{key}_sha"] = np.array(digest(ip, ix, dv))
  rows = np.arange(0, m.shape[0], 97)
  rows = rows[ip[rows + 1] > ip[rows]]
  sel = np.concatenate([np.arange(ip[r], ip[r + 1]) for r in rows])
  out[f"{key}_sample_rows"] = rows
  out[f"{key}_sample_cols"] = ix[sel]
  out[f"{key}_sample_data"] = dv[sel]
  out[f"{key}_nnz"] = np.int64(ix.size)


def spans(out, key, hg, emb):
  ns, es = W.ComputeSpans(hg, embedding=emb, run_in_parallel=False,
                          disable_pbar=True)
  out[f"{key}_node_span"] = np.array([ns[i] for i in sorted(hg.node)], np.float64)
  out[f"{key}_edge_span"] = np.array([es[i] for i in sorted(hg.edge)], np.float64)


def main():
  out = {}
  tiny = Hypergraph()
  with open(os.path.join(HERE, "snap_youtube_tiny.hypergraph.pb"), "rb") as f:
    tiny.ParseFromString(f.read())
  csr = np.load(os.path.join(HERE, "csr_tiny.npz"))
  alg = np.load(os.path.join(HERE, "algdist_tiny.npz"))
  emb_tiny = emb_from(csr["node_ids"], alg["x_20"], csr["edge_ids"], alg["y_20"])

  random.seed(11)
  small = hu.CreateRandomHyperGraph(150, 50, 0.05)
  rs = np.random.RandomState(3)
  nid = np.array(sorted(small.node), np.int64)
  eid = np.array(sorted(small.edge), np.int64)
  X40 = rs.standard_normal((nid.size, 40)).astype(np.float32)
  Y40 = rs.standard_normal((eid.size, 40)).astype(np.float32)
  emb_small = emb_from(nid, X40, eid, Y40)
  X5 = rs.uniform(0, 1, (nid.size, 5)).astype(np.float32)
  Y5 = rs.uniform(0, 1, (eid.size, 5)).astype(np.float32)
  emb_small5 = emb_from(nid, X5, eid, Y5)
  with open(os.path.join(HERE, "weights_small_graph.pb"), "wb") as f:
    f.write(small.SerializeToString())
  out["small_X40"], out["small_Y40"] = X40, Y40
  out["small_X5"], out["small_Y5"] = X5, Y5

  cases = [("tiny_a0", tiny, emb_tiny, 0), ("tiny_a3", tiny, emb_tiny, 0.3),
           ("small40_a0", small, emb_small, 0)]
  for key, hg, emb, alpha in cases:
    n2e, e2n = W.WeightByDistance(hg, alpha, emb, np.linalg.norm, True)
    put(out, f"{key}_dist_n", n2e)
    put(out, f"{key}_dist_e", e2n)
    n2n, e2e = W.WeightBySameTypeDistance(hg, alpha, emb, np.linalg.norm, True)
    put(out, f"{key}_same_n", n2n)
    put(out, f"{key}_same_e", e2e)
    print(key, "done", n2e.nnz, n2n.nnz, e2e.nnz, flush=True)

  # spans with a given embedding, and WeightByAlgebraicSpan over them
  orig = W.ComputeSpans
  for key, hg, emb, alpha in (("tiny_a0", tiny, emb_tiny, 0),
                              ("small5_a3", small, emb_small5, 0.3)):
    spans(out, key, hg, emb)
    W.ComputeSpans = functools.partial(orig, embedding=emb,
                                       run_in_parallel=False,
                                       disable_pbar=True)
    try:
      n2w, e2w = W.WeightByAlgebraicSpan(hg, alpha)
    finally:
      W.ComputeSpans = orig
    put(out, f"{key}_span_n", n2w)
    put(out, f"{key}_span_e", e2w)
  # the default embedding (5-d alg-dist, 10 iterations) under a seed
  np.random.seed(9)
  ns, es = W.ComputeSpans(small, run_in_parallel=False, disable_pbar=True)
  out["small_default_node_span"] = np.array([ns[i] for i in sorted(small.node)])
  out["small_default_edge_span"] = np.array([es[i] for i in sorted(small.edge)])
  out["small_default_seed"] = np.int64(9)
  np.savez_compressed(os.path.join(HERE, "weights_dist.npz"), **out)
  print("wrote weights_dist.npz")


if __name__ == "__main__":
  main()

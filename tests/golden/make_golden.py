#!/usr/bin/env python3
"""Generate the golden fixtures in tests/golden/ by RUNNING THE REFERENCE.

Runs only in the build container (needs /root/reference); the outputs are
plain data (.npz / .pb) that travel with the repo. Usage:

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

What is pinned:
  * snap_youtube_tiny.hypergraph.pb  -- the reference's own test data file,
    copied verbatim (data, not source).
  * csr_*.npz        -- ToCsrMatrix/ToEdgeCsrMatrix(CompressRange(hg)).
  * algdist_*.npz    -- EmbedAlgebraicDistance(seed, k, iters) outputs
    (float32 proto values) + the seed.
  * fobe_*.npz       -- BooleanSamples -> SamplesToModelInput arrays under
    np.random.seed; youtube_tiny stored as sha256 + head rows (724 792 recs).
  * hobe_*.npz       -- AlgebraicDistanceSamples(run_in_parallel=False).
  * probs_tiny.npz   -- HOBE nn/ee/ne probabilities for fixed pair lists.
  * weights_small.npz -- UniformWeight / WeightByNeighborhood CSR values.
"""

import hashlib
import os
import random
import shutil
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import refload  # noqa: E402

ref = refload.load()
hu = ref.hypergraph_util
from hypergraphembedding_amd.proto import Hypergraph  # noqa: E402

TINY_PB = "/root/reference/test_data/snap_youtube_tiny.hypergraph.pb"


def sha(*arrays):
  h = hashlib.sha256()
  for a in arrays:
    h.update(np.ascontiguousarray(a).tobytes())
  return h.hexdigest()


def csr_of(hg):
  c, inv_n, inv_e = hu.CompressRange(hg)
  a = hu.ToCsrMatrix(c)
  at = hu.ToEdgeCsrMatrix(c)
  n_ids = np.array([inv_n[i] for i in range(len(inv_n))], np.int64)
  e_ids = np.array([inv_e[i] for i in range(len(inv_e))], np.int64)
  return c, dict(N=len(c.node), E=len(c.edge), rp_n=a.indptr.astype(np.int32),
                 col_n=a.indices.astype(np.int32),
                 rp_e=at.indptr.astype(np.int32),
                 col_e=at.indices.astype(np.int32), node_ids=n_ids,
                 edge_ids=e_ids)


def emb_arrays(emb, csr):
  """Embedding proto (keyed by ORIGINAL ids) -> compressed-order arrays."""
  X = np.array([emb.node[int(i)].values for i in csr["node_ids"]], np.float32)
  Y = np.array([emb.edge[int(i)].values for i in csr["edge_ids"]], np.float32)
  return X, Y


def model_input(recs, K):
  feat, tg = ref.hg2v_sample.SamplesToModelInput(recs, K, weighted=False)
  F = np.array(feat, dtype=np.int64).T.astype(np.int32)
  T = np.array(tg, dtype=np.float64).T.astype(np.float32)
  return F, T


def random_hg(seed, n, e, p):
  random.seed(seed)
  return hu.CreateRandomHyperGraph(n, e, p)


def main():
  out = HERE
  shutil.copyfile(TINY_PB, os.path.join(out, "snap_youtube_tiny.hypergraph.pb"))
  tiny = Hypergraph()
  with open(TINY_PB, "rb") as f:
    tiny.ParseFromString(f.read())
  tiny_c, tiny_csr = csr_of(tiny)
  np.savez_compressed(os.path.join(out, "csr_tiny.npz"), **tiny_csr)

  small = random_hg(1, 120, 40, 0.06)
  small_c, small_csr = csr_of(small)
  np.savez_compressed(os.path.join(out, "csr_small.npz"), **small_csr)

  # reference test graph (tests/test_embedding.py:14-22)
  th = Hypergraph()
  for n, e in [(0, 0), (1, 0), (1, 1), (2, 1), (2, 2), (3, 2)]:
    hu.AddNodeToEdge(th, n, e)
  th_c, th_csr = csr_of(th)

  # ---- algebraic distance ----
  AD = ref.algebraic_distance
  res = {}
  for iters in (1, 3, 20):
    np.random.seed(0)
    emb = AD.EmbedAlgebraicDistance(tiny, 10, iterations=iters,
                                    run_in_parallel=False, disable_pbar=True)
    X, Y = emb_arrays(emb, tiny_csr)
    res[f"x_{iters}"], res[f"y_{iters}"] = X, Y
    assert emb.method_name == "AlgebraicDistance"
  np.savez_compressed(os.path.join(out, "algdist_tiny.npz"), seed=0, k=10,
                      **res)
  np.random.seed(7)
  # on the COMPRESSED graph, as EmbedHg2vAlgDist's sampler_fn does
  # (embedding.py:399-408 receives the compressed hg from the skeleton)
  emb_small = AD.EmbedAlgebraicDistance(small_c, 10, iterations=20,
                                        run_in_parallel=False,
                                        disable_pbar=True)
  ident = dict(node_ids=np.arange(small_csr["N"]),
               edge_ids=np.arange(small_csr["E"]))
  Xs, Ys = emb_arrays(emb_small, ident)
  np.random.seed(5)
  emb_th = AD.EmbedAlgebraicDistance(th, 2, iterations=3,
                                     run_in_parallel=False, disable_pbar=True)
  Xt, Yt = emb_arrays(emb_th, th_csr)
  np.savez_compressed(os.path.join(out, "algdist_small.npz"), seed=7, k=10,
                      iters=20, x=Xs, y=Ys, th_seed=5, th_k=2, th_iters=3,
                      th_x=Xt, th_y=Yt, **{f"th_{k}": v for k, v in
                                           th_csr.items()})

  # ---- FOBE ----
  BS = ref.hg2v_sample.BooleanSamples
  np.random.seed(3)
  recs = BS(tiny_c, num_neighbors=5, num_samples=200, disable_pbar=True)
  F, T = model_input(recs, 5)
  kinds = np.array([np.count_nonzero(T[:, j]) for j in range(3)])
  np.savez_compressed(os.path.join(out, "fobe_tiny.npz"), seed=3, K=5, S=200,
                      n=F.shape[0], sha=sha(F, T), head_idx=F[:3000],
                      head_tgt=T[:3000], tail_idx=F[-3000:], tail_tgt=T[-3000:],
                      kinds=kinds)
  # small graph with non-unit weights and negatives (HG2V_BOOLEAN_NS path)
  wsmall = hu.CompressRange(small)[0]
  rnd = np.random.RandomState(99)
  for _, node in wsmall.node.items():
    node.weight = float(rnd.choice([0.5, 1.0, 1.5]))
  for _, edge in wsmall.edge.items():
    edge.weight = float(rnd.choice([0.25, 1.0, 2.0]))
  nw = np.array([wsmall.node[i].weight for i in range(len(wsmall.node))],
                np.float32)
  ew = np.array([wsmall.edge[i].weight for i in range(len(wsmall.edge))],
                np.float32)
  np.random.seed(4)
  recs = BS(wsmall, num_neighbors=3, num_samples=12, neg_samples=4,
            disable_pbar=True)
  F, T = model_input(recs, 3)
  np.savez_compressed(os.path.join(out, "fobe_small_ns.npz"), seed=4, K=3,
                      S=12, neg=4, node_weight=nw, edge_weight=ew, idx=F,
                      tgt=T)

  # ---- HOBE ----
  AS = ref.hg2v_sample.AlgebraicDistanceSamples
  np.random.seed(11)
  recs = AS(small_c, emb_small, num_neighbors=3, num_samples=20,
            run_in_parallel=False, disable_pbar=True)
  F, T = model_input(recs, 3)
  np.savez_compressed(os.path.join(out, "hobe_small.npz"), seed=11, K=3, S=20,
                      alg_x=Xs, alg_y=Ys, idx=F, tgt=T)

  # ---- HOBE probabilities on youtube_tiny for fixed pairs ----
  X20, Y20 = res["x_20"], res["y_20"]
  emb20 = ref.HypergraphEmbedding()
  for i in range(len(tiny_c.node)):
    emb20.node[i].values.extend(X20[i])
  for i in range(len(tiny_c.edge)):
    emb20.edge[i].values.extend(Y20[i])
  a = hu.ToCsrMatrix(tiny_c)
  at = hu.ToEdgeCsrMatrix(tiny_c)
  rs = np.random.RandomState(2024)
  N, E = len(tiny_c.node), len(tiny_c.edge)
  nn_nbr = (a * a.T).tocsr()
  nn_a = rs.randint(0, N, 1500)
  nn_b = np.array([rs.choice(nn_nbr[i].nonzero()[1]) if j % 3 else
                   rs.randint(0, N) for j, i in enumerate(nn_a)])
  ee_a = rs.randint(0, E, 400)
  ee_b = rs.randint(0, E, 400)
  ne_a = rs.randint(0, N, 1500)
  ne_b = rs.randint(0, E, 1500)
  S = ref.hg2v_sample
  nn_p = np.array([S._same_type_dist_calc((i, j), a, emb20.node, emb20.edge)
                   for i, j in zip(nn_a, nn_b)], np.float32)
  ee_p = np.array([S._same_type_dist_calc((i, j), at, emb20.edge, emb20.node)
                   for i, j in zip(ee_a, ee_b)], np.float32)
  np.random.seed(0)
  ne_p = np.array([S.DiffTypeDistanceSample((v, e), a, at, 2, emb20)
                   .node_edge_prob for v, e in zip(ne_a, ne_b)], np.float32)
  np.savez_compressed(os.path.join(out, "probs_tiny.npz"), nn_a=nn_a,
                      nn_b=nn_b, nn_p=nn_p, ee_a=ee_a, ee_b=ee_b, ee_p=ee_p,
                      ne_a=ne_a, ne_b=ne_b, ne_p=ne_p)

  # ---- weighting (hg2v_weighting.py:137-198) ----
  W = ref.hg2v_weighting
  u_n, u_e = W.UniformWeight(small_c)
  nb_n, nb_e = W.WeightByNeighborhood(small_c, 0.3)
  nb_n, nb_e = nb_n.tocsr(), nb_e.tocsr()
  nb_n.sort_indices()
  nb_e.sort_indices()
  np.savez_compressed(
      os.path.join(out, "weights_small.npz"), alpha=0.3,
      uniform_n=u_n.toarray(), uniform_e=u_e.toarray(),
      neigh_n=nb_n.toarray().astype(np.float32),
      neigh_e=nb_e.toarray().astype(np.float32))
  print("golden fixtures written to", out)


if __name__ == "__main__":
  main()

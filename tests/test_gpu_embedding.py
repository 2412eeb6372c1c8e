"""End-to-end embedding API on the device, mirroring the reference's
checkEmbedding tests (tests/test_embedding.py:14-64, 176-257) and model
tests (tests/test_hg2v_model.py:14-68), plus Embed(args) with the registry
and UniformWeight's known answer (tests/test_hg2v_weights.py:21-47)."""

import random

import numpy as np
import pytest
import scipy.sparse as sps

from hypergraphembedding_amd import (EMBEDDING_OPTIONS, AddNodeToEdge,
                                     BooleanModel, CreateRandomHyperGraph, Embed,
                                     EmbedAlgebraicDistance, EmbedHg2vAlgDist,
                                     EmbedHg2vBoolean, Hypergraph,
                                     KerasModelToEmbedding, UniformWeight,
                                     UnweightedFloatModel, Relabel)

pytestmark = pytest.mark.gpu


def _test_hypergraph():
  h = Hypergraph()
  for n, e in ((0, 0), (1, 0), (1, 1), (2, 1), (2, 2), (3, 2)):
    AddNodeToEdge(h, n, e)
  return h


def _check(emb, h, dim):
  assert emb.dim == dim
  for i in h.node:
    assert i in emb.node and len(emb.node[i].values) == dim
  for i in h.edge:
    assert i in emb.edge and len(emb.edge[i].values) == dim
  vals = np.array([v.values for v in emb.node.values()], np.float32)
  assert np.isfinite(vals).all()


def test_alg_dist_typical():
  h = _test_hypergraph()
  emb = EmbedAlgebraicDistance(h, 2, iterations=3, disable_pbar=True)
  _check(emb, h, 2)
  # the reference's code sets "AlgebraicDistance" (its test's "ALG_DIST"
  # expectation is a known-broken assertion)
  assert emb.method_name == "AlgebraicDistance"
  v = np.array([emb.node[i].values for i in h.node] +
               [emb.edge[i].values for i in h.edge])
  assert v.min() >= 0 and v.max() <= 1  # joint per-dim rescale


@pytest.mark.parametrize("fn,name", [
    (EmbedHg2vBoolean, "HG2V_BOOLEAN"), (EmbedHg2vAlgDist, "HG2V_ALG_DIST"),
    (EMBEDDING_OPTIONS["HG2V_ADJ_JAC"], "HG2V_ADJ_JAC"),
    (EMBEDDING_OPTIONS["HG2V_NEIGH_JAC"], "HG2V_NEIGH_JAC")])
def test_hg2v_typical_batch_one(fn, name):
  h = _test_hypergraph()
  emb = fn(h, 2, num_neighbors=2, num_samples=2, batch_size=1, epochs=1,
           disable_pbar=True)
  _check(emb, h, 2)
  assert emb.method_name == name


@pytest.mark.parametrize("key", ["HG2V_BOOLEAN", "HG2V_ALG_DIST",
                                 "HG2V_BOOLEAN_NS", "ALG_DIST", "HG2V_ADJ_JAC",
                                 "HG2V_NEIGH_JAC"])
def test_fuzz_random_hypergraphs(key):
  rnd = random.Random(11)
  np.random.seed(11)
  done = 0
  while done < 3:
    h = CreateRandomHyperGraph(25, 25, 0.25)
    max_dim = min(len(h.node), len(h.edge))
    if max_dim <= 1:
      continue
    dim = rnd.randint(1, max_dim - 1)
    if key.startswith("HG2V"):
      fn = EMBEDDING_OPTIONS[key]
      emb = fn(h, dim, num_neighbors=2, num_samples=2, batch_size=1, epochs=1)
    else:
      emb = EMBEDDING_OPTIONS[key](h, dim)
    _check(emb, h, dim)
    done += 1


def test_sparse_ids_keyed_by_original():
  h = Relabel(_test_hypergraph(), {0: 90, 1: 7, 2: 1000, 3: 55},
              {0: 4, 1: 400, 2: 40})
  emb = EmbedHg2vAlgDist(h, 2, num_neighbors=2, num_samples=5, epochs=2)
  _check(emb, h, 2)
  assert set(emb.node) == {90, 7, 1000, 55} and set(emb.edge) == {4, 400, 40}


def test_reproducible_under_numpy_seed():
  h = _test_hypergraph()
  outs = []
  for _ in range(2):
    np.random.seed(5)
    e = EmbedHg2vBoolean(h, 2, num_neighbors=2, num_samples=10, epochs=2)
    outs.append(np.array([e.node[i].values for i in sorted(h.node)]))
  assert np.array_equal(outs[0], outs[1])


class _Args:
  embedding_method = ["HG2V_BOOLEAN", "HG2V_ALG_DIST"]
  embedding_combination_strategy = "CONCATENATE"
  embedding_dimension = 2
  embedding_debug_summary = None


def test_embed_args_concatenate():
  h = _test_hypergraph()
  args = _Args()
  emb = Embed(args, h)
  _check(emb, h, 4)
  assert emb.method_name == "HG2V_BOOLEAN_HG2V_ALG_DIST"


@pytest.mark.parametrize("model_fn", [BooleanModel, UnweightedFloatModel])
def test_model_to_embedding_shapes(model_fn):
  h = Hypergraph()
  AddNodeToEdge(h, 0, 0)
  AddNodeToEdge(h, 2, 2)
  node_map = {0: 0, 2: 1}
  edge_map = {0: 0, 2: 1}
  model = model_fn(h, 5, 2)
  nw, ew = model.get_weights()
  assert nw.shape == (4, 5) and ew.shape == (4, 5)  # max idx + 2 rows
  assert np.abs(nw).max() <= 0.05  # Keras uniform(-0.05, 0.05) init
  emb = KerasModelToEmbedding(h, model, node_map, edge_map)
  assert emb.dim == 5
  for n in h.node:
    assert len(emb.node[node_map[n]].values) == 5
  for e in h.edge:
    assert len(emb.edge[edge_map[e]].values) == 5


def test_uniform_weight_known_answer():
  h = Hypergraph()
  AddNodeToEdge(h, 0, 1)
  AddNodeToEdge(h, 2, 2)
  AddNodeToEdge(h, 3, 2)
  n2w, e2w = UniformWeight(h)
  want_n = sps.csr_matrix([[0, 1, 0], [0, 0, 0], [0, 0, 1], [0, 0, 1]],
                          dtype=np.float32)
  want_e = sps.csr_matrix([[0, 0, 0, 0], [1, 0, 0, 0], [0, 0, 1, 1]],
                          dtype=np.float32)
  assert n2w.shape == want_n.shape and e2w.shape == want_e.shape
  assert abs(n2w - want_n).max() < 1e-5
  assert abs(e2w - want_e).max() < 1e-5


def test_isolated_node_raises_like_reference():
  h = _test_hypergraph()
  h.node[9].name = "isolated"  # present, no edges
  with pytest.raises(ZeroDivisionError):
    EmbedAlgebraicDistance(h, 2, iterations=2)


def test_weighted_jaccard_samples_api():
  """hg2v_sample.WeightedJaccardSamples with the reference's feature
  matrices (UniformWeight / WeightByNeighborhood)."""
  from hypergraphembedding_amd import (WeightedJaccardSamples,
                                       WeightByNeighborhood)
  from hypergraphembedding_amd.hypergraph_util import CompressRange
  h = CompressRange(_test_hypergraph())[0]
  n2f, e2f = WeightByNeighborhood(h, 0.5)
  recs = WeightedJaccardSamples(h, n2f, e2f, num_neighbors=2, num_samples=4)
  assert recs
  for r in recs:
    p = [x for x in (r.node_node_prob, r.edge_edge_prob, r.node_edge_prob)
         if x is not None]
    assert len(p) == 1 and 0.0 <= p[0] <= 1.0


def test_embed_beyond_proto_limit_returns_shards(tmp_path):
  """EmbedHg2vAlgDist on an Incidence whose embedding message exceeds
  protobuf's 2 GiB limit (1.1M rows x 512 floats, ~2.8 GB): the embedder
  returns a ShardedEmbedding with the message surface, written as shards
  that each parse as a HypergraphEmbedding; rows equal the trained tables
  (proto_native.read_embedding, native and per-shard protobuf)."""
  import os
  from hypergraphembedding_amd.embedding import EmbedHg2vAlgDist
  from hypergraphembedding_amd.proto import HypergraphEmbedding
  from hypergraphembedding_amd.proto_native import (PROTO_LIMIT,
                                                    ShardedEmbedding,
                                                    read_embedding)
  from hypergraphembedding_amd.synthetic import random_hypergraph
  inc = random_hypergraph(N=1_000_000, E=100_000, seed=3)
  np.random.seed(0)
  emb = EmbedHg2vAlgDist(inc, 512, num_samples=2, epochs=1)
  assert isinstance(emb, ShardedEmbedding) and emb.ByteSize() > PROTO_LIMIT
  assert emb.dim == 512 and emb.method_name == "HG2V_ALG_DIST"
  assert len(emb.node) == inc.N and len(emb.edge) == inc.E
  assert np.isfinite(emb.node_tab).all() and np.abs(emb.node_tab).max() > 0
  files = emb.write(str(tmp_path / "big.pb"))
  assert len(files) == 2
  rs = np.random.RandomState(1)
  sel = rs.choice(inc.N, 2000, replace=False)
  total = 0
  for f in files:
    m = HypergraphEmbedding()
    with open(f, "rb") as fh:
      m.ParseFromString(fh.read())
    assert m.dim == 512 and m.method_name == "HG2V_ALG_DIST"
    total += len(m.node) + len(m.edge)
    for r in sel:
      k = int(inc.node_ids[r])
      if k in m.node:
        assert np.array_equal(np.array(m.node[k].values, np.float32),
                              emb.node_tab[r])
  assert total == inc.N + inc.E
  back = read_embedding(str(tmp_path / "big.pb"))
  assert np.array_equal(back.node_tab, emb.node_tab)  # ids ascending = rows
  assert np.array_equal(back.edge_tab, emb.edge_tab)
  for f in files:
    os.remove(f)

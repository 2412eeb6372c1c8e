"""Host-side API, restating the reference's own known-answer tests for the
hot path: SamplesToModelInput (tests/test_hg2v_samples.py:13-189),
DictToSparseRow (tests/test_hg2v_weights.py:50-56), CSR orientation
(tests/test_hypergraph_util.py:103-192), Relabel / CompressRange (339-386),
RemoveNode / RemoveEdge (421-475); plus the device-ready Incidence builder
against those scipy matrices. CPU only."""

import random

import numpy as np
import pytest
import scipy.sparse as sps

from hypergraphembedding_amd import (EMBEDDING_OPTIONS, AddNodeToEdge,
                                     CompressRange, CreateRandomHyperGraph,
                                     FromSparseMatrix, Hypergraph,
                                     HypergraphEmbedding, Incidence, Relabel,
                                     RemoveEdge, RemoveNode, SamplesToModelInput,
                                     SimilarityRecord, ToCsrMatrix,
                                     ToEdgeCsrMatrix)
from hypergraphembedding_amd import hg2v_weighting as W
from hypergraphembedding_amd.embedding import (CombineEmbeddings,
                                               method_not_supported)
from hypergraphembedding_amd.hg2v_sample import (ModelInputToArrays,
                                                 records_from_arrays)
from hypergraphembedding_amd.synthetic import random_hypergraph


# ---- SamplesToModelInput (test_hg2v_samples.py:13-189) ----------------------

def _cols(*xs):
  return [[x] for x in xs]


STMI_CASES = [
    # (record, weighted, features, targets)
    (SimilarityRecord(left_node_idx=0, right_node_idx=1, node_node_prob=0.5),
     False, _cols(1, 0, 2, 0, 0, 0, 0, 0), _cols(0.5, 0, 0)),
    (SimilarityRecord(left_edge_idx=0, right_edge_idx=1, edge_edge_prob=0.5),
     False, _cols(0, 1, 0, 2, 0, 0, 0, 0), _cols(0, 0.5, 0)),
    (SimilarityRecord(left_node_idx=0, right_edge_idx=1,
                      neighbor_node_indices=[2], neighbor_edge_indices=[3, 4],
                      node_edge_prob=0.5),
     False, _cols(1, 0, 0, 2, 3, 0, 4, 5), _cols(0, 0, 0.5)),
    (SimilarityRecord(left_node_idx=0, right_node_idx=1, left_weight=0.3,
                      right_weight=0.6, node_node_prob=0.5),
     True, _cols(1, 0, 2, 0, 0.3, 0.6, 0, 0, 0, 0, 0, 0, 0, 0),
     _cols(0.5, 0, 0)),
    (SimilarityRecord(left_edge_idx=0, right_edge_idx=1, left_weight=0.3,
                      right_weight=0.6, neighbor_node_indices=[2],
                      neighbor_node_weights=[0.25],
                      neighbor_edge_indices=[3, 4],
                      neighbor_edge_weights=[0.5, 0.75], node_edge_prob=0.5),
     True, _cols(0, 1, 0, 2, 0.3, 0.6, 3, 0, 0.25, 0, 4, 5, 0.5, .75),
     _cols(0, 0, 0.5)),
    (SimilarityRecord(left_edge_idx=0, right_edge_idx=1, left_weight=0.3,
                      right_weight=0.6, edge_edge_prob=0.5),
     True, _cols(0, 1, 0, 2, 0.3, 0.6, 0, 0, 0, 0, 0, 0, 0, 0),
     _cols(0, 0.5, 0)),
]


@pytest.mark.parametrize("rec,weighted,feat,tgt", STMI_CASES)
def test_samples_to_model_input_known_answers(rec, weighted, feat, tgt):
  assert SamplesToModelInput([rec], num_neighbors=2,
                             weighted=weighted) == (feat, tgt)


def test_model_input_arrays_roundtrip():
  rs = np.random.RandomState(3)
  K = 3
  recs = []
  for _ in range(50):
    kind = rs.randint(3)
    if kind == 0:
      recs.append(SimilarityRecord(left_node_idx=int(rs.randint(9)),
                                   right_node_idx=int(rs.randint(9)),
                                   node_node_prob=float(np.float32(rs.rand()))))
    elif kind == 1:
      recs.append(SimilarityRecord(left_edge_idx=int(rs.randint(9)),
                                   right_edge_idx=int(rs.randint(9)),
                                   edge_edge_prob=float(np.float32(rs.rand()))))
    else:
      recs.append(SimilarityRecord(
          left_node_idx=int(rs.randint(9)), right_edge_idx=int(rs.randint(9)),
          neighbor_node_indices=rs.randint(9, size=K).tolist(),
          neighbor_edge_indices=rs.randint(9, size=K).tolist(),
          node_edge_prob=float(np.float32(rs.rand()))))
  idx, tgt = ModelInputToArrays(*SamplesToModelInput(recs, K, weighted=False))
  assert idx.shape == (50, 4 + 2 * K) and idx.dtype == np.int32
  assert tgt.shape == (50, 3) and tgt.dtype == np.float32
  back = records_from_arrays(idx, tgt, K)
  idx2, tgt2 = ModelInputToArrays(*SamplesToModelInput(back, K, weighted=False))
  assert np.array_equal(idx, idx2) and np.array_equal(tgt, tgt2)


# ---- weighting helpers (test_hg2v_weights.py:50-56; hg2v_weighting.py) -----

def test_dict_to_sparse_row():
  got = W.DictToSparseRow({0: 1, 2: 4, 5: 100})
  want = sps.csr_matrix([1, 0, 4, 0, 0, 100], dtype=np.float32)
  assert got.shape == want.shape and abs(got - want).max() < 1e-5


def test_scale_helpers():
  assert W.ZeroOneScaleValues({}) == {}
  assert W.ZeroOneScaleValues({1: 3, 2: 3}) == {1: 1, 2: 1}
  assert W.ZeroOneScaleValues({1: 2, 2: 4, 3: 3}) == {1: 0, 2: 1, 3: 0.5}
  assert W.OneMinusValues({1: 0.25}) == {1: 0.75}
  assert W.AlphaScaleValues({1: 0.5}, 0.5) == {1: 0.75}
  with pytest.raises(AssertionError):
    W.AlphaScaleValues({1: 0.5}, 2)


# ---- hypergraph_util (test_hypergraph_util.py) -----------------------------

def _same(a, b):
  assert a.shape == b.shape and (a != b).nnz == 0


def test_from_sparse_matrix():
  got = FromSparseMatrix(sps.csr_matrix([[1, 0], [1, 0], [0, 1], [1, 1]]))
  want = Hypergraph()
  for n, es in ((0, [0]), (1, [0]), (2, [1]), (3, [0, 1])):
    want.node[n].edges.extend(es)
  want.edge[0].nodes.extend([0, 1, 3])
  want.edge[1].nodes.extend([2, 3])
  assert got == want
  assert FromSparseMatrix(sps.csr_matrix([])) == Hypergraph()


def test_csr_orientation():
  h = Hypergraph()
  AddNodeToEdge(h, 1, 2)
  _same(ToCsrMatrix(h), sps.csr_matrix([[0, 0, 0], [0, 0, 1]], dtype=bool))
  _same(ToEdgeCsrMatrix(h), sps.csr_matrix([[0, 0], [0, 0], [0, 1]],
                                           dtype=bool))
  h = Hypergraph()
  AddNodeToEdge(h, 1, 1)
  AddNodeToEdge(h, 1, 2)
  AddNodeToEdge(h, 2, 0)
  _same(ToCsrMatrix(h), sps.csr_matrix([[0, 0, 0], [0, 1, 1], [1, 0, 0]],
                                       dtype=bool))
  _same(ToCsrMatrix(Hypergraph()), sps.csr_matrix([]))


def test_csr_roundtrip_fuzz():
  rnd = random.Random(0)
  for _ in range(100):
    h = CreateRandomHyperGraph(rnd.randint(0, 10), rnd.randint(0, 10),
                               rnd.random())
    assert h == FromSparseMatrix(ToCsrMatrix(h))
  h = CreateRandomHyperGraph(100, 100, 0)
  assert h == FromSparseMatrix(ToCsrMatrix(h))


def test_relabel_and_compress_range():
  h = Hypergraph()
  AddNodeToEdge(h, 0, 1)
  AddNodeToEdge(h, 1, 1)
  AddNodeToEdge(h, 1, 2)
  h.name = "KEEP ME"
  got = Relabel(h, {0: 100, 1: 200}, {1: 50, 2: 150})
  assert got.name == "KEEP ME"
  _same(ToCsrMatrix(got), ToCsrMatrix(_edges_hg([(100, 50), (200, 50),
                                                 (200, 150)])))
  for orig in [got] + [CreateRandomHyperGraph(100, 100, 0.01)
                       for _ in range(10)]:
    comp, nmap, emap = CompressRange(orig)
    _same(ToCsrMatrix(orig), ToCsrMatrix(Relabel(comp, nmap, emap)))
    assert len(comp.node) == max(comp.node) + 1 == len(orig.node)
    assert len(comp.edge) == max(comp.edge) + 1 == len(orig.edge)


def _edges_hg(pairs):
  h = Hypergraph()
  for n, e in pairs:
    AddNodeToEdge(h, n, e)
  return h


def test_remove_node_and_edge():
  h = _edges_hg([(0, 0), (0, 1), (1, 0), (1, 1)])
  RemoveNode(h, 0)
  assert h == _edges_hg([(1, 0), (1, 1)])
  h = _edges_hg([(0, 0), (0, 1), (1, 0)])
  RemoveNode(h, 0)
  assert h == _edges_hg([(1, 0)])  # degree-0 edge dropped
  h = _edges_hg([(0, 0), (0, 1), (1, 0), (1, 1)])
  RemoveEdge(h, 0)
  assert h == _edges_hg([(0, 1), (1, 1)])


# ---- Incidence: the device upload format ------------------------------------

@pytest.mark.parametrize("seed", range(5))
def test_incidence_matches_compressed_csr(seed):
  rnd = random.Random(seed)
  h = CreateRandomHyperGraph(rnd.randint(1, 60), rnd.randint(1, 40), 0.15)
  # sparse, shuffled ids as in real data
  nmap = {n: 7 * n + 3 for n in h.node}
  emap = {e: 11 * e + 1 for e in h.edge}
  h = Relabel(h, nmap, emap)
  comp, inv_n, inv_e = CompressRange(h)
  inc = Incidence.from_hypergraph(h)
  a, at = inc.to_scipy()
  if comp.node:
    _same(a, ToCsrMatrix(comp).astype(bool)[:inc.N, :inc.E])
    _same(at, ToEdgeCsrMatrix(comp).astype(bool)[:inc.E, :inc.N])
  assert inc.node_ids.tolist() == [inv_n[i] for i in range(inc.N)]
  assert inc.edge_ids.tolist() == [inv_e[i] for i in range(inc.E)]
  for rp, col in ((inc.rp_n, inc.col_n), (inc.rp_e, inc.col_e)):
    for r in range(len(rp) - 1):
      assert np.all(np.diff(col[rp[r]:rp[r + 1]]) > 0)  # sorted, distinct


def test_incidence_from_scipy_and_transpose():
  m = sps.random(40, 30, density=0.1, random_state=1, format="csr")
  inc = Incidence.from_scipy(m)
  a, at = inc.to_scipy()
  _same(a, (m != 0))
  _same(at, (m != 0).T.tocsr())


def test_synthetic_generator_shape():
  inc = random_hypergraph(N=2000, E=1000, mean_degree=8, seed=1)
  assert inc.N == 2000 and inc.E <= 1000
  assert inc.node_degree().min() >= 1 and inc.edge_size().min() >= 1
  assert abs(inc.nnz / inc.N - 8) < 0.5
  again = random_hypergraph(N=2000, E=1000, mean_degree=8, seed=1)
  assert np.array_equal(inc.col_n, again.col_n)


# ---- registry / combination (embedding.py:51-107, 419-444) -----------------

def test_registry_keys_and_unsupported():
  from hypergraphembedding_amd.embedding import (
      EmbedHg2vAdjJaccard, EmbedHg2vNeighborhoodWeightedJaccard)
  for key in ("ALG_DIST", "HG2V_BOOLEAN", "HG2V_ALG_DIST", "HG2V_BOOLEAN_NS"):
    assert callable(EMBEDDING_OPTIONS[key])
  assert EMBEDDING_OPTIONS["HG2V_ADJ_JAC"] is EmbedHg2vAdjJaccard
  assert EMBEDDING_OPTIONS["HG2V_NEIGH_JAC"] is EmbedHg2vNeighborhoodWeightedJaccard
  for key in ("SVD", "NMF", "AUTO_ENCODER", "N2V5_CLIQUE", "N2V3_BIPARTIDE"):
    with pytest.raises(RuntimeError):
      EMBEDDING_OPTIONS[key](Hypergraph(), 2)
  with pytest.raises(RuntimeError):
    method_not_supported(Hypergraph(), 2)


class _Args:
  embedding_method = ["A", "B"]
  embedding_combination_strategy = "CONCATENATE"
  embedding_dimension = 2


def test_combine_concatenate():
  h = _edges_hg([(0, 5), (1, 5)])
  embs = []
  for off in (0.0, 10.0):
    e = HypergraphEmbedding()
    e.dim = 2
    for n in h.node:
      e.node[n].values.extend([off + n, off + n + 0.5])
    for x in h.edge:
      e.edge[x].values.extend([off - x, off])
    embs.append(e)
  args = _Args()
  comb = CombineEmbeddings(args, h, embs)
  assert comb.dim == 4 and args.embedding_dimension == 4
  assert comb.method_name == "A_B"
  assert list(comb.node[1].values) == [1, 1.5, 11, 11.5]
  assert list(comb.edge[5].values) == [-5, 0, 5, 10]
  args.embedding_combination_strategy = "NOT_A_STRATEGY"
  with pytest.raises(ValueError):
    CombineEmbeddings(args, h, embs)


def test_incidence_samples_equal_the_proto_path():
  """The combiner's array-level samples (positives straight from the CSR,
  SampleMissingConnections' native draws fed the CSR arrays) equal the
  proto path's (node map order, Python-random-exact draws) on the proto of
  the same graph with ascending ids -- the C5 preparation without a
  Python loop per incidence."""
  import random
  from hypergraphembedding_amd import _hgx
  from hypergraphembedding_amd.combine_embeddings_util import (
      incidence_samples, proto_samples)
  from hypergraphembedding_amd.hypergraph_util import CreateRandomHyperGraph
  from hypergraphembedding_amd.proto import Hypergraph
  random.seed(3)
  hg0 = CreateRandomHyperGraph(300, 80, 0.03)
  inc = Incidence.from_hypergraph(hg0)
  hg = Hypergraph()
  hg.ParseFromString(_hgx.write_hypergraph_bytes(inc).tobytes())
  assert list(hg.node) == sorted(hg.node)
  for seed in (0, 1):
    random.seed(seed)
    a = incidence_samples(inc)
    random.seed(seed)
    b = proto_samples(hg, list(hg.node), list(hg.edge))
    for x, y in zip(a, b):
      assert np.array_equal(x, y)


def test_rng_modes_and_state_seed():
  """rng is None or "mt19937" (ValueError otherwise, before any device
  call); the mt19937 table-init seed is derived from numpy's state without
  advancing it; reference-only runs refuse the product's extensions."""
  from hypergraphembedding_amd import embedding
  from hypergraphembedding_amd.runtime import check_rng, numpy_state_seed
  assert check_rng(None) is None and check_rng("mt19937") == "mt19937"
  with pytest.raises(ValueError):
    check_rng("philox")
  np.random.seed(12)
  before = np.random.get_state()[1].copy(), np.random.get_state()[2]
  s1 = numpy_state_seed()
  s2 = numpy_state_seed()
  after = np.random.get_state()
  assert s1 == s2 and 0 <= s1 < 2**63
  assert np.array_equal(before[0], after[1]) and before[1] == after[2]
  np.random.seed(13)
  assert numpy_state_seed() != s1
  with pytest.raises(ValueError):
    embedding.EmbedHg2vBoolean(None, 4, rng="mt19937",
                               row_quota=(np.ones(2), np.ones(2)))
  with pytest.raises(ValueError):
    embedding.EmbedHg2vAlgDist(None, 4, rng="mt19937", group=object())

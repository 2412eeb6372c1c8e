"""The numpy-seeded samplers (rng="mt19937", csrc/hgx_mt.hip) against the
reference's own record streams, and the product API end to end.

  * C1 FOBE (youtube_tiny, S=200, K=5, np.random.seed(3)): the 724,792
    records hash to the sha of the reference's BooleanSamples stream
    (tests/golden/make_golden.py imported the reference to make it), and
    numpy's state afterwards is the reference's (the oracle's MT19937 replica
    after the same draws);
  * the weighted small graph with negatives (HG2V_BOOLEAN_NS path) and the
    HOBE small stream (AlgebraicDistanceSamples, run_in_parallel=False, the
    reference's float32 alg coordinates): every record equal;
  * C1 HOBE: the 755,267 pairs and neighbours equal the oracle replica's,
    the probabilities the reference's for the same coordinates;
  * np.random.seed(3); EmbedHg2vBoolean(youtube_tiny, 16, rng="mt19937")
    through the product API: the stream, every epoch's order (Keras'
    np.random.shuffle), the epochs run and numpy's final state as the
    reference's; the embedding vs the CPU restatement trained on the
    reference stream from the same init: per-row cosine p50 >= 0.9999,
    p1 >= 0.999.
"""

import hashlib

import numpy as np
import pytest

import oracle as O
from conftest import golden

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
  from hypergraphembedding_amd import _hgx
  c = _hgx.Context(0)
  yield c
  c.close()


def _sha(idx, tgt):
  h = hashlib.sha256()
  h.update(np.ascontiguousarray(idx, np.int32).tobytes())
  h.update(np.ascontiguousarray(tgt, np.float32).tobytes())
  return h.hexdigest()


def _next_words(n=16):
  """The next n raw MT19937 words of numpy's global stream (consumed)."""
  return np.random.randint(0, 2**32, size=n, dtype=np.uint32).astype(np.int64)


def _oracle_words(r, n=16):
  return np.array([r.next32() for _ in range(n)], np.int64)


def test_fobe_mt_is_the_reference_stream(ctx, tiny_inc):
  z = golden("fobe_tiny.npz")
  K, S = int(z["K"]), int(z["S"])
  inc = tiny_inc
  ctx.upload(inc)
  np.random.seed(int(z["seed"]))
  n = ctx.sample_fobe_mt(K, np.full(inc.N, S, np.int32), np.full(inc.E, S, np.int32))
  assert n == int(z["n"])
  idx, tgt = ctx.records_get()
  assert np.array_equal(idx[:3000], z["head_idx"])
  assert np.array_equal(tgt[-3000:], z["tail_tgt"])
  assert _sha(idx, tgt) == str(z["sha"])
  assert ctx.records_blocks()[-1] == n
  # numpy is left where the reference leaves it
  r = O.Rng(int(z["seed"]))
  O.fobe_sample(r, inc, np.full(inc.N, S, np.int32), np.full(inc.E, S, np.int32), K)
  assert np.array_equal(_next_words(), _oracle_words(r))


def test_fobe_mt_weighted_with_negatives(ctx, small_inc):
  z = golden("fobe_small_ns.npz")
  K, S, G = int(z["K"]), int(z["S"]), int(z["neg"])
  q = lambda w, m: np.array([int(float(x) * m) for x in w], np.int32)
  nw, ew = z["node_weight"], z["edge_weight"]
  ctx.upload(small_inc)
  np.random.seed(int(z["seed"]))
  n = ctx.sample_fobe_mt(K, q(nw, S), q(ew, S), q(nw, G), q(ew, G))
  idx, tgt = ctx.records_get()
  assert n == z["idx"].shape[0]
  assert np.array_equal(idx, z["idx"]) and np.array_equal(tgt, z["tgt"])
  b = ctx.records_blocks()
  assert b.size == 10 and b[-1] == n


def test_hobe_mt_small_is_the_reference_stream(ctx, small_inc):
  z = golden("hobe_small.npz")
  K, S = int(z["K"]), int(z["S"])
  ctx.upload(small_inc)
  ctx.alg_set(z["alg_x"], z["alg_y"])  # the reference's float32 coordinates
  np.random.seed(int(z["seed"]))
  n = ctx.sample_hobe_mt(K, S)
  idx, tgt = ctx.records_get()
  assert n == z["idx"].shape[0]
  assert np.array_equal(idx, z["idx"])
  assert np.abs(tgt - z["tgt"]).max() <= 1e-6
  # the parent's state after its last pair draw (the neighbour draws ran in
  # the worker's copy)
  r = O.Rng(int(z["seed"]))
  O.hobe_sample(r, small_inc, z["alg_x"], z["alg_y"], S, K)
  assert np.array_equal(_next_words(), _oracle_words(r))


def test_hobe_mt_c1_pairs_and_probabilities(ctx, tiny_inc):
  """C1 HOBE (755,267 records): pairs and neighbours equal the oracle
  replica's record for record; probabilities from the reference's
  20-iteration coordinates equal the oracle's (<= 1e-5)."""
  z = golden("algdist_tiny.npz")
  inc = tiny_inc
  ctx.upload(inc)
  ctx.alg_set(z["x_20"], z["y_20"])
  np.random.seed(7)
  n = ctx.sample_hobe_mt(5, 200)
  assert n == 755_267
  idx, tgt = ctx.records_get()
  oidx, otgt = O.hobe_sample(O.Rng(7), inc, z["x_20"], z["y_20"], 200, 5)
  assert np.array_equal(idx, oidx)
  assert np.abs(tgt - otgt).max() <= 1e-5


def test_mt_stream_refuses_the_record_store(ctx, small_inc):
  """An MT stream is not keyed: the store cannot re-derive it."""
  from hypergraphembedding_amd import _hgx
  z = golden("hobe_small.npz")
  ctx.upload(small_inc)
  ctx.alg_set(z["alg_x"], z["alg_y"])
  ctx.sample_hobe_mt(3, 5)
  ctx.store_reset(0)
  with pytest.raises(_hgx.HgxError):
    ctx.store_append()


def _row_cos(a, b):
  num = (a * b).sum(1)
  den = np.linalg.norm(a, axis=1) * np.linalg.norm(b, axis=1)
  return num / np.maximum(den, 1e-30)


def test_embed_hg2v_boolean_mt_end_to_end(tiny_hypergraph, tiny_inc, monkeypatch):
  """np.random.seed(3); EmbedHg2vBoolean(youtube_tiny, 16, rng="mt19937"):
  the product API with numpy's stream throughout, vs the reference's stream
  trained by the CPU restatement with the same init and epoch orders."""
  from hypergraphembedding_amd import embedding
  from hypergraphembedding_amd.hg2v_model import Hg2vModel
  seen = {}

  class Spy(Hg2vModel):
    def fit(self, *a, **k):
      seen["tables"] = self.ctx.model_get()
      seen["records"] = self.ctx.records_get()
      seen["state"] = np.random.get_state()
      return super().fit(*a, **k)

  monkeypatch.setattr(embedding, "Hg2vModel", Spy)
  z = golden("fobe_tiny.npz")
  K, S, d = int(z["K"]), int(z["S"]), 16
  np.random.seed(int(z["seed"]))
  emb = embedding.EmbedHg2vBoolean(tiny_hypergraph, d, rng="mt19937")
  end_words = _next_words()
  assert emb.method_name == "HG2V_BOOLEAN"
  idx, tgt = seen["records"]
  assert _sha(idx, tgt) == str(z["sha"])
  # numpy's state at fit = the reference's after BooleanSamples
  inc = tiny_inc
  r = O.Rng(int(z["seed"]))
  oidx, otgt = O.fobe_sample(r, inc, np.full(inc.N, S, np.int32),
                             np.full(inc.E, S, np.int32), K)
  rs = np.random.RandomState()
  rs.set_state(seen["state"])
  assert np.array_equal(rs.randint(0, 2**32, 16, dtype=np.uint32).astype(np.int64),
                        _oracle_words(r))
  # Keras' epoch orders from that state; the CPU restatement on the
  # reference stream, the product's init, those orders, EarlyStopping
  rs.set_state(seen["state"])
  perms = np.stack([rs.permutation(oidx.shape[0]) for _ in range(10)])
  nt, et = seen["tables"]
  ont, oet, ol, _, _ = O.train(oidx, otgt, K, nt, et, O.LOSS_KLD, O.ACT_SIGMOID,
                               batch=256, max_epochs=10, perms=perms,
                               min_delta=1e-3)
  # the epochs run drew exactly len(ol) shuffles from numpy's stream
  rs.set_state(seen["state"])
  for _ in range(len(ol)):
    rs.permutation(oidx.shape[0])
  assert np.array_equal(rs.randint(0, 2**32, 16, dtype=np.uint32).astype(np.int64),
                        end_words)
  gn = np.array([emb.node[int(i)].values for i in inc.node_ids], np.float32)
  ge = np.array([emb.edge[int(i)].values for i in inc.edge_ids], np.float32)
  for g, o in ((gn, ont[1:]), (ge, oet[1:])):
    c = _row_cos(g, o)
    assert np.percentile(c, 50) >= 0.9999 and np.percentile(c, 1) >= 0.999, \
        (np.percentile(c, 50), np.percentile(c, 1))


def test_fobe_mt_c2_equals_the_oracle_replica(ctx, capsys):
  """C2 (random 100k/50k, S=200, K=5): the ~34M-record numpy-seeded FOBE
  stream equals the oracle's MT19937 replica record for record, and numpy's
  state afterwards equals the replica's. Timings of both are printed."""
  import time
  from hypergraphembedding_amd.synthetic import random_hypergraph
  inc = random_hypergraph(seed=0)
  S, K = 200, 5
  q_n, q_e = np.full(inc.N, S, np.int32), np.full(inc.E, S, np.int32)
  ctx.upload(inc)
  np.random.seed(21)
  t = time.perf_counter()
  n = ctx.sample_fobe_mt(K, q_n, q_e)
  ctx.synchronize()
  t_dev = time.perf_counter() - t
  assert n > 30_000_000
  r = O.Rng(21)
  t = time.perf_counter()
  oidx, otgt = O.fobe_sample(r, inc, q_n, q_e, K)
  t_cpu = time.perf_counter() - t
  idx, tgt = ctx.records_get()
  assert idx.shape == oidx.shape
  assert np.array_equal(idx, oidx) and np.array_equal(tgt, otgt)
  del idx, tgt, oidx, otgt
  assert np.array_equal(_next_words(), _oracle_words(r))
  with capsys.disabled():
    print(f"\nC2 FOBE rng=mt19937: {n} records, device path {t_dev:.2f} s "
          f"({n / t_dev / 1e6:.1f}M records/s), oracle replica (1 CPU "
          f"thread) {t_cpu:.2f} s")


def test_embed_hg2v_alg_dist_mt_end_to_end(tiny_hypergraph, tiny_inc, monkeypatch):
  """np.random.seed(0); EmbedHg2vAlgDist(youtube_tiny, 16, rng="mt19937"):
  the alg-dist init from numpy (as EmbedAlgebraicDistance draws it), the
  HOBE pairs and (run_in_parallel=False) neighbours of the reference record
  for record, the probabilities from this device's coordinates (within
  5e-4 of the reference's: its coordinates agree to 1e-4), numpy's state at
  fit = the reference's parent state, Keras' epoch orders; the embedding vs
  the CPU restatement trained on the reference stream from the same init
  and orders: per-row cosine p50 >= 0.9999, p1 >= 0.999."""
  from hypergraphembedding_amd import embedding
  from hypergraphembedding_amd.hg2v_model import Hg2vModel
  seen = {}

  class Spy(Hg2vModel):
    def fit(self, *a, **k):
      seen["tables"] = self.ctx.model_get()
      seen["records"] = self.ctx.records_get()
      seen["state"] = np.random.get_state()
      return super().fit(*a, **k)

  monkeypatch.setattr(embedding, "Hg2vModel", Spy)
  z = golden("algdist_tiny.npz")  # the reference's coordinates, seed 0
  inc, K, S, d = tiny_inc, 5, 200, 16
  np.random.seed(int(z["seed"]))
  emb = embedding.EmbedHg2vAlgDist(tiny_hypergraph, d, rng="mt19937")
  end_words = _next_words()
  assert emb.method_name == "HG2V_ALG_DIST"
  r = O.Rng(int(z["seed"]))
  r.random((inc.N, 10))
  r.random((inc.E, 10))
  oidx, otgt = O.hobe_sample(r, inc, z["x_20"], z["y_20"], S, K)
  idx, tgt = seen["records"]
  assert np.array_equal(idx, oidx)
  assert np.abs(tgt - otgt).max() <= 5e-4
  rs = np.random.RandomState()
  rs.set_state(seen["state"])
  assert np.array_equal(rs.randint(0, 2**32, 16, dtype=np.uint32).astype(np.int64),
                        _oracle_words(r))
  rs.set_state(seen["state"])
  perms = np.stack([rs.permutation(oidx.shape[0]) for _ in range(10)])
  nt, et = seen["tables"]
  ont, oet, ol, _, _ = O.train(oidx, otgt, K, nt, et, O.LOSS_MSE, O.ACT_RELU,
                               batch=256, max_epochs=10, perms=perms,
                               min_delta=1e-3)
  rs.set_state(seen["state"])
  for _ in range(len(ol)):
    rs.permutation(oidx.shape[0])
  assert np.array_equal(rs.randint(0, 2**32, 16, dtype=np.uint32).astype(np.int64),
                        end_words)
  gn = np.array([emb.node[int(i)].values for i in inc.node_ids], np.float32)
  ge = np.array([emb.edge[int(i)].values for i in inc.edge_ids], np.float32)
  for g, o in ((gn, ont[1:]), (ge, oet[1:])):
    c = _row_cos(g, o)
    assert np.percentile(c, 50) >= 0.9999 and np.percentile(c, 1) >= 0.999, \
        (np.percentile(c, 50), np.percentile(c, 1))


def test_mt_zero_quotas_still_draw_their_permutations(ctx, small_inc):
  """np.random.choice(cols, 0, replace=False) still draws permutation(|cols|)
  in numpy's legacy RandomState: rows with quota 0 (weight-0 rows, S = 0)
  consume the stream like the reference's. FOBE with a third of the rows at
  quota 0 and HOBE with S = 0 against the oracle replica: records and the
  state afterwards."""
  inc, K = small_inc, 3
  rs = np.random.RandomState(8)
  nq = np.where(rs.random_sample(inc.N) < 0.33, 0, 7).astype(np.int32)
  eq = np.where(rs.random_sample(inc.E) < 0.33, 0, 7).astype(np.int32)
  ctx.upload(inc)
  np.random.seed(31)
  n = ctx.sample_fobe_mt(K, nq, eq)
  r = O.Rng(31)
  oidx, otgt = O.fobe_sample(r, inc, nq, eq, K)
  idx, tgt = ctx.records_get()
  assert n == oidx.shape[0] and np.array_equal(idx, oidx) and np.array_equal(tgt, otgt)
  assert np.array_equal(_next_words(), _oracle_words(r))
  z = golden("hobe_small.npz")
  ctx.alg_set(z["alg_x"], z["alg_y"])
  np.random.seed(32)
  assert ctx.sample_hobe_mt(K, 0) == 0
  r = O.Rng(32)
  assert O.hobe_sample(r, inc, z["alg_x"], z["alg_y"], 0, K)[0].shape[0] == 0
  assert np.array_equal(_next_words(), _oracle_words(r))


def test_mt_isolated_negative_endpoint_raises(ctx):
  """_sample_neighbors on a node without edges raises ValueError in the
  reference (np.random.randint(0) inside np.random.choice, hg2v_sample.py
  49-51): a node-edge negative of an isolated node in the numpy-seeded mode
  fails the same way. numpy's global state is left as it was before the call
  (the reference's would have advanced to the failing draw); without the
  isolated endpoint the same call succeeds."""
  from hypergraphembedding_amd.hypergraph_util import Incidence
  inc = Incidence(3, 2, [0, 2, 3, 3], [0, 1, 1])  # node 2 has no edges
  ctx.upload(inc)
  z3, z2 = np.zeros(3, np.int32), np.zeros(2, np.int32)
  np.random.seed(4)
  before = np.random.get_state()
  with pytest.raises(ValueError):
    ctx.sample_fobe_mt(2, z3, z2, np.array([0, 0, 3], np.int32), z2)
  after = np.random.get_state()
  assert np.array_equal(before[1], after[1]) and before[2] == after[2]
  n = ctx.sample_fobe_mt(2, z3, z2, np.array([3, 3, 0], np.int32), z2)
  assert n > 0

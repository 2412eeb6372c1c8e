"""FOBE/HOBE models (reference: hypergraph_embedding/hg2v_model.py).

The reference builds a Keras graph (two Embedding tables of (max_idx + 2) x d,
uniform(-0.05, 0.05) init, three heads, Adagrad). Here a model is a pair of
tables resident on the device plus its loss/activation; training is libhgx
``hgx_train`` (Keras 2.x Adagrad semantics, see csrc/hgx_train.hip).

BooleanModel      -> sigmoid heads, kullback_leibler_divergence (51-125)
UnweightedFloatModel -> relu heads, mean_squared_error (129-203)
KerasModelToEmbedding -> rows idx + 1 keyed by the original ids (31-48)
"""

from . import _hgx
from .proto import HypergraphEmbedding
from .runtime import get_context, numpy_seed


class Hg2vModel:
  """Two embedding tables on a device context (row 0 = padding)."""

  def __init__(self, node_rows, edge_rows, dimension, num_neighbors, loss, act,
               ctx=None, seed=None):
    self.ctx = ctx or get_context()
    self.dimension = dimension
    self.num_neighbors = num_neighbors
    self.loss = loss
    self.act = act
    self.ctx.model_init(dimension, node_rows, edge_rows,
                        numpy_seed() if seed is None else seed)

  def fit(self, batch_size=256, epochs=10, min_delta=1e-3, lr=0.01, eps=1e-7,
          shuffle_seed=None, perms=None, rng=None):
    """Keras fit(shuffle=True) + EarlyStopping(monitor='loss', min_delta,
    patience=0) over the records resident on the context. rng="mt19937":
    every epoch's order is Keras 2.x's own, np.random.shuffle of
    arange(records) on numpy's global RandomState (training_arrays.fit_loop),
    drawn only for the epochs that run."""
    if rng == "mt19937":
      return self._fit_numpy_order(batch_size, epochs, min_delta, lr, eps)
    return self.ctx.train(batch=batch_size, max_epochs=epochs, lr=lr, eps=eps,
                          loss=self.loss, act=self.act, min_delta=min_delta,
                          shuffle_seed=numpy_seed() if shuffle_seed is None
                          else shuffle_seed, perms=perms)

  def _fit_numpy_order(self, batch_size, epochs, min_delta, lr, eps):
    import numpy as np
    n = self.ctx.records_info()[0]
    md = float(np.float32(min_delta))  # hgx_train compares in double
    best, losses = float("inf"), []
    for _ in range(epochs):
      order = np.arange(n)
      np.random.shuffle(order)
      self.ctx.train(batch=batch_size, max_epochs=1, lr=lr, eps=eps,
                     loss=self.loss, act=self.act, min_delta=-1e30,
                     perms=order[None, :])
      cur = self.ctx.train_loss_sum() / max(n, 1)
      losses.append(cur)
      if cur < best - md:
        best = cur
      else:
        break
    return np.array(losses, np.float32)

  def fit_store(self, budget, batch_size=256, epochs=10, min_delta=1e-3,
                lr=0.01, eps=1e-7, seed=None, on_chunk=None):
    """fit() over the record store of the context (hgx_store_*): a stream
    sampled once and kept as 12-byte entries because its trainer records
    do not fit in HBM (the C4 HOBE stream: 5.9e9 records, 404 GB; the
    reference materialises it and fits with Keras' shuffle=True,
    embedding.py:277-302). Every epoch is one global pseudo-random
    permutation of all records (keyed by record identity and the epoch
    seed), cut into batches of `batch_size` in that order -- Keras'
    semantics -- and trained through chunks of at most `budget` records
    (hgx_store_plan / hgx_store_load): a chunk is the next stretch of the
    epoch's order, and a chunk's last partial batch is completed by the
    next chunk's first records. The epoch loss is the record-weighted mean
    (Keras' batch-size-weighted mean) and EarlyStopping(min_delta,
    patience=0) applies to it. Epoch ep's seed comes from
    RandomState([seed, ep]). Returns the epoch losses; per epoch the
    records may exceed 2^31. on_chunk(epoch, chunk, n_chunks), if given, is
    called after every trained chunk (progress of long epochs)."""
    import numpy as np
    base = numpy_seed() % (2**32) if seed is None else seed
    best, losses = float("inf"), []
    self.records_per_epoch = 0
    self.chunk_stats = []  # (epoch, chunk, step ms, records, batches)
    for ep in range(epochs):
      es = int(np.random.RandomState([base, ep]).randint(0, 2**62, dtype=np.int64))
      bounds, counts = self.ctx.store_plan(es, budget)
      lsum, n = 0.0, 0
      nc = counts.size
      for c in range(nc):
        m = self.ctx.store_load(es, bounds[c], bounds[c + 1], batch_size,
                                c == nc - 1)
        if m == 0:
          continue
        self.ctx.train(batch=batch_size, max_epochs=1, lr=lr, eps=eps,
                       loss=self.loss, act=self.act, min_delta=-1e30)
        lsum += self.ctx.train_loss_sum()
        n += m
        self.chunk_stats.append((ep, c) + tuple(self.ctx.train_stats()))
        if on_chunk is not None:
          on_chunk(ep, c, nc)
      self.records_per_epoch = n
      cur = lsum / max(n, 1)
      losses.append(cur)
      if cur < best - min_delta:
        best = cur
      else:
        break
    return np.array(losses, np.float32)

  def get_weights(self):
    return self.ctx.model_get()


def _rows(hypergraph):
  max_node = max(i for i in hypergraph.node)
  max_edge = max(i for i in hypergraph.edge)
  return max_node + 2, max_edge + 2


def BooleanModel(hypergraph, dimension, num_neighbors):
  n, e = _rows(hypergraph)
  return Hg2vModel(n, e, dimension, num_neighbors, _hgx.LOSS_KLD,
                   _hgx.ACT_SIGMOID)


def UnweightedFloatModel(hypergraph, dimension, num_neighbors):
  n, e = _rows(hypergraph)
  return Hg2vModel(n, e, dimension, num_neighbors, _hgx.LOSS_MSE,
                   _hgx.ACT_RELU)


def KerasModelToEmbedding(hypergraph, model, node_map, edge_map,
                          node_layer_name="node_embedding",
                          edge_layer_name="edge_embedding"):
  """Rows idx + 1 of the trained tables, keyed by node_map / edge_map."""
  del node_layer_name, edge_layer_name
  node_w, edge_w = model.get_weights()
  emb = HypergraphEmbedding()
  emb.dim = int(node_w.shape[1])
  for node_idx in hypergraph.node:
    emb.node[node_map[node_idx]].values.extend(node_w[node_idx + 1].tolist())
  for edge_idx in hypergraph.edge:
    emb.edge[edge_map[edge_idx]].values.extend(edge_w[edge_idx + 1].tolist())
  return emb


__all__ = ["Hg2vModel", "BooleanModel", "UnweightedFloatModel",
           "KerasModelToEmbedding"]

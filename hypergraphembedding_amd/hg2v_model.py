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
          shuffle_seed=None, perms=None):
    """Keras fit(shuffle=True) + EarlyStopping(monitor='loss', min_delta,
    patience=0) over the records resident on the context."""
    return self.ctx.train(batch=batch_size, max_epochs=epochs, lr=lr, eps=eps,
                          loss=self.loss, act=self.act, min_delta=min_delta,
                          shuffle_seed=numpy_seed() if shuffle_seed is None
                          else shuffle_seed, perms=perms)

  def fit_streaming(self, chunk_fn, n_chunks, batch_size=256, epochs=10,
                    min_delta=1e-3, lr=0.01, eps=1e-7, seed=None,
                    chunk_perms=None, side=None):
    """fit() over a record stream too large to keep resident (SURVEY §5:
    "stream samples in chunks"; the reference materialises every record,
    embedding.py:277-284). chunk_fn(c) makes chunk c resident on the context
    and returns its record count; chunks must be the same records every
    epoch (the device samplers are keyed by seed and row, so re-sampling a
    row class reproduces it). Per epoch the chunk order is shuffled and each
    chunk's records are shuffled on the device: a windowed shuffle in place
    of Keras' global one over records that never coexist. The
    chunks are strided row classes (embedding._row_chunks), each a uniform
    slice of the graph, so a window mixes records of the whole id range;
    model state carries across chunks (one-epoch hgx_train calls), the epoch
    loss is the record-weighted mean and EarlyStopping(min_delta,
    patience=0) applies to it. Epoch ep's chunk order and shuffle seeds come
    from RandomState([seed, ep]). chunk_perms[ep][c] (optional) fixes a
    chunk's record order.

    side (optional): a second context on the same device that samples,
    `side.ctx` with `side.sample(c)` -> record count (chunk_fn is then
    unused). Chunk c + 1 is sampled on it while chunk c trains here (each
    context's work on its own stream, on disjoint CUs when both have
    stream_cus set); the host hands the chunk over (hgx_records_copy) once
    both are done -- no cross-stream barrier packet ever waits in a queue.
    Same records, order and seeds as the in-line form, so the same tables
    bit for bit.
    Returns the epoch losses; total records per epoch may exceed 2^31."""
    import threading
    import numpy as np
    base = numpy_seed() % (2**32) if seed is None else seed

    def plan(ep):
      ers = np.random.RandomState([base, ep])
      order = (np.arange(n_chunks) if chunk_perms is not None
               else ers.permutation(n_chunks))
      seeds = ers.randint(0, 2**62, size=n_chunks, dtype=np.int64)
      return [int(c) for c in order], [int(x) for x in seeds]

    def train(c, ep, shuffle_seed, out):
      try:
        perms = (None if chunk_perms is None
                 else chunk_perms[ep][c][None, :])
        self.ctx.train(batch=batch_size, max_epochs=1, lr=lr, eps=eps,
                       loss=self.loss, act=self.act, min_delta=-1e30,
                       shuffle_seed=shuffle_seed, perms=perms)
        out.append(self.ctx.train_loss_sum())
        self.chunk_stats.append((ep, c) + tuple(self.ctx.train_stats()))
      except BaseException as e:  # re-raised by the caller
        out.append(e)

    best, losses = float("inf"), []
    self.records_per_epoch = 0
    self.chunk_stats = []  # (epoch, chunk, step ms, records, batches)
    ahead = None  # (epoch, chunk, records) sampled on `side` ahead of time
    for ep in range(epochs):
      order, seeds = plan(ep)
      lsum, n = 0.0, 0
      for i, c in enumerate(order):
        if side is None:
          m = chunk_fn(c)
          if m == 0:
            continue
          out = []
          train(c, ep, seeds[i], out)
        else:
          if ahead is not None and ahead[:2] == (ep, c):
            m = ahead[2]
          else:
            m = side.sample(c)
          ahead = None
          if m == 0:
            continue
          self.ctx.records_copy_from(side.ctx)
          nxt = ((ep, order[i + 1]) if i + 1 < len(order) else
                 (ep + 1, plan(ep + 1)[0][0]) if ep + 1 < epochs else None)
          out = []
          th = threading.Thread(target=train, args=(c, ep, seeds[i], out))
          th.start()
          try:
            if nxt is not None:
              ahead = (nxt[0], nxt[1], side.sample(nxt[1]))
          finally:
            th.join()
        if isinstance(out[0], BaseException):
          raise out[0]
        lsum += out[0]
        n += m
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

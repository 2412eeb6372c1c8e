"""Keras-style dense models on the MI355X MLP engine (hgx_mlp_*).

The reference builds two small Keras models off the FOBE/HOBE path: the
node/edge classifier of the link-prediction experiment
(evaluation_util.py:471-505) and the combiner MLPs of
combine_embeddings_util.py:80-174. ``DenseModel`` owns one engine for either
and gives it Keras 2.x defaults: Dense kernels glorot_uniform
(limit sqrt(6 / (fan_in + fan_out))) and zero biases drawn from numpy's
global RandomState, Adagrad(lr=0.01, epsilon=1e-7), MSE, batch 256, a shuffle
per epoch and EarlyStopping(monitor='loss', min_delta, patience=0).
Samples are (node row, edge row, label) triples into two tables resident in
HBM; the engine gathers the rows itself.
"""

import numpy as np

from . import _hgx
from .runtime import get_context, numpy_seed

LP_CLASSIFIER = _hgx.MLP_LP_CLASSIFIER
NE_SUPERVISED = _hgx.MLP_NE_SUPERVISED
NE_SEMI_SUPERVISED = _hgx.MLP_NE_SEMI_SUPERVISED


def glorot_uniform_weights(shapes, rs=np.random):
  """Flat weights (per layer: kernel K x N row-major, then bias N)."""
  parts = []
  for k, n in shapes:
    lim = np.sqrt(6.0 / (k + n))
    parts.append(rs.uniform(-lim, lim, (k, n)).astype(np.float32).ravel())
    parts.append(np.zeros(n, np.float32))
  return np.concatenate(parts)


class DenseModel:
  """One Keras model on the device; ``in_dim`` = width of a table row."""

  def __init__(self, kind, in_dim, out_dim=0, ctx=None):
    self.ctx = ctx or get_context()
    self.kind, self.in_dim, self.out_dim = kind, in_dim, out_dim
    self.engine = _hgx.Mlp(self.ctx, kind, in_dim, out_dim)
    self.engine.set_weights(glorot_uniform_weights(self.engine.shapes))
    self.epoch_losses = np.zeros(0, np.float32)

  @property
  def shapes(self):
    return self.engine.shapes

  def set_tables(self, node_tab, edge_tab):
    self.engine.set_tables(node_tab, edge_tab)

  def fit(self, node_row, edge_row, label, epochs, min_delta=0.0, batch=256,
          lr=0.01, eps=1e-7, perms=None):
    """Keras fit(shuffle=True) with EarlyStopping(monitor='loss')."""
    self.engine.set_samples(node_row, edge_row, label)
    seed = numpy_seed()
    self.epoch_losses = self.engine.fit(batch=batch, max_epochs=epochs, lr=lr,
                                        eps=eps, min_delta=min_delta,
                                        seed=seed, perms=perms)
    return self.epoch_losses

  def predict_label(self, node_row, edge_row):
    return self.engine.predict(0, node_row, edge_row)

  def predict_joint(self, which, rows):
    """which 1: JointNode of node-table rows, 2: JointEdge of edge rows."""
    return self.engine.predict(which, rows if which == 1 else None,
                               rows if which == 2 else None)

  def stats(self):
    return self.engine.stats()

  def close(self):
    self.engine.close()

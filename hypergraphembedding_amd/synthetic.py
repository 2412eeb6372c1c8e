"""Synthetic hypergraphs of SURVEY.md §8(d) (BASELINE.json configs 2-5).

* random   (C2/C3): N=100 000 nodes, E=50 000 edges; node degree
  1 + Poisson(19) (mean 20); each node's edges drawn uniformly without
  duplicates; nnz ~ 2.0e6, mean edge size ~ 40.
* powerlaw (C4/C5): N=10 000 000, E=5 000 000; node degree 1 + Poisson(19);
  edge choice proportional to rank^-0.8 (Zipf-like edge sizes). Built by
  libhgx's host generator (numpy sorts of 2e8 keys take minutes).

Both return an :class:`Incidence` directly (no proto: a 2e8-incidence proto
is beyond Python protobuf). Edges that receive no node are dropped, so every
row is non-empty (an isolated row makes the reference's alg-dist divide by
zero, algebraic_distance.py:49). Deterministic for a seed.
"""

import numpy as np

from .hypergraph_util import Incidence


def _dedup_rows(rows, cols, ncols, draw, rng):
  """Redraw duplicate (row, col) pairs until every row's columns are
  distinct (the reference's AddNodeToEdge never stores a duplicate)."""
  for _ in range(64):
    key = rows.astype(np.int64) * ncols + cols
    order = np.argsort(key, kind="stable")
    dup = np.zeros(key.size, bool)
    ks = key[order]
    dup[order[1:]] = ks[1:] == ks[:-1]
    if not dup.any():
      break
    cols[dup] = draw(int(dup.sum()), rng)
  return rows, cols


def _finish(N, E, rows, cols):
  used = np.zeros(E, bool)
  used[cols] = True
  if not used.all():
    remap = np.cumsum(used) - 1
    cols = remap[cols].astype(np.int64)
    E = int(used.sum())
  order = np.lexsort((cols, rows))
  rows, cols = rows[order], cols[order]
  rp = np.zeros(N + 1, np.int64)
  np.add.at(rp, rows + 1, 1)
  rp = np.cumsum(rp)
  return Incidence(N, E, rp.astype(np.int32), cols.astype(np.int32))


def random_hypergraph(N=100_000, E=50_000, mean_degree=20, seed=0):
  rng = np.random.default_rng(seed)
  deg = 1 + rng.poisson(mean_degree - 1, N)
  deg = np.minimum(deg, E)
  rows = np.repeat(np.arange(N, dtype=np.int64), deg)
  draw = lambda n, r: r.integers(0, E, n)
  cols = draw(rows.size, rng)
  rows, cols = _dedup_rows(rows, cols, E, draw, rng)
  return _finish(N, E, rows, cols)


def powerlaw_hypergraph(N=10_000_000, E=5_000_000, mean_degree=20,
                        exponent=0.8, seed=0):
  """C4/C5 shape, generated natively (libhgx hgx_synth_powerlaw: alias-table
  Zipf draws, counting-sort transpose; ~2e8 incidences in seconds)."""
  from . import _hgx
  rp_n, col_n, E_kept = _hgx.synth_powerlaw(N, E, float(mean_degree),
                                           float(exponent), seed)
  rp_e, col_e = _hgx.csr_transpose(N, E_kept, rp_n, col_n)
  return Incidence(N, E_kept, rp_n, col_n, rp_e, col_e)


CONFIGS = {
    "random_100k": lambda seed=0: random_hypergraph(seed=seed),
    "powerlaw_10m": lambda seed=0: powerlaw_hypergraph(seed=seed),
}

"""The samplers' record streams pinned bit for bit (tests/golden/
stream_sha.json, made by tests/golden/make_stream_sha.py on an MI355X):
HOBE and FOBE on a 20k/10k power-law graph with the oracle's alg-dist
coordinates. The samplers' speed work (interleaved probes, LDS membership
walks, Bloom filters of the member sets) must leave every record -- ids,
neighbour lists, probabilities -- unchanged; a deliberate change of the
stream regenerates the file."""

import hashlib
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def stream_shas():
  import oracle as O
  from hypergraphembedding_amd import _hgx
  from hypergraphembedding_amd.synthetic import powerlaw_hypergraph
  inc = powerlaw_hypergraph(N=20_000, E=10_000, seed=5)
  r = O.Rng(3)
  x, y = O.algdist(inc, r.random((inc.N, 10)), r.random((inc.E, 10)), 20)
  ctx = _hgx.Context(0)
  out = {}
  try:
    ctx.upload(inc)
    ctx.alg_set(x.astype(np.float32), y.astype(np.float32))
    for name, n in (("hobe", lambda: ctx.sample_hobe(17, 5, 20)),
                    ("fobe_ns", lambda: ctx.sample_fobe(
                        29, 5, np.full(inc.N, 20, np.int32), np.full(inc.E, 20, np.int32),
                        np.full(inc.N, 7, np.int32), np.full(inc.E, 7, np.int32)))):
      m = n()
      idx, tgt = ctx.records_get()
      h = hashlib.sha256()
      h.update(idx.tobytes())
      h.update(tgt.tobytes())
      out[name] = {"records": int(m), "sha256": h.hexdigest()}
  finally:
    ctx.close()
  return out


def test_sampler_streams_pinned():
  with open(os.path.join(HERE, "golden", "stream_sha.json")) as f:
    want = json.load(f)
  assert stream_shas() == want

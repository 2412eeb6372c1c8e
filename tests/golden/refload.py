"""Load the reference's Keras-free modules in THIS container (golden generation only).

Never imported by the product, by ``-m gpu`` tests, by ``smoke()`` or by
``bench.py``: ``/root/reference`` does not exist on the GPU box. Follows the
loader recipe of SURVEY.md §8(c): the package ``__init__`` (which pulls in
keras via embedding.py:31-36) is bypassed by a stub package whose ``__path__``
points at the reference directory, ``hypergraph_pb2`` is provided by our
runtime-built descriptor (hypergraphembedding_amd/proto.py) and the real
submodules are loaded from their files.
"""

import importlib.util
import os
import sys
import types

REF = "/root/reference/hypergraph_embedding"


def load():
  here = os.path.dirname(os.path.abspath(__file__))
  sys.path.insert(0, os.path.dirname(os.path.dirname(here)))
  from hypergraphembedding_amd import proto

  if "hypergraph_embedding" in sys.modules and hasattr(
      sys.modules["hypergraph_embedding"], "_graft_stub"):
    return sys.modules["hypergraph_embedding"]
  pkg = types.ModuleType("hypergraph_embedding")
  pkg.__path__ = [REF]
  pkg._graft_stub = True
  for n in ("Hypergraph", "HypergraphEmbedding", "EvaluationMetrics",
            "ExperimentalResult"):
    setattr(pkg, n, getattr(proto, n))
  sys.modules["hypergraph_embedding"] = pkg
  pb2 = types.ModuleType("hypergraph_embedding.hypergraph_pb2")
  for n in ("Hypergraph", "HypergraphEmbedding", "EvaluationMetrics",
            "ExperimentalResult"):
    setattr(pb2, n, getattr(proto, n))
  sys.modules["hypergraph_embedding.hypergraph_pb2"] = pb2
  sys.dont_write_bytecode = True
  for mod in ("hypergraph_util", "algebraic_distance", "hg2v_weighting",
              "hg2v_sample"):
    full = f"hypergraph_embedding.{mod}"
    spec = importlib.util.spec_from_file_location(full,
                                                  os.path.join(REF, mod + ".py"))
    m = importlib.util.module_from_spec(spec)
    sys.modules[full] = m
    spec.loader.exec_module(m)
    setattr(pkg, mod, m)
  return pkg

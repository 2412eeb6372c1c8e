"""Native hypergraph.proto I/O for graphs beyond Python protobuf
(runner.py:352-364 reads the proto and writes the
embedding the same way, through Python protobuf).

``read_incidence(path_or_bytes)`` parses a serialized ``Hypergraph``
(hypergraph.proto:6-23) in libhgx and returns the same :class:`Incidence`
as ``Incidence.from_hypergraph(parsed message)``, without building the
message: the C4 graph (2e8 incidences) takes seconds instead of minutes.
The file is memory-mapped, not copied.

``write_embedding(path, inc, node_tab, edge_tab, method_name)`` writes a
``HypergraphEmbedding`` (hypergraph.proto:26-35) keyed by the original ids,
parsing to the same message as ``coords_to_embedding(...)``. Entries are
written in ascending id order.
Messages over 2 GiB are written too (protobuf itself refuses to serialise
them); readers must then stream them.
"""

import mmap
import os

import numpy as np

from . import _hgx
from .hypergraph_util import Incidence


def read_incidence(src):
  """Incidence from a Hypergraph file path or its serialized bytes."""
  if isinstance(src, (str, os.PathLike)):
    with open(src, "rb") as f:
      size = os.fstat(f.fileno()).st_size
      if size == 0:
        return _from_parsed(_hgx.parse_hypergraph(b""))
      with mmap.mmap(f.fileno(), 0, access=mmap.ACCESS_READ) as m:
        parsed = _hgx.parse_hypergraph(m)
    return _from_parsed(parsed)
  return _from_parsed(_hgx.parse_hypergraph(src))


def _from_parsed(p):
  rp_e, col_e = _hgx.csr_transpose(p["N"], p["E"], p["rp_n"], p["col_n"])
  return Incidence(p["N"], p["E"], p["rp_n"], p["col_n"], rp_e, col_e,
                   node_ids=p["node_ids"], edge_ids=p["edge_ids"],
                   node_weight=p["node_weight"], edge_weight=p["edge_weight"])


def embedding_bytes(inc, node_tab, edge_tab, method_name):
  """Wire bytes of the HypergraphEmbedding of compressed rows node_tab[i] /
  edge_tab[j], keyed by inc.node_ids[i] / inc.edge_ids[j]."""
  return _hgx.write_embedding_bytes(inc.node_ids, node_tab, inc.edge_ids,
                                    edge_tab, method_name)


def write_embedding(path, inc, node_tab, edge_tab, method_name):
  buf = embedding_bytes(inc, node_tab, edge_tab, method_name)
  with open(path, "wb") as f:
    f.write(memoryview(buf))
  return buf.size


__all__ = ["read_incidence", "write_embedding", "embedding_bytes"]

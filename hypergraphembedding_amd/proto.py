"""Runtime-built protobuf classes for ``hypergraph.proto``.

The image has no ``protoc``, so instead of a generated ``hypergraph_pb2`` we
build the same ``FileDescriptorProto`` by hand. Field numbers, labels, types
and defaults follow reference ``hypergraph_embedding/hypergraph.proto:1-69``
exactly, so the wire format is byte-compatible with files written by the
reference's ``runner.py`` (runner.py:352-364).

Exports ``Hypergraph``, ``HypergraphEmbedding``, ``EvaluationMetrics`` and
``ExperimentalResult`` (the names the reference re-exports from its package
``__init__``, hypergraph_embedding/__init__.py:18-23).
"""

from google.protobuf import descriptor_pb2
from google.protobuf import descriptor_pool
from google.protobuf import message_factory

_PKG = "hypergraph_embedding"
_F = descriptor_pb2.FieldDescriptorProto


def _field(msg, name, number, ftype, label=_F.LABEL_OPTIONAL, type_name=None,
           default=None):
  f = msg.field.add()
  f.name = name
  f.number = number
  f.type = ftype
  f.label = label
  if type_name is not None:
    f.type_name = type_name
  if default is not None:
    f.default_value = default
  return f


def _map_entry(parent, entry_name, value_type_name):
  """proto2 map<int32, Msg> = repeated nested *Entry{key=1, value=2}."""
  entry = parent.nested_type.add()
  entry.name = entry_name
  entry.options.map_entry = True
  _field(entry, "key", 1, _F.TYPE_INT32)
  _field(entry, "value", 2, _F.TYPE_MESSAGE, type_name=value_type_name)
  return entry


def _build_file():
  fd = descriptor_pb2.FileDescriptorProto()
  fd.name = "hypergraph_embedding/hypergraph.proto"
  fd.package = _PKG
  fd.syntax = "proto2"

  # message Hypergraph (hypergraph.proto:6-23)
  hg = fd.message_type.add()
  hg.name = "Hypergraph"
  nd = hg.nested_type.add()
  nd.name = "NodeData"
  _field(nd, "edges", 1, _F.TYPE_INT32, _F.LABEL_REPEATED)
  _field(nd, "name", 2, _F.TYPE_STRING)
  _field(nd, "weight", 3, _F.TYPE_FLOAT, default="1")
  ed = hg.nested_type.add()
  ed.name = "EdgeData"
  _field(ed, "nodes", 1, _F.TYPE_INT32, _F.LABEL_REPEATED)
  _field(ed, "name", 2, _F.TYPE_STRING)
  _field(ed, "weight", 3, _F.TYPE_FLOAT, default="1")
  _map_entry(hg, "NodeEntry", f".{_PKG}.Hypergraph.NodeData")
  _map_entry(hg, "EdgeEntry", f".{_PKG}.Hypergraph.EdgeData")
  _field(hg, "node", 1, _F.TYPE_MESSAGE, _F.LABEL_REPEATED,
         f".{_PKG}.Hypergraph.NodeEntry")
  _field(hg, "edge", 2, _F.TYPE_MESSAGE, _F.LABEL_REPEATED,
         f".{_PKG}.Hypergraph.EdgeEntry")
  _field(hg, "name", 3, _F.TYPE_STRING)

  # message HypergraphEmbedding (hypergraph.proto:26-35)
  he = fd.message_type.add()
  he.name = "HypergraphEmbedding"
  em = he.nested_type.add()
  em.name = "Embedding"
  _field(em, "values", 1, _F.TYPE_FLOAT, _F.LABEL_REPEATED)
  _map_entry(he, "NodeEntry", f".{_PKG}.HypergraphEmbedding.Embedding")
  _map_entry(he, "EdgeEntry", f".{_PKG}.HypergraphEmbedding.Embedding")
  _field(he, "node", 1, _F.TYPE_MESSAGE, _F.LABEL_REPEATED,
         f".{_PKG}.HypergraphEmbedding.NodeEntry")
  _field(he, "edge", 2, _F.TYPE_MESSAGE, _F.LABEL_REPEATED,
         f".{_PKG}.HypergraphEmbedding.EdgeEntry")
  _field(he, "dim", 3, _F.TYPE_INT32)
  _field(he, "method_name", 4, _F.TYPE_STRING)

  # message EvaluationMetrics (hypergraph.proto:37-58)
  ev = fd.message_type.add()
  ev.name = "EvaluationMetrics"
  for i, n in enumerate(["accuracy", "precision", "recall", "f1"], start=1):
    _field(ev, n, i, _F.TYPE_FLOAT)
  for i, n in enumerate(["num_true_pos", "num_true_neg", "num_false_pos",
                         "num_false_neg"], start=5):
    _field(ev, n, i, _F.TYPE_INT32)
  _field(ev, "experiment_name", 9, _F.TYPE_STRING)
  rec = ev.nested_type.add()
  rec.name = "EvaluationRecord"
  _field(rec, "node_idx", 1, _F.TYPE_INT32)
  _field(rec, "edge_idx", 2, _F.TYPE_INT32)
  _field(rec, "label", 3, _F.TYPE_BOOL)
  _field(rec, "prediction", 4, _F.TYPE_BOOL)
  _field(ev, "records", 10, _F.TYPE_MESSAGE, _F.LABEL_REPEATED,
         f".{_PKG}.EvaluationMetrics.EvaluationRecord")

  # message ExperimentalResult (hypergraph.proto:60-69)
  er = fd.message_type.add()
  er.name = "ExperimentalResult"
  _field(er, "hypergraph", 1, _F.TYPE_MESSAGE, type_name=f".{_PKG}.Hypergraph")
  _field(er, "embedding", 2, _F.TYPE_MESSAGE,
         type_name=f".{_PKG}.HypergraphEmbedding")
  _field(er, "metrics", 3, _F.TYPE_MESSAGE, _F.LABEL_REPEATED,
         f".{_PKG}.EvaluationMetrics")
  _field(er, "removal_probability", 4, _F.TYPE_FLOAT)
  return fd


_pool = descriptor_pool.DescriptorPool()
_file = _pool.Add(_build_file())


def _cls(name):
  return message_factory.GetMessageClass(
      _pool.FindMessageTypeByName(f"{_PKG}.{name}"))


Hypergraph = _cls("Hypergraph")
HypergraphEmbedding = _cls("HypergraphEmbedding")
EvaluationMetrics = _cls("EvaluationMetrics")
ExperimentalResult = _cls("ExperimentalResult")

__all__ = ["Hypergraph", "HypergraphEmbedding", "EvaluationMetrics",
           "ExperimentalResult"]

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
parsing to the same message as ``coords_to_embedding(...)``; entries in
ascending id order. An embedding whose message would exceed protobuf's
2 GiB limit (C4: 10M x 256 floats, ~10 GB) is written as shards
``path-00000-of-0000n``: each shard is a complete ``HypergraphEmbedding``
(same ``dim`` and ``method_name``) under the limit, holding a contiguous
id range; together they are the one message (concatenating the shard
bytes IS its wire encoding: protobuf merges map entries).

``read_embedding(path)`` reads either form back -- natively (any size) or
through Python protobuf one shard at a time -- and merges the shards.

``ShardedEmbedding`` is what the embedders return when the message would
exceed the limit: the tables plus the message surface callers use (``dim``,
``method_name``, ``node`` / ``edge`` maps, ``SerializeToString``) and
``shards()`` / ``write(path)``.
"""

import mmap
import os
import re

import numpy as np

from . import _hgx
from .hypergraph_util import Incidence

# protobuf refuses to parse messages of 2 GiB or more; shards stay below
PROTO_LIMIT = 2**31 - 1
SHARD_BYTES = PROTO_LIMIT - (1 << 20)


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
  edge_tab[j], keyed by inc.node_ids[i] / inc.edge_ids[j] (one message)."""
  return _hgx.write_embedding_bytes(inc.node_ids, node_tab, inc.edge_ids,
                                    edge_tab, method_name)


# ---- sizes of the wire encoding (hgx_proto.hip put_entry) -----------------
def _varint_len(v):
  v = np.asarray(v, np.uint64)
  n = np.ones(v.shape, np.int64)
  for s in range(7, 64, 7):
    n += (v >= np.uint64(1) << np.uint64(s)).astype(np.int64)
  return n


def _entry_bytes(ids, d):
  """Wire bytes of each map<int32, Embedding> entry (unpacked floats)."""
  key = np.asarray(ids, np.int64).astype(np.int32).astype(np.int64)
  body = 1 + _varint_len(key.view(np.uint64)) + 1 + _varint_len(5 * d) + 5 * d
  return 1 + _varint_len(body) + body


def _tail_bytes(d, method_name):
  n = 1 + int(_varint_len(np.int64(d).astype(np.int32).astype(np.int64)
                          .view(np.uint64)))
  if method_name is not None:
    m = len(method_name.encode())
    n += 1 + int(_varint_len(m)) + m
  return n


def message_bytes(node_ids, edge_ids, d, method_name):
  """Serialized size of the whole HypergraphEmbedding (one message)."""
  return int(_entry_bytes(node_ids, d).sum() + _entry_bytes(edge_ids, d).sum()
             + _tail_bytes(d, method_name))


class _Row:
  __slots__ = ("values",)

  def __init__(self, values):
    self.values = values


class _MapView:
  """Read-only view of one map<int32, Embedding> of a ShardedEmbedding."""

  def __init__(self, ids, tab):
    self._ids, self._tab = ids, tab
    self._order = np.argsort(ids, kind="stable")
    self._sorted = ids[self._order]

  def __len__(self):
    return int(self._ids.size)

  def __iter__(self):
    return iter(int(i) for i in self._sorted)

  def _row(self, key):
    j = int(np.searchsorted(self._sorted, key))
    if j >= self._sorted.size or self._sorted[j] != key:
      return -1
    return int(self._order[j])

  def __contains__(self, key):
    return self._row(key) >= 0

  def __getitem__(self, key):
    r = self._row(key)
    if r < 0:
      raise KeyError(key)
    return _Row(self._tab[r].tolist())

  def keys(self):
    return list(iter(self))


class ShardedEmbedding:
  """A HypergraphEmbedding too large for one protobuf message, kept as its
  tables (rows keyed by original ids). Message surface: dim, method_name,
  node / edge maps (len, iteration, membership, [id].values),
  SerializeToString() (the shards concatenated: the wire encoding of the one
  merged message, readable by read_embedding at any size). shards() yields
  HypergraphEmbedding messages under the limit; write(path) stores them as
  shard files."""

  def __init__(self, node_ids, node_tab, edge_ids, edge_tab, dim,
               method_name="", shard_bytes=None):
    self.node_ids = np.ascontiguousarray(node_ids, np.int64)
    self.edge_ids = np.ascontiguousarray(edge_ids, np.int64)
    self.node_tab = np.ascontiguousarray(node_tab, np.float32)
    self.edge_tab = np.ascontiguousarray(edge_tab, np.float32)
    self.dim = int(dim)
    self.method_name = method_name
    # the module value at construction (tests lower it)
    self.shard_bytes = SHARD_BYTES if shard_bytes is None else shard_bytes
    self.node = _MapView(self.node_ids, self.node_tab)
    self.edge = _MapView(self.edge_ids, self.edge_tab)

  def ByteSize(self):
    return message_bytes(self.node_ids, self.edge_ids, self.dim,
                         self.method_name)

  def shard_bytes_iter(self):
    """Wire bytes (uint8 arrays) of each shard, in id order."""
    for sel_n, sel_e in _shard_plan(self.node_ids, self.edge_ids, self.dim,
                                    self.method_name, self.shard_bytes):
      yield _hgx.write_embedding_bytes(self.node_ids[sel_n],
                                       self.node_tab[sel_n],
                                       self.edge_ids[sel_e],
                                       self.edge_tab[sel_e], self.method_name)

  def shards(self):
    from .proto import HypergraphEmbedding
    for b in self.shard_bytes_iter():
      m = HypergraphEmbedding()
      m.ParseFromString(memoryview(b))
      yield m

  def SerializeToString(self):
    return b"".join(bytes(memoryview(b)) for b in self.shard_bytes_iter())

  def write(self, path):
    return _write_shards(path, self.shard_bytes_iter(),
                         len(_shard_plan(self.node_ids, self.edge_ids,
                                         self.dim, self.method_name,
                                         self.shard_bytes)))


def _shard_plan(node_ids, edge_ids, d, method_name, shard_bytes):
  """[(node rows, edge rows)] of each shard: entries in ascending id order
  (nodes, then edges) cut greedily so that each shard's message, dim and
  method_name included, stays within shard_bytes."""
  on = np.argsort(node_ids, kind="stable")
  oe = np.argsort(edge_ids, kind="stable")
  sizes = np.concatenate([_entry_bytes(node_ids[on], d),
                          _entry_bytes(edge_ids[oe], d)])
  cap = shard_bytes - _tail_bytes(d, method_name)
  assert sizes.size == 0 or sizes.max() <= cap, "one entry exceeds the shard size"
  cuts, start, cum = [0], 0, np.cumsum(sizes)
  while start < sizes.size:
    base = cum[start - 1] if start else 0
    end = int(np.searchsorted(cum, base + cap, side="right"))
    cuts.append(end)
    start = end
  if len(cuts) == 1:
    cuts.append(0)
  plan, nn = [], node_ids.size
  for a, b in zip(cuts[:-1], cuts[1:]):
    plan.append((on[min(a, nn):min(b, nn)], oe[max(a - nn, 0):max(b - nn, 0)]))
  return plan


def shard_name(path, i, n):
  return f"{path}-{i:05d}-of-{n:05d}"


def _shard_files(path):
  """Files named exactly as shard_name(path, i, n) names them (i < n, both
  at least five digits): not `path-1-00000-of-00002`, a shard of another
  embedding saved at `path-1`."""
  path = str(path)
  d, base = os.path.split(path)
  pat = re.compile(re.escape(base) + r"-(\d{5,})-of-(\d{5,})")
  out = []
  try:
    names = os.listdir(d or ".")
  except FileNotFoundError:
    return out
  for name in names:
    m = pat.fullmatch(name)
    if m and int(m.group(1)) < int(m.group(2)):
      out.append(os.path.join(d, name) if d else name)
  return out


def _clear_outputs(path):
  """Remove an earlier embedding at `path` (the single file and any shards
  of any count), so that a later read never mixes layouts or shard counts."""
  for name in [str(path)] + _shard_files(path):
    if os.path.isfile(name):
      os.remove(name)


def _write_shards(path, bufs, n):
  _clear_outputs(path)
  if n == 1:
    names = [str(path)]
  else:
    names = [shard_name(path, i, n) for i in range(n)]
  for name, b in zip(names, bufs):
    with open(name, "wb") as f:
      f.write(memoryview(b))
  return names


def write_embedding(path, inc, node_tab, edge_tab, method_name,
                    shard_bytes=None):
  """Write the embedding of compressed rows node_tab / edge_tab keyed by the
  original ids: one file `path` if the message fits protobuf's limit, else
  shards `path-00000-of-0000n` (each a complete HypergraphEmbedding under
  shard_bytes). Returns the file names."""
  node_tab = np.ascontiguousarray(node_tab, np.float32)
  d = int(node_tab.shape[1])
  emb = ShardedEmbedding(inc.node_ids, node_tab, inc.edge_ids, edge_tab, d,
                         method_name, shard_bytes=shard_bytes)
  return emb.write(path)


def save_embedding(path, emb):
  """Write an embedder's result: a HypergraphEmbedding message to `path`
  (runner.py:363-364), or a ShardedEmbedding as its shards. Returns the
  file names."""
  if isinstance(emb, ShardedEmbedding):
    return emb.write(path)
  _clear_outputs(path)
  with open(path, "wb") as f:
    f.write(emb.SerializeToString())
  return [str(path)]


def embedding_files(path):
  """The files of the embedding at `path`: [path] or its shards in order.
  Raises if both layouts, or shards of more than one count, are present (a
  stale earlier write: the caller cannot tell which one is current)."""
  path = str(path)
  names = sorted(_shard_files(path))
  if os.path.exists(path):
    if names:
      raise FileExistsError(f"{path} exists both as one file and as "
                            f"{len(names)} shard files")
    return [path]
  if not names:
    raise FileNotFoundError(path)
  counts = sorted({int(x.rsplit("-of-", 1)[1]) for x in names})
  if len(counts) > 1:
    raise FileExistsError(f"{path}: shards of {counts} different counts")
  n = counts[0]
  want = [shard_name(path, i, n) for i in range(n)]
  missing = sorted(set(want) - set(names))
  if missing:
    raise FileNotFoundError(f"missing embedding shards: {missing[:3]}")
  return want


def read_embedding(path, native=True):
  """ShardedEmbedding-shaped tables (ids ascending, the merged message) of
  the embedding written at `path` (one file or its shards). native: libhgx's
  parser (any size, every shard at once); otherwise Python protobuf, one
  message per shard."""
  files = embedding_files(path)
  if native:
    parts = []
    for name in files:
      with open(name, "rb") as f:
        if os.fstat(f.fileno()).st_size == 0:
          parts.append(_hgx.parse_embedding(b""))
          continue
        with mmap.mmap(f.fileno(), 0, access=mmap.ACCESS_READ) as m:
          parts.append(_hgx.parse_embedding(m))
  else:
    from .proto import HypergraphEmbedding
    parts = []
    for name in files:
      m = HypergraphEmbedding()
      with open(name, "rb") as f:
        m.ParseFromString(f.read())
      parts.append(_message_tables(m))
  return _merge(parts)


def _message_tables(m):
  def tab(mp):
    ids = np.array(sorted(mp.keys()), np.int64)
    w = len(mp[int(ids[0])].values) if ids.size else m.dim
    t = np.empty((ids.size, w), np.float32)
    for i, k in enumerate(ids.tolist()):
      t[i] = mp[k].values
    return ids, t
  ni, nt = tab(m.node)
  ei, et = tab(m.edge)
  return {"node_ids": ni, "node_tab": nt, "edge_ids": ei, "edge_tab": et,
          "dim": m.dim, "method_name": m.method_name}


def _merge(parts):
  """Later parts win on a repeated key, as protobuf's merge does. Shards
  written here hold ascending, disjoint id ranges: then the parts are only
  concatenated (one part: returned as parsed), with no dedup copy."""
  out = {}
  for side in ("node", "edge"):
    tabs = [p[f"{side}_tab"] for p in parts]
    w = max((t.shape[1] for t in tabs if t.size), default=0)
    tabs = [t.reshape(-1, w) if t.size else np.zeros((0, w), np.float32)
            for t in tabs]
    if len(parts) == 1:
      ids, tab = parts[0][f"{side}_ids"], tabs[0]
    else:
      ids = np.concatenate([p[f"{side}_ids"] for p in parts])
      tab = None
    if ids.size < 2 or bool(np.all(ids[1:] > ids[:-1])):
      out[f"{side}_ids"] = ids
      out[f"{side}_tab"] = tab if tab is not None else np.concatenate(tabs)
      continue
    if tab is None:
      tab = np.concatenate(tabs)
    rev = np.argsort(ids[::-1], kind="stable")  # last occurrence first
    first = np.ones(ids.size, bool)
    first[1:] = ids[::-1][rev][1:] != ids[::-1][rev][:-1]
    pick = (ids.size - 1 - rev)[first]
    out[f"{side}_ids"], out[f"{side}_tab"] = ids[pick], tab[pick]
  last = parts[-1] if parts else {"dim": 0, "method_name": ""}
  dims = [p["dim"] for p in parts if p["dim"]]
  names = [p["method_name"] for p in parts if p["method_name"]]
  return ShardedEmbedding(out["node_ids"], out["node_tab"], out["edge_ids"],
                          out["edge_tab"], dims[-1] if dims else last["dim"],
                          names[-1] if names else "")


__all__ = ["read_incidence", "write_embedding", "embedding_bytes",
           "read_embedding", "save_embedding", "ShardedEmbedding",
           "embedding_files",
           "message_bytes", "PROTO_LIMIT", "SHARD_BYTES"]

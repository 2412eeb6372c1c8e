"""Host restatement of the record store's epoch order (csrc/hgx_store.hip:
epoch_keys, epoch_key; hgx::mix64 in csrc/hgx_internal.h) for tests: the
key of entry (w0, w1) under an epoch seed, and the order sorting by it.
Test infrastructure only."""

import numpy as np

M64 = (1 << 64) - 1


def mix64(z):
  """splitmix64 finaliser on uint64 arrays (wrapping arithmetic)."""
  z = np.asarray(z, np.uint64)
  with np.errstate(over="ignore"):
    z = z + np.uint64(0x9e3779b97f4a7c15)
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xbf58476d1ce4e5b9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94d049bb133111eb)
  return z ^ (z >> np.uint64(31))


def epoch_keys(epoch_seed):
  s = np.uint64(epoch_seed & M64)
  return (mix64(s ^ np.uint64(0x53544f52454b3130)),
          mix64(s ^ np.uint64(0x53544f52454b3230)))


def entry_keys(entries, epoch_seed):
  """uint64 epoch keys of (n, 3) uint32 store entries."""
  e = np.asarray(entries, np.uint32)
  k1, k2 = epoch_keys(epoch_seed)
  ident = (e[:, 0].astype(np.uint64) << np.uint64(32)) | e[:, 1].astype(np.uint64)
  return mix64(mix64(ident ^ k1) ^ k2)


def epoch_order(entries, epoch_seed):
  """Positions of the entries in the epoch's global order."""
  return np.argsort(entry_keys(entries, epoch_seed), kind="stable")


def row_sort(idx, tgt):
  """Records sorted as rows (ids then target bits): multiset comparison."""
  a = np.concatenate([idx.astype(np.int64),
                      tgt.view(np.uint32).astype(np.int64)], 1)
  o = np.lexsort(a.T[::-1])
  return a[o]

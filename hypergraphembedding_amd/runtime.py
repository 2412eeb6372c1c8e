"""Per-process device context (one libhgx context per device).

The reference fans work out through fork Pools sharing module globals
(algebraic_distance.py:9, hg2v_sample.py:27). Here every hot-path call goes
through one native context per device; the device is LOCAL_RANK (one process
per GPU under torch.distributed.run) unless set explicitly.
"""

import contextlib
import os
import threading

import numpy as np

from . import _hgx

_lock = threading.Lock()
_contexts = {}


def default_device():
  return int(os.environ.get("HGX_DEVICE", os.environ.get("LOCAL_RANK", "0")))


def get_context(device=None):
  """The process-wide context for `device` (created on first use). Raises if
  libhgx.so or a HIP device is missing -- there is no CPU fallback."""
  dev = default_device() if device is None else int(device)
  with _lock:
    ctx = _contexts.get(dev)
    if ctx is None:
      ctx = _hgx.Context(dev)
      _contexts[dev] = ctx
    return ctx


@contextlib.contextmanager
def scratch_context(device=None):
  """A private context for a side-effect-free call (it neither reads nor
  replaces the incidence, coordinates or records a caller left on the
  process-wide context), closed on exit."""
  ctx = _hgx.Context(default_device() if device is None else int(device))
  try:
    yield ctx
  finally:
    ctx.close()


def numpy_state_seed():
  """A 63-bit device seed derived from numpy's global RandomState WITHOUT
  drawing from it (a hash of its MT19937 key and position): the seed of the
  table init in rng="mt19937" runs, where numpy's stream must advance
  exactly as the reference's does (Keras draws its init from TF, not numpy)."""
  import hashlib
  st = np.random.get_state()
  h = hashlib.blake2b(np.asarray(st[1], np.uint32).tobytes() +
                      int(st[2]).to_bytes(4, "little"), digest_size=8)
  return int.from_bytes(h.digest(), "little") >> 1


RNG_MODES = (None, "mt19937")


def check_rng(rng):
  """rng=None: the device's counter-based draws keyed by a numpy-drawn seed
  (distribution parity); rng="mt19937": numpy's global RandomState stream
  itself, the reference's records and epoch shuffles bit for bit."""
  if rng not in RNG_MODES:
    raise ValueError("rng must be None or 'mt19937', not %r" % (rng,))
  return rng


def numpy_seed():
  """A 63-bit device seed drawn from numpy's global RandomState, so that
  np.random.seed(s) makes a whole embedding run reproducible, as it does for
  the reference (which draws everything from np.random)."""
  return int(np.random.randint(0, 2**62, dtype=np.int64))

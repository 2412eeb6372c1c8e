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


def numpy_seed():
  """A 63-bit device seed drawn from numpy's global RandomState, so that
  np.random.seed(s) makes a whole embedding run reproducible, as it does for
  the reference (which draws everything from np.random)."""
  return int(np.random.randint(0, 2**62, dtype=np.int64))

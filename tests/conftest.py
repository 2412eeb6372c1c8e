import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (ROOT, os.path.join(ROOT, "oracle")):
  if p not in sys.path:
    sys.path.insert(0, p)


def pytest_configure(config):
  config.addinivalue_line(
      "markers", "gpu: needs a real MI355X (runs the HIP path through libhgx)")


def golden(name):
  return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def golden_incidence(name):
  from hypergraphembedding_amd.hypergraph_util import Incidence
  z = golden(name)
  return Incidence(int(z["N"]), int(z["E"]), z["rp_n"], z["col_n"], z["rp_e"],
                   z["col_e"], node_ids=z["node_ids"], edge_ids=z["edge_ids"])


@pytest.fixture(scope="session")
def tiny_hypergraph():
  from hypergraphembedding_amd.proto import Hypergraph
  h = Hypergraph()
  with open(os.path.join(GOLDEN, "snap_youtube_tiny.hypergraph.pb"), "rb") as f:
    h.ParseFromString(f.read())
  return h


@pytest.fixture(scope="session")
def tiny_inc():
  return golden_incidence("csr_tiny.npz")


@pytest.fixture(scope="session")
def small_inc():
  return golden_incidence("csr_small.npz")


class Background:
  """CPU checker work run beside the GPU tests (session-wide): a test runs
  its device part, submits the oracle half here and a test at the end of
  the session (tests/test_gpu_zz_deferred.py) asserts on the result. Four
  workers: the C2 / C3 epoch checkers at 8 OpenMP threads each (the box's
  CPU share is 16) and the two C4 windows' single-threaded oracles."""

  def __init__(self):
    from concurrent.futures import ThreadPoolExecutor
    self.pool = ThreadPoolExecutor(4)
    self.jobs = {}

  def submit(self, key, fn):
    self.jobs[key] = self.pool.submit(fn)

  def result(self, key, fallback):
    """The submitted job's result, or fallback() run here when the device
    half did not run in this session (the deferred test run alone)."""
    job = self.jobs.pop(key, None)
    return job.result() if job is not None else fallback()


@pytest.fixture(scope="session")
def background():
  b = Background()
  yield b
  b.pool.shutdown(wait=True)

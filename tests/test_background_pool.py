"""conftest.Background, the pool the BASELINE-size GPU checkers run on
(CPU only): a submitted job's result comes back to the asserting test, a
job's exception reaches it, and a key never submitted falls back to
running the work inline."""

import pytest

from conftest import Background


def test_submit_then_result():
  b = Background()
  try:
    b.submit("k", lambda: 41 + 1)
    assert b.result("k", lambda: pytest.fail("fallback ran")) == 42
    # the key is consumed: a second result() runs the fallback
    assert b.result("k", lambda: "inline") == "inline"
  finally:
    b.pool.shutdown(wait=True)


def test_job_exception_reaches_the_asserting_test():
  b = Background()
  try:
    def boom():
      raise ValueError("checker failed")
    b.submit("k", boom)
    with pytest.raises(ValueError, match="checker failed"):
      b.result("k", lambda: None)
  finally:
    b.pool.shutdown(wait=True)

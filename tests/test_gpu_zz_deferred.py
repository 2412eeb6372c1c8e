"""The checker halves of the BASELINE-size trainer parity tests
(tests/test_gpu_baseline_parity.py: a full C3 HOBE epoch, ~60M records, and
a full C2 FOBE epoch, ~34M) and of the C4 d = 256 windows
(tests/test_gpu_c4.py), collected last: their CPU checkers ran in the
background while the other GPU tests used the device. Run alone, each test
does its device half itself first."""

import pytest

import test_gpu_baseline_parity as P
import test_gpu_c4 as C4

pytestmark = pytest.mark.gpu


@pytest.mark.timeout(900)
def test_c3_full_hobe_epoch_vs_oracle(background):
  P.assert_checked(background.result(
      "c3", lambda: P.checker(P._device_epoch("c3"))))


@pytest.mark.timeout(900)
def test_c2_full_fobe_epoch_vs_oracle(background):
  P.assert_checked(background.result(
      "c2", lambda: P.checker(P._device_epoch("c2"))))


def _c4_ctx():
  from hypergraphembedding_amd import _hgx
  from hypergraphembedding_amd.synthetic import powerlaw_hypergraph
  g = powerlaw_hypergraph(seed=0)
  ctx = _hgx.Context(0)
  ctx.upload(g)
  return ctx, g


def _window_inline(which):
  ctx, g = _c4_ctx()
  try:
    w = (C4.hobe_window if which == "hobe" else C4.fobe_window)(ctx, g)
  finally:
    ctx.close()
  return C4.window_check(w)


@pytest.mark.timeout(900)
def test_c4_d256_window_vs_oracle(background):
  frac = C4.assert_window(background.result(
      "c4_hobe_window", lambda: _window_inline("hobe")))
  assert frac >= 0.4


@pytest.mark.timeout(900)
def test_c4_fobe_d256_window_vs_oracle(background):
  C4.assert_window(background.result(
      "c4_fobe_window", lambda: _window_inline("fobe")))

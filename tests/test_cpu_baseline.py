"""The multi-threaded CPU baseline trainer (oracle/cpu_train_mt.c, timed by
bench.py) computes what the single-threaded oracle computes, up to the
summation order of duplicate rows."""

import numpy as np

import oracle as O


def test_train_mt_matches_oracle():
  rs = np.random.RandomState(0)
  n, K, N, E, d = 20_000, 5, 3_000, 1_500, 32
  idx = np.zeros((n, 4 + 2 * K), np.int32)
  kind = rs.randint(0, 3, n)
  idx[:, 0] = np.where(kind != 1, rs.randint(1, N + 1, n), 0)
  idx[:, 2] = np.where(kind == 0, rs.randint(1, N + 1, n), 0)
  idx[:, 1] = np.where(kind == 1, rs.randint(1, E + 1, n), 0)
  idx[:, 3] = np.where(kind != 0, rs.randint(1, E + 1, n), 0)
  m2 = kind == 2
  idx[m2, 4:4 + K] = rs.randint(1, N + 1, (m2.sum(), K))
  idx[m2, 4 + K:] = rs.randint(1, E + 1, (m2.sum(), K))
  tgt = np.zeros((n, 3), np.float32)
  tgt[np.arange(n), kind] = rs.uniform(0, 1, n)
  nt = rs.uniform(-0.05, 0.05, (N + 2, d)).astype(np.float32)
  et = rs.uniform(-0.05, 0.05, (E + 2, d)).astype(np.float32)
  for loss, act in ((O.LOSS_MSE, O.ACT_RELU), (O.LOSS_KLD, O.ACT_SIGMOID)):
    ref = O.train(idx, tgt, K, nt, et, loss, act, max_epochs=1,
                  min_delta=-1e30)
    a_nt, a_et = ref[0], ref[1]
    b_nt, b_et, _ = O.train_mt(idx, tgt, K, nt, et, loss, act, epochs=1,
                               threads=4)
    assert np.abs(a_nt - b_nt).max() < 1e-5
    assert np.abs(a_et - b_et).max() < 1e-5

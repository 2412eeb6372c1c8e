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
    # the checker build (the oracle of tests/test_gpu_baseline_parity.py)
    c_nt, c_et, c_loss = O.train_mt(idx, tgt, K, nt, et, loss, act, epochs=1,
                                    threads=4, exact=True)
    assert np.abs(a_nt - c_nt).max() < 1e-6
    assert np.abs(a_et - c_et).max() < 1e-6
    assert np.isclose(c_loss, ref[2][0], rtol=1e-6)


def test_cpu_hobe_sampler_baseline_computes_the_reference_quantities(small_inc):
  """The timed CPU sampler baseline (oracle/cpu_sample_mt.c) samples what
  AlgebraicDistanceSamples samples: per row min(S, |pattern row|) distinct
  valid columns in the four kind blocks, probabilities equal to the oracle's
  (bit-exact, same float formula), neighbours from the right rows."""
  inc, S, K = small_inc, 6, 3
  r = O.Rng(3)
  ax, ay = O.algdist(inc, r.random((inc.N, 10)), r.random((inc.E, 10)), 5)
  ax, ay = ax.astype(np.float32), ay.astype(np.float32)
  nq = np.full(inc.N, S, np.int32)
  eq = np.full(inc.E, S, np.int32)
  nq[::3] = 0
  idx, tgt, b = O.cpu_hobe_sample_mt(inc, ax, ay, nq, eq, K, seed=5, threads=2)
  A = np.zeros((inc.N, inc.E), int)
  A[np.repeat(np.arange(inc.N), np.diff(inc.rp_n)), inc.col_n] = 1
  pats = [A @ A.T > 0, A.T @ A > 0, A @ A.T @ A > 0, A.T @ A @ A.T > 0]
  cols = [(0, 2), (1, 3), (0, 3), (3, 0)]
  for blk in range(4):
    rec = idx[b[blk]:b[blk + 1]]
    q = nq if blk in (0, 2) else eq
    rc, cc = cols[blk]
    rows, cnt = np.unique(rec[:, rc] - 1, return_counts=True)
    want = np.minimum(q, pats[blk].sum(1))
    assert np.array_equal(np.bincount(rows, cnt, minlength=q.size), want)
    assert pats[blk][rec[:, rc] - 1, rec[:, cc] - 1].all()
  nn = slice(b[0], b[1])
  ee = slice(b[1], b[2])
  ne = slice(b[2], b[4])
  assert np.array_equal(tgt[nn, 0], O.hobe_probs(O.HOBE_NN, idx[nn, 0] - 1,
                                                 idx[nn, 2] - 1, inc, ax, ay))
  assert np.array_equal(tgt[ee, 1], O.hobe_probs(O.HOBE_EE, idx[ee, 1] - 1,
                                                 idx[ee, 3] - 1, inc, ax, ay))
  assert np.array_equal(tgt[ne, 2], O.hobe_probs(O.HOBE_NE, idx[ne, 0] - 1,
                                                 idx[ne, 3] - 1, inc, ax, ay))
  for i in range(int(b[2]), int(b[4])):
    v, e = idx[i, 0] - 1, idx[i, 3] - 1
    assert np.isin(idx[i, 4:4 + K] - 1, inc.col_e[inc.rp_e[e]:inc.rp_e[e + 1]]).all()
    assert np.isin(idx[i, 4 + K:] - 1, inc.col_n[inc.rp_n[v]:inc.rp_n[v + 1]]).all()

"""The MLP restatement (oracle/mlpref.c) against an independent float64
autograd formulation of the same Keras models (torch on the CPU): forward
values, the gradient of the Keras loss (sum over outputs of the weighted
batch mean of the per-sample mean squared error) and the Adagrad step.
A large Adagrad epsilon makes the step proportional to the gradient, so a
wrong gradient scale shows (with eps = 1e-7 Adagrad's first step is
lr * sign(g)). The dropout masks are the shared counter-based ones."""

import numpy as np
import pytest
import torch

import oracle as O

M64 = (1 << 64) - 1


def mix64(z):
  z = (z + 0x9e3779b97f4a7c15) & M64
  z = ((z ^ (z >> 30)) * 0xbf58476d1ce4e5b9) & M64
  z = ((z ^ (z >> 27)) * 0x94d049bb133111eb) & M64
  return z ^ (z >> 31)


def rand64(seed, stream, ctr):
  return mix64((mix64(seed ^ mix64((stream + 0x632be59bd9b4e019) & M64)) + ctr)
               & M64)


def drop_mask(seed, stream, M, width):
  in4 = (width + 3) // 4 * 4
  w64 = (in4 + 63) // 64
  mask = np.zeros((M, width), np.float64)
  for p in range(M):
    for k in range(width):
      r = rand64(seed, stream, p * w64 + (k >> 6))
      mask[p, k] = 2.0 if (r >> (k & 63)) & 1 else 0.0
  return mask


def shapes_of(kind, I, D):
  if kind == 0:
    return [(2 * I, I), (I, 1)]
  H = (I + D) // 2
  s = [(I, H), (I, H), (H, D), (H, D)]
  if kind == 2:
    s += [(D, H), (D, H), (H, I), (H, I)]
  return s + [(2 * D, D), (D, 1)]


def torch_step(kind, I, D, flat, nt, et, nr, er, lab, seed, lr, eps):
  """One Keras batch in float64 autograd; returns (new flat weights, loss)."""
  shapes = shapes_of(kind, I, D)
  params, off = [], 0
  for k, n in shapes:
    W = torch.tensor(flat[off:off + k * n].reshape(k, n), dtype=torch.float64,
                     requires_grad=True)
    off += k * n
    b = torch.tensor(flat[off:off + n], dtype=torch.float64, requires_grad=True)
    off += n
    params.append((W, b))
  relu, sig = torch.relu, torch.sigmoid
  dense = lambda x, q, a: a(x @ params[q][0] + params[q][1])
  xn = torch.tensor(nt[nr], dtype=torch.float64)
  xe = torch.tensor(et[er], dtype=torch.float64)
  t = torch.tensor(lab, dtype=torch.float64)
  mse = lambda y, tt: ((y - tt) ** 2).mean(dim=-1).mean()
  stream = 0x44000000  # epoch 0
  if kind == 0:
    h = dense(torch.cat([xn, xe], 1), 0, relu)
    loss = mse(dense(h, 1, sig), t[:, None])
  else:
    M = len(nr)
    dn = xn * torch.tensor(drop_mask(seed, stream, M, I))
    de = xe * torch.tensor(drop_mask(seed, stream + 1, M, I))
    jn = dense(dense(dn, 0, relu), 2, sig)
    je = dense(dense(de, 1, relu), 3, sig)
    q = 4 if kind == 1 else 8
    y = dense(dense(torch.cat([jn, je], 1), q, relu), q + 1, sig)
    loss = mse(y, t[:, None])
    if kind == 2:
      loss = 4 * loss
      # creation order: post_n 4, post_e 5, rec_n 6, rec_e 7
      rn = dense(dense(jn, 4, relu), 6, relu)
      re = dense(dense(je, 5, relu), 7, relu)
      loss = loss + mse(rn, xn) + mse(re, xe)
  loss.backward()
  out = []
  for W, b in params:
    for p in (W, b):
      g = p.grad.numpy().ravel()
      a = g * g
      out.append(p.detach().numpy().ravel() - lr * g / (np.sqrt(a) + eps))
  return np.concatenate(out), float(loss.detach())


@pytest.mark.parametrize("kind", [0, 1, 2])
def test_one_batch_matches_autograd(kind):
  I, D, M = 12, 6, 40
  rng = np.random.default_rng(kind)
  shapes = shapes_of(kind, I, D)
  flat = np.concatenate([np.concatenate([
      rng.uniform(-1, 1, k * n) * np.sqrt(6 / (k + n)),
      rng.normal(0, 0.2, n)]) for k, n in shapes]).astype(np.float32)
  assert flat.size == O.mlp_num_weights(kind, I, D)
  nt = rng.random((30, I)).astype(np.float32)
  et = rng.random((20, I)).astype(np.float32)
  nr = rng.integers(0, 30, M).astype(np.int32)
  er = rng.integers(0, 20, M).astype(np.int32)
  lab = (rng.random(M) < 0.4).astype(np.float32)
  # lr 1, eps 10: the step ~ g/10 is far above the f32 spacing of w
  seed, lr, eps = 1234, 1.0, 10.0
  w, losses = O.mlp_fit(kind, I, D, flat, nt, et, nr, er, lab,
                        np.arange(M)[None, :], batch=M, lr=lr, eps=eps,
                        seed=seed)
  ref, ref_loss = torch_step(kind, I, D, flat.astype(np.float64), nt, et, nr, er,
                             lab, seed, lr, eps)
  assert abs(losses[0] - ref_loss) <= 1e-5 * max(1.0, abs(ref_loss))
  step_ref = ref - flat
  step = w - flat
  # the step is ~lr*g/eps: compare it relative to its own scale
  assert np.abs(step - step_ref).max() <= 1e-3 * np.abs(step_ref).max()
  assert np.abs(step_ref).max() > 0


def test_early_stopping_and_epoch_loss():
  """EarlyStopping(monitor=loss, min_delta, patience=0): stops at the first
  epoch that does not improve the best loss by more than min_delta."""
  kind, I, D, n = 0, 8, 0, 600
  rng = np.random.default_rng(7)
  shapes = shapes_of(kind, I, D)
  flat = np.concatenate([np.concatenate([
      rng.uniform(-1, 1, k * n_) * np.sqrt(6 / (k + n_)), np.zeros(n_)])
      for k, n_ in shapes]).astype(np.float32)
  nt = rng.random((40, I)).astype(np.float32)
  et = rng.random((25, I)).astype(np.float32)
  nr = rng.integers(0, 40, n).astype(np.int32)
  er = rng.integers(0, 25, n).astype(np.int32)
  lab = (rng.random(n) < 0.5).astype(np.float32)
  perms = np.stack([rng.permutation(n) for _ in range(30)])
  _, l_all = O.mlp_fit(kind, I, 0, flat, nt, et, nr, er, lab, perms,
                       min_delta=-1e30)
  assert len(l_all) == 30
  _, l_stop = O.mlp_fit(kind, I, 0, flat, nt, et, nr, er, lab, perms,
                        min_delta=1e-3)
  k = len(l_stop)
  np.testing.assert_array_equal(l_stop, l_all[:k])
  best = np.minimum.accumulate(l_all)
  # every epoch before the stop improved on the best by more than 1e-3
  for e in range(1, k - 1):
    assert l_all[e] + 1e-3 < best[e - 1]
  if k < 30:
    assert not l_all[k - 1] + 1e-3 < best[k - 2]

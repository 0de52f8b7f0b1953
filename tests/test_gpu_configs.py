"""GPU parity at every BASELINE.json configuration shape that fits one GPU.

BASELINE.json ``configs`` (SURVEY.md §8 config sizes):
  1. trainer.py plumbing: 16 clients x 1,206,590 (EMNIST CNN), trainer defaults
     (uniform, step 0.5, clipping + zeroing on, weighted; trainer.py:63-90,
     builder.py:453-525) through ``build_quantization_encode_aggregator``;
  2. 128 clients x 2^20, stochastic "8-bit" (step 1/127, sigma 0.25);
  3. 256 clients x 4,050,748 (StackOverflow LSTM), stochastic step 1.0;
  headline: 1024 clients x 25,000,000, stochastic step 0.5 (bench.py's round),
     and 257 clients x 25 M (more clients than decoder lanes per tile, an odd
     client count for the encoder's multiply-high ticket division);
  5. one-bit SGD codec at P = 25,000,000 (one_bit_sgd.py:45-112).
  4. one GPU's share of config 4: 64 clients x 11,000,000 (ResNet-18), stochastic;
Configs 4 and 5's 8-GPU splits are covered by the distributed tests.

Checks, by what the oracle (CPU restatement) can afford in seconds:
  * codes: byte-identical to the oracle for a subset of clients (all clients
    where the oracle is fast enough);
  * the round's int32 client sum: against the oracle's sum of every client where
    affordable (configs 1-3), else against the sum of the HIP elementwise
    quantiser ``fc_quantize`` (itself bit-exact against the oracle in
    test_gpu_codec.py) -- a size-independent property of the full-size round;
  * the dequantised sum: f32(sum) * step, bit-exact.
"""
import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest
import torch

from federated_amd import _lib
from federated_amd import builder
from federated_amd import codec
from oracle import aggregators as oagg
from oracle import codec as ocodec
from oracle import quantize_utils as oq

pytestmark = pytest.mark.gpu
F32 = np.float32
MODE = {"uniform": _lib.UNIFORM, "stochastic": _lib.STOCHASTIC}
ORACLE_Q = {"uniform": lambda x, s, sd: oq.uniform_quantize(x, s), "stochastic": oq.stochastic_quantize}
WORKERS = max(1, min(16, len(os.sched_getaffinity(0))))


def _host_deltas(C, P, sigma, seed):
  def one(c):
    return (np.random.default_rng(seed + c).standard_normal(P, dtype=np.float32) * F32(sigma))
  with ThreadPoolExecutor(WORKERS) as ex:
    return list(ex.map(one, range(C)))


def _oracle_sum(xs, step, seeds, mode):
  """int32 sum over clients of the oracle's q (thread pool: numpy releases the GIL)."""
  def one(c):
    return ORACLE_Q[mode](xs[c], F32(step), tuple(seeds[c])).astype(np.int64)
  acc = np.zeros(xs[0].size, np.int64)
  with ThreadPoolExecutor(WORKERS) as ex:
    for q in ex.map(one, range(len(xs))):
      acc += q
  return oagg.wrap_i32(acc)


def _hip_quantize_sum(rows, step, seeds, mode):
  """int32 sum of fc_quantize (the oracle-pinned elementwise HIP quantiser)."""
  acc = torch.zeros(rows[0].numel(), dtype=torch.int64, device=rows[0].device)
  for c, r in enumerate(rows):
    q, _ = codec.quantize(r, step, tuple(int(v) for v in seeds[c]), MODE[mode])
    acc += q
  return acc.to(torch.int32)


def _check_codes(batch, xs_host, clients, step, seeds, mode):
  """Byte-exact codes of `clients` against the oracle (quantiser + C coder on a thread pool)."""
  bits = batch.bits()

  def one(c):
    q = ORACLE_Q[mode](xs_host[c], F32(step), tuple(seeds[c]))
    code, nbits = ocodec.run_length_gamma_encode(q)
    return c, nbits, code
  with ThreadPoolExecutor(WORKERS) as ex:
    for c, nbits, code in ex.map(one, clients):
      assert int(bits[c]) == nbits, c
      assert batch.client_code(c) == code, c


def _round(rows, step, seeds, mode):
  # default capacities (4 bits/element): wider codes (config 2's ~10 bits) overflow and
  # exercise the re-encode of just the overflowed clients
  batch = codec.quantize_encode_checked(rows, step, torch.from_numpy(seeds), MODE[mode])
  ovf = codec.check_overflow(batch)
  assert not len(ovf), ovf
  out = torch.empty(rows[0].numel(), dtype=torch.float32, device=rows[0].device)
  s, out, err = codec.decode_accumulate(batch, out=out, step=step)
  assert int(err.item()) == 0
  return batch, s, out


def _release():
  torch.cuda.synchronize()
  torch.cuda.empty_cache()


@pytest.mark.parametrize("C,P,mode,step,sigma,code_clients", [
    (128, 1 << 20, "stochastic", 1.0 / 127, 0.25, (0, 1, 64, 127)),          # config 2
    (256, 4_050_748, "stochastic", 1.0, 1.0, (0, 1, 255)),                  # config 3
], ids=["config2_128x1M_8bit", "config3_256x4.05M"])
def test_config_round_matches_oracle(gpu, C, P, mode, step, sigma, code_clients):
  xs = _host_deltas(C, P, sigma, seed=1000 * C)
  seeds = np.array([[77 + c, 3 * c + 1] for c in range(C)], np.int64)
  rows = [torch.from_numpy(x).to(gpu) for x in xs]
  batch, s, out = _round(rows, step, seeds, mode)
  _check_codes(batch, xs, code_clients, step, seeds, mode)
  want = _oracle_sum(xs, step, seeds, mode)
  np.testing.assert_array_equal(s.cpu().numpy(), want)
  np.testing.assert_array_equal(out.cpu().numpy(), oq.uniform_dequantize(want, F32(step)))
  del rows, batch
  _release()


@pytest.mark.parametrize("C,mode", [(257, "stochastic"), (1024, "stochastic"), (1024, "uniform")],
                         ids=["257x25M_stochastic", "1024x25M_stochastic", "1024x25M_uniform"])
def test_headline_shape_round(gpu, C, mode):
  """25 M elements per client (24,415 tiles, look-backs across the whole client),
  257 or 1024 clients: more clients than the decoder's 128 lanes per tile (each
  lane walks several clients) and the encoder's ticket division at C = 257 / 1024."""
  P, step = 25_000_000, 0.5
  g = torch.Generator(device=gpu)
  rows = []
  for c in range(C):
    g.manual_seed(4242 + c)
    rows.append(torch.randn(P, generator=g, device=gpu, dtype=torch.float32))
  seeds = np.array([[1000 + c, 1000 + c] for c in range(C)], np.int64)
  batch, s, out = _round(rows, step, seeds, mode)
  # sixteen clients' codes byte for byte against the oracle, spread over the batch (the
  # first and last clients, the 32nd-34th, every eighth of the batch)
  picks = sorted(set([0, 1, 2, 31, 32, 33] + [C * k // 8 for k in range(1, 8)] + [C - 3, C - 2, C - 1]))
  _check_codes(batch, {c: rows[c].cpu().numpy() for c in picks}, picks, step, seeds, mode)
  want = _hip_quantize_sum(rows, step, seeds, mode)
  assert torch.equal(s, want)
  np.testing.assert_array_equal(out.cpu().numpy(), oq.uniform_dequantize(want.cpu().numpy(), F32(step)))
  _check_sum_sampled(rows, s, step, seeds, mode, n=100_000)  # every client's term at 100,000 positions
  # whole-batch code length: the sum of every client's bit count is what the decoder consumed
  assert int(batch.bits().min()) > 0
  del rows, batch, s, out, want
  _release()


def _check_sum_sampled(rows, s, step, seeds, mode, n=20_000, seed=8):
  """The full round's int32 sum against the ORACLE at n sampled positions, every
  client's term restated there (oracle.quantize_utils.stochastic_quantize_at: the
  quantiser is elementwise and stream element i needs only its counter)."""
  P = rows[0].numel()
  idx = np.sort(np.random.default_rng(seed).choice(P, n, replace=False))
  it = torch.from_numpy(idx).to(rows[0].device)
  vals = torch.stack([r[it] for r in rows]).cpu().numpy()

  def one(c):
    if mode == "uniform":
      return oq.uniform_quantize(vals[c], F32(step)).astype(np.int64)
    return oq.stochastic_quantize_at(vals[c], idx, F32(step), tuple(seeds[c])).astype(np.int64)
  acc = np.zeros(n, np.int64)
  with ThreadPoolExecutor(WORKERS) as ex:
    for q in ex.map(one, range(len(rows))):
      acc += q
  np.testing.assert_array_equal(s[it].cpu().numpy(), oagg.wrap_i32(acc))


def test_config4_share_round(gpu):
  """One GPU's share of config 4 (CIFAR-100 ResNet-18 deltas, 512 clients x 11 M
  over 8 GPUs): 64 clients x 11,000,000, stochastic step 0.5 (sigma 1), through
  QuantizeEncodeFactory at its default settings.  Codes of three clients
  byte-identical to the oracle; the int32 sum against the oracle at sampled
  positions of every client and against the HIP elementwise quantiser in full;
  the result bit-exact; a second round reuses the first round's code sizes
  (no overflow re-encode)."""
  from federated_amd.aggregators import quantize_encode  # pylint: disable=g-import-not-at-top
  C, P, step = 64, 11_000_000, 0.5
  g = torch.Generator(device=gpu)
  rows = []
  for c in range(C):
    g.manual_seed(11000 + c)
    rows.append(torch.randn(P, generator=g, device=gpu, dtype=torch.float32))
  seeds = np.array([[300 + c, 7 * c + 2] for c in range(C)], np.int64)
  batch, s, out = _round(rows, step, seeds, "stochastic")
  picks = (0, 33, 63)
  _check_codes(batch, {c: rows[c].cpu().numpy() for c in picks}, picks, step, seeds, "stochastic")
  want = _hip_quantize_sum(rows, step, seeds, "stochastic")
  assert torch.equal(s, want)
  _check_sum_sampled(rows, s, step, seeds, "stochastic")
  res_want = oq.uniform_dequantize(want.cpu().numpy(), F32(step))
  np.testing.assert_array_equal(out.cpu().numpy(), res_want)
  process = quantize_encode.QuantizeEncodeFactory(step, rounding_type="stochastic").create((np.float32, (P,)))
  state = process.initialize()
  for _ in range(2):
    r = process.next(state, rows, seeds=seeds)
    np.testing.assert_array_equal(r.result.cpu().numpy(), res_want)
    state = r.state
  del rows, batch, s, out, want
  _release()


def test_config1_trainer_defaults_round(gpu):
  """trainer.py defaults (uniform, step 0.5, clipping + zeroing, weighted by example
  counts) at the EMNIST CNN size, through the builder; oracle: the wrappers restated
  in numpy around oracle.aggregators.quantize_encode_next."""
  C, P = 16, 1_206_590
  xs = _host_deltas(C, P, 0.02, seed=31)
  xs[3] = xs[3] * F32(1000.0)  # a client far above the zeroing threshold
  w = np.random.default_rng(5).integers(200, 2000, C).astype(np.float32)
  f = builder.build_quantization_encode_aggregator()  # trainer defaults
  process = f.create((np.float32, (P,)), (np.float32, ()))
  state = process.initialize()
  out = process.next(state, xs, weight=w)
  # --- oracle: zeroing (linf > 2X + 1), clipping (global L2 vs C), mean weight ---
  linf = np.array([np.max(np.abs(oq.ftz(x))) for x in xs], np.float32)
  zero_thr = F32(F32(state["zeroing_norm"]) * F32(2.0) + F32(1.0))
  keep = ~(linf > zero_thr)
  assert not keep[3] and keep.sum() == C - 1
  l2 = np.array([np.sqrt(np.sum(oq.ftz(x).astype(np.float64) ** 2)) for x in xs], np.float32)
  l2 = np.where(keep, l2, F32(0.0)).astype(np.float32)
  clip = F32(state["clipping_norm"])
  with np.errstate(divide="ignore"):
    inv = np.where(l2 > 0, F32(1.0) / l2, np.float32(np.inf)).astype(np.float32)
  scale = np.where(keep, clip * np.minimum(inv, F32(1.0) / clip), F32(0.0)).astype(np.float32)
  pre = [((x * scale[c]) * w[c]).astype(np.float32) for c, x in enumerate(xs)]
  # uniform rounding draws no randomness: any seeds
  want, meas, _ = oagg.quantize_encode_next(pre, 0.5, "uniform")
  want = (want / F32(np.sum(w, dtype=np.float32))).astype(np.float32)
  np.testing.assert_array_equal(out.result, want)
  assert out.measurements["mean_value"]["avg_bitrate"] == meas["avg_bitrate"]
  assert out.measurements["mean_value"]["avg_sparsity"] == meas["avg_sparsity"]
  assert out.measurements["zeroing_norm"] == zero_thr
  # next state: the quantile estimates moved against the raw estimates
  assert out.state["clipping_norm"] == builder.QuantileEstimate(1.0, 0.8, 0.2).update(clip, l2)
  _release()


def test_config5_onebit_at_25M(gpu):
  """One-bit SGD (config 5's codec) at P = 25 M: masks bit-exact, means and the
  client-order float32 decoded sum against the oracle."""
  C, P = 16, 25_000_000
  xs = _host_deltas(C, P, 1.0, seed=555)
  rows = [torch.from_numpy(x).to(gpu) for x in xs]
  masks, means, dist = codec.onebit_encode(rows, 0.0)
  nw = (P + 31) // 32
  m = masks.cpu().numpy().view(np.uint32).reshape(C, nw)
  for c in (0, C - 1):
    # TF's mask word w holds element 32 w + i in bit i
    bits = np.pad((xs[c] >= 0).astype(np.uint8), (0, nw * 32 - P)).reshape(nw, 32)
    want = np.packbits(bits, axis=1, bitorder="little").view("<u4").reshape(-1)
    np.testing.assert_array_equal(m[c], want)
  res = codec.onebit_decode_sum(masks, means, C, P).cpu().numpy()
  want, meas = oagg.one_bit_sgd_next(xs, 0.0)
  np.testing.assert_allclose(means.cpu().numpy()[1::2],
                             [F32(np.sum(x * (x >= 0), dtype=np.float64) / max(np.sum(x >= 0), 1))
                              for x in xs], rtol=1e-6)
  np.testing.assert_allclose(res, want, rtol=1e-5, atol=1e-5)
  np.testing.assert_allclose(np.mean(dist.cpu().numpy()) / P, meas["avg_distortion"], rtol=1e-5)
  del rows
  _release()


def test_config5_onebit_round_full_size(gpu):
  """Config 5's whole codec round on one GPU: 1024 clients x 25 M, one-bit SGD
  (one_bit_sgd.py:45-112) through distributed.onebit_round (the round the 8-GPU run
  shards).  Oracle checks the size allows:
    * every client's mask bits at 20,000 sampled positions (x >= threshold), and
      four clients' whole masks;
    * 16 clients' means and distortions against numpy float64 over their full rows
      (rtol 1e-6 / 1e-5; TF's float32 reduction order is unspecified);
    * the round's decoded sum at the sampled positions: the client-order float32
      sum of each client's mean selected by its bit (one_bit_sgd.py:87-112), bit
      for bit given the means;
    * measurements: avg_bitrate = (P + 64) / P, avg_distortion."""
  from federated_amd import distributed  # pylint: disable=g-import-not-at-top
  C, P, thr = 1024, 25_000_000, 0.0
  g = torch.Generator(device=gpu)
  rows = []
  for c in range(C):
    g.manual_seed(5000 + c)
    rows.append(torch.randn(P, generator=g, device=gpu, dtype=torch.float32) * (0.5 + (c % 5) * 0.25) + 0.01 * (c % 3))
  rnd = distributed.onebit_round(rows, thr, multi=False)
  masks, means, dist = codec.onebit_encode(rows, thr)  # the round's own encode, for the checks
  res = rnd.result.cpu().numpy()
  nw = (P + 31) // 32
  means_h = means.cpu().numpy().reshape(C, 2)
  dist_h = dist.cpu().numpy()
  # masks at sampled positions, every client
  idx = np.sort(np.random.default_rng(55).choice(P, 20_000, replace=False))
  it = torch.from_numpy(idx).to(gpu)
  vals = torch.stack([r[it] for r in rows]).cpu().numpy()
  words = masks.view(C, nw)[:, torch.from_numpy(idx // 32).to(gpu)].cpu().numpy().view(np.uint32)
  bits = ((words >> (idx % 32).astype(np.uint32)) & 1).astype(bool)
  np.testing.assert_array_equal(bits, oq.ftz(vals) >= F32(thr))
  # whole masks and means / distortions of sampled clients against float64 numpy
  for c in (0, 1, 511, 1023):
    x = oq.ftz(rows[c].cpu().numpy())
    b = np.pad((x >= thr).astype(np.uint8), (0, nw * 32 - P)).reshape(nw, 32)
    np.testing.assert_array_equal(masks.view(C, nw)[c].cpu().numpy().view(np.uint32),
                                  np.packbits(b, axis=1, bitorder="little").view("<u4").reshape(-1))
  for c in range(0, C, C // 16):
    x = oq.ftz(rows[c].cpu().numpy())
    ab = x >= thr
    xd = x.astype(np.float64)
    mb, ma = xd[~ab].sum() / max((~ab).sum(), 1), xd[ab].sum() / max(ab.sum(), 1)
    np.testing.assert_allclose(means_h[c], [mb, ma], rtol=1e-6)
    dec = np.where(ab, means_h[c, 1], means_h[c, 0]).astype(np.float32)
    np.testing.assert_allclose(dist_h[c], ((x - dec).astype(np.float64) ** 2).sum(), rtol=1e-5)
  # the decoded client-order float32 sum at the sampled positions
  acc = np.zeros(idx.size, np.float32)
  for c in range(C):
    acc = (acc + np.where(bits[c], means_h[c, 1], means_h[c, 0]).astype(np.float32)).astype(np.float32)
  np.testing.assert_array_equal(res[idx].view(np.uint32), acc.view(np.uint32))
  m = rnd.measurements
  assert m["avg_bitrate"] == F32((F32(P) + F32(64.0)) / F32(P))
  np.testing.assert_allclose(m["avg_distortion"], np.mean(dist_h / P), rtol=1e-5)
  del rows, masks, means, dist, rnd
  _release()

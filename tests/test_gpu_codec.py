"""GPU parity of the HIP codec kernels against the CPU oracle (bit-exact).

Every check goes through the C ABI (federated_amd/_lib.py -> libfedcodec.so).
"""
import numpy as np
import pytest
import torch

from federated_amd import _lib
from federated_amd import codec
from oracle import codec as ocodec
from oracle import quantize_utils as oq

pytestmark = pytest.mark.gpu

MODES = {"uniform": _lib.UNIFORM, "stochastic": _lib.STOCHASTIC, "dithered": _lib.DITHERED}
ORACLE_Q = {
    "uniform": lambda x, s, seed: oq.uniform_quantize(x, s),
    "stochastic": oq.stochastic_quantize,
    "dithered": oq.dithered_quantize,
}


def special_values():
  f32 = np.float32
  vals = [0.0, -0.0, 1e-45, -1e-45, 1e-39, -1e-39, 1.1754944e-38, -1.1754942e-38, 0.5, -0.5, 1.5,
          2.5, -2.5, 0.25, 0.75, 1.0, -1.0, 3.0, 1e30, -1e30, np.inf, -np.inf, np.nan, 2.0**31,
          -2.0**31, 2.0**31 - 128, 2.0**30, -2.0**30 - 64, 1e-20, 7.0, 1e8]
  return np.array(vals, dtype=f32)


@pytest.mark.parametrize("mode", list(MODES))
@pytest.mark.parametrize("step", [0.5, 0.4, 1.0 / 127, 1.0, 3.7e-3, 1e-30])
def test_quantize_matches_oracle(gpu, mode, step):
  rng = np.random.default_rng(7)
  x = np.concatenate([rng.standard_normal(20000).astype(np.float32) * 3,
                      special_values(),
                      (np.arange(-600, 600, dtype=np.float32) * np.float32(step) * 0.5)])
  for seed in [(0, 0), (1, 1), (2**40 + 7, 3), (-5, 2**62)]:
    q, _ = codec.quantize(torch.from_numpy(x).to(gpu), step, seed, MODES[mode])
    want = ORACLE_Q[mode](x, step, seed)
    got = q.cpu().numpy()
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, (mode, step, seed, x[bad[:5]], got[bad[:5]], want[bad[:5]])


def test_noise_matches_oracle(gpu):
  x = np.zeros(1001, np.float32)
  _, noise = codec.quantize(torch.from_numpy(x).to(gpu), 1.0, (3, 9), _lib.DITHERED, want_noise=True)
  np.testing.assert_array_equal(noise.cpu().numpy(), oq.generate_noise((3, 9), 1001))


def _rand_q(rng, P, kind):
  if kind == "sparse":
    q = rng.integers(-3, 4, P).astype(np.int32)
    q[rng.random(P) < 0.9] = 0
  elif kind == "dense":
    q = np.rint(rng.standard_normal(P) * 3).astype(np.int32)
  elif kind == "wide":
    q = (rng.standard_normal(P) * 2.0**rng.integers(0, 30, P)).astype(np.int64)
    q = np.clip(q, -2**31, 2**31 - 1).astype(np.int32)
  elif kind == "zeros":
    q = np.zeros(P, np.int32)
  elif kind == "runs":
    q = np.zeros(P, np.int32)
    pos = rng.choice(P, size=max(1, P // 5000), replace=False)
    q[pos] = rng.integers(1, 100, pos.size) * rng.choice([-1, 1], pos.size)
  elif kind == "extreme":
    q = rng.choice(np.array([-2**31, 2**31 - 1, 1, -1, 0], np.int32), P)
  else:
    raise ValueError(kind)
  return q


@pytest.mark.parametrize("P", [1, 3, 4, 5, 1023, 1024, 1025, 4096, 4099, 20000, 100003])
@pytest.mark.parametrize("kind", ["sparse", "dense", "wide", "zeros", "runs", "extreme"])
def test_rlgamma_encode_bytes_match_oracle(gpu, P, kind):
  rng = np.random.default_rng(P * 31 + len(kind))
  qs = [_rand_q(rng, P, kind) for _ in range(3)]
  batch = codec.rlgamma_encode([torch.from_numpy(q).to(gpu) for q in qs])
  assert not len(codec.check_overflow(batch))
  bits = batch.bits()
  for c, q in enumerate(qs):
    want, nbits = ocodec.run_length_gamma_encode(q)
    assert bits[c] == nbits
    assert batch.client_code(c) == want, (c, kind, P)
  s, _, err = codec.decode_accumulate(batch)
  assert int(err.item()) == 0
  want_sum = np.sum(np.stack(qs).astype(np.int64), axis=0)
  want_sum = ((want_sum + 2**31) % 2**32 - 2**31).astype(np.int32)
  np.testing.assert_array_equal(s.cpu().numpy(), want_sum)


@pytest.mark.parametrize("mode", list(MODES))
@pytest.mark.parametrize("P,C", [(1, 2), (4097, 3), (50000, 5), (300000, 7)])
def test_quantize_encode_batch_matches_oracle(gpu, mode, P, C):
  rng = np.random.default_rng(P + C)
  step = 0.5 if mode != "dithered" else 0.3
  xs = [(rng.standard_normal(P) * rng.uniform(0.1, 2)).astype(np.float32) for _ in range(C)]
  seeds = np.array([[1000 + c, 77 * c] for c in range(C)], np.int64)
  batch = codec.quantize_encode_checked([torch.from_numpy(x).to(gpu) for x in xs], step,
                                        torch.from_numpy(seeds), MODES[mode])
  bits = batch.bits()
  acc = np.zeros(P, np.int32)
  dists, nnzs = codec.finalize(batch)
  dists = dists.cpu().numpy()
  nnzs = nnzs.cpu().numpy()
  noise_sum = np.zeros(P, np.float32)
  for c in range(C):
    q = ORACLE_Q[mode](xs[c], step, tuple(seeds[c]))
    code, nbits = ocodec.run_length_gamma_encode(q)
    assert bits[c] == nbits
    assert batch.client_code(c) == code
    acc = (acc.astype(np.int64) + q).astype(np.int32)
    if mode == "dithered":
      n = oq.generate_noise(tuple(seeds[c]), P)
      noise_sum = noise_sum + n
      deq = oq.dithered_dequantize(q, step, n)
    else:
      deq = oq.uniform_dequantize(q, step)
    want_d = np.sum((xs[c].astype(np.float64) - deq) ** 2)
    np.testing.assert_allclose(dists[c], want_d, rtol=1e-5, atol=1e-30)
    assert nnzs[c] == np.count_nonzero(q)
  ns = None
  if mode == "dithered":
    ns = codec.noise_sum(torch.from_numpy(seeds), P, gpu)
    np.testing.assert_array_equal(ns.cpu().numpy(), noise_sum)
  out = torch.empty(P, dtype=torch.float32, device=gpu)
  s, out, err = codec.decode_accumulate(batch, out=out, step=step, noise_sum=ns)
  assert int(err.item()) == 0
  np.testing.assert_array_equal(s.cpu().numpy(), acc)
  if mode == "dithered":
    want = oq.dithered_dequantize(acc, step, noise_sum)
  else:
    want = oq.uniform_dequantize(acc, step)
  np.testing.assert_array_equal(out.cpu().numpy(), want)


def test_reference_known_answers(gpu):
  # elias_gamma_encode_test.py:32-37: mean 16 bits; decoded sum = elementwise sum.
  qs = [np.array([-5, 3, 0, 0], np.int32), np.array([-3, 1, 0, 0], np.int32)]
  batch = codec.rlgamma_encode([torch.from_numpy(q).to(gpu) for q in qs])
  assert list(batch.nbytes() * 8) == [16, 16]
  s, _, _ = codec.decode_accumulate(batch)
  np.testing.assert_array_equal(s.cpu().numpy(), [-8, 4, 0, 0])
  # quantize_encode_client_lambda_test.py:93-112 and qsgd_test.py:128-130
  for q, nbits in (([2, 2, 2], 15), ([1, 1, 1], 9), ([0, 0, 0], 5), ([2, 3, 6], 17)):
    b = codec.rlgamma_encode([torch.tensor(q, dtype=torch.int32, device=gpu)])
    assert int(b.bits()[0]) == nbits


@pytest.mark.parametrize("grid,win", [("1", None), ("5", None), ("64", None), ("512", None),
                                      ("default", None), ("512", "4"), ("4096", "64")])
def test_encode_many_tiles_per_workgroup(gpu, grid, win, monkeypatch):
  """Persistent workgroups that each take many tiles (LDS window reuse) and
  look-backs that cross many tiles: with 2 clients x 977 tiles and hundreds of
  waves, the nearest inclusive prefix often lies beyond 64 tiles, so the
  multi-window walk (lookback_deep) runs, with short (4) and full (64)
  prefetch windows."""
  if grid != "default":
    monkeypatch.setenv("FEDCODEC_ENC_GRID", grid)
  if win is not None:
    monkeypatch.setenv("FEDCODEC_LB_WIN", win)
  rng = np.random.default_rng(len(grid) * 7 + (int(win) if win else 0))
  P, C = 1_000_003, 2
  xs = [(rng.standard_normal(P) * 0.7).astype(np.float32) for _ in range(C)]
  xs[1][100_000:900_000] = 0.0  # long zero runs crossing many tiles
  seeds = np.array([[5, 6], [7, 8]], np.int64)
  batch = codec.quantize_encode_checked([torch.from_numpy(x).to(gpu) for x in xs], 0.25,
                                        torch.from_numpy(seeds), _lib.STOCHASTIC)
  acc = np.zeros(P, np.int64)
  for c in range(C):
    q = oq.stochastic_quantize(xs[c], 0.25, tuple(seeds[c]))
    code, nbits = ocodec.run_length_gamma_encode(q)
    assert int(batch.bits()[c]) == nbits
    assert batch.client_code(c) == code
    acc += q
  s, _, err = codec.decode_accumulate(batch)
  assert int(err.item()) == 0
  np.testing.assert_array_equal(s.cpu().numpy(), acc.astype(np.int32))


def test_decode_tile_ranges_match_full_decode(gpu):
  """fc_decode_accumulate_tiles over consecutive tile ranges writes exactly the
  full decode (the multi-GPU path all-reduces finished ranges while later ones
  decode); a range never touches elements outside it."""
  rng = np.random.default_rng(11)
  P, C = 10_000, 3  # 10 tiles, the last partial
  xs = [(rng.standard_normal(P) * 1.3).astype(np.float32) for _ in range(C)]
  seeds = np.array([[1, 2], [3, 4], [5, 6]], np.int64)
  batch = codec.quantize_encode_checked([torch.from_numpy(x).to(gpu) for x in xs], 0.5,
                                        torch.from_numpy(seeds), _lib.STOCHASTIC)
  full, fout, err = codec.decode_accumulate(batch, out=torch.empty(P, device=gpu), step=0.5)
  assert int(err.item()) == 0
  part = torch.full((P,), 12345, dtype=torch.int32, device=gpu)
  pout = torch.full((P,), -7.0, dtype=torch.float32, device=gpu)
  err = torch.zeros(1, dtype=torch.int32, device=gpu)
  for tb, te in ((0, 3), (3, 4), (4, 10)):
    codec.decode_accumulate(batch, sum_out=part, out=pout, step=0.5, err=err, tiles=(tb, te))
    hi = min(P, te * 1024)
    np.testing.assert_array_equal(part[:hi].cpu().numpy(), full[:hi].cpu().numpy())
    assert (part[hi:].cpu().numpy() == 12345).all()
    assert (pout[hi:].cpu().numpy() == -7.0).all()
  np.testing.assert_array_equal(pout.cpu().numpy(), fout.cpu().numpy())
  assert int(err.item()) == 0


def test_noise_sum_many_clients(gpu):
  """fc_noise_sum with more clients than one 256-client key chunk: the client-order
  float32 sum of TF's dither noise, bit-exact against the oracle."""
  P, C = 1001, 300
  seeds = np.array([[3 * c + 1, 7 * c + 2] for c in range(C)], np.int64)
  want = np.zeros(P, np.float32)
  for c in range(C):
    want = want + oq.generate_noise(tuple(seeds[c]), P)
  got = codec.noise_sum(torch.from_numpy(seeds), P, gpu).cpu().numpy()
  np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("step", [1.0 / 127, 0.4, 0.1, 1.0 / 3, 0.7, 3.7e-3, 0.275, 1.9999999])
@pytest.mark.parametrize("mode", ["uniform", "stochastic"])
def test_encoder_division_matches_ieee_over_whole_binades(gpu, step, mode):
  """The encoder forms x / step without a division for host-known steps (a
  multiply for powers of two; Markstein's RN(1/step) + FMA remainder correction
  otherwise; the IEEE division for an all-ones significand such as 1.9999999).
  Every float32 of whole binades of x (|x / step| in [1, 2), [63, 128) and
  [4096, 8192), both signs: 2^25 consecutive bit patterns plus the tie points)
  must quantise exactly as the elementwise kernel, which divides with the IEEE
  division and is bit-exact against the oracle (test_quantize_matches_oracle)."""
  s = np.float32(step)
  parts = []
  for k, sign in ((0, 1), (6, -1), (12, 1)):
    lo = np.float32(s * np.float32(2.0**k)).view(np.uint32)
    bits = lo + np.arange(1 << 23, dtype=np.uint32)
    parts.append(bits.view(np.float32) * np.float32(sign))
  ties = (np.arange(-3000, 3000, dtype=np.float32) + np.float32(0.5)) * s
  x = np.concatenate(parts + [ties, np.nextafter(ties, np.float32(np.inf)),
                              np.nextafter(ties, np.float32(-np.inf))]).astype(np.float32)
  xt = torch.from_numpy(x).to(gpu)
  seed = (12, 34)
  batch = codec.quantize_encode_checked([xt], float(s), torch.tensor([seed], dtype=torch.int64), MODES[mode])
  got, _, err = codec.decode_accumulate(batch)
  assert int(err.item()) == 0
  want, _ = codec.quantize(xt, float(s), seed, MODES[mode])
  bad = torch.nonzero(got != want).flatten()
  assert bad.numel() == 0, (x[bad[:5].cpu().numpy()], got[bad[:5]].cpu(), want[bad[:5]].cpu())

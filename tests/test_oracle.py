"""CPU oracle pinned against the reference's known answers (no GPU).

Pins: Random123 Philox4x32-10 known-answer vectors; the reference's own
known-answer tests (file:line in each test); the committed golden fixtures.
"""
import os

import numpy as np
import pytest

from oracle import aggregators as oagg
from oracle import codec as ocodec
from oracle import philox
from oracle import quantize_utils as oq

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "golden.npz")


# Random123 kat_vectors for philox4x32 10 rounds (the TF block function).
@pytest.mark.parametrize("ctr,key,want", [
    ((0, 0, 0, 0), (0, 0), (0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8)),
    ((0xffffffff,) * 4, (0xffffffff, 0xffffffff), (0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd)),
    ((0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344), (0xa4093822, 0x299f31d0),
     (0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1)),
])
def test_philox_random123_kat(ctr, key, want):
  got = philox.philox4x32_10([np.uint32(c) for c in ctr], key)
  assert tuple(int(g) for g in got) == want


def test_uint32_to_float_range():
  r = np.array([0, 0x7FFFFF, 0x800000, 0xFFFFFFFF], np.uint32)
  u = philox.uint32_to_float(r)
  assert u[0] == 0.0 and u[2] == 0.0 and u[1] < 1.0 and u[3] < 1.0
  noise = philox.stateless_uniform(1000, (1, 2), -0.5, 0.5)
  assert noise.min() >= -0.5 and noise.max() < 0.5


# elias_gamma_encode_test.py:32-37, 91-116
def test_elias_gamma_known_answers():
  codes = [ocodec.run_length_gamma_encode(q)[0] for q in ([-5, 3, 0, 0], [-3, 1, 0, 0])]
  assert np.mean([ocodec.get_bitstring_length(c) for c in codes]) == 16
  rank2 = ocodec.run_length_gamma_encode(np.array([[-5, 3, 0, 0], [-3, 1, 0, 0]]).reshape(-1))[0]
  assert ocodec.get_bitstring_length(rank2) == 32
  s, rate, _ = oagg.elias_gamma_sum_next([[-5, 3, 0, 0], [-3, 1, 0, 0]])
  np.testing.assert_array_equal(s, [-8, 4, 0, 0])
  assert rate == 16 / 4


# quantize_encode_client_lambda_test.py:93-112 and qsgd_test.py:128-130
@pytest.mark.parametrize("q,bits,nbytes", [([2, 2, 2], 15, 2), ([1, 1, 1], 9, 2), ([0, 0, 0], 5, 1),
                                           ([2, 3, 6], 17, 3)])
def test_code_lengths_known_answers(q, bits, nbytes):
  code, nb = ocodec.run_length_gamma_encode(q)
  assert nb == bits and len(code) == nbytes


def test_gamma_code_lengths_closed_form():
  # cross_entropy.py:32-35: an Elias gamma code of v has 2*floor(log2 v)+1 bits
  for v in [1, 2, 3, 4, 7, 8, 1000, 2**20, 2**31 - 1]:
    n = int(np.floor(np.log2(v)))
    # one nonzero v at position 0, no trailing zeros: Gamma(1) + sign + Gamma(v)
    assert ocodec.encoded_bits([v]) == 1 + 1 + 2 * n + 1


# quantize_utils_test.py:46-59
def test_uniform_known_answers():
  np.testing.assert_array_equal(oq.uniform_quantize(np.full(3, 2.0, np.float32), 0.4), [5, 5, 5])
  np.testing.assert_allclose(oq.uniform_dequantize(np.full(3, 5, np.int32), 0.4), [2.0] * 3, rtol=1e-7)


def test_round_half_to_even_and_x86_cast():
  x = np.array([0.5, 1.5, 2.5, -0.5, -1.5, np.nan, np.inf, -np.inf, 3e9, -3e9], np.float32)
  np.testing.assert_array_equal(oq.uniform_quantize(x, 1.0)[:5], [0, 2, 2, 0, -2])
  assert (oq.uniform_quantize(x, 1.0)[5:] == np.int32(-2**31)).all()


def test_ftz_daz():
  x = np.array([1e-39, -1e-39, 1e-20], np.float32)  # denormal inputs read as zero (DAZ)
  np.testing.assert_array_equal(oq.uniform_quantize(x, 1e-25), [0, 0, 100000])
  # a normal input whose quotient is denormal is flushed (FTZ): rounds to 0
  assert oq.uniform_quantize(np.array([1e-30], np.float32), 1e10)[0] == 0


# quantize_utils_test.py:64-97 (stochastic properties)
def test_stochastic_properties():
  rng = np.random.default_rng(0)
  v = rng.uniform(-5, 5, 1000).astype(np.float32)
  q0 = oq.stochastic_quantize(v, 0.4, (0, 0))
  q1 = oq.stochastic_quantize(v, 0.4, (1, 1))
  assert not np.all(q0 == q1)
  fl = np.floor(v / np.float32(0.4)).astype(np.int32)
  assert np.all((q0 == fl) | (q0 == fl + 1))
  ints = rng.integers(-5, 5, 3).astype(np.float32)
  np.testing.assert_array_equal(oq.stochastic_quantize(ints, 1.0, (0, 0)), ints)
  np.testing.assert_array_equal(oq.stochastic_quantize(np.zeros(1000, np.float32), 0.4, (0, 0)), 0)
  # unbiased: mean of q * step close to mean of v
  big = rng.uniform(-1, 1, 200000).astype(np.float32)
  qb = oq.stochastic_quantize(big, 0.5, (7, 7)).astype(np.float64) * 0.5
  assert abs(qb.mean() - big.mean()) < 5e-3


# quantize_utils_test.py:102-152 (dither bounds)
def test_dithered_properties():
  rng = np.random.default_rng(1)
  v = rng.uniform(-5, 5, 1000).astype(np.float32)
  q = oq.dithered_quantize(v, 0.4, (0, 0))
  noise = oq.generate_noise((0, 0), v.size)
  deq = oq.dithered_dequantize(q, 0.4, noise)
  assert np.max(np.abs(deq - v)) <= 0.5 * 0.4 + 1e-6
  ints = rng.integers(-5, 5, 3).astype(np.float32)
  np.testing.assert_array_equal(oq.dithered_quantize(ints, 1.0, (0, 0)), ints)


# quantize_utils_test.py:157-186
def test_schedules():
  assert [float(oq.linear_decay(2., 0., r, 4)) for r in range(4)] == [2., 1.5, 1., 0.5]
  np.testing.assert_allclose([oq.exponential_decay(2., 0., r, 1.) for r in range(4)],
                             [2., 2. * np.exp(-1.), 2. * np.exp(-2.), 2. * np.exp(-3.)], rtol=1e-6)
  assert [float(oq.step_decay(2., 0., r, 2)) for r in range(4)] == [2., 2., 1., 1.]


# quantize_utils_test.py:19-40
def test_normalizers():
  v = np.array([0.0, 1.0, 2.0], np.float32)
  assert np.isclose(oq.mean_magnitude(v), 1.0)
  assert oq.max_magnitude(v) == 2.0
  assert np.isclose(oq.dimensionless_norm(v), np.sqrt(5.0 / 3.0))


# quantize_encode_test.py:154-206 (uniform and stochastic, step 1.0, two clients of ones[3])
@pytest.mark.parametrize("mode", ["uniform", "stochastic"])
def test_quantize_encode_round_known_answers(mode):
  res, meas, _ = oagg.quantize_encode_next([np.ones(3, np.float32)] * 2, 1.0, mode)
  np.testing.assert_array_equal(res, [2.0, 2.0, 2.0])
  assert meas["avg_bitrate"] == np.float64(16.0 / 3.0)
  assert meas["avg_distortion"] == 0.0 and meas["avg_sparsity"] == 0.0 and meas["step_size"] == 1.0


# quantize_encode_test.py:211-226
def test_quantize_encode_dithered_bound():
  res, _, _ = oagg.quantize_encode_next([np.ones(3, np.float32)] * 2, 1.0, "dithered")
  assert np.max(np.abs(res - 2.0)) <= 1.0


# stochastic_quantize_test.py:86-110
def test_stochastic_quantize_factory_known_answer():
  res, qsum = oagg.stochastic_quantize_next([np.full(3, 2.0, np.float32)] * 2, 0.4, [(0, 0), (1, 1)])
  np.testing.assert_array_equal(qsum, [10, 10, 10])
  np.testing.assert_allclose(res, [4.0] * 3, rtol=1e-6)


# one_bit_sgd_test.py:100-202
@pytest.mark.parametrize("values,thr,want,dist", [
    ([[-1.0] * 3] * 2, 0.0, [-2.0] * 3, 0.0),
    ([[0.0, 2.0, -1.0]] * 2, 0.0, [2.0, 2.0, -2.0], 2. / 3.),
    ([[-1.0, 1.0, 2.0]] * 2, 2.0, [0.0, 0.0, 4.0], 2. / 3.),
    ([[-1.0, 1.0, 2.0]], 2.0, [0.0, 0.0, 2.0], 2. / 3.),
    ([[-1.0, 1.0, 2.0], [1.0, 1.0, 1.0]], 2.0, [1.0, 1.0, 3.0], 2. / 6.),
])
def test_one_bit_sgd_known_answers(values, thr, want, dist):
  res, meas = oagg.one_bit_sgd_next(values, thr)
  np.testing.assert_allclose(res, want, rtol=1e-6, atol=1e-6)
  np.testing.assert_allclose(meas["avg_distortion"], dist, rtol=1e-6)
  assert meas["avg_bitrate"] == np.float32((3 + 64) / 3)


@pytest.mark.parametrize("kind", ["sparse", "dense", "extreme", "zeros"])
def test_rlgamma_round_trip(kind):
  rng = np.random.default_rng(3)
  P = 10007
  q = {"sparse": np.where(rng.random(P) < 0.9, 0, rng.integers(-9, 9, P)),
       "dense": rng.integers(-1000, 1000, P),
       "extreme": rng.choice([-2**31, 2**31 - 1, 1, -1, 0], P),
       "zeros": np.zeros(P)}[kind].astype(np.int32)
  code, nbits = ocodec.run_length_gamma_encode(q)
  assert len(code) == (nbits + 7) // 8
  np.testing.assert_array_equal(ocodec.run_length_gamma_decode(code, P), q)
  acc = np.ones(P, np.int32)
  ocodec.decode_accumulate(code, acc)
  np.testing.assert_array_equal(acc, (q.astype(np.int64) + 1).astype(np.int32) if kind != "extreme"
                                else oagg.wrap_i32(q.astype(np.int64) + 1))


def test_malformed_stream_rejected():
  with pytest.raises(ValueError):
    ocodec.run_length_gamma_decode(b"\x00\x00", 5)


def test_golden_fixtures_reproduce():
  """The oracle still produces the committed fixtures bit for bit."""
  import sys  # pylint: disable=g-import-not-at-top
  sys.path.insert(0, os.path.dirname(GOLDEN))
  import make_golden  # pylint: disable=g-import-not-at-top
  g = np.load(GOLDEN, allow_pickle=False)
  x = g["q_x"]
  for m in make_golden.MODES:
    for si, s in enumerate(make_golden.STEPS):
      for ki, sd in enumerate(make_golden.SEEDS):
        np.testing.assert_array_equal(make_golden.QFN[m](x, np.float32(s), sd), g["q_%s_%d_%d" % (m, si, ki)])
  for name in [k[6:] for k in g.files if k.startswith("rl_in_")]:
    code, nbits = ocodec.run_length_gamma_encode(g["rl_in_" + name])
    assert nbits == int(g["rl_bits_" + name])
    assert code == g["rl_code_" + name].tobytes()


# qsgd_test.py:72-141 (known answers of the QSGD round)
@pytest.mark.parametrize("values,num_steps,want,bitrate", [
    ([[1.0]], 1.0, [1.0], 40.0),                                     # :72-94
    ([[1.0], [2.0]], 2.0, [3.0], 40.0),                              # :96-118
    ([[2.0, 3.0, 6.0]] * 2, 7.0, [4.0, 6.0, 12.0], 56.0 / 3.0),      # :120-142
])
def test_qsgd_known_answers(values, num_steps, want, bitrate):
  res, m, _ = oagg.qsgd_next(values, num_steps, seeds=[(1, 2), (3, 4)])
  np.testing.assert_allclose(res, want, rtol=1e-6)
  assert m["avg_bitrate"] == np.float64(bitrate)
  assert m["avg_distortion"] == 0.0 and m["avg_sparsity"] == 0.0


def test_qsgd_different_clients_bounds():
  # qsgd_test.py:144-172: result within the stochastic-rounding bounds
  res, m, _ = oagg.qsgd_next([[2.0, 3.0, 6.0], [1.0, 1.0, 1.0]], 7.0, seeds=[(5, 6), (7, 8)])
  lo = np.sqrt(3.0) / 7.0 * 4.0
  hi = np.sqrt(3.0) / 7.0 * 5.0
  assert np.all(res - np.array([2.0 + lo, 3.0 + lo, 6.0 + lo]) >= -1e-6)
  assert np.all(res - np.array([2.0 + hi, 4.0 + hi, 6.0 + hi]) <= 1e-6)
  assert m["avg_bitrate"] == np.float64(56.0 / 3.0)
  assert m["avg_distortion"] <= max(1.0 - lo, hi - 1.0) ** 2 / 2.0


def test_client_lambda_known_answer():
  # quantize_encode_client_lambda_test.py:80-132: options [0.5, 1, 2], lambda 1, two
  # clients of ones(3): losses [16/3, 16/3, 1 + 8/3] -> both vote for 2.0
  res, m, next_step = oagg.client_lambda_next([np.ones(3, np.float32)] * 2, 1.0, 1.0,
                                              [0.5, 1.0, 2.0])
  np.testing.assert_array_equal(res, [2.0, 2.0, 2.0])
  np.testing.assert_array_equal(m["step_size_vote_counts"], [0, 0, 2])
  assert next_step == 2.0 and m["step_size"] == 1.0
  onehot, losses = oagg.vote_step_size(np.ones(3, np.float32), [0.5, 1.0, 2.0], 1.0, "uniform", (0, 0))
  np.testing.assert_allclose(losses, [16 / 3, 16 / 3, 1 + 8 / 3], rtol=1e-6)


# drive_test.py:92-201 known answers
@pytest.mark.parametrize("values,scaling,want,dist", [
    ([[-1.0, 0.0, 2.0]] * 2, "min_distortion", [-2.0, 2.0, 2.0], 2. / 3.),
    ([[1.0, -1.0, 0.0], [0.0, 0.0, 0.0]], "min_distortion", [2. / 3., -2. / 3., 2. / 3.], 1. / 9.),
    ([[1.0, 1.0, 1.0]], "unbiased", [1.0, 1.0, 1.0], 0.0),
    ([[-1.0, 0.0, 2.0]] * 2, "unbiased", [-10. / 3., 10. / 3., 10. / 3.], 10. / 9.),
    ([[1.0, -1.0, 0.0], [0.0, 0.0, 0.0]], "unbiased", [1.0, -1.0, 1.0], 1. / 6.),
])
def test_drive_known_answers(values, scaling, want, dist):
  res, m = oagg.drive_next(values, scaling)
  np.testing.assert_allclose(res, want, rtol=1e-6)
  np.testing.assert_allclose(m["avg_distortion"], dist, rtol=1e-6)
  np.testing.assert_allclose(m["avg_bitrate"], 35.0 / 3.0, rtol=1e-6)


def test_hadamard_oracle_is_orthonormal():
  rng = np.random.default_rng(1)
  for P in (1, 3, 4, 1000, 4097):
    x = rng.standard_normal(P).astype(np.float32)
    y = oagg.hadamard_forward(x, (5, 6))
    np.testing.assert_allclose(np.linalg.norm(y), np.linalg.norm(x), rtol=1e-6)
    np.testing.assert_allclose(oagg.hadamard_inverse(y, (5, 6), P), x, atol=1e-6)

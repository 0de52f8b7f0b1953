"""GPU parity of the reference-shaped aggregation processes (ExecutionTest halves).

Each case mirrors a reference execution test (file:line) and additionally
checks bit-exactness against the CPU oracle on seeded inputs and the committed
golden fixtures.
"""
import os

import numpy as np
import pytest
import torch

from federated_amd import _lib
from federated_amd import builder
from federated_amd import codec
from federated_amd.aggregators import elias_gamma_encode
from federated_amd.aggregators import quantize_encode
from federated_amd.aggregators import stochastic_quantize
from federated_amd.aggregators import sum_factory
from federated_amd.aggregators.comparison_methods import one_bit_sgd
from federated_amd.aggregators.utils import quantize_utils
from oracle import aggregators as oagg

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "golden.npz")
SEEDS = [(0, 0), (1, 1), (2**40 + 7, 3)]


# quantize_encode_test.py:154-206
@pytest.mark.parametrize("rounding", ["uniform", "stochastic"])
def test_quantize_encode_reference_execution(gpu, rounding):
  process = quantize_encode.QuantizeEncodeFactory(1.0, rounding_type=rounding).create(
      (np.float32, (3,)))
  out = process.next(process.initialize(), [np.ones(3, np.float32)] * 2)
  np.testing.assert_array_equal(out.result, [2.0, 2.0, 2.0])
  m = out.measurements
  assert m["avg_bitrate"] == np.float64(16.0 / 3.0)
  assert m["avg_distortion"] == 0.0 and m["avg_sparsity"] == 0.0 and m["step_size"] == 1.0
  assert out.state["round_num"] == 1.0 and out.state["step_size"] == 1.0


# quantize_encode_test.py:211-226
def test_quantize_encode_dithered_execution(gpu):
  process = quantize_encode.QuantizeEncodeFactory(1.0, rounding_type="dithered").create(
      (np.float32, (3,)))
  out = process.next(process.initialize(), [np.ones(3, np.float32)] * 2)
  assert np.max(np.abs(out.result - 2.0)) <= 1.0


@pytest.mark.parametrize("rounding", ["uniform", "stochastic", "dithered"])
def test_quantize_encode_matches_golden_round(gpu, rounding):
  g = np.load(GOLDEN, allow_pickle=False)
  xs = list(g["round_x"])
  process = quantize_encode.QuantizeEncodeFactory(0.5, rounding_type=rounding).create(
      (np.float32, (xs[0].size,)))
  out = process.next(process.initialize(), xs, seeds=np.array(SEEDS))
  np.testing.assert_array_equal(out.result, g["round_%s_result" % rounding])
  assert out.measurements["avg_bitrate"] == g["round_%s_bitrate" % rounding]
  np.testing.assert_allclose(out.measurements["avg_distortion"], g["round_%s_distortion" % rounding],
                             rtol=1e-5)
  assert out.measurements["avg_sparsity"] == g["round_%s_sparsity" % rounding]


@pytest.mark.parametrize("norm", ["mean_magnitude", "max_magnitude", "dimensionless_norm"])
def test_quantize_encode_normalized_matches_oracle(gpu, norm):
  rng = np.random.default_rng(5)
  xs = [(rng.standard_normal(4097) * (c + 1)).astype(np.float32) for c in range(3)]
  process = quantize_encode.QuantizeEncodeFactory(0.25, rounding_type="stochastic",
                                                  normalization_type=norm).create(
                                                      (np.float32, (4097,)))
  out = process.next(process.initialize(), xs, seeds=np.array(SEEDS))
  want, meas, _ = oagg.quantize_encode_next(xs, 0.25, "stochastic", seeds=SEEDS,
                                            normalization_type=norm)
  # the norm is the correctly rounded float32 of a float64 reduction on both sides
  # (TF reduces in float32 in an unspecified order: parity unpinned beyond that)
  np.testing.assert_array_equal(out.result, want)
  assert out.measurements["avg_bitrate"] == meas["avg_bitrate"]


@pytest.mark.parametrize("norm", ["mean_magnitude", "max_magnitude", "dimensionless_norm"])
def test_builder_normalized_weighted_matches_oracle(gpu, norm):
  """behind the clipping / mean wrappers the normaliser sees the
  pre-scaled value (x * clip) * weight, as QuantizeEncode does inside TFF's
  MeanFactory / clipping_factory (builder.py:100-109, quantize_encode.py:145)."""
  rng = np.random.default_rng(11)
  P = 5000
  xs = [(rng.standard_normal(P) * (0.3 + c)).astype(np.float32) for c in range(4)]
  w = np.array([1.0, 3.0, 0.5, 7.25], np.float32)
  f = builder.build_quantization_encode_aggregator(step_size=0.25, rounding_type="stochastic",
                                                   normalization_type=norm, zeroing=False)
  process = f.create((np.float32, (P,)), (np.float32, ()))
  state = process.initialize()
  out = process.next(state, xs, weight=w, seeds=np.array(SEEDS + [(9, 9)]))
  # oracle: the inner codec on the pre-scaled values the wrappers hand it
  l2 = np.array([np.sqrt(np.sum(x.astype(np.float64) ** 2)) for x in xs], np.float32)
  clip = np.float32(state["clipping_norm"])
  scale = (clip * np.minimum(np.float32(1.0) / l2, np.float32(1.0) / clip)).astype(np.float32)
  pre = [((x * scale[c]) * w[c]).astype(np.float32) for c, x in enumerate(xs)]
  want, meas, _ = oagg.quantize_encode_next(pre, 0.25, "stochastic", seeds=SEEDS + [(9, 9)],
                                            normalization_type=norm)
  want = want / np.float32(np.sum(w, dtype=np.float32))
  np.testing.assert_array_equal(out.result, want.astype(np.float32))
  assert out.measurements["mean_value"]["avg_bitrate"] == meas["avg_bitrate"]


def test_elias_gamma_factory_reference_execution(gpu):
  # elias_gamma_encode_test.py:80-116
  process = elias_gamma_encode.EliasGammaEncodedSumFactory().create((np.int32, (4,)))
  out = process.next((), [[-5, 3, 0, 0], [-3, 1, 0, 0]])
  np.testing.assert_array_equal(out.result, [-8, 4, 0, 0])
  assert out.measurements["avg_bitrate"] == 16 / 4
  process2 = elias_gamma_encode.EliasGammaEncodedSumFactory().create((np.int32, (2, 4)))
  out2 = process2.next((), [[[-5, 3, 0, 0], [-3, 1, 0, 0]]] * 2)
  np.testing.assert_array_equal(out2.result, [[-10, 6, 0, 0], [-6, 2, 0, 0]])
  assert out2.measurements["avg_bitrate"] == 32 / 8


def test_stochastic_quantize_reference_execution(gpu):
  # stochastic_quantize_test.py:86-110
  f = stochastic_quantize.StochasticQuantizeFactory(0.4, sum_factory.add_sum_measurements())
  process = f.create((np.float32, (3,)))
  out = process.next((), [np.full(3, 2.0, np.float32)] * 2)
  np.testing.assert_array_equal(out.measurements, [10, 10, 10])
  np.testing.assert_allclose(out.result, [4.0] * 3, rtol=1e-6)
  ps = f.create([(np.float32, (2,)), (np.float32, (3,))])
  out = ps.next((), [[np.full(2, 2.0, np.float32), np.full(3, 2.0, np.float32)]] * 2)
  np.testing.assert_allclose(out.result[1], [4.0] * 3, rtol=1e-6)


# one_bit_sgd_test.py:100-202
@pytest.mark.parametrize("values,thr,want,dist", [
    ([[-1.0] * 3] * 2, 0.0, [-2.0] * 3, 0.0),
    ([[0.0, 2.0, -1.0]] * 2, 0.0, [2.0, 2.0, -2.0], 2. / 3.),
    ([[-1.0, 1.0, 2.0]] * 2, 2.0, [0.0, 0.0, 4.0], 2. / 3.),
    ([[-1.0, 1.0, 2.0]], 2.0, [0.0, 0.0, 2.0], 2. / 3.),
    ([[-1.0, 1.0, 2.0], [1.0, 1.0, 1.0]], 2.0, [1.0, 1.0, 3.0], 2. / 6.),
])
def test_one_bit_sgd_reference_execution(gpu, values, thr, want, dist):
  process = one_bit_sgd.OneBitSGDFactory(thr).create((np.float32, (3,)))
  out = process.next((), [np.array(v, np.float32) for v in values])
  np.testing.assert_allclose(out.result, want, rtol=1e-6, atol=1e-6)
  np.testing.assert_allclose(out.measurements["avg_distortion"], dist, rtol=1e-6)
  assert out.measurements["avg_bitrate"] == np.float32(67 / 3)


def test_one_bit_matches_golden(gpu):
  g = np.load(GOLDEN, allow_pickle=False)
  xs = list(g["round_x"])
  out = one_bit_sgd.OneBitSGDFactory(0.1).create((np.float32, (xs[0].size,))).next((), xs)
  np.testing.assert_allclose(out.result, g["onebit_result"], rtol=1e-6, atol=1e-6)
  np.testing.assert_allclose(out.measurements["avg_distortion"], g["onebit_distortion"], rtol=1e-5)


def test_quantize_utils_device_functions(gpu):
  # quantize_utils_test.py:46-59
  q = quantize_utils.uniform_quantize(torch.full((3,), 2.0), 0.4, (0, 0))
  np.testing.assert_array_equal(q.cpu().numpy(), [5, 5, 5])
  d = quantize_utils.uniform_dequantize(torch.full((3,), 5, dtype=torch.int32), 0.4)
  np.testing.assert_allclose(d.cpu().numpy(), [2.0] * 3, rtol=1e-7)
  assert float(quantize_utils.max_magnitude(torch.tensor([0.0, 1.0, 2.0]))) == 2.0
  np.testing.assert_allclose(float(quantize_utils.mean_magnitude(torch.tensor([0.0, 1.0, 2.0]))), 1.0)
  noise = quantize_utils.generate_noise((3, 9), (1001,))
  g = np.load(GOLDEN, allow_pickle=False)
  np.testing.assert_array_equal(noise.cpu().numpy(), g["noise_3_9"])


def test_quantizer_matches_golden_fixtures(gpu):
  g = np.load(GOLDEN, allow_pickle=False)
  x = torch.from_numpy(g["q_x"]).cuda()
  steps = [0.5, 0.4, 1.0 / 127, 1.0]
  for mi, m in enumerate(["uniform", "stochastic", "dithered"]):
    for si, s in enumerate(steps):
      for ki, sd in enumerate(SEEDS):
        q, _ = codec.quantize(x, np.float32(s), sd, mi)
        np.testing.assert_array_equal(q.cpu().numpy(), g["q_%s_%d_%d" % (m, si, ki)])


def test_rlgamma_matches_golden_fixtures(gpu):
  g = np.load(GOLDEN, allow_pickle=False)
  names = [k[6:] for k in g.files if k.startswith("rl_in_")]
  for name in names:
    b = codec.rlgamma_encode([torch.from_numpy(g["rl_in_" + name]).cuda()])
    assert int(b.bits()[0]) == int(g["rl_bits_" + name]), name
    assert b.client_code(0) == g["rl_code_" + name].tobytes(), name


def test_builder_round_runs_and_clips(gpu):
  f = builder.build_quantization_encode_aggregator(step_size=0.01, rounding_type="uniform")
  process = f.create([(np.float32, (2, 3)), (np.float32, (4,))], (np.float32, ()))
  state = process.initialize()
  rng = np.random.default_rng(9)
  values = [[rng.standard_normal((2, 3)).astype(np.float32) * 0.1,
             rng.standard_normal(4).astype(np.float32) * 0.1] for _ in range(4)]
  weights = [1.0, 2.0, 3.0, 4.0]
  out = process.next(state, values, weights, seeds=np.array([[i, i] for i in range(4)]))
  # weighted mean of clipped values (norms < 1 => unclipped), quantised with step 0.01
  flat = [np.concatenate([v[0].reshape(-1), v[1]]) for v in values]
  want = sum(w * x for w, x in zip(weights, flat)) / sum(weights)
  got = np.concatenate([out.result[0].reshape(-1), out.result[1]])
  assert np.max(np.abs(got - want)) <= 0.01 * 0.5 * 4 / sum(weights) + 1e-6
  assert out.state["clipping_norm"] != state["clipping_norm"]


def test_decoder_rejects_malformed_stream(gpu):
  b = codec.rlgamma_encode([torch.tensor([5, 0, -3, 7], dtype=torch.int32, device="cuda")])
  b.stream.zero_()  # a run of zeros longer than 31 bits is not a gamma code
  _, _, err = codec.decode_accumulate(b)
  assert int(err.item()) != 0


# qsgd_test.py:72-142 known answers, through the HIP path
@pytest.mark.parametrize("values,num_steps,want,bitrate", [
    ([[1.0]], 1.0, [1.0], 40.0),
    ([[1.0], [2.0]], 2.0, [3.0], 40.0),
    ([[2.0, 3.0, 6.0]] * 2, 7.0, [4.0, 6.0, 12.0], 56.0 / 3.0),
])
def test_qsgd_reference_execution(gpu, values, num_steps, want, bitrate):
  from federated_amd.aggregators.comparison_methods import qsgd  # pylint: disable=g-import-not-at-top
  process = qsgd.QSGDFactory(num_steps).create((np.float32, (len(values[0]),)))
  out = process.next(process.initialize(), [np.asarray(v, np.float32) for v in values])
  np.testing.assert_array_equal(out.result, np.asarray(want, np.float32))
  assert out.measurements["avg_bitrate"] == np.float64(bitrate)
  assert out.measurements["avg_distortion"] == 0.0 and out.measurements["avg_sparsity"] == 0.0


@pytest.mark.parametrize("P,C", [(5, 2), (4099, 3), (300007, 6)])
def test_qsgd_matches_oracle(gpu, P, C):
  from federated_amd.aggregators.comparison_methods import qsgd  # pylint: disable=g-import-not-at-top
  rng = np.random.default_rng(P + C)
  xs = [(rng.standard_normal(P) * rng.uniform(0.01, 3)).astype(np.float32) for _ in range(C)]
  seeds = np.array([[40 + c, 7 * c] for c in range(C)], np.int64)
  process = qsgd.QSGDFactory(127.0).create((np.float32, (P,)))
  out = process.next(process.initialize(), xs, seeds=seeds)
  want, m, codes = oagg.qsgd_next(xs, 127.0, seeds=seeds)
  # the norm (correctly rounded float64 sum on both sides), q, the codes and the
  # client-order float32 server sum are all exact
  np.testing.assert_array_equal(out.result, want)
  assert out.measurements["avg_bitrate"] == m["avg_bitrate"]
  assert out.measurements["avg_sparsity"] == m["avg_sparsity"]
  np.testing.assert_allclose(out.measurements["avg_distortion"], m["avg_distortion"], rtol=1e-5)
  # deterministic run to run (round 1 summed with LDS float atomics)
  out2 = process.next(process.initialize(), xs, seeds=seeds)
  np.testing.assert_array_equal(out2.result, out.result)


@pytest.mark.parametrize("qmax", [None, 41, 127], ids=["int32rows", "int8rows41", "int8rows127"])
@pytest.mark.parametrize("P,C,group", [(4099, 5, 2), (2048, 300, 7), (1025, 3, 3)])
def test_decode_scaled_client_order(gpu, P, C, group, qmax):
  """fc_decode_accumulate_scaled in client groups (a workspace of `group` int32
  rows; with a bound qmax <= 127 the rows are int8, four times as many per group):
  acc = fsum_in, then acc + f32(q_c) * s_c in client order, bit for bit."""
  rng = np.random.default_rng(P * 7 + C)
  qs = [rng.integers(-40, 41, P).astype(np.int32) * (rng.random(P) < 0.6) for _ in range(C)]
  qs[0][: P // 3] = 0  # long zero runs
  batch = codec.rlgamma_encode([torch.from_numpy(q.astype(np.int32)).to(gpu) for q in qs])
  scale = (rng.random(C) * 3 + 1e-3).astype(np.float32)
  fin = rng.standard_normal(P).astype(np.float32)
  stride = (P + 3) // 4 * 4
  ws = torch.empty(group * stride * 4, dtype=torch.uint8, device=gpu)
  out, err = codec.decode_accumulate_scaled(batch, scale, fsum_in=torch.from_numpy(fin).to(gpu), workspace=ws,
                                            qmax=qmax)
  assert int(err.item()) == 0
  acc = fin.copy()
  for c in range(C):
    acc = (acc + (qs[c].astype(np.float32) * scale[c]).astype(np.float32)).astype(np.float32)
  np.testing.assert_array_equal(out.cpu().numpy(), acc)


def test_decode_scaled_int8_rows_flag_values_past_the_bound(gpu):
  """A declared bound the codes break (|q| = 200 > 127) is reported through err."""
  P = 3000
  q = np.zeros(P, np.int32)
  q[[5, 1000, 2999]] = [3, -200, 7]
  batch = codec.rlgamma_encode([torch.from_numpy(q).to(gpu)])
  _, err = codec.decode_accumulate_scaled(batch, np.array([0.5], np.float32), qmax=127)
  assert int(err.item()) != 0
  out, err = codec.decode_accumulate_scaled(batch, np.array([0.5], np.float32))
  assert int(err.item()) == 0
  np.testing.assert_array_equal(out.cpu().numpy(), q.astype(np.float32) * np.float32(0.5))


def test_qsgd_codes_bit_exact(gpu):
  """The fused encoder with a per-client step reproduces the oracle's bytes."""
  rng = np.random.default_rng(11)
  P, C = 70001, 3
  xs = [(rng.standard_normal(P) * 0.1).astype(np.float32) for _ in range(C)]
  seeds = np.array([[9, c] for c in range(C)], np.int64)
  _, _, codes = oagg.qsgd_next(xs, 15.0, seeds=seeds)
  norms = np.array([oagg.l2_norm(x) for x in xs], np.float32)
  steps = torch.from_numpy((norms / np.float32(15.0)).astype(np.float32)).to(gpu)
  batch = codec.quantize_encode_checked([torch.from_numpy(x).to(gpu) for x in xs], 1.0,
                                        torch.from_numpy(seeds), _lib.STOCHASTIC, norms=steps)
  for c in range(C):
    assert batch.client_code(c) == codes[c]


# quantize_encode_client_lambda_test.py:80-132
def test_client_lambda_reference_execution(gpu):
  from federated_amd.aggregators import quantize_encode_client_lambda as qecl  # pylint: disable=g-import-not-at-top
  process = qecl.QuantizeEncodeClientLambdaFactory(1.0, 1.0, [0.5, 1.0, 2.0]).create(
      (np.float32, (3,)))
  out = process.next(process.initialize(), [np.ones(3, np.float32)] * 2)
  np.testing.assert_array_equal(out.result, [2.0, 2.0, 2.0])
  np.testing.assert_array_equal(out.measurements["step_size_vote_counts"], [0, 0, 2])
  assert out.measurements["step_size"] == 1.0 and out.state["step_size"] == 2.0


@pytest.mark.parametrize("rounding", ["uniform", "stochastic", "dithered"])
@pytest.mark.parametrize("P,C", [(7, 2), (5000, 3), (200003, 4)])
def test_vote_lengths_match_oracle(gpu, rounding, P, C):
  """Per-option code lengths are exact; distortions within float tolerance."""
  from oracle import codec as ocodec  # pylint: disable=g-import-not-at-top
  from oracle import quantize_utils as oq  # pylint: disable=g-import-not-at-top
  rng = np.random.default_rng(P * 3 + C)
  xs = [(rng.standard_normal(P) * rng.uniform(0.05, 2)).astype(np.float32) for _ in range(C)]
  xs[0][: P // 3] = 0.0  # long zero runs across tiles
  options = [0.05, 0.1, 0.5, 1.0, 2.0, 7.0, 1e-3]
  seeds = np.array([[3 + c, 11 * c] for c in range(C)], np.int64)
  bits, dist = codec.vote_lengths([torch.from_numpy(x).to(gpu) for x in xs], options, seeds,
                                  {"uniform": 0, "stochastic": 1, "dithered": 2}[rounding])
  bits, dist = bits.cpu().numpy(), dist.cpu().numpy()
  qfn = {"uniform": lambda x, s, sd: oq.uniform_quantize(x, s), "stochastic": oq.stochastic_quantize,
         "dithered": oq.dithered_quantize}[rounding]
  for c in range(C):
    noise = oq.generate_noise(tuple(seeds[c]), P) if rounding == "dithered" else None
    for k, step in enumerate(options):
      q = qfn(xs[c], np.float32(step), tuple(seeds[c]))
      assert bits[c, k] == ocodec.encoded_bits(q), (c, k)
      deq = oq.dithered_dequantize(q, np.float32(step), noise) if noise is not None else \
          oq.uniform_dequantize(q, np.float32(step))
      want = np.sum((oq.ftz(xs[c]) - deq).astype(np.float64) ** 2)
      np.testing.assert_allclose(dist[c, k], want, rtol=1e-5, atol=1e-12)


def test_client_lambda_matches_oracle(gpu):
  from federated_amd.aggregators import quantize_encode_client_lambda as qecl  # pylint: disable=g-import-not-at-top
  rng = np.random.default_rng(21)
  P, C = 3001, 6
  xs = [rng.uniform(-1.0 / (c + 1), 1.0 / (c + 1), P).astype(np.float32) for c in range(C)]
  options = [0.01, 0.1, 0.5, 1.0, 2.0]
  seeds = np.array([[c, c + 1] for c in range(C)], np.int64)
  process = qecl.QuantizeEncodeClientLambdaFactory(0.001, 0.5, options, "stochastic").create(
      (np.float32, (P,)))
  out = process.next(process.initialize(), xs, seeds=seeds)
  want, m, next_step = oagg.client_lambda_next(xs, 0.001, 0.5, options, "stochastic", seeds=seeds)
  np.testing.assert_array_equal(out.result, want)
  np.testing.assert_array_equal(out.measurements["step_size_vote_counts"], m["step_size_vote_counts"])
  assert out.state["step_size"] == next_step


@pytest.mark.parametrize("values,scaling,want,dist", [
    ([[-1.0, 0.0, 2.0]] * 2, "min_distortion", [-2.0, 2.0, 2.0], 2. / 3.),
    ([[1.0, -1.0, 0.0], [0.0, 0.0, 0.0]], "min_distortion", [2. / 3., -2. / 3., 2. / 3.], 1. / 9.),
    ([[1.0, 1.0, 1.0]], "unbiased", [1.0, 1.0, 1.0], 0.0),
    ([[-1.0, 0.0, 2.0]] * 2, "unbiased", [-10. / 3., 10. / 3., 10. / 3.], 10. / 9.),
    ([[1.0, -1.0, 0.0], [0.0, 0.0, 0.0]], "unbiased", [1.0, -1.0, 1.0], 1. / 6.),
])
def test_drive_reference_execution(gpu, values, scaling, want, dist):
  from federated_amd.aggregators.comparison_methods import drive  # pylint: disable=g-import-not-at-top
  process = drive.DRIVEFactory(scaling).create((np.float32, (3,)))
  out = process.next(process.initialize(), [np.asarray(v, np.float32) for v in values])
  np.testing.assert_allclose(out.result, want, rtol=1e-6)
  np.testing.assert_allclose(out.measurements["avg_distortion"], dist, rtol=1e-6)
  np.testing.assert_allclose(out.measurements["avg_bitrate"], 35.0 / 3.0, rtol=1e-6)


@pytest.mark.parametrize("scaling", ["unbiased", "min_distortion"])
def test_drive_matches_oracle(gpu, scaling):
  from federated_amd.aggregators.comparison_methods import drive  # pylint: disable=g-import-not-at-top
  rng = np.random.default_rng(4)
  P, C = 100003, 5
  xs = [(rng.standard_normal(P) * (c + 0.5)).astype(np.float32) for c in range(C)]
  out = drive.DRIVEFactory(scaling).create((np.float32, (P,))).next((), xs)
  want, m = oagg.drive_next(xs, scaling)
  np.testing.assert_allclose(out.result, want, rtol=1e-5, atol=1e-5)
  np.testing.assert_allclose(out.measurements["avg_distortion"], m["avg_distortion"], rtol=1e-5)


@pytest.mark.parametrize("P", [1, 3, 4096, 5000, 1 << 17, 300001, (1 << 21) + 5])  # last: 3 passes
def test_hadamard_matches_oracle_and_round_trips(gpu, P):
  rng = np.random.default_rng(P)
  x = rng.standard_normal(P).astype(np.float32)
  n = 1 << max(0, (P - 1).bit_length())
  t = torch.zeros(n, dtype=torch.float32, device=gpu)
  t[:P] = torch.from_numpy(x).to(gpu)
  codec.hadamard_([t], (7, 9))
  y = t.cpu().numpy()
  want = oagg.hadamard_forward(x, (7, 9))
  np.testing.assert_allclose(y, want, rtol=1e-4, atol=1e-5 * max(1.0, np.sqrt(np.log2(n))))
  codec.hadamard_([t], (7, 9), inverse=True)
  np.testing.assert_allclose(t.cpu().numpy()[:P], x, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("P", [1, 2, 3, 32, 1000, 4097, 1 << 17, 300_001, 2_000_006])
def test_dft_matches_oracle_and_round_trips(gpu, P):
  """The DFT rotation (builder.py:70-71): signs from the same Philox stream as the
  Hadamard rotation, unitary FFT of the n/2 complex numbers (fc_dft_rotate: Stockham
  passes for powers of two -- m = 16, 2^16 -- Bluestein otherwise, m = 1,000,003 a
  prime); against a float64 numpy restatement, norm-preserving, and inverted back
  to x."""
  rng = np.random.default_rng(P + 1)
  x = rng.standard_normal(P).astype(np.float32)
  n = P + P % 2
  t = torch.zeros(n, dtype=torch.float32, device=gpu)
  t[:P] = torch.from_numpy(x).to(gpu)
  codec.dft_([t], (7, 9))
  y = t.cpu().numpy()
  np.testing.assert_allclose(y, oagg.dft_forward(x, (7, 9)), rtol=1e-4, atol=1e-5 * max(1.0, np.log2(n)))
  np.testing.assert_allclose(np.linalg.norm(y.astype(np.float64)), np.linalg.norm(x.astype(np.float64)), rtol=1e-5)
  codec.dft_([t], (7, 9), inverse=True)
  np.testing.assert_allclose(t.cpu().numpy()[:P], x, rtol=1e-4, atol=1e-5)


def test_dft_rows_at_25M(gpu):
  """fc_dft_rotate over two rows of 25,000,000 (m = 12.5 M complex, Bluestein length
  2^25): each row against numpy's float64 FFT (relative L2 error), and back."""
  P = 25_000_000
  rng = np.random.default_rng(25)
  xs = [rng.standard_normal(P).astype(np.float32) for _ in range(2)]
  ts = [torch.from_numpy(x).to(gpu) for x in xs]
  codec.dft_(ts, (3, 4))
  for x, t in zip(xs, ts):
    y = t.cpu().numpy().astype(np.float64)
    want = oagg.dft_forward(x, (3, 4))
    assert np.linalg.norm(y - want) <= 1e-5 * np.linalg.norm(want)
  codec.dft_(ts, (3, 4), inverse=True)
  for x, t in zip(xs, ts):
    back = t.cpu().numpy().astype(np.float64)
    assert np.linalg.norm(back - x) <= 1e-5 * np.linalg.norm(x)
  del ts
  torch.cuda.empty_cache()


@pytest.mark.parametrize("rotation", ["dft", "hadamard"])
def test_quantize_encode_with_rotation_end_to_end(gpu, rotation):
  """build_quantization_encode_aggregator(rotation=...) (builder.py:68-71): the round's
  result is the weighted mean within the quantiser's error in the rotated basis,
  and a linear inner aggregator makes the rotation invisible."""
  rng = np.random.default_rng(9)
  P, C = 3001, 4
  xs = [(rng.standard_normal(P) * 0.1).astype(np.float32) for _ in range(C)]
  agg = builder.build_quantization_encode_aggregator(step_size=0.001, rotation=rotation, zeroing=False,
                                                     clipping=False, weighted=False)
  process = agg.create((np.float32, (P,)))
  out = process.next(process.initialize(), xs)
  mean = np.mean(np.stack(xs), axis=0)
  res = np.asarray(out.result)
  assert res.shape == (P,)
  assert np.max(np.abs(res - mean)) < 0.002  # |error| <= step / 2 per coordinate, rotated back
  factory = builder.DiscreteFourierTransformFactory if rotation == "dft" else builder.HadamardTransformFactory
  from federated_amd.aggregators import sum_factory  # pylint: disable=g-import-not-at-top
  proc = factory(sum_factory.SumFactory()).create((np.float32, (P,)))
  out = proc.next(proc.initialize(), xs)
  np.testing.assert_allclose(np.asarray(out.result), np.sum(np.stack(xs).astype(np.float64), 0), rtol=1e-4,
                             atol=1e-4)


def test_drive_with_hadamard_rotation_end_to_end(gpu):
  rng = np.random.default_rng(8)
  P, C = 5000, 4
  xs = [(rng.standard_normal(P) * 0.01).astype(np.float32) for _ in range(C)]
  agg = builder.build_drive_aggregator(zeroing=False, clipping=False, weighted=False)
  process = agg.create((np.float32, (P,)))
  out = process.next(process.initialize(), xs)
  res = np.asarray(out.result)
  assert res.shape == (P,)
  # unweighted mean of the clients, approximated by 1-bit DRIVE in the rotated basis
  mean = np.mean(np.stack(xs), axis=0)
  assert np.linalg.norm(res - mean) < np.linalg.norm(mean) * 1.5


@pytest.mark.parametrize("P", [1, 31, 2047, 2049, 70_001])
def test_mask_encoders_many_tiles(gpu, P):
  """k_mask_encode (one-bit SGD, DRIVE) over full and partial 2048-element tiles:
  masks bit-exact (bit i of word w = element 32w + i), means and distortion
  against float64 numpy within float32 tolerance; client_norms likewise."""
  rng = np.random.default_rng(P)
  xs = [(rng.standard_normal(P) * (1 + c)).astype(np.float32) for c in range(3)]
  xs[1][: P // 2] = 0.0
  dev = [torch.from_numpy(x).to(gpu) for x in xs]
  nw = (P + 31) // 32

  def want_masks(ab):
    bits = np.zeros(nw * 32, bool)
    bits[:P] = ab
    return np.packbits(bits.reshape(-1, 32)[:, ::-1], axis=1).view(">u4").ravel().astype(np.uint32)

  masks, means, dist = codec.onebit_encode(dev, 0.1)
  masks = masks.cpu().numpy().view(np.uint32).reshape(3, nw)
  means = means.cpu().numpy().reshape(3, 2)
  for c, x in enumerate(xs):
    ab = ~(x < np.float32(0.1))
    np.testing.assert_array_equal(masks[c], want_masks(ab))
    mb = x[~ab].astype(np.float64).sum() / max((~ab).sum(), 1)
    ma = x[ab].astype(np.float64).sum() / max(ab.sum(), 1)
    np.testing.assert_allclose(means[c], [mb, ma], rtol=1e-5, atol=1e-7)
    dec = np.where(ab, means[c, 1], means[c, 0]).astype(np.float32)
    np.testing.assert_allclose(float(dist[c]), float(((x - dec).astype(np.float64) ** 2).sum()), rtol=1e-5)

  masks, means, dist = codec.drive_encode(dev)
  masks = masks.cpu().numpy().view(np.uint32).reshape(3, nw)
  means = means.cpu().numpy().reshape(3, 2)
  for c, x in enumerate(xs):
    np.testing.assert_array_equal(masks[c], want_masks(~(x < 0)))
    n1 = np.abs(x.astype(np.float64)).sum()
    scale = (np.sqrt((x.astype(np.float64) ** 2).sum()) ** 2 / n1) if n1 else 0.0
    np.testing.assert_allclose(means[c], [-scale, scale], rtol=1e-5)

  for kind, fn in ((_lib.NORM_L2, lambda x: np.sqrt((x.astype(np.float64) ** 2).sum())),
                   (_lib.NORM_MAX_MAGNITUDE, lambda x: np.abs(x).max())):
    got = codec.client_norms(dev, kind).cpu().numpy()
    np.testing.assert_allclose(got, [fn(x) for x in xs], rtol=1e-6)


@pytest.mark.parametrize("C", [1, 16, 64, 128])
def test_client_split_passes(gpu, C):
  """Few clients per GPU: k_client_norms and k_mask_encode cut each client's row
  over several workgroups (fc's client_parts: up to 16 parts here) and add the
  float64 parts in order.  Masks bit-exact; the L2 / max norms equal the oracle's
  correctly rounded float32 (oracle.aggregators.l2_norm); means, distortion and
  DRIVE scales against float64 numpy (one_bit_sgd.py:56-81, drive.py:58-76)."""
  P = (1 << 21) + 5
  rng = np.random.default_rng(C)
  xs = [(rng.standard_normal(P) * (0.5 + (c % 7))).astype(np.float32) for c in range(C)]
  dev = [torch.from_numpy(x).to(gpu) for x in xs]
  nw = (P + 31) // 32
  l2 = codec.client_norms(dev, _lib.NORM_L2).cpu().numpy()
  mx = codec.client_norms(dev, _lib.NORM_MAX_MAGNITUDE).cpu().numpy()
  both = codec.client_norms(dev, _lib.NORM_L2_LINF).cpu().numpy()
  masks, means, dist = codec.onebit_encode(dev, 0.0)
  masks = masks.cpu().numpy().view(np.uint32).reshape(C, nw)
  means = means.cpu().numpy().reshape(C, 2)
  dist = dist.cpu().numpy()
  _, dmeans, _ = codec.drive_encode(dev)
  dmeans = dmeans.cpu().numpy().reshape(C, 2)
  for c in range(0, C, max(1, C // 8)):
    x = xs[c]
    assert l2[c] == oagg.l2_norm(x)
    assert mx[c] == np.abs(x).max() and both[1, c] == mx[c] and both[0, c] == l2[c]
    ab = x >= 0
    bits = np.pad(ab.astype(np.uint8), (0, nw * 32 - P)).reshape(nw, 32)
    np.testing.assert_array_equal(masks[c], np.packbits(bits, axis=1, bitorder="little").view("<u4").reshape(-1))
    xd = x.astype(np.float64)
    mb, ma = xd[~ab].sum() / max((~ab).sum(), 1), xd[ab].sum() / max(ab.sum(), 1)
    np.testing.assert_allclose(means[c], [mb, ma], rtol=1e-6)
    dec = np.where(ab, means[c, 1], means[c, 0]).astype(np.float32)
    np.testing.assert_allclose(dist[c], ((x - dec).astype(np.float64) ** 2).sum(), rtol=1e-6)
    scale = (xd ** 2).sum() / np.abs(xd).sum()
    np.testing.assert_allclose(dmeans[c], [-scale, scale], rtol=1e-6)


def test_client_split_is_deterministic(gpu, monkeypatch):
  """the client split's float64 sums are formed per reduction block of
  64 x 2048 elements in an order fixed by P alone, so the norms, the one-bit / DRIVE
  means and the distortion of a client are the same bits whether it is encoded with
  1024 clients on one GPU (few parts per client) or in a 128- or 16-client share of
  an 8-GPU round (many parts), and for any forced part count."""
  P = (1 << 20) + 4099  # 9 reduction blocks, the last one partial
  C = 1024
  g = torch.Generator(device=gpu)
  g.manual_seed(77)
  xs = torch.randn(C, P, generator=g, device=gpu, dtype=torch.float32)
  xs[5] += 1000.0  # a client whose one-pass distortion cancels (k_mask_distortion)
  rows = [xs[c] for c in range(C)]

  def run(sub):
    both = codec.client_norms(sub, _lib.NORM_L2_LINF).cpu().numpy()
    mean = codec.client_norms(sub, _lib.NORM_MEAN_MAGNITUDE).cpu().numpy()
    rms = codec.client_norms(sub, _lib.NORM_DIMENSIONLESS).cpu().numpy()
    masks, means, dist = codec.onebit_encode(sub, 0.0)
    _, dmeans, ddist = codec.drive_encode(sub)
    return (both.reshape(2, -1), mean, rms, masks.cpu().numpy().reshape(len(sub), -1),
            means.cpu().numpy().reshape(-1, 2), dist.cpu().numpy(), dmeans.cpu().numpy().reshape(-1, 2),
            ddist.cpu().numpy())

  full = run(rows)
  for lo, hi in ((0, 128), (128, 144), (5, 6)):
    part = run(rows[lo:hi])
    for a, b in zip(full, part):
      a = a[:, lo:hi] if a.ndim == 2 and a.shape[0] == 2 and a.shape[1] == C else a[lo:hi]
      np.testing.assert_array_equal(a.view(np.uint8), b.view(np.uint8))
  monkeypatch.setenv("FEDCODEC_OB_PARTS", "3")
  forced = run(rows[:16])
  for a, b in zip(full, forced):
    a = a[:, :16] if a.ndim == 2 and a.shape[0] == 2 and a.shape[1] == C else a[:16]
    np.testing.assert_array_equal(a.view(np.uint8), b.view(np.uint8))
  del xs, rows
  torch.cuda.empty_cache()

"""Reference-shaped API surface, host-side logic only (no GPU).

Mirrors the ComputationTest halves of the reference tests: constructor
validation, create() type checks, initialize() state structure.
"""
import collections

import numpy as np
import pytest

from federated_amd import builder
from federated_amd import tff_compat as tc
from federated_amd.aggregators import elias_gamma_encode
from federated_amd.aggregators import quantize_encode
from federated_amd.aggregators import stochastic_quantize
from federated_amd.aggregators import sum_factory
from federated_amd.aggregators.comparison_methods import one_bit_sgd
from federated_amd.aggregators.utils import quantize_utils


# quantize_encode_test.py:30-65
@pytest.mark.parametrize("rounding", ["uniform", "stochastic", "dithered"])
def test_quantize_encode_initialize_state(rounding):
  process = quantize_encode.QuantizeEncodeFactory(1.0, rounding_type=rounding).create(
      (np.float32, (3,)))
  state = process.initialize()
  assert isinstance(state, collections.OrderedDict)
  assert list(state) == ["round_num", "step_size", "inner_state"]
  assert state["round_num"].dtype == np.float32 and state["round_num"] == 0.0
  assert state["step_size"].dtype == np.float32 and state["step_size"] == 1.0
  assert state["inner_state"] == ()


# quantize_encode_test.py:136-146
@pytest.mark.parametrize("value_type", [(np.int32, (3,)), [(np.float32, (2,)), (np.float32, (3,))]])
def test_quantize_encode_create_raises(value_type):
  with pytest.raises(ValueError):
    quantize_encode.QuantizeEncodeFactory(1.0).create(value_type)


@pytest.mark.parametrize("kw,msg", [
    (dict(rounding_type="bogus"), "rounding_type"),
    (dict(normalization_type="bogus"), "normalization_type"),
    (dict(schedule="bogus"), "schedule"),
])
def test_quantize_encode_ctor_raises(kw, msg):
  with pytest.raises(ValueError, match=msg):
    quantize_encode.QuantizeEncodeFactory(0.5, **kw)


# elias_gamma_encode_test.py:40-77
def test_elias_gamma_create():
  process = elias_gamma_encode.EliasGammaEncodedSumFactory().create((np.int32, (4,)))
  assert process.initialize() == ()
  for bad in [(np.float32, (3,)), [(np.int32, (2,)), (np.int32, (3,))]]:
    with pytest.raises(ValueError):
      elias_gamma_encode.EliasGammaEncodedSumFactory().create(bad)
  assert elias_gamma_encode.get_bitstring_length(b"ab") == 16.0


def test_stochastic_quantize_create():
  f = stochastic_quantize.StochasticQuantizeFactory(0.4, sum_factory.add_sum_measurements())
  assert f.create((np.float32, (3,))).initialize() == ()
  with pytest.raises(ValueError):
    f.create((np.int32, (3,)))


def test_one_bit_create():
  assert one_bit_sgd.OneBitSGDFactory().create((np.float32, (3,))).initialize() == ()
  with pytest.raises(ValueError):
    one_bit_sgd.OneBitSGDFactory().create((np.int32, (3,)))


# builder_test.py / builder.py:498-516
@pytest.mark.parametrize("kw,msg", [
    (dict(rounding_type="x"), "rounding_type"),
    (dict(normalization_type="x"), "normalization_type"),
    (dict(step_size_sched="x"), "step_size_sched"),
])
def test_builder_validation(kw, msg):
  with pytest.raises(ValueError, match=msg):
    builder.build_quantization_encode_aggregator(**kw)


def test_builder_default_state():
  f = builder.build_quantization_encode_aggregator(rounding_type="stochastic", zeroing=False)
  process = f.create([(np.float32, (2, 3)), (np.float32, (4,))], (np.float32, ()))
  state = process.initialize()
  assert state["clipping_norm"] == np.float32(1.0)
  assert state["zeroing_norm"] == ()
  assert list(state["inner_state"]) == ["round_num", "step_size", "inner_state"]
  with pytest.raises(ValueError):
    builder.configure_aggregator(quantize_encode.QuantizeEncodeFactory(0.5), rotation="bogus")


def test_quantile_estimate_geometric_update():
  q = builder.QuantileEstimate(1.0, 0.8, 0.2)
  # all norms below the estimate -> estimate shrinks by exp(-0.2 * 0.2)
  assert np.isclose(q.update(np.float32(1.0), [0.1, 0.2]), np.exp(-0.2 * 0.2), rtol=1e-6)
  z = builder.QuantileEstimate(10.0, 0.98, np.log(10.0), multiplier=2.0, increment=1.0)
  assert z.report(np.float32(10.0)) == 21.0


def test_quantile_estimate_counts_against_the_raw_estimate():
  # TFF applies multiplier / increment to the reported value only: the quantile
  # query compares every record with the raw estimate X (10), not 2X + 1 (21).
  z = builder.QuantileEstimate(10.0, 0.98, np.log(10.0), multiplier=2.0, increment=1.0)
  norms = np.array([5.0, 9.0, 15.0, 20.0], np.float32)  # 2 of 4 <= X; all 4 <= 2X + 1
  got = z.update(np.float32(10.0), norms)
  want = np.float32(10.0) * np.exp(-np.float32(np.log(10.0)) * (np.float32(0.5) - np.float32(0.98)))
  assert np.isclose(got, want, rtol=1e-6)
  assert got > 10.0  # only half the clients are below X: the estimate grows


def test_tff_adapter_imports_without_tff():
  from federated_amd import tff_adapter  # pylint: disable=g-import-not-at-top
  try:
    import tensorflow_federated  # noqa: F401  pylint: disable=g-import-not-at-top,unused-import
    pytest.skip("TFF present")
  except ImportError:
    pass
  with pytest.raises(ImportError, match="tensorflow_federated"):
    tff_adapter.as_tff_factory(quantize_encode.QuantizeEncodeFactory(0.5))


# quantize_utils_test.py:157-186 (host scalar schedules of the product package)
def test_product_schedules():
  assert [float(quantize_utils.linear_decay(2., 0., r, 4)) for r in range(4)] == [2., 1.5, 1., 0.5]
  assert [float(quantize_utils.step_decay(2., 0., r, 2)) for r in range(4)] == [2., 2., 1., 1.]
  np.testing.assert_allclose([quantize_utils.exponential_decay(2., 0., r, 1.) for r in range(4)],
                             [2., 2. * np.exp(-1.), 2. * np.exp(-2.), 2. * np.exp(-3.)], rtol=1e-6)


def test_schedule_state_update_is_host_side():
  f = quantize_encode.QuantizeEncodeFactory(2.0, schedule="step_decay", schedule_hparam=2,
                                            min_step_size=0.1)
  assert f._schedule_fn(np.float32(3.0)) == np.float32(1.0)


def test_to_type():
  t = tc.to_type((np.float32, (2, 4)))
  assert t.num_elements == 8 and t.is_tensor()
  s = tc.to_type([(np.float32, (2,)), (np.int32, (3,))])
  assert not s.is_tensor() and not tc.is_structure_of_floats(s)


def test_qsgd_create():
  from federated_amd.aggregators.comparison_methods import qsgd  # pylint: disable=g-import-not-at-top
  process = qsgd.QSGDFactory(7.0).create((np.float32, (3,)))
  assert process.initialize() == ()
  with pytest.raises(ValueError):  # qsgd_test.py:60-66
    qsgd.QSGDFactory(1.0).create((np.int32, (3,)))


def test_client_lambda_create_and_builder():
  from federated_amd.aggregators import quantize_encode_client_lambda as qecl  # pylint: disable=g-import-not-at-top
  process = qecl.QuantizeEncodeClientLambdaFactory(1.0, 1.0, [0.5, 1.0, 2.0]).create(
      (np.float32, (3,)))
  state = process.initialize()
  assert list(state.keys()) == ["step_size", "inner_state"] and state["step_size"] == 1.0
  with pytest.raises(ValueError, match="rounding_type"):
    qecl.QuantizeEncodeClientLambdaFactory(1.0, 1.0, [1.0], rounding_type="nearest")
  with pytest.raises(ValueError):
    qecl.QuantizeEncodeClientLambdaFactory(1.0, 1.0, [1.0]).create((np.int32, (3,)))
  with pytest.raises(ValueError, match="step_size"):  # builder.py:562-565
    builder.build_vote_step_size_aggregator(0.3)
  with pytest.raises(ValueError, match="rounding_type"):
    builder.build_vote_step_size_aggregator(0.5, rounding_type="x")
  agg = builder.build_vote_step_size_aggregator(0.5)
  inner = agg._inner  # pylint: disable=protected-access
  assert inner._lagrange_multiplier == 0.03430265272  # pylint: disable=protected-access
  opts = inner._step_size_options  # pylint: disable=protected-access
  assert len(opts) == 7 and abs(opts[3] - 0.5) < 1e-12


def test_vote_losses_and_ties():
  from federated_amd.aggregators import quantize_encode_client_lambda as qecl  # pylint: disable=g-import-not-at-top
  loss = qecl.vote_losses([[15, 9, 5]], [[0.0, 0.0, 3.0]], 3, 3, 1.0)
  np.testing.assert_allclose(loss, [[16 / 3, 16 / 3, 1 + 8 / 3]], rtol=1e-6)
  np.testing.assert_array_equal(qecl.votes_from_losses([[1.0, 1.0, 2.0]]), [[1, 0, 0]])  # first on ties


def test_drive_create_and_builders():
  from federated_amd.aggregators.comparison_methods import drive  # pylint: disable=g-import-not-at-top
  with pytest.raises(ValueError, match="scaling_factor"):  # drive.py:36-38
    drive.DRIVEFactory("biased")
  with pytest.raises(ValueError):
    drive.DRIVEFactory().create((np.int32, (3,)))
  assert drive.DRIVEFactory().create((np.float32, (3,))).initialize() == ()
  agg = builder.build_drive_aggregator()  # rotation defaults to hadamard (builder.py:272-273)
  assert isinstance(agg._inner, builder.HadamardTransformFactory)  # pylint: disable=protected-access
  from federated_amd.aggregators.comparison_methods import qsgd  # pylint: disable=g-import-not-at-top
  assert isinstance(builder.build_qsgd_aggregator(7.0)._inner, qsgd.QSGDFactory)  # pylint: disable=protected-access
  assert isinstance(builder.build_drive_aggregator(rotation="dft")._inner,  # pylint: disable=protected-access
                    builder.DiscreteFourierTransformFactory)
  with pytest.raises(ValueError):
    builder.build_one_bit_sgd_aggregator(rotation="fft")


def test_min_segments_bounds():
  """Tensors longer than one encoder row (2^26 - 1) are always segmented, into rows
  of at most that many elements; beyond FC_MAX_ELEMS (2^30 - 2^26): ValueError."""
  from federated_amd import _lib, codec  # pylint: disable=g-import-not-at-top
  assert codec.min_segments(_lib.MAX_ROW_ELEMS) == 1
  for P in (_lib.MAX_ROW_ELEMS + 1, (1 << 26) + 5, 100_000_000, _lib.MAX_ELEMS):
    k = codec.min_segments(P)
    assert 2 <= k <= 63 and P // k // 2048 * 2048 <= _lib.MAX_ROW_ELEMS
    assert P - k * (P // k // 2048 * 2048) <= _lib.MAX_ROW_ELEMS
    assert codec.auto_segments(1024, P) >= k and codec.auto_segments(2, P) >= k
  with pytest.raises(ValueError):
    codec.min_segments(_lib.MAX_ELEMS + 1)


def test_per_stream_workspaces_are_lru_bounded():
  """codec keeps one encoder workspace per stream, the least recently used dropped past
  _WS_STREAMS (a side stream's buffer is recorded on that stream, so dropping it is safe)."""
  from federated_amd import codec  # pylint: disable=g-import-not-at-top
  bufs = {}
  for k in range(codec._WS_STREAMS + 3):  # pylint: disable=protected-access
    assert codec._ws_slot(bufs, ("dev", k), None) is None  # pylint: disable=protected-access
    bufs[("dev", k)] = k
  codec._ws_slot(bufs, ("dev", 4), None)  # pylint: disable=protected-access
  assert len(bufs) <= codec._WS_STREAMS + 1  # pylint: disable=protected-access
  assert ("dev", 4) in bufs and list(bufs)[-1] == ("dev", 4)  # most recently used last
  assert ("dev", 0) not in bufs

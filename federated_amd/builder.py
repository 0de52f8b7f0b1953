"""Aggregator-factory surface of compressed_communication/builder.py, MI355X-backed.

``build_quantization_encode_aggregator`` is the drop-in point
(builder.py:453-525): same name, keyword arguments, defaults and ValueError
messages.  It wraps ``QuantizeEncodeFactory`` with ``configure_aggregator``
(builder.py:37-119) in the reference order: concat -> (weighted) mean ->
adaptive clipping -> adaptive zeroing.  TFF is not installed here, so those TFF
wrappers are restated (``WrappedAggregationFactory`` below):

* concat_factory: each client's list of tensors is flattened and concatenated
  (on device);
* MeanFactory (builder.py:100-101): value * weight, inner sum, / sum(weight)
  (divide_no_nan); UnweightedMeanFactory: / number of clients;
* clipping_factory with ``PrivateQuantileEstimationProcess.no_noise(
  initial_estimate=1.0, target_quantile=0.8, learning_rate=0.2)``
  (builder.py:104-109): scale = C * min(1 / ||x||_2, 1 / C) as
  ``tf.clip_by_global_norm``, geometric update C <- C * exp(-lr * (frac(||x||
  <= C) - q));
* zeroing_factory with ``no_noise(10.0, 0.98, log(10), multiplier=2,
  increment=1)`` (builder.py:110-117): a client whose max |x| exceeds
  2 * X + 1 is zeroed; same geometric update on X.

The clip scale and the client weight are fused into the HIP encoder as a
per-client pre-scale (``fc_quantize_encode`` prescale), so they cost no extra
HBM pass.  Parity of the wrappers with TFF is **unpinned** (TFF absent; no
fixture in the reference holds their outputs).
"""
import collections
import inspect
import math

import numpy as np
import torch

from federated_amd import _lib
from federated_amd import builder_configs
from federated_amd import codec
from federated_amd import tff_compat as tc
from federated_amd.aggregators import _values
from federated_amd.aggregators import quantize_encode
from federated_amd.aggregators import quantize_encode_client_lambda
from federated_amd.aggregators.comparison_methods import drive
from federated_amd.aggregators.comparison_methods import one_bit_sgd
from federated_amd.aggregators.comparison_methods import qsgd

F32 = np.float32


def _accepts(fn, name):
  """Whether a process's next function takes keyword `name` (AggregationProcess.next
  forwards *args / **kwargs: the wrapped next_fn's signature decides)."""
  fn = getattr(getattr(fn, "__self__", None), "_next_fn", fn)
  try:
    return name in inspect.signature(fn).parameters
  except (TypeError, ValueError):
    return False


def call_inner(process, state, rows, seeds=None, prescale=None):
  """process.next(state, rows, ...) passing the optional seeds / fused pre-scales
  only to processes that take them; otherwise the pre-scales (x * clip) * weight
  are applied on the device first."""
  kw = {}
  if seeds is not None and _accepts(process.next, "seeds"):
    kw["seeds"] = seeds
  if prescale is not None:
    if _accepts(process.next, "prescale"):
      kw["prescale"] = prescale
    else:
      ps = np.asarray(prescale, np.float32).reshape(len(rows), 2)
      rows = [(r * float(ps[c, 0])) * float(ps[c, 1]) for c, r in enumerate(rows)]
  return process.next(state, rows, **kw)


class HadamardTransformFactory(tc.UnweightedAggregationFactory):
  """tff.aggregators.HadamardTransformFactory (builder.py:68-69) restated on MI355X.

  Each client's flattened value is zero-padded to n = 2^k and rotated by
  y = H D x / sqrt(n) (``fc_hadamard``: D = Rademacher signs of the round seed);
  the inner factory aggregates the rotated values; the server applies the
  inverse x = D H y / sqrt(n) to the aggregate and drops the padding.  The sign
  stream and seed schedule of TFF's implementation are not available here:
  parity unpinned (round-trip and linearity are tested).
  """

  def __init__(self, inner_agg_factory):
    self._inner = inner_agg_factory

  def create(self, value_type):
    value_type = tc.to_type(value_type)
    if not tc.is_structure_of_floats(value_type) or not value_type.is_tensor():
      raise ValueError("Expect value_type to be a float tensor, found %s." % (value_type,))
    shape = value_type.shape
    P = value_type.num_elements
    n = 1 << max(0, (P - 1).bit_length())
    inner = self._inner.create(tc.TensorType(np.float32, (n,)))

    def init_fn():
      return collections.OrderedDict(round_seed=np.zeros(2, np.int64), inner_state=inner.initialize())

    def next_fn(state, value, seeds=None, prescale=None, rotation_seed=None):
      rows, vshape, host = _values.to_device_rows(value, torch.float32)
      if vshape != shape:
        raise ValueError("client value shape %s != %s" % (vshape, shape))
      if prescale is not None:
        ps = np.asarray(prescale, np.float32).reshape(len(rows), 2)
        rows = [(r * float(ps[c, 0])) * float(ps[c, 1]) for c, r in enumerate(rows)]
      if rotation_seed is None:
        rotation_seed = quantize_encode.clock_seeds(1)[0]
      rotation_seed = np.asarray(rotation_seed, np.int64).reshape(2)
      padded = []
      for r in rows:
        t = torch.zeros(n, dtype=torch.float32, device=r.device)
        t[:P] = r
        padded.append(t)
      codec.hadamard_(padded, rotation_seed)
      out = call_inner(inner, state["inner_state"], padded, seeds=seeds)
      res = torch.as_tensor(out.result).cuda().reshape(-1).to(torch.float32).contiguous()
      codec.hadamard_([res], rotation_seed, inverse=True)
      new_state = collections.OrderedDict(round_seed=rotation_seed, inner_state=out.state)
      return tc.MeasuredProcessOutput(state=new_state,
                                      result=_values.finish(res[:P].contiguous(), shape, host),
                                      measurements=out.measurements)

    return tc.AggregationProcess(init_fn, next_fn)


class DiscreteFourierTransformFactory(tc.UnweightedAggregationFactory):
  """tff.aggregators.DiscreteFourierTransformFactory (builder.py:70-71) restated on MI355X.

  Each client's flattened value is zero-padded to an even length n, sign-flipped by
  the round's Rademacher signs D (``fc_sign_flip``) and rotated by the unitary DFT of
  its n / 2 complex numbers (first half real, second half imaginary parts; the
  hand-written FFT of fc_dft_rotate); the inner factory aggregates the rotated values; the server applies
  the inverse rotation and drops the padding.  TFF's own pairing of real and
  imaginary parts, sign stream and seed schedule are not available here: parity
  unpinned (round trip, norm preservation and linearity are tested).
  """

  def __init__(self, inner_agg_factory):
    self._inner = inner_agg_factory

  def create(self, value_type):
    value_type = tc.to_type(value_type)
    if not tc.is_structure_of_floats(value_type) or not value_type.is_tensor():
      raise ValueError("Expect value_type to be a float tensor, found %s." % (value_type,))
    shape = value_type.shape
    P = value_type.num_elements
    n = P + (P % 2)
    inner = self._inner.create(tc.TensorType(np.float32, (n,)))

    def init_fn():
      return collections.OrderedDict(round_seed=np.zeros(2, np.int64), inner_state=inner.initialize())

    def next_fn(state, value, seeds=None, prescale=None, rotation_seed=None):
      rows, vshape, host = _values.to_device_rows(value, torch.float32)
      if vshape != shape:
        raise ValueError("client value shape %s != %s" % (vshape, shape))
      if prescale is not None:
        ps = np.asarray(prescale, np.float32).reshape(len(rows), 2)
        rows = [(r * float(ps[c, 0])) * float(ps[c, 1]) for c, r in enumerate(rows)]
      if rotation_seed is None:
        rotation_seed = quantize_encode.clock_seeds(1)[0]
      rotation_seed = np.asarray(rotation_seed, np.int64).reshape(2)
      padded = []
      for r in rows:
        t = torch.zeros(n, dtype=torch.float32, device=r.device)
        t[:P] = r
        padded.append(t)
      codec.dft_(padded, rotation_seed)
      out = call_inner(inner, state["inner_state"], padded, seeds=seeds)
      res = torch.as_tensor(out.result).cuda().reshape(-1).to(torch.float32).contiguous()
      codec.dft_([res], rotation_seed, inverse=True)
      new_state = collections.OrderedDict(round_seed=rotation_seed, inner_state=out.state)
      return tc.MeasuredProcessOutput(state=new_state,
                                      result=_values.finish(res[:P].contiguous(), shape, host),
                                      measurements=out.measurements)

    return tc.AggregationProcess(init_fn, next_fn)


class QuantileEstimate:
  """``PrivateQuantileEstimationProcess.no_noise`` (geometric update) restated.

  The process keeps a raw estimate X.  ``report()`` is the affine map
  multiplier * X + increment that TFF applies to the reported value only
  (``EstimationProcess.map``); the quantile query itself records, per client,
  whether the client's norm is <= the RAW estimate X (tensorflow_privacy
  ``QuantileEstimatorQuery``), and moves X geometrically:
  X <- X * exp(-lr * (frac_below - target_quantile)).  For zeroing (2X + 1,
  q = 0.98) X therefore tracks the 98th percentile of the client norms and the
  zeroing threshold sits at about twice it.
  """

  def __init__(self, initial_estimate, target_quantile, learning_rate, multiplier=1.0,
               increment=0.0):
    self.initial_estimate = F32(initial_estimate)
    self.target_quantile = F32(target_quantile)
    self.learning_rate = F32(learning_rate)
    self.multiplier = F32(multiplier)
    self.increment = F32(increment)

  def report(self, estimate):
    return F32(estimate * self.multiplier + self.increment)

  def update(self, estimate, norms):
    below = F32(np.mean((np.asarray(norms, np.float32) <= F32(estimate)).astype(np.float32)))
    return F32(estimate * np.exp(-self.learning_rate * (below - self.target_quantile)))


class WrappedAggregationFactory(tc.WeightedAggregationFactory):
  """concat -> mean -> clipping -> zeroing around an inner codec factory."""

  def __init__(self, inner, concatenate=True, weighted=True, clipping=True, zeroing=True):
    self._inner = inner
    self._concatenate = concatenate
    self._weighted = weighted
    self._clip = QuantileEstimate(1.0, 0.8, 0.2) if clipping else None
    self._zero = (QuantileEstimate(10.0, 0.98, math.log(10.0), multiplier=2.0, increment=1.0)
                  if zeroing else None)

  def create(self, value_type, weight_type=None):
    value_type = tc.to_type(value_type)
    parts = list(value_type) if isinstance(value_type, tc.StructType) else [value_type]
    if not self._concatenate and len(parts) != 1:
      raise NotImplementedError("concatenate=False over a structure is not supported")
    P = int(sum(t.num_elements for t in parts))
    inner = self._inner.create(tc.TensorType(np.float32, (P,)))
    wrap = self

    def init_fn():
      return collections.OrderedDict(
          zeroing_norm=wrap._zero.initial_estimate if wrap._zero else (),
          clipping_norm=wrap._clip.initial_estimate if wrap._clip else (),
          inner_state=inner.initialize())

    def flat(v):
      seq = v if isinstance(v, (list, tuple)) and len(parts) > 1 else [v]
      ts = [torch.as_tensor(np.asarray(x, np.float32) if not isinstance(x, torch.Tensor) else x)
            .cuda().reshape(-1).to(torch.float32) for x in seq]
      return torch.cat(ts) if len(ts) > 1 else ts[0].contiguous()

    def unflat(t):
      out, off = [], 0
      for ty in parts:
        n = ty.num_elements
        out.append(t[off:off + n].reshape(ty.shape).cpu().numpy())
        off += n
      return out if len(parts) > 1 else out[0]

    def next_fn(state, value, weight=None, seeds=None):
      rows = [flat(v) for v in value]
      C = len(rows)
      w = (np.asarray(weight, np.float32).reshape(C) if (wrap._weighted and weight is not None)
           else np.ones(C, np.float32))
      s0 = np.ones(C, np.float32)
      zero_norm = clip_norm = ()
      if wrap._zero or wrap._clip:
        # both wrapper norms from ONE read pass over the round's deltas
        l2, linf = codec.client_norms(rows, _lib.NORM_L2_LINF).cpu().numpy()
      if wrap._zero:
        zero_norm = wrap._zero.report(state["zeroing_norm"])
        keep = ~(linf > zero_norm)
        s0 = np.where(keep, s0, F32(0.0)).astype(np.float32)
      if wrap._clip:
        l2 = np.where(s0 == 0, F32(0.0), l2).astype(np.float32)  # zeroed clients have norm 0
        clip_norm = wrap._clip.report(state["clipping_norm"])
        with np.errstate(divide="ignore"):
          inv = np.where(l2 > 0, F32(1.0) / l2, np.float32(np.inf)).astype(np.float32)
        scale = (clip_norm * np.minimum(inv, F32(1.0) / clip_norm)).astype(np.float32)
        s0 = (s0 * scale).astype(np.float32)
      prescale = np.stack([s0, w], axis=1)
      out = call_inner(inner, state["inner_state"], rows, seeds=seeds, prescale=prescale)
      denom = F32(np.sum(w, dtype=np.float32)) if wrap._weighted else F32(C)
      res = torch.as_tensor(out.result).cuda().reshape(-1)
      # divide_no_nan: an IEEE float32 division by a device scalar (a Python-scalar
      # divisor would be turned into a multiply by its reciprocal)
      res = (res / torch.full((1,), float(denom), dtype=res.dtype, device=res.device)
             if denom != 0 else torch.zeros_like(res))
      new_state = collections.OrderedDict(
          zeroing_norm=(wrap._zero.update(state["zeroing_norm"], linf) if wrap._zero else ()),
          clipping_norm=(wrap._clip.update(state["clipping_norm"], l2) if wrap._clip else ()),
          inner_state=out.state)
      measurements = collections.OrderedDict(
          zeroing_norm=zero_norm, clipping_norm=clip_norm,
          mean_value=out.measurements)
      return tc.MeasuredProcessOutput(state=new_state, result=unflat(res),
                                      measurements=measurements)

    return tc.AggregationProcess(init_fn, next_fn)


def configure_aggregator(factory,
                         rotation: str = "identity",
                         concatenate: bool = True,
                         zeroing: bool = True,
                         clipping: bool = True,
                         weighted: bool = True,
                         group_layers: bool = False,
                         task: str = ""):
  """builder.py:37-119 (see module docstring for what is restated)."""
  del task
  if rotation == "hadamard":
    factory = HadamardTransformFactory(factory)
  elif rotation == "dft":
    factory = DiscreteFourierTransformFactory(factory)
  elif rotation != "identity":
    raise ValueError(
        "Provided `rotation` must be one of 'dft', 'hadamard' or 'identity'.")
  if group_layers:
    raise NotImplementedError("group_layers is out of scope (SURVEY.md 2a, group.py)")
  return WrappedAggregationFactory(factory, concatenate=concatenate, weighted=weighted,
                                   clipping=clipping, zeroing=zeroing)


def build_quantization_encode_aggregator(
    step_size: float = 0.5,
    rounding_type: str = "uniform",
    normalization_type: str = "constant",
    step_size_sched: str = "fixed",
    step_size_sched_hparam: float = 0.,
    min_step_size: float = 0.01,
    rotation: str = "identity",
    concatenate: bool = True,
    zeroing: bool = True,
    clipping: bool = True,
    weighted: bool = True):
  """Creates an aggregation factory for quantization and entropy coding."""
  if rounding_type not in ["uniform", "stochastic", "dithered"]:
    raise ValueError("Expected `rounding_type` to be one one of [\"uniform\", "
                     f"\"stochastic\", \"dithered\"], found {rounding_type}.")

  if normalization_type not in [
      "constant", "mean_magnitude", "max_magnitude", "dimensionless_norm"
  ]:
    raise ValueError(
        "Expected `normalization_type` to be one one of [\"constant\", "
        "\"mean_magnitude\", \"max_magnitude\", \"dimensionless_norm\"], found "
        f"{normalization_type}.")

  if step_size_sched not in [
      "fixed", "linear_decay", "exponential_decay", "step_decay"
  ]:
    raise ValueError(
        "Expected `step_size_sched` to be one one of [\"fixed\", "
        "\"linear_decay\", \"exponential_decay\", \"step_decay\"], found "
        f"{step_size_sched}.")

  factory = quantize_encode.QuantizeEncodeFactory(step_size, rounding_type,
                                                  normalization_type,
                                                  step_size_sched,
                                                  step_size_sched_hparam,
                                                  min_step_size)

  return configure_aggregator(factory, rotation, concatenate, zeroing, clipping,
                              weighted)


def build_vote_step_size_aggregator(
    step_size: float,
    rounding_type: str = "uniform",
    sampling_width: float = 1.15,
    rotation: str = "identity",
    concatenate: bool = True,
    zeroing: bool = True,
    clipping: bool = True,
    weighted: bool = True):
  """Creates an aggregation factory for client voting experiments (builder.py:528-579)."""
  if step_size not in builder_configs.LAGRANGE_MULTIPLIER_VALUES.keys():
    raise ValueError(
        "Expected `step_size` to be one one of [0.05, 0.1, 0.25, 0.5, 1.0, "
        f"2.0, 2.5, 3.75, 5.0, 7.5, 10.0], found {step_size}.")
  if rounding_type not in ["uniform", "stochastic", "dithered"]:
    raise ValueError("Expected `rounding_type` to be one one of [\"uniform\", "
                     f"\"stochastic\", \"dithered\"], found {rounding_type}.")

  lagrange_multiplier = builder_configs.LAGRANGE_MULTIPLIER_VALUES[step_size]
  step_size_options = [
      step_size * scale for scale in sampling_width**np.linspace(-3, 3, 7)
  ]
  factory = quantize_encode_client_lambda.QuantizeEncodeClientLambdaFactory(
      lagrange_multiplier, step_size, step_size_options, rounding_type)

  return configure_aggregator(factory, rotation, concatenate, zeroing, clipping,
                              weighted)


def build_drive_aggregator(
    rotation: str = "hadamard",
    concatenate: bool = True,
    zeroing: bool = True,
    clipping: bool = True,
    weighted: bool = True):
  """Creates an aggregation factory for comparing to DRIVE (builder.py:272-298)."""
  factory = drive.DRIVEFactory()
  return configure_aggregator(factory, rotation, concatenate, zeroing, clipping,
                              weighted)


def build_one_bit_sgd_aggregator(
    rotation: str = "identity",
    concatenate: bool = True,
    zeroing: bool = True,
    clipping: bool = True,
    weighted: bool = True):
  """Creates an aggregation factory for comparing to 1-bit SGD (builder.py:301-327)."""
  factory = one_bit_sgd.OneBitSGDFactory()
  return configure_aggregator(factory, rotation, concatenate, zeroing, clipping,
                              weighted)


def build_qsgd_aggregator(
    num_steps: float,
    rotation: str = "identity",
    concatenate: bool = True,
    zeroing: bool = True,
    clipping: bool = True,
    weighted: bool = True):
  """Creates an aggregation factory for comparing to QSGD (builder.py:330-358)."""
  factory = qsgd.QSGDFactory(num_steps=num_steps)
  return configure_aggregator(factory, rotation, concatenate, zeroing, clipping,
                              weighted)

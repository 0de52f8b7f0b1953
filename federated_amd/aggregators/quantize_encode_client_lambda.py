"""Client step-size vote + quantise + encode aggregator on MI355X.

Mirrors ``compressed_communication/aggregators/quantize_encode_client_lambda.py``
(``QuantizeEncodeClientLambdaFactory``, :28-184): same constructor arguments and
ValueError messages; state ``OrderedDict(step_size=f32, inner_state=())``;
measurements ``OrderedDict(step_size, step_size_options,
step_size_vote_counts)``.

What runs where (one round, :146-182):
  * client ``quantize`` with the broadcast step (:97-103) + run-length gamma
    encode: ONE fused HIP launch (``fc_quantize_encode``); server decode + int32
    sum + dequantise (with the dithered noise sum): ONE launch, as in
    ``QuantizeEncodeFactory``;
  * client ``vote_step_size`` (:105-130): for every step option the client
    quantises, measures D = sum (x - deq)^2 / P and R = bitstring bits / P and
    votes for argmin D + lambda R.  The reference runs a full TFC encode per
    option to learn R; here one length-only launch (``fc_vote_lengths``)
    computes every option's exact code length and distortion, drawing the TF
    random stream once per element for all options;
  * the argmin, vote count and next step (:161-166): host scalar math.

Seeds: as in ``QuantizeEncodeFactory``, ``next`` takes optional ``seeds`` (the
quantise draw) and ``vote_seeds`` (the vote's draw; the reference draws both
from ``tf.timestamp()`` at different moments).
"""
import collections

import numpy as np
import torch

from federated_amd import _lib
from federated_amd import codec
from federated_amd import tff_compat as tc
from federated_amd.aggregators import _values
from federated_amd.aggregators.quantize_encode import clock_seeds

F32 = np.float32
_ROUNDING = {"uniform": _lib.UNIFORM, "stochastic": _lib.STOCHASTIC, "dithered": _lib.DITHERED}


def vote_losses(bits, dist, P, options_count, lagrange_multiplier):
  """quantize_encode_client_lambda.py:118-127 from per-option code bits and sum of
  squared errors: loss = D + lambda * R, float32 as in the reference."""
  size = F32(P)
  distortion = (np.asarray(dist, np.float64).astype(np.float32) / size).astype(np.float32)
  nbytes = (np.asarray(bits, np.int64) + 7) // 8
  rate = ((8.0 * nbytes.astype(np.float64)).astype(np.float32) / size).astype(np.float32)
  loss = (distortion + F32(lagrange_multiplier) * rate).astype(np.float32)
  assert loss.shape[-1] == options_count
  return loss


def votes_from_losses(loss):
  """tf.one_hot(tf.argmin(objective)) per client (first index on ties)."""
  loss = np.atleast_2d(loss)
  onehot = np.zeros(loss.shape, np.int32)
  onehot[np.arange(loss.shape[0]), np.argmin(loss, axis=1)] = 1
  return onehot


class QuantizeEncodeClientLambdaFactory(tc.UnweightedAggregationFactory):
  r"""Aggregator that quantizes and encodes input tensor elements over training.

  Every round, each client additionally quantizes according to step sizes in
  `step_size_options` and reports the step size within those options that
  minimizes `D + \lambda * R` for the given `lambda`; the `step_size` moves to
  the option with the most votes.
  """

  def __init__(self, lagrange_multiplier, step_size, step_size_options,
               rounding_type="uniform"):
    self._lagrange_multiplier = lagrange_multiplier
    self._step_size = step_size
    self._step_size_options = step_size_options
    if rounding_type not in _ROUNDING:
      raise ValueError("Expected `rounding_type` to be one one of "
                       "[\"uniform\", \"stochastic\", \"dithered\"], found "
                       f"{rounding_type}.")
    self._rounding_type = rounding_type
    self._mode = _ROUNDING[rounding_type]

  def create(self, value_type):
    value_type = tc.to_type(value_type)
    if not tc.is_structure_of_floats(value_type) or not value_type.is_tensor():
      raise ValueError("Expect value_type to be a float tensor, "
                       f"found {value_type}.")
    shape = value_type.shape
    P = value_type.num_elements
    factory = self
    options = np.asarray(self._step_size_options, np.float32)

    def init_fn():
      return collections.OrderedDict(step_size=F32(factory._step_size), inner_state=())

    def next_fn(state, value, seeds=None, vote_seeds=None, prescale=None):
      rows, vshape, host = _values.to_device_rows(value, torch.float32)
      if vshape != shape:
        raise ValueError("client value shape %s != %s" % (vshape, shape))
      C = len(rows)
      if prescale is not None:  # TFF wrapper scales (builder.configure_aggregator): (x * clip) * weight
        ps = np.asarray(prescale, np.float32).reshape(C, 2)
        rows = [(r * float(ps[c, 0])) * float(ps[c, 1]) for c, r in enumerate(rows)]
      step_size = F32(state["step_size"])
      seeds = clock_seeds(C) if seeds is None else np.asarray(seeds, np.int64).reshape(C, 2)
      vote_seeds = seeds if vote_seeds is None else np.asarray(vote_seeds, np.int64).reshape(C, 2)
      seeds_dev = torch.as_tensor(seeds).cuda()
      # quantize (:97-103) + inner EliasGammaEncodedSum (:157) + dequantize (:158-159)
      batch = codec.quantize_encode_checked(rows, step_size, seeds_dev, factory._mode)
      noise_sum = codec.noise_sum(seeds_dev, P, rows[0].device) if factory._mode == _lib.DITHERED else None
      out = torch.empty(P, dtype=torch.float32, device=rows[0].device)
      _, out, err = codec.decode_accumulate(batch, want_sum=False, out=out, step=float(step_size),
                                            noise_sum=noise_sum)
      # vote_step_size (:105-130) for every client, then the vote count (:161-166)
      bits, dist = codec.vote_lengths(rows, options, vote_seeds, factory._mode)
      if int(err.item()):
        raise RuntimeError("malformed run-length gamma code")
      loss = vote_losses(bits.cpu().numpy(), dist.cpu().numpy(), P, len(options),
                         factory._lagrange_multiplier)
      counts = votes_from_losses(loss).sum(axis=0).astype(np.int32)
      next_step = F32(options[int(np.argmax(counts))])
      next_state = collections.OrderedDict(step_size=next_step, inner_state=state["inner_state"])
      measurements = collections.OrderedDict(
          step_size=step_size,
          step_size_options=list(factory._step_size_options),
          step_size_vote_counts=counts)
      return tc.MeasuredProcessOutput(state=next_state, result=_values.finish(out, shape, host),
                                      measurements=measurements)

    return tc.AggregationProcess(init_fn, next_fn)

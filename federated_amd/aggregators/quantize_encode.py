"""Quantise + run-length-gamma encode aggregator on MI355X (the default trainer codec).

Mirrors ``compressed_communication/aggregators/quantize_encode.py``
(``QuantizeEncodeFactory``, :27-213): same constructor arguments, defaults and
ValueError messages; ``create(value_type)`` requires a single float tensor;
the process state is ``OrderedDict(round_num=f32, step_size=f32,
inner_state=())`` and ``next`` returns ``MeasuredProcessOutput(state, result,
measurements=OrderedDict(avg_bitrate=f64, avg_distortion=f32,
avg_sparsity=f32, step_size=f32))``.

What runs where (one round, :173-211):
  * client ``quantize`` (:139-156) for every client of the round and
    ``tfc.run_length_gamma_encode`` (elias_gamma_encode.py:97-99): ONE fused HIP
    launch (``fc_quantize_encode``) over the whole batch;
  * server decode + int32 sum (elias_gamma_encode.py:63-88) and the server
    ``dequantize`` (:169-171, 189-190): ONE HIP launch (``fc_decode_accumulate``);
  * dithered ``noise_sum`` (:183): ``fc_noise_sum`` regenerates every client's
    noise from its seed in client order;
  * schedules and measurements: host scalar float32/float64 math.

Seeds: the reference seeds each client with ``tf.timestamp()*1e6`` (:141-144),
which is not reproducible; here ``next`` takes an optional ``seeds`` int64
[C, 2] argument and otherwise derives distinct seeds from the clock.
"""
import collections
import time

import numpy as np
import torch

from federated_amd import _lib
from federated_amd import codec
from federated_amd import distributed
from federated_amd import tff_compat as tc
from federated_amd.aggregators import _values
from federated_amd.aggregators.utils import quantize_utils

F32 = np.float32

_ROUNDING = {"uniform": _lib.UNIFORM, "stochastic": _lib.STOCHASTIC, "dithered": _lib.DITHERED}
_NORMS = {"mean_magnitude": _lib.NORM_MEAN_MAGNITUDE, "max_magnitude": _lib.NORM_MAX_MAGNITUDE,
          "dimensionless_norm": _lib.NORM_DIMENSIONLESS}


def clock_seeds(n, base=None):
  """``tf.cast(tf.stack([tf.timestamp()*1e6]*2), tf.int64)`` per client, made distinct
  (client i gets base + i; ``base`` defaults to this process's clock)."""
  base = int(time.time() * 1e6) if base is None else int(base)
  return np.array([[base + i, base + i] for i in range(n)], dtype=np.int64).reshape(n, 2)


class QuantizeEncodeFactory(tc.UnweightedAggregationFactory):
  """Aggregator that quantizes and encodes input tensor elements over training."""

  def __init__(self,
               initial_step_size,
               rounding_type="uniform",
               normalization_type="constant",
               schedule="fixed",
               schedule_hparam=None,
               min_step_size=0.01):
    self._initial_step_size = initial_step_size
    self._step_size = initial_step_size
    self._min_step_size = min_step_size

    if normalization_type == "constant":
      self._norm_kind = None
    elif normalization_type in _NORMS:
      self._norm_kind = _NORMS[normalization_type]
    else:
      raise ValueError("Expected `normalization_type` to be one one of "
                       "[\"constant\", \"mean_magnitude\", \"max_magnitude\", "
                       f"\"dimensionless_norm\"], found {normalization_type}.")

    if rounding_type not in _ROUNDING:
      raise ValueError("Expected `rounding_type` to be one one of "
                       "[\"uniform\", \"stochastic\", \"dithered\"], found "
                       f"{rounding_type}.")
    self._rounding_type = rounding_type
    self._mode = _ROUNDING[rounding_type]

    if schedule == "fixed":
      self._schedule_fn = lambda _: F32(self._step_size)
    elif schedule == "linear_decay":
      self._schedule_fn = lambda round_num: quantize_utils.linear_decay(
          initial_step_size, min_step_size, round_num, total_rounds=schedule_hparam)
    elif schedule == "exponential_decay":
      self._schedule_fn = lambda round_num: quantize_utils.exponential_decay(
          initial_step_size, min_step_size, round_num, exp=schedule_hparam)
    elif schedule == "step_decay":
      self._schedule_fn = lambda round_num: quantize_utils.step_decay(
          initial_step_size, min_step_size, round_num, freq=schedule_hparam)
    else:
      raise ValueError("Expected `schedule` to be one one of [\"fixed\", "
                       "\"linear_decay\", \"exponential_decay\", "
                       f"\"step_decay\"], found {schedule}.")

  def create(self, value_type):
    value_type = tc.to_type(value_type)
    if not tc.is_structure_of_floats(value_type) or not value_type.is_tensor():
      raise ValueError("Expect value_type to be a float tensor, "
                       f"found {value_type}.")
    shape = value_type.shape
    P = value_type.num_elements
    factory = self

    def init_fn():
      return collections.OrderedDict(
          round_num=F32(0.0),
          step_size=F32(factory._step_size),
          inner_state=())

    # host-side process memory (not TFF state): the previous round's code sizes
    # size this round's stream capacities (codec.CapacityHint)
    cap_hint = codec.CapacityHint()

    def next_fn(state, value, seeds=None, prescale=None, sharded=False, group=None):
      """``sharded``: this process holds one rank's block of the round's clients
      (``value``, ``seeds`` and ``prescale`` are that block's, possibly empty);
      the int32 sums and the measurements are reduced over ``group`` (default:
      the torch.distributed world; distributed.aggregate_round) and every rank
      returns the round's global result.  The state is replicated: every rank
      steps it the same way."""
      multi = bool(sharded) and distributed.is_multi(group)
      # multi: one small all-reduce before the round's collectives -- a rank-local
      # error is raised on every rank, and clock seeds come from ONE base (rank 0's)
      # offset by the global client index, so no two clients of the round share a stream
      rows, host, lo, base = _values.sharded_rows(value, shape, sharded, multi, group)
      C = len(rows)
      step_size = F32(state["step_size"])
      if seeds is None:
        seeds = clock_seeds(C) if base is None else clock_seeds(C, base=base + lo)
      seeds = torch.as_tensor(np.asarray(seeds, np.int64).reshape(C, 2)).cuda()
      if prescale is not None:  # fused TFF wrapper scales (builder.configure_aggregator)
        prescale = torch.as_tensor(np.asarray(prescale, np.float32).reshape(C, 2)).cuda()
      # normalize_fn sees the value behind the clipping / mean wrappers (:145): the
      # norm of the pre-scaled elements, as the encoder quantises them
      norms = (codec.client_norms(rows, factory._norm_kind, prescale=prescale)
               if factory._norm_kind and C else None)
      # encode (quantize :139-156 + tfc encode), decode + int32 sum, dequantise with
      # the un-normalised state step (:189-190), measurements (:150-155, 184-185;
      # elias_gamma_encode.py:100-108)
      rnd = distributed.aggregate_round(rows, step_size, seeds, factory._mode, group=group, prescale=prescale,
                                        norms=norms, caps=cap_hint.caps(P, C), P=P,
                                        multi=multi)
      if rnd.batch is not None:
        cap_hint.update(rnd.batch)
      next_round = F32(state["round_num"] + F32(1.0))
      next_state = collections.OrderedDict(
          round_num=next_round,
          step_size=F32(factory._schedule_fn(next_round)),
          inner_state=state["inner_state"])
      measurements = collections.OrderedDict(rnd.measurements)
      measurements["step_size"] = step_size
      return tc.MeasuredProcessOutput(state=next_state,
                                      result=_values.finish(rnd.result, shape, host),
                                      measurements=measurements)

    return tc.AggregationProcess(init_fn, next_fn)

"""Stochastic quantisation of a structure of tensors on MI355X.

Mirrors ``compressed_communication/aggregators/stochastic_quantize.py``
(``StochasticQuantizeFactory``, :22-90): every float tensor of each client's
structure is stochastically quantised with ``scale_factor`` (one seed per
client shared by its tensors, :57-63), the int32 structure goes to the inner
aggregation process, and the inner result is dequantised (:72-76).  State and
measurements pass through from the inner process (:80-88).
"""
import numpy as np
import torch

from federated_amd import _lib
from federated_amd import codec
from federated_amd import tff_compat as tc
from federated_amd.aggregators import quantize_encode


def _as_list(t):
  return list(t) if isinstance(t, tc.StructType) else None


class StochasticQuantizeFactory(tc.UnweightedAggregationFactory):
  """Aggregator that stochastically quantizes input tensor elements."""

  def __init__(self, scale_factor, inner_agg_factory):
    self.scale_factor = scale_factor
    self.inner_agg_factory = inner_agg_factory

  def create(self, value_type):
    value_type = tc.to_type(value_type)
    if not tc.is_structure_of_floats(value_type):
      raise ValueError("Expect value_type to be structure of "
                       f"float tensors, found {value_type}.")
    members = _as_list(value_type)
    types = members if members is not None else [value_type]
    qtypes = [tc.TensorType(np.int32, t.shape) for t in types]
    inner = self.inner_agg_factory.create(
        tc.StructType(qtypes) if members is not None else qtypes[0])
    scale = float(self.scale_factor)

    def quantize(value, seed):
      parts = value if members is not None else [value]
      out = []
      for t, v in zip(types, parts):
        x = torch.as_tensor(np.asarray(v, np.float32) if not isinstance(v, torch.Tensor) else v)
        q, _ = codec.quantize(x.cuda().reshape(-1), scale, seed, _lib.STOCHASTIC)
        out.append(q.reshape(t.shape))
      return out if members is not None else out[0]

    def dequantize(value):
      parts = value if members is not None else [value]
      out = []
      for t, v in zip(types, parts):
        v = torch.as_tensor(v).cuda().reshape(-1).to(torch.int32)
        out.append(codec.dequantize(v, scale).reshape(t.shape).cpu().numpy())
      return out if members is not None else out[0]

    def init_fn():
      return inner.initialize()

    def next_fn(state, value, seeds=None):
      if seeds is None:
        seeds = quantize_encode.clock_seeds(len(value))
      quantized = [quantize(v, seeds[i]) for i, v in enumerate(value)]
      inner_out = inner.next(state, quantized)
      return tc.MeasuredProcessOutput(state=inner_out.state,
                                      result=dequantize(inner_out.result),
                                      measurements=inner_out.measurements)

    return tc.AggregationProcess(init_fn, next_fn)

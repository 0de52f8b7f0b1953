"""One-bit SGD codec on MI355X (BASELINE config 5).

Mirrors ``compressed_communication/aggregators/comparison_methods/one_bit_sgd.py``
(``OneBitSGDFactory``, :21-130): per client ``mask = x >= threshold``, the two
masked means, distortion ``sum (x - decode)^2 / P`` and bitrate ``(P + 64) / P``
(:56-81); the server decodes every client and sums in float32 in client order
(:87-112).  Masks are kept bit-packed in HBM (1 bit per element), which is the
wire format the bitrate already assumes.
"""
import collections

import numpy as np
import torch

from federated_amd import codec
from federated_amd import tff_compat as tc
from federated_amd.aggregators import _values

F32 = np.float32


class OneBitSGDFactory(tc.UnweightedAggregationFactory):
  """Aggregator that quantizes to 1 bit."""

  def __init__(self, threshold=0.):
    self._threshold = threshold

  def create(self, value_type):
    value_type = tc.to_type(value_type)
    if not tc.is_structure_of_floats(value_type) or not value_type.is_tensor():
      raise ValueError("Expect value_type to be a float tensor, "
                       f"found {value_type}.")
    shape = value_type.shape
    P = value_type.num_elements

    def next_fn(state, value):
      rows, vshape, host = _values.to_device_rows(value, torch.float32)
      if vshape != shape:
        raise ValueError("client value shape %s != %s" % (vshape, shape))
      masks, means, dist = codec.onebit_encode(rows, self._threshold)
      out = codec.onebit_decode_sum(masks, means, len(rows), P)
      size = F32(P)
      bitrate = F32((size + F32(64.0)) / size)
      distortion = (dist.cpu().numpy().astype(np.float32) / size).astype(np.float32)
      return tc.MeasuredProcessOutput(
          state=state,
          result=_values.finish(out, shape, host),
          measurements=collections.OrderedDict(
              avg_bitrate=bitrate,
              avg_distortion=F32(np.mean(distortion, dtype=np.float32))))

    return tc.AggregationProcess(lambda: (), next_fn)

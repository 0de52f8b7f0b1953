"""DRIVE codec on MI355X.

Mirrors ``compressed_communication/aggregators/comparison_methods/drive.py``
(``DRIVEFactory``, :21-124): per client the sign mask (1 bit per element) and
one float scale -- ``||x||_2^2 / ||x||_1`` ("unbiased", divide_no_nan) or
``||x||_1 / P`` ("min_distortion") -- bitrate ``(P + 32) / P``, distortion
``sum (x - decode)^2 / P`` (:58-76); the server decodes ``+-scale`` and sums in
float32 in client order (:80-103).  Like the reference it assumes the random
rotation was applied already (builder ``rotation="hadamard"``).

What runs where: ``fc_drive_encode`` (one workgroup per client: masks + float64
norms, then the distortion pass) and ``fc_onebit_decode_sum`` (decode + client-
order float32 sum).  The norms are float64 sums rounded to float32 (TF reduces
in float32 in an unspecified order): the scale matches within an ulp.
"""
import collections

import numpy as np
import torch

from federated_amd import codec
from federated_amd import tff_compat as tc
from federated_amd.aggregators import _values

F32 = np.float32


class DRIVEFactory(tc.UnweightedAggregationFactory):
  """Aggregator that implements DRIVE algorithm."""

  def __init__(self, scaling_factor="unbiased"):
    if scaling_factor not in ["unbiased", "min_distortion"]:
      raise ValueError("Expect scaling_factor to be one of [\"unbiased\", "
                       f"\"min_distortion\"], found {scaling_factor}.")
    self._scaling_factor = scaling_factor

  def create(self, value_type):
    value_type = tc.to_type(value_type)
    if not tc.is_structure_of_floats(value_type) or not value_type.is_tensor():
      raise ValueError("Expect value_type to be a float tensor, "
                       f"found {value_type}.")
    shape = value_type.shape
    P = value_type.num_elements
    min_distortion = self._scaling_factor == "min_distortion"

    def next_fn(state, value):
      rows, vshape, host = _values.to_device_rows(value, torch.float32)
      if vshape != shape:
        raise ValueError("client value shape %s != %s" % (vshape, shape))
      masks, means, dist = codec.drive_encode(rows, min_distortion)
      out = codec.onebit_decode_sum(masks, means, len(rows), P)
      size = F32(P)
      bitrate = F32((size + F32(32.0)) / size)                                      # :66
      distortion = (dist.cpu().numpy().astype(np.float32) / size).astype(np.float32)  # :69-70
      return tc.MeasuredProcessOutput(
          state=state,
          result=_values.finish(out, shape, host),
          measurements=collections.OrderedDict(
              avg_bitrate=bitrate,
              avg_distortion=F32(np.mean(distortion, dtype=np.float32))))

    return tc.AggregationProcess(lambda: (), next_fn)

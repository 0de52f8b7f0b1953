"""Run-length Elias-gamma encoded integer sum on MI355X.

Mirrors ``compressed_communication/aggregators/elias_gamma_encode.py``:
``get_bitstring_length`` (:22-24) and ``EliasGammaEncodedSumFactory`` (:27-116).
Per client the int32 tensor is coded by the HIP encoder (tfc.run_length_gamma_encode
semantics, :97-99); the server decodes every code and sums in int32 (the
federated_aggregate accumulate/merge of :63-88) in one HIP decode pass.
"""
import collections

import numpy as np
import torch

from federated_amd import codec
from federated_amd import tff_compat as tc
from federated_amd.aggregators import _values


def get_bitstring_length(value):
  """Size in bits of an encoded value (bytes or an EncodedBatch row count)."""
  return np.float64(8.0 * len(value))


class EliasGammaEncodedSumFactory(tc.UnweightedAggregationFactory):
  """Aggregator that encodes input integer tensor elements (see module doc)."""

  def create(self, value_type):
    value_type = tc.to_type(value_type)
    if not tc.is_structure_of_integers(value_type) or not value_type.is_tensor():
      raise ValueError("Expect value_type to be an integer tensor, "
                       f"found {value_type}.")
    shape = value_type.shape

    def init_fn():
      return ()

    def next_fn(state, value):
      rows, vshape, host = _values.to_device_rows(value, torch.int32)
      if vshape != shape:
        raise ValueError("client value shape %s != %s" % (vshape, shape))
      batch = codec.rlgamma_encode(rows)
      nbytes = batch.nbytes().astype(np.float64)
      avg_bitstring_length = np.mean(8.0 * nbytes)
      num_elements = np.float64(value_type.num_elements)
      avg_bitrate = (np.float64(avg_bitstring_length / num_elements)
                     if num_elements else np.float64(0.0))
      s, _, err = codec.decode_accumulate(batch)
      if int(err.item()):
        raise RuntimeError("malformed run-length gamma code")
      return tc.MeasuredProcessOutput(
          state=state,
          result=_values.finish(s, shape, host),
          measurements=collections.OrderedDict(avg_bitrate=avg_bitrate))

    return tc.AggregationProcess(init_fn, next_fn)

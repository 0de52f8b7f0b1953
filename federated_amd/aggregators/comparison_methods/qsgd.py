"""QSGD codec on MI355X.

Mirrors ``compressed_communication/aggregators/comparison_methods/qsgd.py``
(``QSGDFactory``, :35-146):

* client ``quantize_encode`` (:62-79): norm = ||x||_2, step = norm / num_steps,
  stochastic quantisation with that step, client-side dequantisation for the
  distortion / sparsity measurements, ``tfc.run_length_gamma_encode`` of q,
  and the norm sent beside the code;
* server ``sum_encoded_value`` (:85-112): decode every client, dequantise with
  its own step, and sum in float32.

What runs where: the per-client L2 norms (``fc_client_norms``, float64
accumulation), then ONE fused HIP quantise + encode launch over the batch with
a per-client step, then ONE decode launch that dequantises each client with its
step and sums in float32 in client order (``fc_decode_accumulate_scaled``).  The per-client
step ``norm / num_steps`` is divided on the host in float32 (IEEE), so the
quantiser sees exactly the step TF would compute from the same norm.

Parity: q and the bitstream are bit-exact against the oracle given the norm;
the norm itself is TF's float32 reduction in an unspecified order (here a
correctly rounded float64 sum, as the oracle's).  The server sum adds the
clients in client order in float32 exactly as the reference's accumulate does
(the decoder writes each client group's q rows, ``k_sum_planes`` adds them in
order), so with the oracle's norm it is bit-exact and deterministic.
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


def get_bitstring_length(nbytes):
  """qsgd.py:27-32: 32 bits of norm + 8 * code bytes, float64."""
  return 32. + 8. * np.asarray(nbytes, dtype=np.float64)


class QSGDFactory(tc.UnweightedAggregationFactory):
  """Aggregator that implements QSGD.

  Expects `value_type` to be a `TensorType`.

  Paper: https://arxiv.org/abs/1610.02132
  """

  def __init__(self, num_steps):
    self._num_steps = num_steps

  def create(self, value_type):
    value_type = tc.to_type(value_type)
    if not tc.is_structure_of_floats(value_type) or not value_type.is_tensor():
      raise ValueError("Expect value_type to be a float tensor, "
                       f"found {value_type}.")
    shape = value_type.shape
    P = value_type.num_elements
    num_steps = F32(self._num_steps)

    def next_fn(state, value, seeds=None):
      rows, vshape, host = _values.to_device_rows(value, torch.float32)
      if vshape != shape:
        raise ValueError("client value shape %s != %s" % (vshape, shape))
      C = len(rows)
      if seeds is None:
        seeds = clock_seeds(C)
      seeds = torch.as_tensor(np.asarray(seeds, np.int64).reshape(C, 2)).cuda()
      norms = codec.client_norms(rows, _lib.NORM_L2).cpu().numpy().astype(np.float32)   # :66
      with np.errstate(divide="ignore", invalid="ignore"):
        steps = (norms / num_steps).astype(np.float32)                                  # :67
      steps_dev = torch.from_numpy(steps).cuda()
      # client step = steps[c] * 1.0 (exact); stochastic rounding (:68-69)
      batch = codec.quantize_encode_checked(rows, 1.0, seeds, _lib.STOCHASTIC, norms=steps_dev)
      # |q| <= num_steps + 1 whenever every client step is positive and finite (|x| <=
      # ||x||_2): the server's q rows can then be int8
      qmax = int(np.ceil(num_steps)) + 1
      if not (np.all(steps > 0) and np.all(np.isfinite(steps)) and qmax <= 127):
        qmax = None
      out, err = codec.decode_accumulate_scaled(batch, steps_dev, qmax=qmax)           # :85-112
      dist, nnz = codec.finalize(batch)
      if int(err.item()):
        raise RuntimeError("malformed run-length gamma code")
      size = F32(P)
      distortion = (dist.cpu().numpy().astype(np.float32) / size).astype(np.float32)   # :72-74
      nz = nnz.cpu().numpy().astype(np.float32)
      sparsity = ((size - nz) / size).astype(np.float32)                               # :75-77
      lengths = get_bitstring_length(batch.nbytes())                                    # :127
      avg_bitrate = np.float64(np.mean(lengths) / np.float64(P)) if P else np.float64(0.0)
      measurements = collections.OrderedDict(
          avg_bitrate=avg_bitrate,
          avg_distortion=F32(np.mean(distortion, dtype=np.float32)),
          avg_sparsity=F32(np.mean(sparsity, dtype=np.float32)))
      return tc.MeasuredProcessOutput(state=state, result=_values.finish(out, shape, host),
                                      measurements=measurements)

    return tc.AggregationProcess(lambda: (), next_fn)

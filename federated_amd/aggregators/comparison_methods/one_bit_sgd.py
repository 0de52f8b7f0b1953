"""One-bit SGD codec on MI355X (BASELINE config 5).

Mirrors ``compressed_communication/aggregators/comparison_methods/one_bit_sgd.py``
(``OneBitSGDFactory``, :21-130): per client ``mask = x >= threshold``, the two
masked means, distortion ``sum (x - decode)^2 / P`` and bitrate ``(P + 64) / P``
(:56-81); the server decodes every client and sums in float32 in client order
(:87-112).  Masks are kept bit-packed in HBM (1 bit per element), which is the
wire format the bitrate already assumes.
"""
from federated_amd import distributed
from federated_amd import tff_compat as tc
from federated_amd.aggregators import _values


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

    def next_fn(state, value, sharded=False, group=None, slabs=4):
      """``sharded``: this process holds one rank's block of the round's clients
      (possibly empty); the float32 partial sums are all-reduced over ``group``
      (config 5's 8-GPU split, distributed.onebit_round) and the distortion mean
      is global.  The multi-rank float association differs from one process's
      client-order sum: compare with a tolerance."""
      multi = bool(sharded) and distributed.is_multi(group)
      rows, host, _, _ = _values.sharded_rows(value, shape, sharded, multi, group)
      rnd = distributed.onebit_round(rows, self._threshold, group=group, P=P, slabs=slabs, multi=multi)
      return tc.MeasuredProcessOutput(
          state=state,
          result=_values.finish(rnd.result, shape, host),
          measurements=rnd.measurements)

    return tc.AggregationProcess(lambda: (), next_fn)

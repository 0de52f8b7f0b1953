"""Plain integer/float sum over clients (``tff.aggregators.SumFactory`` stand-in).

``add_measurements`` mirrors ``tff.aggregators.add_measurements(SumFactory(),
client_measurement_fn=tff.federated_sum)`` as used by
compressed_communication/aggregators/stochastic_quantize_test.py:36-37.
"""
import collections

import torch

from federated_amd import tff_compat as tc


def _sum(values):
  first = values[0]
  if isinstance(first, (list, tuple)):
    return [_sum([v[i] for v in values]) for i in range(len(first))]
  acc = torch.zeros_like(torch.as_tensor(first).cuda())
  for v in values:
    acc = acc + torch.as_tensor(v).cuda()
  return acc.cpu().numpy()


class SumFactory(tc.UnweightedAggregationFactory):

  def __init__(self, measure_sum=False):
    self._measure_sum = measure_sum

  def create(self, value_type):
    def next_fn(state, value):
      s = _sum(value)
      return tc.MeasuredProcessOutput(state=state, result=s,
                                      measurements=s if self._measure_sum else collections.OrderedDict())
    return tc.AggregationProcess(lambda: (), next_fn)


def add_sum_measurements():
  return SumFactory(measure_sum=True)

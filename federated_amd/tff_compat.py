"""Minimal stand-ins for the TFF template types the reference aggregators use.

TFF is not installed in this image, so the drop-in surface mirrors the
protocol, not the TFF classes: an aggregation factory has ``create(value_type)``
returning a process with ``initialize()`` and ``next(state, client_values)``,
and ``next`` returns a ``MeasuredProcessOutput(state, result, measurements)``
(``tff.templates.AggregationProcess`` / ``MeasuredProcessOutput`` as used at
compressed_communication/aggregators/quantize_encode.py:161-213).  When TFF is
present, ``federated_amd.tff_adapter`` (lazy import) wraps these into real TFF
computations (``quantize_encode_process`` / ``as_tff_factory``; untested here
because TFF is absent).
"""
import collections
from typing import Any, Callable, Sequence

import numpy as np

MeasuredProcessOutput = collections.namedtuple("MeasuredProcessOutput",
                                               ["state", "result", "measurements"])


class TensorType:
  """``tff.TensorType(dtype, shape)`` stand-in."""

  def __init__(self, dtype, shape=()):
    self.dtype = np.dtype(dtype)
    self.shape = tuple(int(s) for s in (shape if isinstance(shape, (tuple, list)) else (shape,)))

  def is_tensor(self):
    return True

  @property
  def num_elements(self):
    return int(np.prod(self.shape)) if self.shape else 1

  def __repr__(self):
    return "TensorType(%s, %s)" % (self.dtype.name, list(self.shape))

  def __eq__(self, other):
    return isinstance(other, TensorType) and (self.dtype, self.shape) == (other.dtype, other.shape)


class StructType(list):
  """A structure of TensorTypes (``tff.StructType`` stand-in)."""

  def is_tensor(self):
    return False


def to_type(spec):
  """``tff.to_type``: (dtype, shape) -> TensorType; list -> StructType."""
  if isinstance(spec, (TensorType, StructType)):
    return spec
  if isinstance(spec, tuple) and len(spec) == 2 and not isinstance(spec[0], tuple):
    dtype = spec[0]
    if hasattr(dtype, "as_numpy_dtype"):  # a tf.DType
      dtype = dtype.as_numpy_dtype
    return TensorType(dtype, spec[1])
  if isinstance(spec, (list, tuple)):
    return StructType([to_type(s) for s in spec])
  raise TypeError("cannot convert %r to a type" % (spec,))


def is_structure_of_floats(t):
  if isinstance(t, TensorType):
    return np.issubdtype(t.dtype, np.floating)
  return all(is_structure_of_floats(s) for s in t)


def is_structure_of_integers(t):
  if isinstance(t, TensorType):
    return np.issubdtype(t.dtype, np.integer)
  return all(is_structure_of_integers(s) for s in t)


class AggregationProcess:
  """``tff.templates.AggregationProcess(initialize_fn, next_fn)`` stand-in."""

  def __init__(self, initialize_fn: Callable[[], Any],
               next_fn: Callable[[Any, Sequence[Any]], MeasuredProcessOutput]):
    self._initialize_fn = initialize_fn
    self._next_fn = next_fn

  def initialize(self):
    return self._initialize_fn()

  def next(self, state, value, *args, **kwargs):
    return self._next_fn(state, value, *args, **kwargs)


class UnweightedAggregationFactory:
  """Marker base class (``tff.aggregators.UnweightedAggregationFactory``)."""

  def create(self, value_type):  # pragma: no cover - interface
    raise NotImplementedError


class WeightedAggregationFactory:
  """Marker base class (``tff.aggregators.WeightedAggregationFactory``)."""

  def create(self, value_type, weight_type):  # pragma: no cover - interface
    raise NotImplementedError

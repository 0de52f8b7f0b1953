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


class FileProgramStateManager:
  """``tff.program.FileProgramStateManager`` stand-in (the trainer's checkpoints:
  utils/training_utils.py:26-55, saved every ``rounds_per_checkpoint`` = 25 rounds by
  ``tff.simulation.run_training_process``, trainer.py:108, 345-354).

  ``save(program_state, version)`` writes one ``.npz`` per version under
  ``root_dir``: every leaf of the nested (Ordered)dict / list / tuple state flattened
  under its key path, with its dtype and shape kept (no pickles: ``np.load`` with
  ``allow_pickle=False`` restores it).  ``load(version, structure)`` rebuilds a state
  shaped like ``structure`` from the saved leaves; ``load_latest(structure)``
  returns ``(state, version)`` of the newest save, or ``(None, 0)``.
  """

  def __init__(self, root_dir, prefix="program_state_"):
    import os  # pylint: disable=g-import-not-at-top
    self._root = root_dir
    self._prefix = prefix
    os.makedirs(root_dir, exist_ok=True)

  def _path(self, version):
    import os  # pylint: disable=g-import-not-at-top
    return os.path.join(self._root, "%s%d.npz" % (self._prefix, int(version)))

  @staticmethod
  def _flatten(state, path, out):
    if isinstance(state, dict):
      for k, v in state.items():
        FileProgramStateManager._flatten(v, path + (str(k),), out)
    elif isinstance(state, (list, tuple)) and not isinstance(state, np.ndarray):
      if not state:
        out["/".join(path + ("<empty>",))] = np.zeros(0, np.int8)
      for i, v in enumerate(state):
        FileProgramStateManager._flatten(v, path + (str(i),), out)
    else:
      out["/".join(path)] = np.asarray(state)

  @staticmethod
  def _rebuild(structure, path, leaves):
    if isinstance(structure, dict):
      items = [(k, FileProgramStateManager._rebuild(v, path + (str(k),), leaves)) for k, v in structure.items()]
      return type(structure)(items)
    if isinstance(structure, (list, tuple)) and not isinstance(structure, np.ndarray):
      vals = [FileProgramStateManager._rebuild(v, path + (str(i),), leaves) for i, v in enumerate(structure)]
      return type(structure)(vals)
    a = leaves["/".join(path)]
    return a[()] if a.ndim == 0 else a

  def get_versions(self):
    import os  # pylint: disable=g-import-not-at-top
    vs = []
    for f in os.listdir(self._root):
      if f.startswith(self._prefix) and f.endswith(".npz"):
        vs.append(int(f[len(self._prefix):-4]))
    return sorted(vs) or None

  def save(self, program_state, version):
    import os  # pylint: disable=g-import-not-at-top
    leaves = {}
    self._flatten(program_state, (), leaves)
    tmp = self._path(version) + ".tmp.npz"
    np.savez(tmp, **leaves)
    os.replace(tmp, self._path(version))

  def load(self, version, structure):
    with np.load(self._path(version), allow_pickle=False) as z:
      leaves = {k: z[k] for k in z.files}
    return self._rebuild(structure, (), leaves)

  def load_latest(self, structure):
    vs = self.get_versions()
    if not vs:
      return None, 0
    return self.load(vs[-1], structure), vs[-1]

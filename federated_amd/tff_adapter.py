"""TFF adapter: the MI355X codec behind real ``tff.templates.AggregationProcess`` objects.

TensorFlow / TFF are NOT installed in this image, so this module imports them
lazily (first call) and cannot be exercised here; ``tests/test_api_cpu.py``
checks only that it imports without TFF and fails with a clear error.

The adapter keeps the reference's federated structure
(``aggregators/quantize_encode.py:173-213`` around
``aggregators/elias_gamma_encode.py:63-116``) and swaps what the TF ops
compute for the HIP codec, called through ``tf.numpy_function``:

* client ``quantize`` (quantize_encode.py:139-156) + ``tfc.run_length_gamma_encode``
  (elias_gamma_encode.py:98) -> one ``fc_quantize_encode`` launch for the client;
  the client step is ``normalize_fn(value) * step`` (quantize_encode.py:145; the
  norm from ``fc_client_norms``).  The client's message is the reference's: ONE
  ``tf.string``, the TFC byte string (elias_gamma_encode.py:97-109), so stock
  reference clients and these interoperate in either direction;
* server ``federated_aggregate`` accumulate (elias_gamma_encode.py:69-73) ->
  ``fc_build_index`` (the decoder index rebuilt on the device from the bare bytes,
  as ``tfc.run_length_gamma_decode(code, shape)`` needs nothing else) +
  ``fc_decode_accumulate`` of the client into the running int32 sum; merge
  (:75-77) is an int32 add;
* server ``dequantize`` (quantize_encode.py:169-171) -> ``fc_dequantize``.

TFF's executor maps clients one at a time, so this path encodes batches of
one; the batched path (``federated_amd.aggregators.quantize_encode``) encodes a
whole round's cohort in one launch and is what ``bench.py`` measures.
"""
import collections

import numpy as np


def _tf():
  try:
    import tensorflow as tf  # pylint: disable=g-import-not-at-top
    import tensorflow_federated as tff  # pylint: disable=g-import-not-at-top
  except ImportError as e:  # pragma: no cover - TFF absent in this image
    raise ImportError("federated_amd.tff_adapter needs tensorflow and tensorflow_federated; "
                      "use federated_amd.builder (TFF-free protocol stand-ins) without them") from e
  return tf, tff


def _encode_one(x, step, seed, mode, norm_kind=None):
  """numpy_function body: one client -> (code bytes, distortion, sparsity, noise).

  ``norm_kind``: the factory's normalisation (quantize_encode.py:145: the client
  step is ``normalize_fn(value) * step``), None for "constant"."""
  import torch  # pylint: disable=g-import-not-at-top
  from federated_amd import _lib  # pylint: disable=g-import-not-at-top
  from federated_amd import codec  # pylint: disable=g-import-not-at-top
  x = torch.from_numpy(np.ascontiguousarray(x, np.float32).reshape(-1)).cuda()
  P = x.numel()
  seeds = torch.as_tensor(np.asarray(seed, np.int64).reshape(1, 2))
  norms = codec.client_norms([x], norm_kind) if norm_kind else None
  batch = codec.quantize_encode_checked([x], float(step), seeds, int(mode), norms=norms)
  dist, nnz = codec.finalize(batch)
  code = batch.client_code(0)
  size = np.float32(P)
  distortion = np.float32(dist.cpu().numpy()[0] / size)
  sparsity = np.float32((size - np.float32(nnz.cpu().numpy()[0])) / size)
  if int(mode) == _lib.DITHERED:
    noise = codec.noise_sum(seeds, P, x.device).cpu().numpy()
  else:
    noise = np.zeros(P, np.float32)
  return code, distortion, sparsity, noise


def _decode_accumulate_one(acc, code):
  """numpy_function body: acc + tfc.run_length_gamma_decode(code, shape) (int32,
  wrapping) from the bare byte string: the index is rebuilt on the device."""
  import torch  # pylint: disable=g-import-not-at-top
  from federated_amd import codec  # pylint: disable=g-import-not-at-top
  acc = torch.from_numpy(np.ascontiguousarray(acc, np.int32).reshape(-1)).cuda()
  batch = codec.from_codes([bytes(code)], acc.numel(), device=acc.device)  # ValueError if malformed
  s, _, err = codec.decode_accumulate(batch, sum_in=acc)
  if int(err.item()):
    raise ValueError("malformed run-length gamma code")
  return s.cpu().numpy()


def quantize_encode_process(value_type, factory):
  """A ``tff.templates.AggregationProcess`` for ``factory`` (a
  federated_amd QuantizeEncodeFactory) over ``value_type`` (a tff.TensorType)."""
  tf, tff = _tf()
  shape = value_type.shape
  P = int(np.prod(shape)) if len(shape) else 1
  mode = factory._mode  # pylint: disable=protected-access
  norm_kind = factory._norm_kind  # pylint: disable=protected-access

  @tff.tf_computation(value_type, tf.float32)
  def quantize(value, step_size):
    seed = tf.cast(tf.stack([tf.timestamp() * 1e6, tf.timestamp() * 1e6]), dtype=tf.int64)
    code, distortion, sparsity, noise = tf.numpy_function(
        lambda x, s, sd: _encode_one(x, s, sd, mode, norm_kind), [value, step_size, seed],
        [tf.string, tf.float32, tf.float32, tf.float32])
    return tf.reshape(code, []), tf.reshape(noise, shape), distortion, sparsity

  @tff.tf_computation
  def zero():
    return tf.zeros(shape, tf.int32)

  @tff.tf_computation
  def accumulate(acc, code):
    out = tf.numpy_function(_decode_accumulate_one, [acc, code], tf.int32)
    return tf.reshape(out, shape)

  @tff.tf_computation
  def merge(a, b):
    return a + b

  @tff.tf_computation
  def report(a):
    return a

  @tff.tf_computation
  def bitstring_length(message):
    return tf.cast(8 * tf.strings.length(message), tf.float64)

  @tff.tf_computation(tff.TensorType(tf.int32, shape), tf.float32,
                      tff.TensorType(tf.float32, shape))
  def dequantize(value, step_size, noise_sum):
    return (tf.cast(value, tf.float32) + noise_sum) * step_size

  @tff.federated_computation()
  def init_fn():
    return tff.federated_zip(collections.OrderedDict(
        round_num=tff.federated_value(0.0, tff.SERVER),
        step_size=tff.federated_value(float(factory._step_size), tff.SERVER),  # pylint: disable=protected-access
        inner_state=tff.federated_value((), tff.SERVER)))

  @tff.federated_computation(init_fn.type_signature.result, tff.type_at_clients(value_type))
  def next_fn(state, value):
    step_size = state["step_size"]
    message, noise, distortion, sparsity = tff.federated_map(
        quantize, (value, tff.federated_broadcast(step_size)))
    noise_sum = tff.federated_sum(noise)
    total = tff.federated_aggregate(message, zero(), accumulate, merge, report)
    avg_len = tff.federated_mean(tff.federated_map(bitstring_length, message))
    avg_bitrate = tff.federated_map(
        tff.tf_computation(lambda x: tf.math.divide_no_nan(x, tf.constant(P, tf.float64))), avg_len)
    result = tff.federated_map(dequantize, (total, step_size, noise_sum))
    next_round = tff.federated_map(tff.tf_computation(lambda x: x + 1.0), state["round_num"])
    next_step = tff.federated_map(
        tff.tf_computation(lambda r: tf.numpy_function(
            lambda rr: np.float32(factory._schedule_fn(np.float32(rr))),  # pylint: disable=protected-access
            [r], tf.float32)), next_round)
    return tff.templates.MeasuredProcessOutput(
        state=tff.federated_zip(collections.OrderedDict(
            round_num=next_round, step_size=next_step, inner_state=state["inner_state"])),
        result=result,
        measurements=tff.federated_zip(collections.OrderedDict(
            avg_bitrate=avg_bitrate, avg_distortion=tff.federated_mean(distortion),
            avg_sparsity=tff.federated_mean(sparsity), step_size=step_size)))

  return tff.templates.AggregationProcess(init_fn, next_fn)


def as_tff_factory(factory):
  """Wraps a federated_amd QuantizeEncodeFactory as a
  ``tff.aggregators.UnweightedAggregationFactory`` whose ``create`` returns
  ``quantize_encode_process``; compose it with TFF's own MeanFactory /
  clipping_factory / zeroing_factory exactly as builder.py:77-117 does."""
  _, tff = _tf()

  class _Factory(tff.aggregators.UnweightedAggregationFactory):

    def create(self, value_type):
      if not value_type.is_tensor() or not np.issubdtype(value_type.dtype.as_numpy_dtype, np.floating):
        raise ValueError("Expect value_type to be a float tensor, found %s." % (value_type,))
      return quantize_encode_process(value_type, factory)

  return _Factory()

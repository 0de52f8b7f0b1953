"""``quantize_utils.py`` restated in numpy with TF-CPU numerics (TEST INFRASTRUCTURE ONLY).

Follows ``compressed_communication/aggregators/utils/quantize_utils.py``
function by function (line numbers below).  TF-CPU numerics restated:

* TF's Eigen worker threads run with FTZ+DAZ (``port::ScopedFlushDenormal``):
  denormal inputs read as signed zero, denormal results are flushed.
* ``tf.round`` is round-half-to-even (``np.rint``).
* ``tf.cast(float32 -> int32)`` compiles to x86 ``cvttps2dq``: NaN, +-Inf and
  values outside [-2^31, 2^31) become INT32_MIN.
* ``tf.cast(int32 -> float32)`` rounds to nearest even.
"""
import numpy as np

from oracle import philox

F32 = np.float32
FLT_MIN = np.float32(1.17549435e-38)
INT_MIN = np.int32(-2**31)


def ftz(a):
  """Flush denormals to signed zero (x86 FTZ/DAZ as TF-CPU runs)."""
  a = np.asarray(a, dtype=np.float32)
  return np.where(np.abs(a) < FLT_MIN, np.copysign(F32(0), a), a).astype(np.float32)


def f32_to_i32(v):
  """x86 ``cvttps2dq`` semantics for float32 -> int32."""
  v = np.asarray(v, dtype=np.float32)
  ok = (v >= F32(-2147483648.0)) & (v < F32(2147483648.0))
  safe = np.where(ok, v, F32(0))
  return np.where(ok, np.trunc(safe).astype(np.int64), np.int64(INT_MIN)).astype(np.int32)


def _div(value, step_size):
  with np.errstate(over="ignore", invalid="ignore", divide="ignore"):
    return ftz(ftz(value) / ftz(F32(step_size)))


# quantize_utils.py:20-21
def mean_magnitude(value):
  value = ftz(value)
  return F32(np.mean(np.abs(value), dtype=np.float64))


# quantize_utils.py:24-25
def max_magnitude(value):
  return F32(np.max(np.abs(ftz(value))))


# quantize_utils.py:28-29
def dimensionless_norm(value):
  value = ftz(value).astype(np.float64)
  return F32(np.sqrt(np.mean(value * value)))


# quantize_utils.py:33-36
def uniform_quantize(value, step_size, seed=None):
  del seed
  return f32_to_i32(np.rint(_div(value, step_size)))


# quantize_utils.py:39-42
def uniform_dequantize(value, step_size, noise_sum=None):
  del noise_sum
  return ftz(np.asarray(value, np.int32).astype(np.float32) * F32(step_size))


# quantize_utils.py:46-53
def stochastic_quantize(value, step_size, seed):
  value = np.asarray(value, np.float32).reshape(-1)
  scaled = _div(value, step_size)
  fl = np.floor(scaled)
  with np.errstate(invalid="ignore"):
    prob = ftz(scaled - fl)
  rnd = philox.stateless_uniform(value.size, seed)
  rounded = np.where(rnd <= prob, np.ceil(scaled), fl)
  return f32_to_i32(rounded)


def stochastic_quantize_at(values, idx, step_size, seed):
  """``stochastic_quantize(x, step_size, seed)[idx]`` from ``values = x[idx]``
  (elementwise: element i needs only x[i] and stream element i)."""
  scaled = _div(np.asarray(values, np.float32), step_size)
  fl = np.floor(scaled)
  with np.errstate(invalid="ignore"):
    prob = ftz(scaled - fl)
  rnd = philox.uint32_to_float(philox.random_bits_at(idx, seed))
  return f32_to_i32(np.where(rnd <= prob, np.ceil(scaled), fl))


# quantize_utils.py:57-59
def generate_noise(seed, n):
  return philox.stateless_uniform(n, seed, -0.5, 0.5)


# quantize_utils.py:62-66
def dithered_quantize(value, step_size, seed):
  value = np.asarray(value, np.float32).reshape(-1)
  scaled = _div(value, step_size)
  noise = generate_noise(seed, value.size)
  with np.errstate(invalid="ignore"):
    return f32_to_i32(np.rint(ftz(scaled - noise)))


# quantize_utils.py:69-84
def dithered_dequantize(value, step_size, noise_sum):
  s = ftz(np.asarray(value, np.int32).astype(np.float32) + ftz(noise_sum))
  return ftz(s * F32(step_size))


# quantize_utils.py:88-91
def linear_decay(initial_value, min_value, round_num, total_rounds):
  delta = F32(round_num) / F32(total_rounds) * (F32(initial_value) - F32(min_value))
  return np.maximum(F32(initial_value) - delta, F32(min_value)).astype(np.float32)


# quantize_utils.py:94-95
def exponential_decay(initial_value, min_value, round_num, exp):
  return F32((F32(initial_value) - F32(min_value)) *
             np.exp(F32(-round_num) * F32(exp)).astype(np.float32) + F32(min_value))


# quantize_utils.py:98-100
def step_decay(initial_value, min_value, round_num, freq):
  return np.maximum(F32(initial_value) * F32(0.5) ** np.floor(F32(round_num) / F32(freq)),
                    F32(min_value)).astype(np.float32)

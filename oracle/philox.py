"""TF ``stateless_random_uniform`` restated in numpy (TEST INFRASTRUCTURE ONLY).

The reference draws its stochastic-rounding and dither noise with
``tf.random.stateless_uniform(shape, seed=int64[2], dtype=float32)``
(``compressed_communication/aggregators/utils/quantize_utils.py:49, 58-59``).
TensorFlow is not installed here, so its published algorithm is restated:

* Philox4x32-10 block function (TF ``lib/random/philox_random.h``; identical to
  Random123 -- pinned by the Random123 known-answer vectors in
  ``tests/test_oracle.py``).
* Seed scramble (TF ``kernels/stateless_random_ops.cc`` ``GenerateKey``):
  ``ctr = {lo(s0), hi(s0), lo(s1), hi(s1)}``, ``mix = Philox(ctr, {0x3ec8f720,
  0x02461e29})``, ``key = {mix0, mix1}``, ``counter = {0, 0, mix2, mix3}``.
  **parity unpinned** (no reference test or fixture holds TF's stream).
* Output element ``i`` is lane ``i % 4`` of the block at counter ``counter +
  i // 4`` (128-bit little-endian increment, TF ``FillPhiloxRandom`` group
  size 4), converted by ``Uint32ToFloat``: ``bitcast(0x3f800000 | (r &
  0x7fffff)) - 1.0f``.  **parity unpinned** (same reason).
"""
import numpy as np

M_A = np.uint64(0xD2511F53)
M_B = np.uint64(0xCD9E8D57)
W_A = 0x9E3779B9
W_B = 0xBB67AE85
SCRAMBLE_KEY = (0x3EC8F720, 0x02461E29)
_M32 = 0xFFFFFFFF


def philox4x32_10(ctr, key):
  """Philox4x32-10 on arrays.  ``ctr``: 4 uint32 arrays (broadcastable).

  ``key``: two python ints.  Returns 4 uint32 arrays.
  """
  c0, c1, c2, c3 = (np.asarray(c, dtype=np.uint32) for c in ctr)
  k0, k1 = int(key[0]) & _M32, int(key[1]) & _M32
  for _ in range(10):
    p0 = M_A * c0.astype(np.uint64)
    p1 = M_B * c2.astype(np.uint64)
    hi0 = (p0 >> np.uint64(32)).astype(np.uint32)
    lo0 = (p0 & np.uint64(_M32)).astype(np.uint32)
    hi1 = (p1 >> np.uint64(32)).astype(np.uint32)
    lo1 = (p1 & np.uint64(_M32)).astype(np.uint32)
    c0, c1, c2, c3 = (hi1 ^ c1 ^ np.uint32(k0), lo1,
                      hi0 ^ c3 ^ np.uint32(k1), lo0)
    k0 = (k0 + W_A) & _M32
    k1 = (k1 + W_B) & _M32
  return c0, c1, c2, c3


def seed_to_key_counter(seed):
  """TF ``GenerateKey``: int64[2] seed -> (key (2 ints), counter (4 ints))."""
  s0 = int(seed[0]) & 0xFFFFFFFFFFFFFFFF
  s1 = int(seed[1]) & 0xFFFFFFFFFFFFFFFF
  ctr = [np.uint32(s0 & _M32), np.uint32(s0 >> 32),
         np.uint32(s1 & _M32), np.uint32(s1 >> 32)]
  mix = philox4x32_10(ctr, SCRAMBLE_KEY)
  mix = [int(m) for m in mix]
  return (mix[0], mix[1]), (0, 0, mix[2], mix[3])


def uint32_to_float(r):
  """TF ``random::Uint32ToFloat``: 23 mantissa bits -> [0, 1)."""
  bits = np.uint32(0x3F800000) | (np.asarray(r, np.uint32) & np.uint32(0x7FFFFF))
  return bits.view(np.float32) - np.float32(1.0)


def random_bits(n, seed):
  """The raw uint32 stream element i of ``stateless_uniform([n], seed)`` uses."""
  key, counter = seed_to_key_counter(seed)
  ngroups = (n + 3) // 4
  g = np.arange(ngroups, dtype=np.uint64)
  # 128-bit add of g to {0, 0, c2, c3}; g < 2^32 for every shape TF allows here.
  c0 = (g & np.uint64(_M32)).astype(np.uint32)
  c1 = (g >> np.uint64(32)).astype(np.uint32)
  r = philox4x32_10([c0, c1, np.uint32(counter[2]), np.uint32(counter[3])], key)
  out = np.stack(r, axis=1).reshape(-1)
  return out[:n]


def random_bits_at(idx, seed):
  """``random_bits(n, seed)[idx]`` for element indices ``idx`` only (the same
  counter arithmetic: element i is lane i % 4 of counter + i // 4), so sampled
  positions of a large tensor can be checked without drawing the whole stream."""
  key, counter = seed_to_key_counter(seed)
  idx = np.asarray(idx, np.int64)
  g = (idx // 4).astype(np.uint64)
  c0 = (g & np.uint64(_M32)).astype(np.uint32)
  c1 = (g >> np.uint64(32)).astype(np.uint32)
  r = np.stack(philox4x32_10([c0, c1, np.uint32(counter[2]), np.uint32(counter[3])], key), axis=1)
  return r[np.arange(idx.size), idx % 4]


def stateless_uniform(n, seed, minval=0.0, maxval=1.0):
  """``tf.random.stateless_uniform([n], seed, minval, maxval, float32)``.

  TF computes ``u * (maxval - minval) + minval`` in float32
  (``stateless_random_ops.py``); for (0, 1) and (-0.5, 0.5) this is exact.
  """
  u = uint32_to_float(random_bits(n, seed))
  scale = np.float32(maxval) - np.float32(minval)
  return (u * scale + np.float32(minval)).astype(np.float32)

"""The decoder's compile-time tables (fc_decode_tables, no GPU) against the
run-length Elias-gamma code format (elias_gamma_encode.py:30-45 via the oracle).

k_decode reads 12 window bits at a time: `lut` gives the up-to-two complete codes
they begin (run d <= 31, |v| <= 31 each), `glut` the structure of the one code
they begin whenever everything up to its magnitude's leading 1 lies in them.  Here
both are restated from the code format itself -- a code is gamma(d), a sign bit
(1 = positive), gamma(|v|); gamma(n) = floor(log2 n) zeros, then n in binary --
and every full code the oracle's encoder writes is decoded through the tables.
"""
import ctypes

import numpy as np
import pytest

from federated_amd import _lib
from oracle import codec as ocodec

BITS = 12


def _gamma_at(bits, pos):
  """(value, next position) of the gamma code at bits[pos:], None past the end."""
  z = 0
  while pos + z < len(bits) and bits[pos + z] == "0":
    z += 1
  if pos + 2 * z + 1 > len(bits):
    return None
  return int(bits[pos + z:pos + 2 * z + 1], 2), pos + 2 * z + 1


def _code_at(bits, pos):
  g = _gamma_at(bits, pos)
  if g is None or g[1] >= len(bits):
    return None
  d, p = g
  sign = bits[p] == "1"
  g = _gamma_at(bits, p + 1)
  if g is None:
    return None
  m, end = g
  return d, (m if sign else -m), end


def _want_lut(i):
  bits = format(i, "0%db" % BITS)
  e, pos = 0, 0
  for c in range(2):
    code = _code_at(bits, pos)
    if code is None:
      break
    d, v, end = code
    if d > 31 or abs(v) > 31:
      break
    e |= ((4 * d) << (7 * c)) | ((v & 63) << (14 + 6 * c))
    pos = end
  return e | (pos << 26) if pos else 0


def _want_glut(i):
  bits = format(i, "0%db" % BITS)
  g = _gamma_at(bits, 0)
  if g is None or g[0] > 31 or g[1] >= BITS:
    return 0
  d, p = g
  neg = 0 if bits[p] == "1" else 1
  z2 = 0
  while p + 1 + z2 < BITS and bits[p + 1 + z2] == "0":
    z2 += 1
  if p + 1 + z2 >= BITS:  # the magnitude's leading 1 is past the index bits
    return 0
  L = p + 1 + 2 * z2 + 1
  return L | ((z2 + 1) << 5) | (neg << 10) | (d << 11)


@pytest.fixture(scope="module")
def tables():
  lib = _lib.load()
  lut = (ctypes.c_uint32 * 4096)()
  glut = (ctypes.c_uint16 * 4096)()
  assert lib.fc_decode_tables(lut, glut, 4096) == 4096
  assert lib.fc_decode_tables(lut, glut, 100) == -1
  return np.frombuffer(lut, np.uint32).copy(), np.frombuffer(glut, np.uint16).copy()


def test_two_code_table_matches_the_code_format(tables):
  lut, _ = tables
  want = np.array([_want_lut(i) for i in range(4096)], np.uint32)
  np.testing.assert_array_equal(lut, want)


def test_single_code_table_matches_the_code_format(tables):
  _, glut = tables
  want = np.array([_want_glut(i) for i in range(4096)], np.uint16)
  np.testing.assert_array_equal(glut, want)


def test_single_code_table_decodes_oracle_streams(tables):
  """Every code of oracle-encoded dense streams (8-bit steps, runs up to 40, |q| up
  to 3000) decoded as k_decode's LONG loop does -- the table entry of the next 12
  bits, m = bits [32 - L, 32 - L + n) of the top 32 -- or, for an entry of 0, by the
  gamma format; the sum of the decoded runs and values equals the input."""
  _, glut = tables
  rng = np.random.default_rng(5)
  q = np.round(rng.standard_normal(20_000) * 40).astype(np.int32)
  q[rng.choice(q.size, 300, replace=False)] = 0
  q[1000:1040] = 0
  q[rng.choice(q.size, 50, replace=False)] = rng.integers(-3000, 3000, 50)
  code, nbits = ocodec.run_length_gamma_encode(q)
  bits = "".join(format(b, "08b") for b in code)[:nbits] + "0" * 64
  pos, idx, got, used = 0, -1, np.zeros_like(q), 0
  while idx + 1 < q.size and pos < nbits:
    top = int(bits[pos:pos + 32], 2)
    e = int(glut[top >> 20])
    L = e & 31
    if L:
      n = (e >> 5) & 31
      m = (top >> (32 - L)) & ((1 << n) - 1)
      v = -m if (e >> 10) & 1 else m
      d = e >> 11
      used += 1
    else:
      d, v, end = _code_at(bits, pos)
      L = end - pos
    idx += d
    if idx >= q.size:  # the trailing run code
      break
    got[idx] = v
    pos += L
  np.testing.assert_array_equal(got, q)
  assert used > 0.95 * np.count_nonzero(q)

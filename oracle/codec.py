"""ctypes binding of ``oracle/rlgamma.c`` (TEST INFRASTRUCTURE ONLY).

Restates ``tfc.run_length_gamma_encode`` / ``tfc.run_length_gamma_decode`` as
called at ``compressed_communication/aggregators/elias_gamma_encode.py:71-72,
97-99`` (see the header of ``rlgamma.c`` for what is pinned and what is not).
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SRC = os.path.join(_HERE, "rlgamma.c")
_BUILD = os.path.join(_HERE, "_build")
_LIB = os.path.join(_BUILD, "liboracle.so")
_lib = None


def build(force=False):
  """Compile rlgamma.c with gcc (the recipe; outputs only under oracle/_build)."""
  if not force and os.path.exists(_LIB) and os.path.getmtime(_LIB) >= os.path.getmtime(_SRC):
    return _LIB
  os.makedirs(_BUILD, exist_ok=True)
  tmp = _LIB + ".tmp.%d" % os.getpid()
  subprocess.check_call(["gcc", "-O2", "-fPIC", "-shared", "-o", tmp, _SRC])
  os.replace(tmp, _LIB)
  return _LIB


def lib():
  global _lib
  if _lib is None:
    _lib = ctypes.CDLL(build())
    i64, p = ctypes.c_int64, ctypes.c_void_p
    _lib.rlg_encoded_bits.argtypes = [p, i64]
    _lib.rlg_encoded_bits.restype = i64
    _lib.rlg_encode.argtypes = [p, i64, p, i64]
    _lib.rlg_encode.restype = i64
    _lib.rlg_decode.argtypes = [p, i64, i64, p]
    _lib.rlg_decode.restype = ctypes.c_int
    _lib.rlg_decode_accumulate.argtypes = [p, i64, i64, p]
    _lib.rlg_decode_accumulate.restype = ctypes.c_int
  return _lib


def _i32(q):
  return np.ascontiguousarray(np.asarray(q, dtype=np.int32).reshape(-1))


def encoded_bits(q):
  q = _i32(q)
  return int(lib().rlg_encoded_bits(q.ctypes.data, q.size))


def run_length_gamma_encode(q):
  """Returns (bytes, nbits)."""
  q = _i32(q)
  nbits = encoded_bits(q)
  out = np.zeros((nbits + 7) // 8 + 8, dtype=np.uint8)
  got = lib().rlg_encode(q.ctypes.data, q.size, out.ctypes.data, out.size)
  assert got == nbits, (got, nbits)
  return out[:(nbits + 7) // 8].tobytes(), nbits


def run_length_gamma_decode(code, n):
  buf = np.frombuffer(bytes(code), dtype=np.uint8)
  out = np.zeros(n, dtype=np.int32)
  rc = lib().rlg_decode(buf.ctypes.data if buf.size else None, buf.size, n, out.ctypes.data)
  if rc != 0:
    raise ValueError("malformed run-length gamma stream (code %d)" % rc)
  return out


def decode_accumulate(code, acc):
  buf = np.frombuffer(bytes(code), dtype=np.uint8)
  assert acc.dtype == np.int32 and acc.flags.c_contiguous
  rc = lib().rlg_decode_accumulate(buf.ctypes.data if buf.size else None, buf.size, acc.size,
                                   acc.ctypes.data)
  if rc != 0:
    raise ValueError("malformed run-length gamma stream (code %d)" % rc)
  return acc


def get_bitstring_length(code):
  """elias_gamma_encode.py:22-24: 8 * bytes as float64."""
  return np.float64(8.0 * len(code))

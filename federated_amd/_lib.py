"""ctypes binding of libfedcodec.so (the C ABI declared in include/fedcodec.h).

The product path has no CPU fallback: if the HIP library is missing or no GPU
is visible, every entry point raises.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("FEDCODEC_LIB") or os.path.join(_HERE, "libfedcodec.so")

UNIFORM, STOCHASTIC, DITHERED = 0, 1, 2
NORM_MEAN_MAGNITUDE, NORM_MAX_MAGNITUDE, NORM_DIMENSIONLESS, NORM_L2, NORM_LINF, NORM_L2_LINF = 1, 2, 3, 4, 5, 6
TILE_ELEMS = 1024
OVERFLOW_CAPACITY, OVERFLOW_STALL = 1, 2  # FC_OVERFLOW_* bits of the encoders' overflow[]
MAX_ELEMS = (1 << 30) - (1 << 26)  # FC_MAX_ELEMS: one client tensor
MAX_ROW_ELEMS = (1 << 26) - 1  # FC_MAX_ROW_ELEMS: one encoder row (longer tensors are segmented)

# (name, restype, argtypes); every symbol declared in include/fedcodec.h.
_P = ctypes.c_void_p
_I32 = ctypes.c_int32
_I64 = ctypes.c_int64
_F32 = ctypes.c_float
_INT = ctypes.c_int
SIGNATURES = {
    "fc_last_error": (ctypes.c_char_p, []),
    "fc_version": (ctypes.c_char_p, []),
    "fc_num_tiles": (_I64, [_I64]),
    "fc_decode_tables": (_I32, [_P, _P, _I32]),
    "fc_encode_workspace_bytes": (_I64, [_I32, _I64]),
    "fc_quantize": (_INT, [_P, _I64, _F32, _I64, _I64, _INT, _P, _P, _P]),
    "fc_quantize_encode": (_INT, [_P, _I32, _I64, _F32, _P, _P, _P, _INT, _P, _P, _P, _P, _P,
                                  _P, _P, _P, _P, _I64, _P]),
    "fc_rlgamma_encode": (_INT, [_P, _I32, _I64, _P, _P, _P, _P, _P, _P, _P, _I64, _P]),
    "fc_rlgamma_encode_segmented": (_INT, [_P, _I32, _I64, _I32, _I64, _P, _P, _P, _P, _P, _P, _P, _I64, _P]),
    "fc_quantize_encode_hinted": (_INT, [_P, _I32, _I64, _F32, _P, _P, _P, _INT, _P, _P, _P, _P, _P,
                                         _P, _P, _P, _P, _I64, _I64, _P]),
    "fc_quantize_encode_quarters": (_INT, [_P, _I32, _I64, _F32, _P, _P, _P, _INT, _P, _P, _P, _P, _P, _P,
                                           _P, _P, _P, _P, _I64, _P]),
    "fc_segmented_workspace_bytes": (_I64, [_I32, _I64, _I32, _I64]),
    "fc_quantize_encode_segmented_split": (_INT, [_P, _I32, _I64, _F32, _P, _P, _P, _INT, _I32, _I64, _P, _P, _P,
                                                  _P, _P, _P, _P, _P, _P, _I64, _P, _P]),
    "fc_decode_accumulate_segmented": (_INT, [_P, _I64, _I32, _I64, _I32, _I64, _I32, _I32, _P, _P, _P, _F32, _P,
                                              _P, _P]),
    "fc_quantize_encode_segmented": (_INT, [_P, _I32, _I64, _F32, _P, _P, _P, _INT, _I32, _I64, _P, _P, _P, _P,
                                            _P, _P, _P, _P, _P, _I64, _P]),
    "fc_decode_accumulate": (_INT, [_P, _P, _P, _P, _I32, _I64, _P, _P, _P, _F32, _P, _P, _P]),
    "fc_index_workspace_bytes": (_I64, [_I32, _I64]),
    "fc_build_index": (_INT, [_P, _P, _P, _I32, _I64, _I64, _P, _P, _P, _P, _P, _I64, _P]),
    "fc_decode_scaled_workspace_bytes": (_I64, [_I32, _I64]),
    "fc_decode_accumulate_scaled": (_INT, [_P, _P, _P, _P, _I32, _I64, _P, _P, _P, _P, _P, _I64, _P]),
    "fc_decode_accumulate_scaled_bounded": (_INT, [_P, _P, _P, _P, _I32, _I64, _P, _P, _P, _P, _I32, _P, _I64,
                                                   _P]),
    "fc_decode_accumulate_tiles": (_INT, [_P, _P, _P, _P, _I32, _I64, _I32, _I32, _P, _P, _P, _F32, _P, _P,
                                          _P]),
    "fc_decode_accumulate_quarters": (_INT, [_P, _P, _P, _P, _P, _I32, _I64, _I32, _I32, _P, _P, _P, _F32, _P,
                                             _P, _P]),
    "fc_vote_workspace_bytes": (_I64, [_I32, _I64, _I32]),
    "fc_vote_lengths": (_INT, [_P, _I32, _I64, _P, _I32, _P, _INT, _P, _P, _P, _I64, _P]),
    "fc_dequantize": (_INT, [_P, _I64, _F32, _P, _P, _P]),
    "fc_copy": (_INT, [_P, _P, _I64, _P]),
    "fc_diag_occupy": (_INT, [ctypes.c_uint32, _I64, _P, _P]),
    "fc_quantize_floor": (_INT, [_P, _I32, _I64, _F32, _P, _INT, _P, _P, _P, _I64, _P]),
    "fc_noise_sum": (_INT, [_P, _I32, _I64, _P, _P]),
    "fc_client_norms": (_INT, [_P, _I32, _I64, _INT, _P, _P]),
    "fc_client_norms_scaled": (_INT, [_P, _I32, _I64, _INT, _P, _P, _P]),
    "fc_finalize": (_INT, [_P, _P, _I32, _I64, _P, _P, _P]),
    "fc_onebit_encode": (_INT, [_P, _I32, _I64, _F32, _P, _P, _P, _P]),
    "fc_drive_encode": (_INT, [_P, _I32, _I64, _INT, _P, _P, _P, _P]),
    "fc_hadamard": (_INT, [_P, _I32, _I64, _INT, _I64, _I64, _P]),
    "fc_sign_flip": (_INT, [_P, _I32, _I64, _I64, _I64, _P]),
    "fc_dft_workspace_bytes": (_I64, [_I64]),
    "fc_dft_rotate": (_INT, [_P, _I32, _I64, _INT, _I64, _I64, _P, _I64, _P]),
    "fc_onebit_decode_sum": (_INT, [_P, _P, _I32, _I64, _P, _P]),
    "fc_onebit_decode_sum_range": (_INT, [_P, _P, _I32, _I64, _I64, _I64, _P, _P]),
}

_lib = None


class FedCodecError(RuntimeError):
  pass


def load():
  """Load libfedcodec.so (no GPU needed).  Raises if it was not built."""
  global _lib
  if _lib is None:
    if not os.path.exists(LIB_PATH):
      raise FedCodecError(
          "libfedcodec.so is not built (%s); run `python -c 'import __graft_entry__ as g; "
          "g.build()'`" % LIB_PATH)
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
      fn = getattr(lib, name)
      fn.restype = res
      fn.argtypes = args
    _lib = lib
  return _lib


def check(rc):
  if rc != 0:
    raise FedCodecError(load().fc_last_error().decode() or "fedcodec error %d" % rc)


def call(name, *args):
  check(getattr(load(), name)(*args))


def ptr(t):
  """Device pointer of a torch tensor (None -> NULL)."""
  if t is None:
    return None
  return ctypes.c_void_p(t.data_ptr())


def stream_handle(stream=None):
  import torch  # pylint: disable=g-import-not-at-top
  s = stream if stream is not None else torch.cuda.current_stream()
  return ctypes.c_void_p(s.cuda_stream)


def require_gpu():
  import torch  # pylint: disable=g-import-not-at-top
  if not torch.cuda.is_available():
    raise FedCodecError("fedcodec needs an MI355X (gfx950) GPU; none is visible")
  load()

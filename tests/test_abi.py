"""The C ABI library loads and exports every symbol include/fedcodec.h declares (no GPU)."""
import ctypes
import os
import re

import pytest

from federated_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
  hdr = open(os.path.join(ROOT, "include", "fedcodec.h")).read()
  hdr = re.sub(r"/\*.*?\*/", "", hdr, flags=re.S)
  return sorted(set(re.findall(r"\b(fc_[a-z0-9_]+)\s*\(", hdr)))


def test_header_declares_the_expected_surface():
  syms = declared_symbols()
  for s in ["fc_quantize", "fc_quantize_encode", "fc_rlgamma_encode", "fc_decode_accumulate",
            "fc_dequantize", "fc_noise_sum", "fc_client_norms", "fc_finalize"]:
    assert s in syms


def test_library_exports_every_declared_symbol():
  lib = _lib.load()
  for s in declared_symbols():
    assert hasattr(lib, s), s
    assert s in _lib.SIGNATURES, "ctypes signature missing for %s" % s


def test_host_only_entry_points():
  lib = _lib.load()
  assert lib.fc_version().startswith(b"fedcodec")
  assert lib.fc_num_tiles(25_000_000) == 24415
  assert lib.fc_num_tiles(0) == 0
  assert lib.fc_encode_workspace_bytes(128, 25_000_000) >= 128 * 24415 * 16


def test_index_workspace_follows_the_chunk_choice():
  """fc_build_index's chunk lanes: the largest of 8192 / 4096 / 2048 bits giving about
  600 K lanes, min(31, chunk / 256 - 1) checkpoints each; the workspace holds five int64
  and the checkpoints per lane, plus an int32 per client."""
  lib = _lib.load()

  def want(n, max_bytes):
    cb = 8192
    while cb > 2048 and n * -(-8 * max_bytes // cb) < 600_000:
      cb //= 2
    lanes = n * max(1, -(-8 * max_bytes // cb))
    return (5 + min(31, cb // 256 - 1)) * 8 * lanes + ((4 * n + 255) & ~255)

  for n, mb in [(1024, 12_300_000), (256, 1_400_000), (128, 1_360_000), (2, 100), (1, 0), (300, 15_872)]:
    assert lib.fc_index_workspace_bytes(n, mb) == want(n, mb), (n, mb)
  assert lib.fc_index_workspace_bytes(0, 10) == -1


def test_argument_validation_without_gpu():
  lib = _lib.load()
  # rejected before any device work: bad sizes / null pointers / bad mode
  rc = lib.fc_quantize_encode(None, 0, 10, 1.0, None, None, None, 0, None, None, None, None, None,
                              None, None, None, None, 0, None)
  assert rc != 0 and b"nclients" in lib.fc_last_error()
  rc = lib.fc_quantize(None, 10, 1.0, 0, 0, 7, None, None, None)
  assert rc != 0
  rc = lib.fc_client_norms(None, 1, 10, 9, None, None)
  assert rc != 0 and b"norm" in lib.fc_last_error()
  rc = lib.fc_decode_accumulate(None, None, None, None, 1, (1 << 26), None, None, None, 1.0, None,
                                None, None)
  assert rc != 0
  dummy = ctypes.c_int64(0)
  p = ctypes.addressof(dummy)
  for tb, te in ((0, 0), (1, 1), (-1, 2), (0, 99)):  # P = 5000: 5 tiles
    rc = lib.fc_decode_accumulate_tiles(p, p, p, p, 1, 5000, tb, te, None, p, None, 1.0, None, p, None)
    assert rc != 0 and b"tile range" in lib.fc_last_error()


def test_product_package_never_imports_the_oracle():
  pkg = os.path.join(ROOT, "federated_amd")
  for dirpath, _, files in os.walk(pkg):
    for f in files:
      if f.endswith(".py"):
        src = open(os.path.join(dirpath, f)).read()
        assert "import oracle" not in src and "from oracle" not in src, f


def test_missing_library_fails_loudly(monkeypatch, tmp_path):
  monkeypatch.setattr(_lib, "LIB_PATH", str(tmp_path / "nope.so"))
  monkeypatch.setattr(_lib, "_lib", None)
  with pytest.raises(_lib.FedCodecError):
    _lib.load()

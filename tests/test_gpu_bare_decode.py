"""Server decode of BARE run-length gamma codes (no encoder index).

The reference's client message is the single tf.string
``tfc.run_length_gamma_encode`` returns (elias_gamma_encode.py:97-109) and the
server decodes it with ``tfc.run_length_gamma_decode(code, shape)`` -- bytes and
shape only (:69-73).  ``codec.from_codes`` rebuilds the decoder index on the
device from the bytes (fc_build_index) and the usual decoder sums the batch.

Checked here:
  * codes produced by the ORACLE (the CPU restatement of the TFC coder), decoded
    and summed on the GPU with no encoder index: the int32 sum bit for bit against
    the oracle's q at config 2 (128 x 2^20, 8-bit steps), config 3 (256 x
    4,050,748, step 1) and 3 x 25 M (the headline's tensor);
  * the rebuilt index (and quarter index) equal to the HIP encoder's, entry for
    entry, and the rebuilt bit lengths equal to the oracle's;
  * edge cases: P = 1, all-zero tensors (one trailing run code), no trailing run,
    runs across many tiles, codes ending on a lane-chunk boundary (2048-, 4096- and
    8192-bit chunks), |q| =
    2^31 (INT_MIN), 63-bit magnitude codes, very sparse and very dense streams;
  * malformed codes rejected: truncated, a byte appended, bits flipped, an empty
    code, a code of another element count.
"""
import numpy as np
import pytest
import torch

from federated_amd import _lib
from federated_amd import codec
from oracle import codec as ocodec
from oracle import quantize_utils as oq

pytestmark = pytest.mark.gpu

F32 = np.float32

# fc_build_index picks 2048-, 4096- or 8192-bit chunk lanes by the batch's size; the
# tests below run at each (FEDCODEC_IDX_CHUNK) -- small batches would otherwise all
# take 2048-bit chunks
CHUNKS = [2048, 4096, 8192]


@pytest.fixture(params=CHUNKS, ids=lambda v: "chunk%d" % v)
def chunk(request, monkeypatch):
  monkeypatch.setenv("FEDCODEC_IDX_CHUNK", str(request.param))
  return request.param


def _oracle_codes(qs):
  return [ocodec.run_length_gamma_encode(q)[0] for q in qs]


def _check_sum(codes, qs_cycle, C, P, quarters=None):
  """Decode C codes (codes[c % len(codes)]) with a rebuilt index; compare with the
  int32 (wrapping) sum of the oracle's q."""
  n = len(codes)
  batch = codec.from_codes([codes[c % n] for c in range(C)], P, quarters=quarters)
  want_bits = np.array([ocodec.encoded_bits(qs_cycle[c % n]) for c in range(C)], np.int64)
  np.testing.assert_array_equal(batch.bits(), want_bits)
  s, _, err = codec.decode_accumulate(batch)
  assert int(err.item()) == 0
  acc = np.zeros(P, np.int64)
  for k in range(n):
    mult = len(range(k, C, n))
    acc += mult * qs_cycle[k].astype(np.int64)
  want = acc.astype(np.int64).astype(np.uint32).view(np.int32)  # int32 wrap
  np.testing.assert_array_equal(s.cpu().numpy(), want)
  return batch


def test_config2_oracle_codes(gpu):
  """Config 2: 128 x 2^20, sigma 0.25, step 1/127 (~10 bits per element)."""
  P, C = 1 << 20, 128
  rng = np.random.default_rng(2)
  qs = [oq.stochastic_quantize((rng.standard_normal(P) * 0.25).astype(F32), F32(1.0 / 127), (k, 7)) for k in range(16)]
  codes = _oracle_codes(qs)
  for quarters in (True, False):
    _check_sum(codes, qs, C, P, quarters=quarters)


def test_config3_oracle_codes(gpu):
  """Config 3: 256 x 4,050,748 (StackOverflow LSTM), sigma 1, step 1 (3-bit)."""
  P, C = 4_050_748, 256
  rng = np.random.default_rng(3)
  qs = [oq.stochastic_quantize(rng.standard_normal(P).astype(F32), F32(1.0), (k, 1)) for k in range(8)]
  _check_sum(_oracle_codes(qs), qs, C, P)


def test_headline_tensor_oracle_codes(gpu):
  """Three 25 M-element clients (the headline's tensor), sigma 1, step 0.5."""
  P, C = 25_000_000, 3
  rng = np.random.default_rng(25)
  qs = [oq.stochastic_quantize(rng.standard_normal(P).astype(F32), F32(0.5), (100 + k, k)) for k in range(C)]
  _check_sum(_oracle_codes(qs), qs, C, P)


@pytest.mark.parametrize("C,P,quarters", [(5, 70_001, False), (5, 70_001, True), (300, 9_000, False)])
def test_rebuilt_index_equals_encoder_index(gpu, chunk, C, P, quarters):
  """The index rebuilt from the bytes equals the HIP encoder's own, entry for entry
  (quarter entries too), for mixed-density clients."""
  rng = np.random.default_rng(C + P)
  scales = [0.02, 0.3, 1.0, 8.0, 60.0]
  xs = [(rng.standard_normal(P) * scales[c % len(scales)]).astype(F32) for c in range(C)]
  rows = [torch.from_numpy(x).to(gpu) for x in xs]
  seeds = torch.tensor([[c, 3 * c + 1] for c in range(C)], dtype=torch.int64)
  enc = codec.quantize_encode(rows, 0.5, seeds, _lib.STOCHASTIC, caps=[codec.worst_case_capacity(P)] * C,
                              segments=1, quarters=quarters)
  assert not len(codec.check_overflow(enc))
  codes = [enc.client_code(c) for c in range(C)]
  bare = codec.from_codes(codes, P, quarters=quarters)
  np.testing.assert_array_equal(bare.idx.cpu().numpy(), enc.idx.cpu().numpy())
  np.testing.assert_array_equal(bare.bits(), enc.bits())
  if quarters:
    np.testing.assert_array_equal(bare.idxq.cpu().numpy(), enc.idxq.cpu().numpy())
  s1, _, e1 = codec.decode_accumulate(bare)
  s2, _, e2 = codec.decode_accumulate(enc)
  assert int(e1.item()) == 0 and int(e2.item()) == 0
  assert torch.equal(s1, s2)


def _edge_qs():
  """Named int32 tensors covering the parser's edge cases."""
  rng = np.random.default_rng(11)
  out = {}
  out["p1_zero"] = np.zeros(1, np.int32)
  out["p1_nonzero"] = np.array([-3], np.int32)
  out["all_zero"] = np.zeros(300_000, np.int32)
  q = np.zeros(200_003, np.int32)
  q[-1] = 5
  out["no_trailing_run"] = q
  q = np.zeros(500_000, np.int32)
  q[[0, 7, 100_000, 100_001, 250_000, 499_998]] = [1, -2, 3, 40000, -7, 1]
  out["long_runs"] = q
  q = np.zeros(50_000, np.int32)
  q[::3] = np.resize(np.array([np.iinfo(np.int32).min, np.iinfo(np.int32).max, -1], np.int32), q[::3].size)
  out["int_min_max"] = q
  out["dense_wide"] = rng.integers(-(1 << 30), 1 << 30, 40_000).astype(np.int32)
  q = np.zeros(2_000_000, np.int32)
  nz = rng.choice(q.size, 300, replace=False)
  q[nz] = rng.integers(1, 9, 300) * rng.choice([-1, 1], 300)
  out["very_sparse"] = q
  out["unit_codes"] = np.ones(70_000, np.int32)  # 3-bit codes: every chunk boundary mid-code
  out["ends_at_4095"] = np.ones(1365, np.int32)  # 1365 three-bit codes: 4095 bits, no trailing run
  q = np.concatenate([np.ones(1365, np.int32), np.zeros(1, np.int32)])  # trailing run code "010": 4098 bits
  out["trailing_across_chunk"] = q
  q = np.concatenate([np.ones(2730, np.int32), np.full(10, 2, np.int32)])  # code start at bit 8190
  out["two_chunks"] = q
  # last element nonzero and the code ends exactly on a chunk boundary (no trailing run):
  # 681 * 3 + 5 = 2048, 1362 * 3 + 2 * 5 = 4096, 2729 * 3 + 5 = 8192 bits
  out["ends_at_2048"] = np.concatenate([np.ones(681, np.int32), np.full(1, 2, np.int32)])
  out["ends_at_4096"] = np.concatenate([np.ones(1362, np.int32), np.full(2, 2, np.int32)])
  out["ends_at_8192"] = np.concatenate([np.ones(2729, np.int32), np.full(1, 2, np.int32)])
  return out


@pytest.mark.parametrize("name", sorted(_edge_qs()))
def test_edge_case_codes(gpu, chunk, name):
  q = _edge_qs()[name]
  P = q.size
  code = ocodec.run_length_gamma_encode(q)[0]
  for quarters in (False, True):
    batch = codec.from_codes([code, code], P, quarters=quarters)
    assert list(batch.bits()) == [ocodec.encoded_bits(q)] * 2
    s, _, err = codec.decode_accumulate(batch)
    assert int(err.item()) == 0
    want = (2 * q.astype(np.int64)).astype(np.uint32).view(np.int32)
    np.testing.assert_array_equal(s.cpu().numpy(), want)


def test_chunk_boundary_sweep(gpu, chunk):
  """Codes of every length around 4096 bits (a lane-chunk boundary at every chunk size):
  a code start, a code's middle and the trailing run landing on each boundary."""
  rng = np.random.default_rng(5)
  codes, qs = [], []
  for extra in range(0, 40):
    q = np.concatenate([np.ones(1365 - 20 + extra, np.int32),
                        rng.integers(-3, 4, 17).astype(np.int32), np.zeros(extra % 5, np.int32)])
    qs.append(q)
  P = max(q.size for q in qs)
  qs = [np.concatenate([q, np.zeros(P - q.size, np.int32)]) for q in qs]
  codes = _oracle_codes(qs)
  _check_sum(codes, qs, len(codes), P)


def _good_code(P=100_000, seed=1):
  rng = np.random.default_rng(seed)
  q = oq.stochastic_quantize(rng.standard_normal(P).astype(F32), F32(0.5), (seed, 0))
  return q, ocodec.run_length_gamma_encode(q)[0]


@pytest.mark.parametrize("how", ["truncated", "appended", "empty", "other_P", "garbage"])
def test_malformed_codes_rejected(gpu, chunk, how):
  q, code = _good_code()
  P = q.size
  if how == "truncated":
    bad = code[:len(code) // 2]
  elif how == "appended":
    bad = code + b"\x80"
  elif how == "empty":
    bad = b""
  elif how == "other_P":
    bad = ocodec.run_length_gamma_encode(q[:-10])[0]
  else:
    bad = bytes(len(code))  # all zero bits: no gamma code terminates
  with pytest.raises(ValueError):
    codec.from_codes([code, bad, code], P)
  # the good codes alone still decode
  batch = codec.from_codes([code, code], P)
  s, _, err = codec.decode_accumulate(batch)
  assert int(err.item()) == 0
  np.testing.assert_array_equal(s.cpu().numpy(), 2 * q)

"""Segmented encode (fc_quantize_encode_segmented): few clients, each cut into
element segments encoded as independent rows and stitched.  The stitched
batch must equal the one-piece encode bit for bit -- code bytes, bit counts,
decoder index -- and the oracle's restatement; measurements equal up to float
summation order.  Cases: a remainder segment or none, all-zero segments (runs
crossing whole segments), a zero tail (the trailing run code moves to the
client's end), every rounding mode, norms and fused pre-scales, and overflow.
"""
import numpy as np
import pytest
import torch

from federated_amd import _lib
from federated_amd import codec
from oracle import codec as ocodec
from oracle import quantize_utils as oq

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True, params=["1", "0"], ids=["split", "inorder"])
def _stitch_mode(monkeypatch, request):
  """Both stitch orders: on a second stream beside the decode of the unstitched
  segments (default), and in order before anything else."""
  monkeypatch.setenv("FEDCODEC_SPLIT_STITCH", request.param)
  return request.param
F32 = np.float32
MODES = {"uniform": _lib.UNIFORM, "stochastic": _lib.STOCHASTIC, "dithered": _lib.DITHERED}
ORACLE_Q = {"uniform": lambda x, s, sd: oq.uniform_quantize(x, s), "stochastic": oq.stochastic_quantize,
            "dithered": oq.dithered_quantize}


def _data(kind, C, P, seed):
  rng = np.random.default_rng(seed)
  xs = []
  for c in range(C):
    x = rng.standard_normal(P).astype(np.float32)
    if kind == "sparse":  # long zero stretches: whole segments quantise to 0
      x = np.where(rng.random(P) < 0.0005, x * 8, 0.0).astype(np.float32)
      x[P // 3:2 * P // 3] = 0.0
    elif kind == "zero_tail":
      x[P - P // 5:] = 0.0
    elif kind == "zero_head":
      x[:P // 2] = 0.0
    elif kind == "all_zero" and c == 1:
      x[:] = 0.0
    xs.append(x)
  return xs


def _same(a, b):
  assert np.array_equal(a.bits(), b.bits())
  for c in range(a.nclients):
    assert a.client_code(c) == b.client_code(c), c
  np.testing.assert_array_equal(a.idx.cpu().numpy(), b.idx.cpu().numpy())
  da, na = codec.finalize(a)
  db, nb = codec.finalize(b)
  np.testing.assert_array_equal(na.cpu().numpy(), nb.cpu().numpy())
  np.testing.assert_allclose(da.cpu().numpy(), db.cpu().numpy(), rtol=1e-6, atol=1e-30)


@pytest.mark.parametrize("C,P,K,mode,kind", [
    (3, 70_000, 4, "stochastic", "gauss"),       # 16,384-element segments + a 4,464 remainder
    (5, 1 << 18, 8, "uniform", "gauss"),         # no remainder
    (2, 300_001, 16, "dithered", "gauss"),
    (4, 200_000, 6, "stochastic", "sparse"),     # all-zero segments
    (3, 150_000, 5, "stochastic", "zero_tail"),
    (3, 150_000, 5, "uniform", "zero_head"),
    (3, 120_000, 4, "stochastic", "all_zero"),
])
def test_segmented_equals_one_piece_and_oracle(gpu, C, P, K, mode, kind):
  xs = _data(kind, C, P, seed=C * 1000 + K)
  rows = [torch.from_numpy(x).to(gpu) for x in xs]
  seeds = torch.tensor([[9 + c, 3 * c + 1] for c in range(C)], dtype=torch.int64)
  step = 0.5 if mode != "dithered" else 0.3
  caps = [codec.worst_case_capacity(P) // 4] * C
  one = codec.quantize_encode(rows, step, seeds, MODES[mode], caps=caps, segments=1)
  seg = codec.quantize_encode(rows, step, seeds, MODES[mode], caps=caps, segments=K)
  assert not len(codec.check_overflow(one)) and not len(codec.check_overflow(seg))
  _same(seg, one)
  q = ORACLE_Q[mode](xs[0], F32(step), (9, 1))
  code, nbits = ocodec.run_length_gamma_encode(q)
  assert seg.client_code(0) == code and int(seg.bits()[0]) == nbits
  s, _, err = codec.decode_accumulate(seg)
  assert int(err.item()) == 0
  want = np.zeros(P, np.int64)
  for c in range(C):
    want += ORACLE_Q[mode](xs[c], F32(step), (9 + c, 3 * c + 1))
  np.testing.assert_array_equal(s.cpu().numpy(), want.astype(np.int32))


def test_segmented_with_norms_and_prescale(gpu):
  C, P, K = 4, 180_000, 7
  xs = _data("gauss", C, P, seed=77)
  rows = [torch.from_numpy(x).to(gpu) for x in xs]
  pre = torch.tensor([[0.5, 2.0], [1.0, 1.0], [3.0, 0.25], [1.5, 1.5]], dtype=torch.float32, device=gpu)
  norms = codec.client_norms(rows, _lib.NORM_MAX_MAGNITUDE, prescale=pre)
  seeds = torch.tensor([[c, c + 5] for c in range(C)], dtype=torch.int64)
  caps = [codec.worst_case_capacity(P) // 4] * C
  one = codec.quantize_encode(rows, 0.05, seeds, _lib.STOCHASTIC, norms=norms, prescale=pre, caps=caps, segments=1)
  seg = codec.quantize_encode(rows, 0.05, seeds, _lib.STOCHASTIC, norms=norms, prescale=pre, caps=caps, segments=K)
  _same(seg, one)


def test_segmented_overflow_then_checked_reencode(gpu):
  """A capacity too small for one client's code: that client is flagged (its bit
  count still exact) and quantize_encode_checked re-encodes only it."""
  C, P = 3, 200_000
  xs = _data("gauss", C, P, seed=5)
  xs[1] = xs[1] * F32(40.0)  # wide codes
  rows = [torch.from_numpy(x).to(gpu) for x in xs]
  seeds = torch.tensor([[c, c] for c in range(C)], dtype=torch.int64)
  caps = [P // 2] * C
  seg = codec.quantize_encode(rows, 0.5, seeds, _lib.STOCHASTIC, caps=caps, segments=6)
  assert list(codec.check_overflow(seg)) == [1]
  one = codec.quantize_encode(rows, 0.5, seeds, _lib.STOCHASTIC, caps=[codec.worst_case_capacity(P)] * C,
                              segments=1)
  assert np.array_equal(seg.bits(), one.bits())
  fixed = codec.quantize_encode_checked(rows, 0.5, seeds, _lib.STOCHASTIC, caps=caps, segments=6)
  assert not len(codec.check_overflow(fixed))
  for c in range(C):
    assert fixed.client_code(c) == one.client_code(c)


def test_segmented_at_the_8gpu_share_shape(gpu):
  """128 clients x 25 M (one GPU's share of the 8-GPU headline), the automatic
  segmentation (8 segments): equal to the one-piece encode for a client subset's
  bytes and for every client's bit count and index."""
  C, P = 128, 25_000_000
  assert codec.auto_segments(C, P) == 8
  g = torch.Generator(device=gpu)
  rows = []
  for c in range(C):
    g.manual_seed(600 + c)
    rows.append(torch.randn(P, generator=g, device=gpu, dtype=torch.float32))
  seeds = torch.tensor([[1000 + c, 1000 + c] for c in range(C)], dtype=torch.int64)
  caps = [P // 2 + 4096] * C
  seg = codec.quantize_encode(rows, 0.5, seeds, _lib.STOCHASTIC, caps=caps)
  one = codec.quantize_encode(rows, 0.5, seeds, _lib.STOCHASTIC, caps=caps, segments=1)
  assert np.array_equal(seg.bits(), one.bits())
  np.testing.assert_array_equal(seg.idx.cpu().numpy(), one.idx.cpu().numpy())
  for c in (0, 77, 127):
    assert seg.client_code(c) == one.client_code(c)
  s1, _, e1 = codec.decode_accumulate(seg)
  s2, _, e2 = codec.decode_accumulate(one)
  assert int(e1.item()) == 0 and int(e2.item()) == 0 and torch.equal(s1, s2)
  del rows, seg, one
  torch.cuda.empty_cache()


@pytest.mark.parametrize("span", ["1", "2"])
def test_unstitched_decode_tile_ranges(gpu, span, monkeypatch, _stitch_mode):
  """Tile-range decodes (the multi-GPU slabs) straight from the segments, before the
  stitch is joined: ranges starting and ending at odd tiles and inside segments,
  two-tile lane segments that would straddle a segment end -- equal to the one-piece
  batch's decode."""
  monkeypatch.setenv("FEDCODEC_DEC_SPAN", span)
  C, P, K = 3, 150_001, 5  # 28,672-element segments (28 tiles) + a 6,641-element remainder
  xs = _data("gauss", C, P, seed=31)
  rows = [torch.from_numpy(x).to(gpu) for x in xs]
  seeds = torch.tensor([[c, 2 * c] for c in range(C)], dtype=torch.int64)
  caps = [codec.worst_case_capacity(P) // 4] * C
  seg = codec.quantize_encode(rows, 0.5, seeds, _lib.STOCHASTIC, caps=caps, segments=K)
  one = codec.quantize_encode(rows, 0.5, seeds, _lib.STOCHASTIC, caps=caps, segments=1)
  assert (seg.seg is not None) == (_stitch_mode == "1")  # split: decoded before the stitch is joined
  T = seg.T
  want, _, e1 = codec.decode_accumulate(one)
  part = torch.full((P,), 77, dtype=torch.int32, device=gpu)
  err = torch.zeros(1, dtype=torch.int32, device=gpu)
  bounds = [0, 3, 27, 29, 57, 84, 85, 140, T]
  for tb, te in zip(bounds[:-1], bounds[1:]):
    codec.decode_accumulate(seg, sum_out=part, err=err, tiles=(tb, te))
  assert int(err.item()) == 0 and int(e1.item()) == 0
  np.testing.assert_array_equal(part.cpu().numpy(), want.cpu().numpy())
  _same(seg, one)


def test_segmented_skewed_client_fits_hint_capacity(gpu):
  """Clients whose nonzeros all sit in ONE segment (model deltas are uneven across
  layers), with the capacities QuantizeEncodeFactory uses from its second round on
  (codec.CapacityHint: the previous round's largest code + 1/8 + 4 KiB): every
  segment's staging holds the client's whole code, so no client overflows (and none
  is re-encoded); the result equals the one-piece encode."""
  C, P = 4, 1 << 22
  K = codec.auto_segments(C, P)
  assert K >= 8
  rng = np.random.default_rng(8)
  xs = [np.zeros(P, np.float32) for _ in range(C)]
  for c in range(C):
    lo = (3 * c % K) * (P // K)
    xs[c][lo:lo + P // K] = (rng.standard_normal(P // K) * 4).astype(np.float32)
  rows = [torch.from_numpy(x).to(gpu) for x in xs]
  worst = [codec.worst_case_capacity(P)] * C
  prev = codec.quantize_encode(rows, 0.5, torch.tensor([[c, c] for c in range(C)], dtype=torch.int64),
                               _lib.STOCHASTIC, caps=worst, segments=1)
  hint = codec.CapacityHint()
  hint.update(prev)
  seeds = torch.tensor([[90 + c, 3 * c] for c in range(C)], dtype=torch.int64)
  seg = codec.quantize_encode(rows, 0.5, seeds, _lib.STOCHASTIC, caps=hint.caps(P, C))
  assert not len(codec.check_overflow(seg))
  one = codec.quantize_encode(rows, 0.5, seeds, _lib.STOCHASTIC, caps=worst, segments=1)
  _same(seg, one)

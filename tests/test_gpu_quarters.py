"""Quarter-tile decoder index (fc_quantize_encode_quarters / fc_decode_accumulate_quarters).

Batches of fewer than 256 clients that are not segmented carry the quarter
index by default, so every small-batch parity test in the suite already decodes
through quarter-tile lane segments; this module checks the index itself against
entries computed from the oracle's q (bit offset of the first code at or after
each 256-element boundary, 1 + the last nonzero before it), the exact path's
entries (tiles with codes beyond the fast path), the overflow repack, tile-range
decodes, and then re-runs the decoding parity tests with the index off
(FEDCODEC_QUARTERS=0: one-tile lane segments).
"""
import numpy as np
import pytest
import torch

from federated_amd import _lib
from federated_amd import codec
from oracle import codec as ocodec
from oracle import quantize_utils as oq
from test_gpu_aggregators import (  # noqa: F401  (collected again below, index off)
    test_decoder_rejects_malformed_stream, test_quantize_encode_matches_golden_round)
from test_gpu_codec import (  # noqa: F401
    test_decode_tile_ranges_match_full_decode, test_quantize_encode_batch_matches_oracle,
    test_reference_known_answers)
from test_gpu_configs import test_config_round_matches_oracle  # noqa: F401

pytestmark = pytest.mark.gpu
MASK36 = (1 << 36) - 1


@pytest.fixture(autouse=True)
def _index_off_for_reruns(request, monkeypatch):
  """The imported parity tests run with the quarter index off (one-tile lane
  segments); this module's own tests keep the default."""
  if request.function.__module__ != __name__:
    monkeypatch.setenv("FEDCODEC_QUARTERS", "0")


def _glen(d):
  return 2 * (int(d).bit_length() - 1) + 1


def _boundary_entries(q, unit=256):
  """Decoder entries at every `unit`-element boundary of q (and the end), from the
  code lengths of run-length gamma (elias_gamma_encode.py:30-45)."""
  P = q.size
  nz = np.nonzero(q)[0]
  lens = np.empty(nz.size, np.int64)
  prev = -1
  for k, i in enumerate(nz):
    lens[k] = _glen(i - prev) + 1 + _glen(abs(int(q[i])))
    prev = i
  cum = np.concatenate([[0], np.cumsum(lens)])
  nb = (P + unit - 1) // unit
  bounds = np.arange(nb + 1, dtype=np.int64) * unit
  bounds[-1] = P
  k = np.searchsorted(nz, bounds, side="left")  # nonzeros before each boundary
  last = np.where(k > 0, nz[np.maximum(k - 1, 0)], -1)
  return (cum[k] & MASK36) | ((last + 1).astype(np.int64) << 36)


def _check_index(batch, qs):
  T = batch.T
  idx = batch.idx.cpu().numpy().astype(np.int64).reshape(batch.nclients, T + 1)
  idxq = batch.idxq.cpu().numpy().astype(np.int64).reshape(batch.nclients, T, 3)
  for c, q in enumerate(qs):
    want = _boundary_entries(q)  # boundaries 0, 256, ... below P, then P
    nq = 4 * T
    full = np.empty(nq + 1, np.int64)
    full[:want.size - 1] = want[:-1]
    full[want.size - 1:] = want[-1]  # quarters past P (a partial last tile): the end entry
    np.testing.assert_array_equal(idx[c, :], full[0:nq + 1:4], err_msg="tile entries, client %d" % c)
    for s in range(1, 4):
      np.testing.assert_array_equal(idxq[c, :, s - 1], full[s:nq:4], err_msg="quarter %d, client %d" % (s, c))


@pytest.mark.parametrize("P,kind", [(1, "gauss"), (300, "gauss"), (1024, "gauss"), (1100, "gauss"),
                                    (70_001, "gauss"), (50_000, "sparse"), (40_000, "dense8"),
                                    (30_000, "zero_quarters")])
def test_quarter_entries_match_oracle_and_decode(gpu, P, kind):
  rng = np.random.default_rng(P + len(kind))
  C = 5
  step = 1.0 / 127 if kind == "dense8" else 0.5
  xs = []
  for c in range(C):
    x = rng.standard_normal(P).astype(np.float32)
    if kind == "sparse":
      x = np.where(rng.random(P) < 0.01, x * 4, 0.0).astype(np.float32)
    elif kind == "dense8":
      x = (x * 0.25).astype(np.float32)
    elif kind == "zero_quarters":  # whole quarters and tiles of zeros
      x[256:768] = 0.0
      x[2048:5000] = 0.0
      x[P - 700:] = 0.0
    xs.append(x)
  seeds = np.array([[40 + c, 3 * c] for c in range(C)], np.int64)
  rows = [torch.from_numpy(x).to(gpu) for x in xs]
  caps = [codec.worst_case_capacity(P)] * C
  qb = codec.quantize_encode(rows, step, torch.from_numpy(seeds), _lib.STOCHASTIC, caps=caps, quarters=True)
  tb = codec.quantize_encode(rows, step, torch.from_numpy(seeds), _lib.STOCHASTIC, caps=caps, quarters=False)
  assert qb.quarters and not tb.quarters
  qs = [oq.stochastic_quantize(xs[c], np.float32(step), tuple(seeds[c])) for c in range(C)]
  for c in range(C):
    code, nbits = ocodec.run_length_gamma_encode(qs[c])
    assert qb.client_code(c) == code and int(qb.bits()[c]) == nbits
  np.testing.assert_array_equal(qb.idx.cpu().numpy(), tb.idx.cpu().numpy())
  _check_index(qb, qs)
  want = np.sum(np.stack(qs).astype(np.int64), axis=0).astype(np.int32)
  for b in (qb, tb):
    s, _, err = codec.decode_accumulate(b)
    assert int(err.item()) == 0
    np.testing.assert_array_equal(s.cpu().numpy(), want)


def test_quarter_entries_from_the_exact_path(gpu):
  """Tiles with codes past the fast path (|q| ~ 2^21: 43-bit codes) send their
  client to k_encode_exact, which writes that client's quarter entries."""
  rng = np.random.default_rng(3)
  P, C = 9000, 3
  xs = [rng.standard_normal(P).astype(np.float32) for _ in range(C)]
  xs[1][1500] = 1e6
  xs[1][2100:2110] = -3e6
  xs[2][8999] = 5e5
  seeds = np.array([[1, 1], [2, 2], [3, 3]], np.int64)
  rows = [torch.from_numpy(x).to(gpu) for x in xs]
  b = codec.quantize_encode(rows, 0.5, torch.from_numpy(seeds), _lib.STOCHASTIC,
                            caps=[codec.worst_case_capacity(P)] * C, quarters=True)
  qs = [oq.stochastic_quantize(xs[c], np.float32(0.5), tuple(seeds[c])) for c in range(C)]
  _check_index(b, qs)
  s, _, err = codec.decode_accumulate(b)
  assert int(err.item()) == 0
  np.testing.assert_array_equal(s.cpu().numpy(), np.sum(np.stack(qs).astype(np.int64), axis=0).astype(np.int32))


def test_quarter_index_survives_overflow_repack(gpu):
  rng = np.random.default_rng(9)
  P, C = 20_000, 4
  xs = [(rng.standard_normal(P) * (30.0 if c == 2 else 0.3)).astype(np.float32) for c in range(C)]
  seeds = np.array([[c, 7] for c in range(C)], np.int64)
  rows = [torch.from_numpy(x).to(gpu) for x in xs]
  b = codec.quantize_encode_checked(rows, 0.5, torch.from_numpy(seeds), _lib.STOCHASTIC, caps=[P // 2] * C)
  assert b.quarters
  qs = [oq.stochastic_quantize(xs[c], np.float32(0.5), tuple(seeds[c])) for c in range(C)]
  _check_index(b, qs)
  s, _, err = codec.decode_accumulate(b)
  assert int(err.item()) == 0
  np.testing.assert_array_equal(s.cpu().numpy(), np.sum(np.stack(qs).astype(np.int64), axis=0).astype(np.int32))


def test_quarter_decode_tile_ranges(gpu):
  rng = np.random.default_rng(21)
  P, C = 10_300, 3
  xs = [(rng.standard_normal(P) * 1.1).astype(np.float32) for _ in range(C)]
  seeds = np.array([[1, 2], [3, 4], [5, 6]], np.int64)
  b = codec.quantize_encode([torch.from_numpy(x).to(gpu) for x in xs], 0.5, torch.from_numpy(seeds),
                            _lib.STOCHASTIC, caps=[codec.worst_case_capacity(P)] * C)
  assert b.quarters
  full, fout, err = codec.decode_accumulate(b, out=torch.empty(P, device=gpu), step=0.5)
  assert int(err.item()) == 0
  part = torch.full((P,), 999, dtype=torch.int32, device=gpu)
  pout = torch.full((P,), -1.0, dtype=torch.float32, device=gpu)
  err = torch.zeros(1, dtype=torch.int32, device=gpu)
  for tb, te in ((0, 1), (1, 6), (6, 11)):
    codec.decode_accumulate(b, sum_out=part, out=pout, step=0.5, err=err, tiles=(tb, te))
    hi = min(P, te * 1024)
    np.testing.assert_array_equal(part[:hi].cpu().numpy(), full[:hi].cpu().numpy())
    assert (part[hi:].cpu().numpy() == 999).all()
  np.testing.assert_array_equal(pout.cpu().numpy(), fout.cpu().numpy())
  assert int(err.item()) == 0


@pytest.mark.parametrize("inject", ["runs", "big", "huge", "all"])
def test_dense_single_code_table_with_unresolvable_codes(gpu, inject):
  """Dense streams (8-bit steps: every wave of quarter segments takes the LONG
  loop, which reads the single-code table first) with codes the 12-bit table
  cannot resolve mixed in: runs of 32+ zeros (the run code's prefix is too long),
  |q| >= 1024 (the magnitude's leading 1 is past the index bits), |q| ~ 2^17 (codes
  past 32 bits: slow_code and a reader restart), both signs, at unit starts and
  ends.  Codes byte-identical to the oracle, the int32 sum exact."""
  rng = np.random.default_rng(7 + len(inject))
  P, C, step = 40_000, 6, 1.0 / 127
  xs = []
  for c in range(C):
    x = (rng.standard_normal(P) * 0.25).astype(np.float32)
    if inject in ("runs", "all"):
      for s in rng.choice(P - 200, 40, replace=False):
        x[s:s + int(rng.integers(32, 140))] = 0.0
      x[256:256 + 33] = 0.0   # a run from a unit start
      x[1024 - 40:1024] = 0.0  # a run up to a tile end
    if inject in ("big", "all"):
      pos = rng.choice(P, 60, replace=False)
      x[pos] = (rng.integers(1024, 6000, pos.size) * rng.choice([-1, 1], pos.size) * step).astype(np.float32)
      x[255] = np.float32(-2047 * step)
      x[512] = np.float32(4095 * step)
    if inject in ("huge", "all"):
      pos = rng.choice(P, 8, replace=False)
      x[pos] = (rng.integers(1 << 16, 1 << 18, pos.size) * rng.choice([-1, 1], pos.size) * step).astype(np.float32)
    xs.append(x)
  seeds = np.array([[90 + c, 5 * c + 1] for c in range(C)], np.int64)
  rows = [torch.from_numpy(x).to(gpu) for x in xs]
  b = codec.quantize_encode(rows, step, torch.from_numpy(seeds), _lib.STOCHASTIC,
                            caps=[codec.worst_case_capacity(P)] * C, quarters=True)
  assert b.quarters
  qs = [oq.stochastic_quantize(xs[c], np.float32(step), tuple(seeds[c])) for c in range(C)]
  for c in range(C):
    code, nbits = ocodec.run_length_gamma_encode(qs[c])
    assert b.client_code(c) == code and int(b.bits()[c]) == nbits
  assert float(np.mean(b.bits().astype(np.float64))) / P >= 8.0  # dense: mostly LONG-loop waves
  s, _, err = codec.decode_accumulate(b)
  assert int(err.item()) == 0
  np.testing.assert_array_equal(s.cpu().numpy(),
                                np.sum(np.stack(qs).astype(np.int64), axis=0).astype(np.int32))

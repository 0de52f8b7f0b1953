"""GPU edge cases of the round plumbing against the oracle.

* One-bit SGD / DRIVE distortion on offset, low-variance clients (x = 1000 +-
  1e-3): the one-pass expansion sum x^2 - 2 m sum x + n m^2 cancels there, so
  those clients are recomputed term by term (k_mask_distortion), as TF computes
  sum (x - decoded)^2 (one_bit_sgd.py:76-78, drive.py:69-70).
* Partial overflow: in a batch of small and large clients only some overflow
  their stream capacity; only those are re-encoded and the batch is re-packed
  (codec._repack) -- every mode, with per-client norms and fused pre-scales.
* A client zeroed by the zeroing wrapper (or weighted 0) under a normalisation:
  norm 0, client step 0, x / 0 = NaN, cast to int32 = INT32_MIN on TF-CPU's x86
  cast (quantize_utils.py:33-36 with quantize_encode.py:145) -- the HIP path
  reproduces that literally.  The reference's behaviour here is parity unpinned
  (no reference test covers it); the oracle restates TF's semantics.
* Stream capacities sized from the previous round (codec.CapacityHint): a dense
  round (~10 bits / element) overflows the default capacity once, then not.
"""
import numpy as np
import pytest
import torch

from federated_amd import _lib
from federated_amd import codec
from federated_amd.aggregators import quantize_encode
from oracle import aggregators as oagg
from oracle import codec as ocodec
from oracle import quantize_utils as oq

pytestmark = pytest.mark.gpu
F32 = np.float32
MODES = {"uniform": _lib.UNIFORM, "stochastic": _lib.STOCHASTIC, "dithered": _lib.DITHERED}
ORACLE_Q = {"uniform": lambda x, s, sd: oq.uniform_quantize(x, s), "stochastic": oq.stochastic_quantize,
            "dithered": oq.dithered_quantize}


def _offset_clients(P):
  rng = np.random.default_rng(17)
  return [
      (F32(1000.0) + rng.standard_normal(P).astype(np.float32) * F32(1e-3)).astype(np.float32),
      (F32(-250.0) + rng.standard_normal(P).astype(np.float32) * F32(1e-4)).astype(np.float32),
      np.where(rng.random(P) < 0.5, F32(500.0), F32(-500.0)).astype(np.float32)
      + (rng.standard_normal(P) * 1e-3).astype(np.float32),
      rng.standard_normal(P).astype(np.float32),
  ]


@pytest.mark.parametrize("P", [4099, 300_001])
def test_onebit_distortion_offset_low_variance(gpu, P):
  xs = _offset_clients(P)
  masks, means, dist = codec.onebit_encode([torch.from_numpy(x).to(gpu) for x in xs], 0.0)
  d = dist.cpu().numpy()
  m = means.cpu().numpy()
  for c, x in enumerate(xs):
    _, meas = oagg.one_bit_sgd_next([x], 0.0)
    # the oracle's distortion with the HIP means (isolates the distortion sum
    # from the float32 means' own reduction order)
    dec = np.where(x >= 0, m[2 * c + 1], m[2 * c]).astype(np.float32)
    want = np.sum((x - dec).astype(np.float64) ** 2)
    np.testing.assert_allclose(d[c], want, rtol=1e-6)
    np.testing.assert_allclose(d[c] / P, meas["avg_distortion"], rtol=1e-4)


@pytest.mark.parametrize("scaling", ["unbiased", "min_distortion"])
def test_drive_distortion_offset_low_variance(gpu, scaling):
  P = 70_001
  xs = _offset_clients(P)
  _, means, dist = codec.drive_encode([torch.from_numpy(x).to(gpu) for x in xs],
                                      min_distortion=scaling == "min_distortion")
  d = dist.cpu().numpy()
  m = means.cpu().numpy()
  for c, x in enumerate(xs):
    dec = np.where(x < 0, m[2 * c], m[2 * c + 1]).astype(np.float32)
    np.testing.assert_allclose(d[c], np.sum((x - dec).astype(np.float64) ** 2), rtol=1e-6)
    _, meas = oagg.drive_next([x], scaling)
    np.testing.assert_allclose(d[c] / P, meas["avg_distortion"], rtol=1e-4)


@pytest.mark.parametrize("mode", list(MODES))
def test_partial_overflow_repack_matches_oracle(gpu, mode):
  """Clients 1, 4 and 5 code at ~8-10 bits / element and overflow a 3-bit/element
  capacity; the others fit.  Norms (max magnitude: bit-exact) and fused
  pre-scales (x * s0) * w are on.  Bytes, bit counts, the decoder index (via the
  decoded sum) and the measurements must equal the oracle."""
  P, C, step = 50_003, 7, 0.05
  rng = np.random.default_rng(3)
  sig = [0.01, 2.0, 0.02, 0.001, 1.5, 3.0, 0.005]
  dense = {1, 4, 5}  # max-magnitude normalisation: q spans +-20 wherever x is nonzero
  xs = [(rng.standard_normal(P) * s * (1.0 if c in dense else (rng.random(P) < 0.02))).astype(np.float32)
        for c, s in enumerate(sig)]
  pre = np.array([[1.0, 1.0], [0.5, 3.0], [1.0, 0.25], [2.0, 1.0], [1.0, 1.0], [0.75, 1.5], [1.0, 2.0]],
                 np.float32)
  seeds = np.array([[40 + c, 9 * c] for c in range(C)], np.int64)
  rows = [torch.from_numpy(x).to(gpu) for x in xs]
  pre_d = torch.from_numpy(pre).to(gpu)
  norms = codec.client_norms(rows, _lib.NORM_MAX_MAGNITUDE, prescale=pre_d)
  caps = [codec._round_up(3 * P // 8 + 256, 64)] * C  # pylint: disable=protected-access
  first = codec.quantize_encode(rows, step, torch.from_numpy(seeds), MODES[mode], norms=norms, caps=caps,
                                prescale=pre_d)
  ovf = set(codec.check_overflow(first).tolist())
  assert ovf and len(ovf) < C, ovf
  batch = codec.quantize_encode_checked(rows, step, torch.from_numpy(seeds), MODES[mode], norms=norms, caps=caps,
                                        prescale=pre_d)
  assert not len(codec.check_overflow(batch))
  acc = np.zeros(P, np.int64)
  dists, nnzs = codec.finalize(batch)
  for c in range(C):
    v = ((xs[c] * pre[c, 0]) * pre[c, 1]).astype(np.float32)
    s = F32(oq.max_magnitude(v) * F32(step))
    q = ORACLE_Q[mode](v, s, tuple(seeds[c]))
    code, nbits = ocodec.run_length_gamma_encode(q)
    assert int(batch.bits()[c]) == nbits, c
    assert batch.client_code(c) == code, c
    assert int(nnzs[c]) == np.count_nonzero(q)
    acc += q
  s, _, err = codec.decode_accumulate(batch)
  assert int(err.item()) == 0
  np.testing.assert_array_equal(s.cpu().numpy(), oagg.wrap_i32(acc))


@pytest.mark.parametrize("norm", ["mean_magnitude", "max_magnitude", "dimensionless_norm"])
def test_zeroed_client_under_normalization(gpu, norm):
  P = 5000
  rng = np.random.default_rng(8)
  xs = [rng.standard_normal(P).astype(np.float32), np.zeros(P, np.float32),
        rng.standard_normal(P).astype(np.float32)]
  seeds = np.array([[1, 2], [3, 4], [5, 6]], np.int64)
  process = quantize_encode.QuantizeEncodeFactory(0.5, "stochastic", normalization_type=norm).create(
      (np.float32, (P,)))
  out = process.next(process.initialize(), xs, seeds=seeds)
  want, meas, codes = oagg.quantize_encode_next(xs, 0.5, "stochastic", seeds=seeds, normalization_type=norm)
  assert oq.stochastic_quantize(xs[1], F32(0.0), (3, 4))[0] == np.iinfo(np.int32).min
  np.testing.assert_array_equal(out.result.view(np.uint32), want.view(np.uint32))
  assert out.measurements["avg_bitrate"] == meas["avg_bitrate"]
  assert out.measurements["avg_sparsity"] == meas["avg_sparsity"]


def test_capacity_hint_sizes_the_next_round(gpu):
  """8-bit steps (~10 bits / element) overflow the default 4-bit capacity in the
  first round only; the second round is sized from the first."""
  P, C, step = 1 << 18, 6, 1.0 / 127
  rows = [torch.randn(P, device=gpu) * 0.25 for _ in range(C)]
  seeds = torch.tensor([[c, c] for c in range(C)], dtype=torch.int64)
  hint = codec.CapacityHint()
  b1 = codec.quantize_encode(rows, step, seeds, _lib.STOCHASTIC, caps=hint.caps(P, C))
  assert len(codec.check_overflow(b1)) == C
  hint.update(b1)
  b2 = codec.quantize_encode(rows, step, seeds + 100, _lib.STOCHASTIC, caps=hint.caps(P, C))
  assert not len(codec.check_overflow(b2))
  assert hint.caps(P, C)[0] < codec.worst_case_capacity(P)
  np.testing.assert_array_equal(b2.bits() > 9 * P, np.ones(C, bool))


def _gamma_bits(n):
  """Elias gamma of n >= 1 as a bit string (TFC run-length gamma, elias_gamma_encode.py:30-45)."""
  b = bin(int(n))[2:]
  return "0" * (len(b) - 1) + b


def test_oversized_run_inside_a_segment_is_flagged(gpu):
  """the decoder reduces a run modulo 2^28 only for a segment's FIRST code
  (whose run starts at the index's previous nonzero, kept modulo 2^28).  A later code
  whose run leaves the tile is malformed and must set err -- before the fix, a run of
  2^28 + 5 from element 0 wrapped back to element 5 and was summed, unflagged.  The
  stream is decoded through an encoder-style index (not rebuilt from the bytes)."""
  P = 1024
  bits = _gamma_bits(1) + "1" + _gamma_bits(1)                # element 0: +1
  bits += _gamma_bits((1 << 28) + 5) + "1" + _gamma_bits(1)  # run 2^28 + 5 (57 bits): out of the tile
  nbits = len(bits)
  padded = bits + "0" * (-nbits % 8)
  code = bytes(int(padded[i:i + 8], 2) for i in range(0, len(padded), 8))
  batch = codec.EncodedBatch(P, 1, [256], gpu)
  buf = np.zeros(batch.stream.numel(), np.uint8)
  buf[:len(code)] = np.frombuffer(code, np.uint8)
  batch.stream.copy_(torch.from_numpy(buf).to(gpu))
  # encoder index of one tile: starts at bit 0 with no earlier nonzero; the tile's
  # codes end at nbits (no trailing code), its last nonzero claimed at element 5
  batch.idx.copy_(torch.tensor([0, nbits | (6 << 36)], dtype=torch.int64, device=gpu))
  batch.total_bits.fill_(nbits)
  s, _, err = codec.decode_accumulate(batch)
  assert int(err.item()) != 0
  # the well-formed prefix alone (element 0 only) decodes cleanly
  ok_bits = _gamma_bits(1) + "1" + _gamma_bits(1) + _gamma_bits(P)
  padded = ok_bits + "0" * (-len(ok_bits) % 8)
  code = bytes(int(padded[i:i + 8], 2) for i in range(0, len(padded), 8))
  buf[:] = 0
  buf[:len(code)] = np.frombuffer(code, np.uint8)
  batch.stream.copy_(torch.from_numpy(buf).to(gpu))
  head = len(ok_bits) - len(_gamma_bits(P))
  batch.idx.copy_(torch.tensor([0, head | (1 << 36)], dtype=torch.int64, device=gpu))
  s, _, err = codec.decode_accumulate(batch)
  assert int(err.item()) == 0
  want = np.zeros(P, np.int32)
  want[0] = 1
  np.testing.assert_array_equal(s.cpu().numpy(), want)

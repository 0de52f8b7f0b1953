"""The chained pair table of the super-tile encoder (k_encode2), against the oracle.

The chained table carries each lane's run state (distance from the lane's last
nonzero, 1-6, or "far") across the lane's four chunks; a nonzero after a far run
is coded without its run code and flagged, and the kernel prepends the exact
one from the lane's nonzero mask; a chunk off the pair table (|q| > 7 somewhere
in the wave) takes the code-table or exponent path and hands its state on.
These inputs are integer-valued, so every rounding gives q = x exactly and the
patterns below land where intended:
  - zero runs of every length 0..20 in front of nonzeros, at every offset of a
    4-element chunk and of a lane's 16 elements (states 1..6, far, lane starts);
  - lanes whose only nonzero follows a far run, and all-zero lanes;
  - isolated |q| in 8..40 that push single wave-chunks off the pair table,
    between chunks that stay on it;
  - a partial last tile.
Reference: the run-length gamma layout of elias_gamma_encode.py:97-99 (TFC),
restated in oracle/codec.py.
"""
import numpy as np
import pytest
import torch

from federated_amd import codec
from oracle import codec as ocodec
from test_gpu_codec import MODES, ORACLE_Q

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True, params=["2", "4", "8"], ids=["2tiles", "4tiles", "8tiles"])
def _super_tiles(monkeypatch, request):
  monkeypatch.setenv("FEDCODEC_ENC2", "1")
  monkeypatch.setenv("FEDCODEC_ENC_NT", request.param)


def _pattern(rng, P, outlier_rate):
  """Integer-valued float32: runs of zeros of length 0..20 (a third of them far:
  >= 6), values in +-1..7, and rare outliers 8..40 in magnitude."""
  x = np.zeros(P, np.float32)
  i = 0
  while i < P:
    r = rng.integers(0, 21) if rng.random() < 0.35 else rng.integers(0, 4)
    i += int(r)
    if i >= P:
      break
    mag = rng.integers(8, 41) if rng.random() < outlier_rate else rng.integers(1, 8)
    x[i] = float(mag if rng.random() < 0.5 else -mag)
    i += 1
  return x


def _check(gpu, xs, mode, step=1.0):
  C, P = len(xs), xs[0].size
  seeds = np.array([[7 + c, 3 * c + 1] for c in range(C)], np.int64)
  batch = codec.quantize_encode_checked([torch.from_numpy(x).to(gpu) for x in xs], step,
                                        torch.from_numpy(seeds), MODES[mode])
  bits = batch.bits()
  acc = np.zeros(P, np.int64)
  for c in range(C):
    q = ORACLE_Q[mode](xs[c], step, tuple(seeds[c]))
    if mode != "dithered":
      np.testing.assert_array_equal(q, xs[c].astype(np.int32))  # integer inputs: q = x
    code, nbits = ocodec.run_length_gamma_encode(q)
    assert bits[c] == nbits, c
    assert batch.client_code(c) == code, c
    acc += q
  s, _, err = codec.decode_accumulate(batch)
  assert int(err.item()) == 0
  np.testing.assert_array_equal(s.cpu().numpy(), acc.astype(np.int32))


@pytest.mark.parametrize("mode", ["uniform", "stochastic"])
@pytest.mark.parametrize("outlier_rate", [0.0, 0.002, 0.05])
def test_chain_runs_and_outliers_match_oracle(gpu, mode, outlier_rate):
  rng = np.random.default_rng(int(outlier_rate * 1000) + len(mode))
  P = 3 * 4096 + 777  # partial last tile
  xs = [_pattern(rng, P, outlier_rate) for _ in range(4)]
  _check(gpu, xs, mode)


def test_chain_every_run_length_at_every_chunk_offset(gpu):
  """One nonzero per lane: lane l's 16 elements hold a single +-k after a run that
  starts in the previous lane, so the run crosses lane and chunk boundaries at
  every offset; plus lanes with two nonzeros d apart (states 1..6 and far inside
  the lane)."""
  P = 4 * 4096
  x = np.zeros(P, np.float32)
  for lane in range(P // 16):
    base = 16 * lane
    if lane % 3 == 0:
      continue  # all-zero lane
    k = 1 + (lane % 7)
    pos = (lane * 5) % 16
    x[base + pos] = k if lane % 2 else -k
    if lane % 3 == 1:
      d = 1 + (lane // 3) % 15  # second nonzero d after the first, inside the lane
      if pos + d < 16:
        x[base + pos + d] = -(1 + (lane % 5))
  y = x.copy()
  y[::97] = 9.0  # a sprinkle of off-table chunks
  _check(gpu, [x, y, -x], "uniform")


def test_chain_dithered_partial_tile(gpu):
  """Dithered rounding (the masked partial-tile variant of the chunk code) on sparse
  small values: q is not x here, the oracle decides."""
  rng = np.random.default_rng(5)
  P = 2 * 4096 + 1001
  xs = [(_pattern(rng, P, 0.01) * np.float32(0.3)).astype(np.float32) for _ in range(3)]
  _check(gpu, xs, "dithered", step=0.3)

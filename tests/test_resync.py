"""The self-synchronisation fc_build_index relies on (CPU).

fc_build_index parses each 4096-bit chunk of a bare run-length gamma code from a
GUESSED start (the chunk's first bit) and stitches the chunks by replaying that
parse beside the true one until they meet.  That is cheap only if a parse from a
random bit reaches a true code start within a small fraction of a chunk.  Measured
here on the oracle's codes (the CPU restatement of TFC's coder) over densities from
0.2 to 10 bits per element: from random bits, the distance to the first true code
start a parse lands on.
"""
import numpy as np

from oracle import codec as ocodec
from oracle import quantize_utils as oq

F32 = np.float32


def _bits(code):
  return np.unpackbits(np.frombuffer(code, np.uint8))


def _parse_code(b, p):
  """One (run, sign, magnitude) code at bit p: the next start, or -1 if it does not parse."""
  n = b.size
  for part in range(2):
    z = 0
    while p < n and b[p] == 0:
      z += 1
      p += 1
      if z > 31:
        return -1
    if p + z + 1 > n:
      return -1
    p += z + 1
    if part == 0:
      if p >= n:
        return -1
      p += 1  # sign bit
  return p


def _sync_distances(q, starts):
  code, _ = ocodec.run_length_gamma_encode(q)
  b = _bits(code)
  true_starts = set()
  p = 0
  while p >= 0 and p < b.size:
    true_starts.add(p)
    p = _parse_code(b, p)
  out = []
  for s in starts:
    p = int(s)
    while p >= 0 and p not in true_starts:
      p = _parse_code(b, p)
    out.append(p - s if p >= 0 else -1)
  return np.array(out), b.size


def test_random_start_parses_resynchronise_within_a_chunk_fraction():
  rng = np.random.default_rng(1)
  P = 1 << 17
  x = rng.standard_normal(P).astype(F32)
  cases = {
      "headline 3.8 bits": oq.stochastic_quantize(x, F32(0.5), (1, 1)),
      "8-bit steps 10 bits": oq.stochastic_quantize(x * F32(0.25), F32(1.0 / 127), (1, 1)),
      "config 3, 2.7 bits": oq.stochastic_quantize(x, F32(1.0), (1, 1)),
      "sparse 1 bit": oq.stochastic_quantize(x * F32(0.1), F32(0.5), (1, 1)),
      "very sparse 0.2 bits": oq.stochastic_quantize(x * F32(0.01), F32(0.5), (1, 1)),
  }
  for name, q in cases.items():
    nbits = ocodec.encoded_bits(q)
    starts = np.sort(rng.integers(0, max(1, nbits - 4096), 300))
    d, _ = _sync_distances(q, starts)
    ok = d[d >= 0]
    assert ok.size >= 0.95 * d.size, name  # (a parse may fail: k_idx_sync then takes the true parse)
    assert ok.mean() < 100 and ok.max() < 2048, (name, ok.mean(), ok.max())

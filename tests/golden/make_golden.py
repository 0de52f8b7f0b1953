"""Generate the committed golden fixtures from the CPU oracle.

python tests/golden/make_golden.py   (writes tests/golden/golden.npz)

The oracle itself is pinned by the reference's known-answer tests and the
Random123 Philox vectors (tests/test_oracle.py); these fixtures freeze its
outputs on small seeded inputs (every rounding mode, several steps and seeds,
special values, ragged sizes, all-zero / no-zero / extreme integer tensors) so
the HIP path can be checked against them without recomputing the oracle.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle import aggregators as oagg  # noqa: E402
from oracle import codec as ocodec  # noqa: E402
from oracle import quantize_utils as oq  # noqa: E402

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden.npz")

SPECIAL = np.array([0.0, -0.0, 1e-45, -1e-45, 1e-39, 1.1754944e-38, 0.5, -0.5, 1.5, 2.5, -2.5,
                    0.25, 0.75, 1.0, -1.0, 3.0, 1e30, -1e30, np.inf, -np.inf, np.nan, 2.0**31,
                    -2.0**31, 2.0**31 - 128, 1e-20, 7.0], np.float32)
SEEDS = [(0, 0), (1, 1), (2**40 + 7, 3)]
STEPS = [0.5, 0.4, 1.0 / 127, 1.0]
MODES = ["uniform", "stochastic", "dithered"]
QFN = {"uniform": lambda x, s, sd: oq.uniform_quantize(x, s), "stochastic": oq.stochastic_quantize,
       "dithered": oq.dithered_quantize}


def int_cases(rng):
  cases = {}
  for P in (1, 3, 4, 5, 1023, 4099):
    q = rng.integers(-3, 4, P).astype(np.int32)
    q[rng.random(P) < 0.7] = 0
    cases["sparse_%d" % P] = q
  cases["zeros_4099"] = np.zeros(4099, np.int32)
  cases["nozero_777"] = (rng.integers(1, 50, 777) * rng.choice([-1, 1], 777)).astype(np.int32)
  cases["extreme_64"] = rng.choice(np.array([-2**31, 2**31 - 1, 1, -1, 0], np.int32), 64)
  cases["ref_a"] = np.array([-5, 3, 0, 0], np.int32)   # elias_gamma_encode_test.py:32-37
  cases["ref_b"] = np.array([-3, 1, 0, 0], np.int32)
  return cases


def main():
  rng = np.random.default_rng(20251015)
  g = {}
  x = np.concatenate([rng.standard_normal(700).astype(np.float32) * 3, SPECIAL])
  g["q_x"] = x
  for m in MODES:
    for si, s in enumerate(STEPS):
      for ki, sd in enumerate(SEEDS):
        g["q_%s_%d_%d" % (m, si, ki)] = QFN[m](x, np.float32(s), sd)
  g["noise_3_9"] = oq.generate_noise((3, 9), 1001)
  for name, q in int_cases(rng).items():
    code, nbits = ocodec.run_length_gamma_encode(q)
    g["rl_in_" + name] = q
    g["rl_code_" + name] = np.frombuffer(code, np.uint8)
    g["rl_bits_" + name] = np.int64(nbits)
  xs = [(rng.standard_normal(5000) * 0.8).astype(np.float32) for _ in range(3)]
  g["round_x"] = np.stack(xs)
  for m in MODES:
    res, meas, codes = oagg.quantize_encode_next(xs, 0.5, m, seeds=SEEDS)
    g["round_%s_result" % m] = res
    g["round_%s_bitrate" % m] = meas["avg_bitrate"]
    g["round_%s_distortion" % m] = meas["avg_distortion"]
    g["round_%s_sparsity" % m] = meas["avg_sparsity"]
    for c, code in enumerate(codes):
      g["round_%s_code_%d" % (m, c)] = np.frombuffer(code, np.uint8)
  res, meas = oagg.one_bit_sgd_next(xs, 0.1)
  g["onebit_result"] = res
  g["onebit_distortion"] = meas["avg_distortion"]
  np.savez_compressed(OUT, **g)
  print("wrote %s (%d arrays, %d bytes)" % (OUT, len(g), os.path.getsize(OUT)))


if __name__ == "__main__":
  main()

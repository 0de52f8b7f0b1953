"""Diagnostic: time the auxiliary kernels of the §8 rows at bench-like sizes.

client norms (QSGD / wrappers), dithered noise sum, step-size vote lengths,
elementwise quantise / dequantise, Hadamard rotation.  Prints ms and the fp32-read rate of each.
"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from federated_amd import _lib, codec  # noqa: E402

dev = torch.device("cuda:0")


def timed(name, fn, nbytes, reps=3):
  fn()
  torch.cuda.synchronize()
  t0 = time.perf_counter()
  for _ in range(reps):
    fn()
  torch.cuda.synchronize()
  dt = (time.perf_counter() - t0) / reps
  print("%-34s %9.2f ms  %7.0f GB/s" % (name, dt * 1e3, nbytes / dt / 1e9), flush=True)


P = 25_000_000
C = int(os.environ.get("C", 256))
g = torch.Generator(device=dev)
rows = []
for c in range(C):
  g.manual_seed(11 + c)
  rows.append(torch.randn(P, generator=g, device=dev))
seeds = torch.tensor([[c, c + 1] for c in range(C)], dtype=torch.int64, device=dev)
timed("client_norms L2 (C x 25M)", lambda: codec.client_norms(rows, _lib.NORM_L2), C * P * 4)
timed("noise_sum dithered (C x 25M)", lambda: codec.noise_sum(seeds, P, dev), P * 4)
timed("vote_lengths K=4 (64 x 25M)",
      lambda: codec.vote_lengths(rows[:64], np.array([0.25, 0.5, 1.0, 2.0], np.float32), seeds[:64],
                                 _lib.STOCHASTIC), 64 * P * 4, reps=1)
big = torch.randn(1 << 25, generator=g, device=dev)  # 128 MiB (P limit 2^26 - 1)
timed("quantize stochastic (2^25, q out)", lambda: codec.quantize(big, 0.5, (1, 2), _lib.STOCHASTIC), (1 << 25) * 8)
timed("dequantize (2^25)", lambda: codec.dequantize(big.view(torch.int32), 0.5), (1 << 25) * 8)
del big
H = [torch.randn(1 << 24, generator=g, device=dev) for _ in range(64)]
timed("hadamard 64 x 2^24 (fwd)", lambda: codec.hadamard_(H, (1, 2)), 64 * (1 << 24) * 4 * 2)
del H
# QSGD server sum (qsgd.py:85-112): the clients' q rows decoded into int32 planes (groups of <= 1 GiB), then
# k_sum_planes adds float(q_c) * step_c in client order.  Traffic: code read + 4P write + 4P read per client.
ns = codec.client_norms(rows, _lib.NORM_L2)
steps = (ns / 16.0).contiguous()  # num_steps 16
qb = codec.quantize_encode_checked(rows, 1.0, seeds, _lib.STOCHASTIC, norms=steps)
code_bytes = int(qb.nbytes().sum())
ws = torch.empty(int(_lib.load().fc_decode_scaled_workspace_bytes(C, P)), dtype=torch.uint8, device=dev)
qout = torch.empty(P, dtype=torch.float32, device=dev)
timed("qsgd decode+ordered sum (C x 25M)", lambda: codec.decode_accumulate_scaled(qb, steps, out=qout, workspace=ws),
      code_bytes + C * P * 8)
timed("qsgd decode+ordered sum, int8 rows", lambda: codec.decode_accumulate_scaled(qb, steps, out=qout, workspace=ws,
                                                                              qmax=17), code_bytes + C * P * 3)
timed("int32 sum decode, same codes", lambda: codec.decode_accumulate(qb, want_sum=False, out=qout, step=1.0),
      code_bytes + P * 4)
# Server decode of bare TFC strings (VERDICT r03 "next" 2): the decoder index rebuilt from the code bytes
# alone (fc_build_index), then the same decode -- against the decode with the encoder's index above.
nbq = np.asarray(qb.nbytes(), np.int64)
nbt = torch.from_numpy(nbq).to(dev)
timed("fc_build_index, same codes (bare strings)",
      lambda: codec.index_codes(qb, nbt, int(nbq.max()), quarters=codec.quarter_index_wanted(C), check=False),
      code_bytes)

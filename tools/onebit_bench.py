"""Diagnostic: time the one-bit SGD codec (fc_onebit_encode + fc_onebit_decode_sum) and DRIVE encode on C x P."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from federated_amd import codec  # noqa: E402

P = int(os.environ.get("P", 25_000_000))
C = int(os.environ.get("C", 1024))
dev = torch.device("cuda:0")
g = torch.Generator(device=dev)
rows = []
for c in range(C):
  g.manual_seed(7 + c)
  rows.append(torch.randn(P, generator=g, device=dev))
for it in range(3):
  torch.cuda.synchronize()
  t0 = time.perf_counter()
  masks, means, dist = codec.onebit_encode(rows)
  torch.cuda.synchronize()
  t1 = time.perf_counter()
  out = codec.onebit_decode_sum(masks, means, C, P)
  torch.cuda.synchronize()
  t2 = time.perf_counter()
  codec.drive_encode(rows)
  torch.cuda.synchronize()
  t3 = time.perf_counter()
  print("onebit C=%d P=%d: encode %.2f ms (%.0f GB/s fp32 read), decode-sum %.2f ms, DRIVE encode %.2f ms" % (
      C, P, (t1 - t0) * 1e3, C * P * 4 / (t1 - t0) / 1e9, (t2 - t1) * 1e3, (t3 - t2) * 1e3))

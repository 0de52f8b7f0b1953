"""Diagnostic: time k_decode alone on C clients x P (encode once, decode N times).

C, P, STEP (0.5), SIGMA (1.0), ITERS from the environment."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from federated_amd import _lib, codec  # noqa: E402

P = int(os.environ.get("P", 25_000_000))
C = int(os.environ.get("C", 128))
STEP = float(os.environ.get("STEP", 0.5))
SIGMA = float(os.environ.get("SIGMA", 1.0))
dev = torch.device("cuda:0")
g = torch.Generator(device=dev)
g.manual_seed(1)
pool = [torch.randn(P, generator=g, device=dev) * SIGMA for _ in range(4)]
rows = [pool[c % 4] for c in range(C)]
ptrs = torch.tensor([r.data_ptr() for r in rows], dtype=torch.int64, device=dev)
seeds = torch.tensor([[c, c] for c in range(C)], dtype=torch.int64, device=dev)
batch = codec.EncodedBatch(P, C, [2 * P + 1024] * C, dev)  # 16 bits per element
codec.quantize_encode(None, STEP, seeds, _lib.STOCHASTIC, ptrs=ptrs, P=P, out=batch)
out = torch.empty(P, dtype=torch.float32, device=dev)
print("code bytes %d (%.3f bits per element)" % (int(batch.nbytes().sum()), 8.0 * batch.nbytes().sum() / (C * P)),
      flush=True)
ts = []
for it in range(int(os.environ.get("ITERS", 3))):
  torch.cuda.synchronize()
  t0 = time.perf_counter()
  codec.decode_accumulate(batch, want_sum=False, out=out, step=STEP)
  torch.cuda.synchronize()
  ts.append((time.perf_counter() - t0) * 1e3)
  print("decode %d clients: %.3f ms" % (C, ts[-1]))
if len(ts) > 1:  # the last line: the median of the calls after the first
  rest = sorted(ts[1:])
  print("decode %d clients: median %.3f ms" % (C, rest[len(rest) // 2]))

"""Diagnostic: cost of the exact-path re-encode (a client with one value past the fast path's |q| < 8192)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from federated_amd import _lib, codec  # noqa: E402

P = int(os.environ.get("P", 25_000_000))
C = int(os.environ.get("C", 1024))
dev = torch.device("cuda:0")
g = torch.Generator(device=dev)
rows = []
for c in range(C):
  g.manual_seed(77 + c)
  rows.append(torch.randn(P, generator=g, device=dev))
ptrs = torch.tensor([r.data_ptr() for r in rows], dtype=torch.int64, device=dev)
seeds = torch.tensor([[c, c] for c in range(C)], dtype=torch.int64, device=dev)
batch = codec.EncodedBatch(P, C, [P + 1024] * C, dev)
for nslow in [0, 1, 4, 16]:
  for c in range(nslow):
    rows[c][12345] = 1e6  # |q| = 2e6 at step 0.5: a code past the fast path
  ts = []
  for it in range(3):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    codec.quantize_encode(None, 0.5, seeds, _lib.STOCHASTIC, ptrs=ptrs, P=P, out=batch)
    e1.record()
    torch.cuda.synchronize()
    if it:
      ts.append(e0.elapsed_time(e1))
  print("slow clients %2d: encode %.2f ms" % (nslow, min(ts)), flush=True)

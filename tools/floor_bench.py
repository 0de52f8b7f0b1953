"""Diagnostic: the encoder's arithmetic floor at the headline size (VERDICT r03 "next" 5).

fc_quantize_floor reads x, draws TF's Philox stream and applies the exact
quantiser + distortion + nonzero count, with no coding; fc_quantize_encode does
all of that plus the run-length gamma code.  Same 1024 x 25 M deltas, same seeds;
HIP-event times on one stream, and the floor's per-tile nonzero counts checked
against the encoder's (same q).
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from federated_amd import _lib, codec  # noqa: E402

HBM = 8.0e12
dev = torch.device("cuda:0")
C, P = int(os.environ.get("C", 1024)), 25_000_000
T = codec.num_tiles(P)
g = torch.Generator(device=dev)
rows = []
for c in range(C):
  g.manual_seed(20251015 + c)
  rows.append(torch.randn(P, generator=g, device=dev))
ptrs = torch.tensor([r.data_ptr() for r in rows], dtype=torch.int64, device=dev)
seeds = torch.tensor([[1000 + c, 1000 + c] for c in range(C)], dtype=torch.int64, device=dev)
dist = torch.empty(C * T, dtype=torch.float32, device=dev)
nnz = torch.empty(C * T, dtype=torch.int32, device=dev)
ws = torch.empty(16 * C, dtype=torch.uint8, device=dev)
batch = codec.EncodedBatch(P, C, [int(P * 0.56)] * C, dev)


def ev(fn, reps=5):
  fn()
  torch.cuda.synchronize()
  e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
  e0.record()
  for _ in range(reps):
    fn()
  e1.record()
  torch.cuda.synchronize()
  return e0.elapsed_time(e1) / reps


for name, mode in (("stochastic", _lib.STOCHASTIC), ("uniform", _lib.UNIFORM)):
  floor = lambda: _lib.call("fc_quantize_floor", _lib.ptr(ptrs), C, P, 0.5, _lib.ptr(seeds), mode, _lib.ptr(dist),
                            _lib.ptr(nnz), _lib.ptr(ws), ws.numel(), _lib.stream_handle())
  t_floor = ev(floor)
  t_enc = ev(lambda: codec.quantize_encode(None, 0.5, seeds, mode, ptrs=ptrs, P=P, out=batch))
  assert not len(codec.check_overflow(batch))
  same = bool(torch.equal(nnz.view(C, T).sum(1), batch.nnz_part.view(C, T).sum(1)))
  S = float(batch.nbytes().astype(np.float64).sum())
  print("%-10s floor %.2f ms (%.3f of 8 TB/s on the 4P read)  encode %.2f ms (%.3f on 4P + code)  "
        "nonzeros equal: %s" % (name, t_floor, C * 4.0 * P / (t_floor * 1e-3) / HBM, t_enc,
                                (C * 4.0 * P + S) / (t_enc * 1e-3) / HBM, same), flush=True)

"""Diagnostic: k_encode(2) time of several library builds on ONE set of inputs.

LIBS="a.so b.so ..." C=1024 P=25000000 python tools/diag/enc_ablate.py
Encode only (ablation builds write streams the decoder must not be fed); HIP
events, median of REPS, stochastic and uniform modes, step 0.5.  CAP: stream capacity
in bytes per element (it is also the encoder's density hint).
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from federated_amd import _lib, codec  # noqa: E402

P = int(os.environ.get("P", 25_000_000))
C = int(os.environ.get("C", 1024))
REPS = int(os.environ.get("REPS", 5))
SEG = int(os.environ["SEGMENTS"]) if os.environ.get("SEGMENTS") else None  # None: codec.auto_segments
dev = torch.device("cuda:0")
g = torch.Generator(device=dev)
rows = []
for c in range(C):
  g.manual_seed(77 + c)
  rows.append(torch.randn(P, generator=g, device=dev))
ptrs = torch.tensor([r.data_ptr() for r in rows], dtype=torch.int64, device=dev)
seeds = torch.tensor([[c, c] for c in range(C)], dtype=torch.int64, device=dev)
batch = codec.EncodedBatch(P, C, [int(P * float(os.environ.get("CAP", 1.0))) + 1024] * C, dev)  # CAP bytes/element (< 0.8: four-tile tickets)
s = torch.cuda.current_stream()
for path in os.environ["LIBS"].split():
  _lib._lib = None  # pylint: disable=protected-access
  _lib.LIB_PATH = path
  codec._WS.buf = None  # pylint: disable=protected-access
  for mode in (_lib.STOCHASTIC, _lib.UNIFORM):
    ts = []
    for it in range(REPS + 1):
      e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
      e0.record(s)
      codec.quantize_encode(None, 0.5, seeds, mode, ptrs=ptrs, P=P, out=batch, stream=s, segments=SEG)
      e1.record(s)
      torch.cuda.synchronize()
      if it:
        ts.append(e0.elapsed_time(e1))
    ts.sort()
    print("%-34s mode=%d C=%d seg=%s enc2=%s  encode %.3f ms" % (os.path.basename(path), mode, C, SEG,
          os.environ.get("FEDCODEC_ENC2", "auto"), ts[len(ts) // 2]), flush=True)

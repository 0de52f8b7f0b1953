"""Diagnostic: does a decode co-scheduled with the encoder hide under it?

Encodes batch B (1024 x 25 M, stochastic step 0.5) on one stream while batch A
(the same deltas, other seeds, encoded beforehand) decodes on a second stream --
independent work, so the pair shows what co-residency of the VALU-bound encoder
and the latency-bound decoder can buy before building a fused work-queue kernel
(VERDICT r03 "next" 3).  Sequential pair vs concurrent pair, over encoder grid
caps (FEDCODEC_ENC_GRID, waves) and decoder grids (FEDCODEC_DEC_GRID, workgroups).
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from federated_amd import _lib, codec  # noqa: E402

dev = torch.device("cuda:0")
C, P = int(os.environ.get("C", 1024)), 25_000_000
g = torch.Generator(device=dev)
rows = []
for c in range(C):
  g.manual_seed(20251015 + c)
  rows.append(torch.randn(P, generator=g, device=dev))
ptrs = torch.tensor([r.data_ptr() for r in rows], dtype=torch.int64, device=dev)
sa = torch.tensor([[1000 + c, 1000 + c] for c in range(C)], dtype=torch.int64, device=dev)
sb = sa + 7919
caps = [int(P * 0.56)] * C
A = codec.EncodedBatch(P, C, caps, dev)
B = codec.EncodedBatch(P, C, caps, dev)
codec.quantize_encode(None, 0.5, sa, _lib.STOCHASTIC, ptrs=ptrs, P=P, out=A)
torch.cuda.synchronize()  # (A's encode done before any encode on another stream starts)
out = torch.empty(P, dtype=torch.float32, device=dev)
s1 = torch.cuda.Stream()
s2 = torch.cuda.Stream()


def enc(stream):
  codec.quantize_encode(None, 0.5, sb, _lib.STOCHASTIC, ptrs=ptrs, P=P, out=B, stream=stream)


def dec(stream):
  codec.decode_accumulate(A, want_sum=False, out=out, step=0.5, stream=stream)


def timeit(fn, reps=3):
  fn()
  torch.cuda.synchronize()
  t0 = time.perf_counter()
  for _ in range(reps):
    fn()
  torch.cuda.synchronize()
  return (time.perf_counter() - t0) / reps * 1e3


def seq():
  enc(s1)
  dec(s1)


def conc():
  ev = torch.cuda.Event()
  ev.record(torch.cuda.current_stream())
  s1.wait_event(ev)
  s2.wait_event(ev)
  dec(s2)  # decoder first: its workgroups are placed before the persistent encoder fills the CUs
  enc(s1)
  torch.cuda.current_stream().wait_stream(s1)
  torch.cuda.current_stream().wait_stream(s2)


def setenv(k, v):
  if v is None:
    os.environ.pop(k, None)
  else:
    os.environ[k] = str(v)


for eg, dg in [(None, None), (3072, None), (3072, 256), (3072, 512), (3584, 256), (None, 256)]:
  setenv("FEDCODEC_ENC_GRID", eg)
  setenv("FEDCODEC_DEC_GRID", dg)
  te = timeit(lambda: enc(s1))
  td = timeit(lambda: dec(s1))
  ts = timeit(seq)
  tc = timeit(conc)
  print("enc grid %-5s dec grid %-5s: encode %.2f  decode %.2f  sequential %.2f  concurrent %.2f ms" % (
      eg, dg, te, td, ts, tc), flush=True)
assert not len(codec.check_overflow(B))

"""Diagnostic: the headline round in two client halves, the first half's decode
overlapped with the second half's encode (two streams, kernel-boundary ordering
only: no in-kernel cross-XCD hand-off).

  one stream:  enc(1024) -> dec(1024)
  halves:      enc(A) -> dec(A) -> enc(B) -> dec(B, + A's int32 sum)
  overlapped:  s1: enc(A) -> enc(B) -> [wait dec(A)] -> dec(B, + A's sum)
               s2:          [wait enc(A)] dec(A)
The result is the same int32 sum (checked bit for bit against the one-stream round).
Knobs swept: FEDCODEC_DEC_GRID (the concurrent decoder's workgroups), FEDCODEC_ENC_GRID.
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from federated_amd import _lib, codec  # noqa: E402

dev = torch.device("cuda:0")
C, P = int(os.environ.get("C", 1024)), 25_000_000
H = C // 2
g = torch.Generator(device=dev)
rows = []
for c in range(C):
  g.manual_seed(20251015 + c)
  rows.append(torch.randn(P, generator=g, device=dev))
ptrs = torch.tensor([r.data_ptr() for r in rows], dtype=torch.int64, device=dev)
seeds = torch.tensor([[1000 + c, 1000 + c] for c in range(C)], dtype=torch.int64, device=dev)
cap = int(P * 0.56)
FULL = codec.EncodedBatch(P, C, [cap] * C, dev)
A = codec.EncodedBatch(P, H, [cap] * H, dev)
B = codec.EncodedBatch(P, C - H, [cap] * (C - H), dev)
pa, pb = ptrs[:H].contiguous(), ptrs[H:].contiguous()
sa, sb = seeds[:H].contiguous(), seeds[H:].contiguous()
out = torch.empty(P, dtype=torch.float32, device=dev)
sumA = torch.empty(P, dtype=torch.int32, device=dev)
sum1 = torch.empty(P, dtype=torch.int32, device=dev)
sum2 = torch.empty(P, dtype=torch.int32, device=dev)
s1 = torch.cuda.Stream()
s2 = torch.cuda.Stream()


def one_stream():
  codec.quantize_encode(None, 0.5, seeds, _lib.STOCHASTIC, ptrs=ptrs, P=P, out=FULL, stream=s1)
  codec.decode_accumulate(FULL, sum_out=sum1, out=out, step=0.5, stream=s1)


def halves():
  codec.quantize_encode(None, 0.5, sa, _lib.STOCHASTIC, ptrs=pa, P=P, out=A, stream=s1)
  codec.decode_accumulate(A, sum_out=sumA, stream=s1)
  codec.quantize_encode(None, 0.5, sb, _lib.STOCHASTIC, ptrs=pb, P=P, out=B, stream=s1)
  codec.decode_accumulate(B, sum_in=sumA, sum_out=sum2, out=out, step=0.5, stream=s1)


A_GRID = None  # the side decode's workgroups only (FEDCODEC_DEC_GRID around that launch)


def overlapped():
  codec.quantize_encode(None, 0.5, sa, _lib.STOCHASTIC, ptrs=pa, P=P, out=A, stream=s1)
  e1 = torch.cuda.Event()
  e1.record(s1)
  s2.wait_event(e1)
  if A_GRID:
    os.environ["FEDCODEC_DEC_GRID"] = str(A_GRID)
  codec.decode_accumulate(A, sum_out=sumA, stream=s2)
  if A_GRID:
    os.environ.pop("FEDCODEC_DEC_GRID", None)
  e2 = torch.cuda.Event()
  e2.record(s2)
  codec.quantize_encode(None, 0.5, sb, _lib.STOCHASTIC, ptrs=pb, P=P, out=B, stream=s1)
  s1.wait_event(e2)
  codec.decode_accumulate(B, sum_in=sumA, sum_out=sum2, out=out, step=0.5, stream=s1)


def timeit(fn, reps=4):
  fn()
  torch.cuda.synchronize()
  t0 = time.perf_counter()
  for _ in range(reps):
    fn()
  torch.cuda.synchronize()
  return (time.perf_counter() - t0) / reps * 1e3


def setenv(k, v):
  if v is None:
    os.environ.pop(k, None)
  else:
    os.environ[k] = str(v)


t1 = timeit(one_stream)
th = timeit(halves)
print("one stream %.2f ms   halves in order %.2f ms" % (t1, th), flush=True)
for dg, eg in [(None, None), (768, None)]:
  setenv("FEDCODEC_DEC_GRID", dg)
  setenv("FEDCODEC_ENC_GRID", eg)
  to = timeit(overlapped)
  print("overlapped: dec grid %-5s enc grid %-5s %.2f ms" % (dg, eg, to), flush=True)
setenv("FEDCODEC_DEC_GRID", None)
setenv("FEDCODEC_ENC_GRID", None)
for ag in (256, 384, 512, 768):
  A_GRID = ag
  print("overlapped: side decode grid %d only: %.2f ms" % (ag, timeit(overlapped)), flush=True)
A_GRID = None
one_stream()
overlapped()
torch.cuda.synchronize()
assert not len(codec.check_overflow(FULL)) and not len(codec.check_overflow(A)) and not len(codec.check_overflow(B))
print("sums equal:", bool(torch.equal(sum1, sum2)), flush=True)

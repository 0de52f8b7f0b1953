"""Diagnostic: encode of client group g+1 overlapped with the decode of group g (two streams).

C clients x P split into G groups; stream E encodes the groups in order, stream D
decodes group g (accumulating the int32 sum) once its encode is done.  The
encoder's persistent grid is capped (FEDCODEC_ENC_GRID) so decoder workgroups
find room beside it.  Prints the serial and the overlapped round times.

C=1024 G=4 ENC_GRID=3072 python tools/overlap_bench.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from federated_amd import _lib, codec  # noqa: E402

P = int(os.environ.get("P", 25_000_000))
C = int(os.environ.get("C", 1024))
G = int(os.environ.get("G", 4))
REPS = int(os.environ.get("REPS", 3))
dev = torch.device("cuda:0")
g = torch.Generator(device=dev)
rows = []
for c in range(C):
  g.manual_seed(77 + c)
  rows.append(torch.randn(P, generator=g, device=dev))
Cg = C // G
ptrs = [torch.tensor([r.data_ptr() for r in rows[k * Cg:(k + 1) * Cg]], dtype=torch.int64, device=dev)
        for k in range(G)]
seeds = [torch.tensor([[c, c] for c in range(k * Cg, (k + 1) * Cg)], dtype=torch.int64, device=dev)
         for k in range(G)]
batches = [codec.EncodedBatch(P, Cg, [P + 1024] * Cg, dev) for _ in range(G)]
full = codec.EncodedBatch(P, C, [P + 1024] * C, dev)
allp = torch.tensor([r.data_ptr() for r in rows], dtype=torch.int64, device=dev)
alls = torch.tensor([[c, c] for c in range(C)], dtype=torch.int64, device=dev)
out = torch.empty(P, device=dev)
isum = torch.empty(P, dtype=torch.int32, device=dev)
err = torch.zeros(1, dtype=torch.int32, device=dev)
sE = torch.cuda.Stream()
sD = torch.cuda.Stream()


def serial():
  codec.quantize_encode(None, 0.5, alls, _lib.STOCHASTIC, ptrs=allp, P=P, out=full, stream=sE)
  codec.decode_accumulate(full, want_sum=False, out=out, step=0.5, err=err, stream=sE)


def overlapped():
  evs = []
  for k in range(G):
    codec.quantize_encode(None, 0.5, seeds[k], _lib.STOCHASTIC, ptrs=ptrs[k], P=P, out=batches[k], stream=sE)
    e = torch.cuda.Event()
    e.record(sE)
    evs.append(e)
  for k in range(G):
    sD.wait_event(evs[k])
    last = k == G - 1
    codec.decode_accumulate(batches[k], sum_in=isum if k else None, sum_out=None if last else isum,
                            out=out if last else None, want_sum=not last, step=0.5, err=err, stream=sD)


for name, fn in (("serial", serial), ("overlapped", overlapped)):
  ts = []
  for it in range(REPS + 1):
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(sE)
    fn()
    sE.wait_stream(sD)
    e1.record(sE)
    torch.cuda.synchronize()
    if it:
      ts.append(e0.elapsed_time(e1))
  print("%-10s C=%d G=%d enc_grid=%s  %.3f ms" % (name, C, G, os.environ.get("FEDCODEC_ENC_GRID", "auto"),
                                                   min(ts)), flush=True)

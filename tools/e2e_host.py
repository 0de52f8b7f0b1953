"""Host-resident round rate: H2D of the client deltas + encode + decode + D2H.

The reference round starts and ends in host memory (TFF simulation executor ->
aggregator -> server optimizer).  bench.py's headline is device-resident; this
tool times the PCIe-inclusive variant of the same round so DESIGN.md can quote
both.  Clients are copied from pinned host buffers in batches on a copy stream
while the previous batch encodes (double-buffered), then decoded and the f32
result copied back.

--codec onebit: config 5's codec (one-bit SGD, one_bit_sgd.py:45-112): the batches
are mask-encoded as they arrive, the server sum decodes all clients in order.

usage: python tools/e2e_host.py [--clients 64] [--batch 16] [--P 25000000] [--codec rlgamma|onebit]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from federated_amd import _lib, codec  # noqa: E402


def main():
  ap = argparse.ArgumentParser()
  ap.add_argument("--clients", type=int, default=64)
  ap.add_argument("--batch", type=int, default=16)
  ap.add_argument("--P", type=int, default=25_000_000)
  ap.add_argument("--reps", type=int, default=3)
  ap.add_argument("--codec", default="rlgamma", choices=["rlgamma", "onebit"])
  args = ap.parse_args()
  dev = torch.device("cuda:0")
  C, B, P = args.clients, args.batch, args.P
  assert C % B == 0
  g = torch.Generator().manual_seed(1)
  host = [torch.randn(P, generator=g).pin_memory() for _ in range(B)]  # B distinct pinned deltas, reused
  dbuf = [[torch.empty(P, device=dev) for _ in range(B)] for _ in range(2)]
  copy_s = torch.cuda.Stream()
  comp_s = torch.cuda.current_stream()
  seeds = torch.tensor([[c, c] for c in range(B)], dtype=torch.int64, device=dev)
  cap = codec._round_up(P + 256, 64)
  batches = [codec.EncodedBatch(P, B, [cap] * B, dev) for _ in range(C // B)] if args.codec == "rlgamma" else []
  out = torch.empty(P, device=dev)
  isum = torch.zeros(P, dtype=torch.int32, device=dev)
  err = torch.zeros(1, dtype=torch.int32, device=dev)
  out_host = torch.empty(P).pin_memory()
  onebit = args.codec == "onebit"
  nw = (P + 31) // 32
  if onebit:
    masks = torch.empty(C * nw, dtype=torch.int32, device=dev)
    means = torch.empty(2 * C, dtype=torch.float32, device=dev)
    dist = torch.empty(C, dtype=torch.float64, device=dev)
  h = _lib.stream_handle(comp_s)

  def round_once():
    ev = [torch.cuda.Event() for _ in range(2)]
    nb = C // B
    with torch.cuda.stream(copy_s):
      for i in range(B):
        dbuf[0][i].copy_(host[i], non_blocking=True)
      ev[0].record(copy_s)
    for k in range(nb):
      cur = k % 2
      comp_s.wait_event(ev[cur])
      if k + 1 < nb:  # next batch's H2D overlaps this batch's encode
        with torch.cuda.stream(copy_s):
          copy_s.wait_stream(comp_s)
          for i in range(B):
            dbuf[1 - cur][i].copy_(host[i], non_blocking=True)
          ev[1 - cur].record(copy_s)
      ptrs = torch.tensor([t.data_ptr() for t in dbuf[cur]], dtype=torch.int64, device=dev)
      if onebit:
        _lib.call("fc_onebit_encode", _lib.ptr(ptrs), B, P, 0.0, _lib.ptr(masks[k * B * nw:]),
                  _lib.ptr(means[2 * k * B:]), _lib.ptr(dist[k * B:]), h)
      else:
        codec.quantize_encode(None, 0.5, seeds, _lib.STOCHASTIC, ptrs=ptrs, P=P, out=batches[k], stream=comp_s)
    if onebit:
      _lib.call("fc_onebit_decode_sum", _lib.ptr(masks), _lib.ptr(means), C, P, _lib.ptr(out), h)
      out_host.copy_(out, non_blocking=True)
      torch.cuda.synchronize()
      return
    for k in range(nb):
      last = k == nb - 1
      codec.decode_accumulate(batches[k], sum_in=isum if k else None, sum_out=None if last else isum,
                              out=out if last else None, step=0.5, err=err, stream=comp_s,
                              want_sum=not last)
    out_host.copy_(out, non_blocking=True)
    torch.cuda.synchronize()

  round_once()
  ts = []
  for _ in range(args.reps):
    t0 = time.perf_counter()
    round_once()
    ts.append(time.perf_counter() - t0)
  t = min(ts)
  print(json.dumps({"metric": "host-resident round (H2D + encode + decode + D2H)", "codec": args.codec,
                    "clients": C, "P": P,
                    "seconds": round(t, 4), "GiB_per_s": round(C * P * 4 / t / 2**30, 2),
                    "h2d_GB": round(C * P * 4 / 1e9, 2)}))


if __name__ == "__main__":
  main()

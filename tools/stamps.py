"""Diagnostic: per-phase cycle shares of k_encode (FC_STAMPS build).

FEDCODEC_LIB=federated_amd/libfedcodec_stamps.so python tools/stamps.py
"""
import ctypes
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from federated_amd import _lib, codec  # noqa: E402

P = int(os.environ.get("P", 25_000_000))
C = int(os.environ.get("C", 128))
mode = int(os.environ.get("MODE", _lib.STOCHASTIC))
lib = _lib.load()
HAVE = hasattr(lib, "fc_debug_stamps")
if HAVE:
  lib.fc_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
dev = torch.device("cuda:0")
g = torch.Generator(device=dev)
g.manual_seed(1)
NPOOL = int(os.environ.get("POOL", 4)) or C  # POOL=0: a distinct delta per client
SIGMA = float(os.environ.get("SIGMA", 1.0))
pool = [torch.randn(P, generator=g, device=dev).mul_(SIGMA) for _ in range(NPOOL)]
rows = [pool[c % NPOOL] for c in range(C)]
ptrs = torch.tensor([r.data_ptr() for r in rows], dtype=torch.int64, device=dev)
seeds = torch.tensor([[c, c] for c in range(C)], dtype=torch.int64, device=dev)
batch = codec.EncodedBatch(P, C, [P + 1024] * C, dev)
buf = (ctypes.c_ulonglong * 16)()
for it in range(3):
  if HAVE:
    lib.fc_debug_stamps(buf, 1)
  torch.cuda.synchronize()
  t0 = time.perf_counter()
  codec.quantize_encode(None, float(os.environ.get("STEP", 0.5)), seeds, mode, ptrs=ptrs, P=P, out=batch)
  torch.cuda.synchronize()
  dt = time.perf_counter() - t0
  if HAVE:
    lib.fc_debug_stamps(buf, 0)
tiles = C * codec.num_tiles(P)
if not HAVE:
  print("encode %.2f ms (no stamps in this build)" % (dt * 1e3))
  sys.exit(0)
names = ["loop/ticket", "A load+quant+code", "B-D scans+emit", "D tail+reductions", "publish agg",
         "pending lookback+prefix", "pending store"]
if os.environ.get("ENC2"):  # k_encode2's stamps (intervals ending at each stamp)
  names = ["scans+emit tile 0", "wait staged tile 1", "quant+code (both tiles)", "scans+emit tile 1",
           "wait end (next stage, lb window)", "reductions+publish", "look-back", "finish: idx+stores+clear"]
tot = sum(buf[i] for i in range(len(names)))
print("encode %.2f ms, %d tiles, %.0f cycles/tile total (memtime units)" % (dt * 1e3, tiles, tot / tiles))
for i, n in enumerate(names):
  print("  %-22s %8.0f  %5.1f%%" % (n, buf[i] / tiles, 100.0 * buf[i] / tot))
cn = {8: "vec lookbacks", 9: "re-polls", 10: "no prefix in 64", 11: "short-body fallback", 12: "predecessor prefix", 13: "sum fold depth"}
for i, n in cn.items():
  print("  %-22s %12d  (%.3f per tile)" % (n, buf[i], buf[i] / tiles))

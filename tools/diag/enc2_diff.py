"""Diagnostic: k_encode vs k_encode2 (FEDCODEC_ENC2) on the same batch.

python tools/diag/enc2_diff.py  -- prints the first differing idx entries / stream
bytes per client (QSGD-like input: per-client norms, step 1/127, stochastic).
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from federated_amd import _lib, codec  # noqa: E402

P = int(os.environ.get("P", 300007))
C = int(os.environ.get("C", 6))
STEP = float(os.environ.get("STEP", 1.0 / 127.0))
rng = np.random.default_rng(P + C)
xs = [(rng.standard_normal(P) * rng.uniform(0.01, 3)).astype(np.float32) for _ in range(C)]
dev = torch.device("cuda:0")
rows = [torch.from_numpy(x).to(dev) for x in xs]
norms = torch.tensor([float(np.linalg.norm(x)) for x in xs], dtype=torch.float32, device=dev)
if os.environ.get("NONORM"):
  norms = None
seeds = torch.tensor([[40 + c, 7 * c] for c in range(C)], dtype=torch.int64, device=dev)
mode = int(os.environ.get("MODE", _lib.STOCHASTIC))
outs = []
for v in ("0", "1"):
  os.environ["FEDCODEC_ENC2"] = v
  b = codec.quantize_encode(rows, STEP, seeds, mode, norms=norms)
  torch.cuda.synchronize()
  outs.append(b)
a, b = outs
print("overflow", codec.check_overflow(a), codec.check_overflow(b))
ta, tb = a.total_bits.cpu().numpy(), b.total_bits.cpu().numpy()
print("total_bits equal:", np.array_equal(ta, tb), ta[:4], tb[:4])
ia = a.idx.cpu().numpy().reshape(C, -1)
ib = b.idx.cpu().numpy().reshape(C, -1)
for c in range(C):
  d = np.nonzero(ia[c] != ib[c])[0]
  if len(d):
    t = d[0]
    print("client %d: %d idx differ, first tile %d: %x vs %x (bits %d vs %d, last %d vs %d)" % (
        c, len(d), t, ia[c, t], ib[c, t], ia[c, t] & ((1 << 36) - 1), ib[c, t] & ((1 << 36) - 1),
        (ia[c, t] >> 36) - 1, (ib[c, t] >> 36) - 1))
  sa = a.stream[int(a.offs_host[c]):int(a.offs_host[c]) + int((ta[c] + 7) // 8)].cpu().numpy()
  sb = b.stream[int(b.offs_host[c]):int(b.offs_host[c]) + int((tb[c] + 7) // 8)].cpu().numpy()
  n = min(len(sa), len(sb))
  d = np.nonzero(sa[:n] != sb[:n])[0]
  if len(d) or len(sa) != len(sb):
    print("client %d: stream bytes differ: %d (first at byte %d = bit %d, tile ~%d)" % (
        c, len(d), d[0] if len(d) else -1, 8 * d[0] if len(d) else -1,
        np.searchsorted(ia[c] & ((1 << 36) - 1), 8 * d[0], side="right") - 1 if len(d) else -1))
da = a.dist_part.cpu().numpy().reshape(C, -1).sum(1)
db = b.dist_part.cpu().numpy().reshape(C, -1).sum(1)
print("dist sums", da, db)
# detail: the first differing tile of client 0 (decoded positions around the first stream diff)
c = 0
d = np.nonzero(ia[c] != ib[c])[0]
if len(d):
  t = d[0]
  M = (1 << 36) - 1
  for u in range(max(0, t - 3), t + 1):
    print("tile %d: old bits %d last %d | new bits %d last %d" % (u, ia[c, u] & M, (ia[c, u] >> 36) - 1,
                                                           ib[c, u] & M, (ib[c, u] >> 36) - 1))
  # quantised values the oracle-free way: decode both streams tile by tile with the decoder
  for name, bb in (("old", a), ("new", b)):
    acc = torch.zeros(P, dtype=torch.int32, device=dev)
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    s_, _, e_ = codec.decode_accumulate(bb, want_sum=True, err=err)
    print(name, "decode err", int(e_.item()))
  sa_, _, _ = codec.decode_accumulate(a, want_sum=True)
  sb_, _, _ = codec.decode_accumulate(b, want_sum=True)
  x = sa_.cpu().numpy(); y = sb_.cpu().numpy()
  dd = np.nonzero(x != y)[0]
  print("sum differs at", len(dd), "positions; first", dd[:10], "tiles", np.unique(dd // 1024)[:10])

"""Diagnostic: HIP-event time of k_encode / k_decode for one library build.

FEDCODEC_LIB=federated_amd/libfedcodec_<variant>.so C=1024 P=25000000 MODE=1 STEP=0.5 [CLIP=3.7] \
    python tools/enc_bench.py
Prints one line: variant, encode ms (median of REPS), decode ms, bits/element.
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from federated_amd import _lib, codec  # noqa: E402

P = int(os.environ.get("P", 25_000_000))
C = int(os.environ.get("C", 1024))
MODE = int(os.environ.get("MODE", _lib.STOCHASTIC))
STEP = float(os.environ.get("STEP", 0.5))
SIGMAS = [float(v) for v in os.environ.get("SIGMA", "1.0").split(",")]
REPS = int(os.environ.get("REPS", 5))
DEC = os.environ.get("DEC", "1") != "0"
dev = torch.device("cuda:0")
g = torch.Generator(device=dev)
# LAYOUT: sep = one allocation per client row (2 MiB-aligned bases); pack = rows back to
# back in one buffer; skew = one buffer, rows 2 MiB-aligned plus c * SKEW bytes
LAYOUT = os.environ.get("LAYOUT", "sep")
rows = []
if LAYOUT == "sep":
  for c in range(C):
    g.manual_seed(77 + c)
    rows.append(torch.randn(P, generator=g, device=dev))
else:
  skew = int(os.environ.get("SKEW", 16384)) // 4
  pitch = P if LAYOUT == "pack" else -(-P // (1 << 19)) * (1 << 19)
  off = [c * pitch + (skew * (c % 64) if LAYOUT == "skew" else 0) for c in range(C)]
  big = torch.empty(off[-1] + P, device=dev)
  for c in range(C):
    g.manual_seed(77 + c)
    r = big[off[c]:off[c] + P]
    r.copy_(torch.randn(P, generator=g, device=dev))
    rows.append(r)
CLIP = float(os.environ.get("CLIP", 0))  # > 0: rows clamped to [-CLIP, CLIP] (e.g. every |q| <= 7)
if CLIP > 0:
  for r in rows:
    r.clamp_(-CLIP, CLIP)
print("row bases mod 2 MiB:", sorted(set(r.data_ptr() % (1 << 21) for r in rows))[:8], flush=True)
ptrs = torch.tensor([r.data_ptr() for r in rows], dtype=torch.int64, device=dev)
seeds = torch.tensor([[c, c] for c in range(C)], dtype=torch.int64, device=dev)
batch = codec.EncodedBatch(P, C, [int(P * float(os.environ.get("CAP", 1.0))) + 1024] * C, dev)
out = torch.empty(P, dtype=torch.float32, device=dev)
err = torch.zeros(1, dtype=torch.int32, device=dev)
prev = 1.0
for SIGMA in SIGMAS:
  for r in rows:
    r.mul_(SIGMA / prev)
  prev = SIGMA if SIGMA else 1.0
  s = torch.cuda.current_stream()
  enc, dec = [], []
  for it in range(REPS + 1):
    e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    e[0].record(s)
    codec.quantize_encode(None, STEP, seeds, MODE, ptrs=ptrs, P=P, out=batch, stream=s)
    e[1].record(s)
    if DEC:  # DEC=0: encode only (ablation builds write streams the decoder must not be fed)
      codec.decode_accumulate(batch, want_sum=False, out=out, step=STEP, err=err, stream=s)
    e[2].record(s)
    torch.cuda.synchronize()
    if it:
      enc.append(e[0].elapsed_time(e[1]))
      dec.append(e[1].elapsed_time(e[2]))
  enc.sort()
  dec.sort()
  bits = float(batch.bits().sum()) / (C * P)
  ok = not len(codec.check_overflow(batch)) and int(err.item()) == 0
  print("%-6s %-28s C=%d P=%d mode=%d step=%g sigma=%g  encode %.3f ms  decode %.3f ms  %.3f bits/elt  %s" % (
      LAYOUT, os.path.basename(_lib.LIB_PATH), C, P, MODE, STEP, SIGMA, enc[len(enc) // 2], dec[len(dec) // 2], bits,
      "ok" if ok else "ERROR"), flush=True)

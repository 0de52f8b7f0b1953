"""Debug: which decode of the pipelined round flags err (64 clients x 2^18, quarters)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from federated_amd import _lib, codec  # noqa: E402

gpu = torch.device("cuda:0")
C, P = 64, 1 << 18
F32 = np.float32
rng = np.random.default_rng(C * P)
rows = [torch.from_numpy((rng.standard_normal(P) * (0.5 + c % 3)).astype(F32)).to(gpu) for c in range(C)]
ptrs = torch.tensor([r.data_ptr() for r in rows], dtype=torch.int64, device=gpu)
seeds = torch.tensor([[3 + c, 5 * c] for c in range(C)], dtype=torch.int64, device=gpu)
pre = torch.from_numpy(np.stack([np.full(C, 0.9, F32), np.arange(1, C + 1, dtype=F32)], 1)).to(gpu)
caps = [codec.worst_case_capacity(P) // 4] * C
H = C // 2
for label, kw in (("no prescale", {}), ("prescale", {"prescale": pre})):
  plain = codec.quantize_encode(None, 0.25, seeds, _lib.STOCHASTIC, ptrs=ptrs, P=P, caps=caps, **kw)
  s, _, err = codec.decode_accumulate(plain)
  print(label, "plain err", int(err.item()), "overflow", list(codec.check_overflow(plain)), flush=True)
  for lo, hi in ((0, H), (H, C)):
    p2 = {"prescale": pre[lo:hi].contiguous()} if kw else {}
    b = codec.quantize_encode(None, 0.25, seeds[lo:hi].contiguous(), _lib.STOCHASTIC, ptrs=ptrs[lo:hi].contiguous(),
                              P=P, caps=caps[lo:hi], **p2)
    s2, _, e2 = codec.decode_accumulate(b)
    e3 = torch.zeros(1, dtype=torch.int32, device=gpu)
    codec.decode_accumulate(b, err=e3, tiles=(0, b.T))
    same = bool(torch.equal(b.stream[:int(b.nbytes()[0])], plain.stream[int(plain.offs_host[lo]):int(plain.offs_host[lo]) + int(b.nbytes()[0])]))
    print(label, "half", lo, hi, "err", int(e2.item()), "tiles err", int(e3.item()), "quarters", b.quarters,
          "ovf", list(codec.check_overflow(b)), "bits equal", np.array_equal(b.bits(), plain.bits()[lo:hi]),
          "client0 bytes equal", same, flush=True)

"""Diagnostic: cost of the server decode of BARE codes (fc_build_index + decode).

The reference server gets only the TFC byte strings (elias_gamma_encode.py:69-73,
97-109); codec.from_codes / fc_build_index rebuild the decoder index on the
device.  Per config: the HIP encoder's codes of C0 distinct clients, copied into a
bare batch of C clients (code c % C0; the rebuild's cost does not depend on the
codes being distinct), then HIP-event times of fc_build_index and of the decode,
the rebuilt index checked against the encoder's.

  python tools/index_bench.py [headline|config2|config3 ...]
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from federated_amd import _lib, codec  # noqa: E402

dev = torch.device("cuda:0")
CONFIGS = {  # name: (C, C0 distinct, P, sigma, step)
    "headline": (1024, 128, 25_000_000, 1.0, 0.5),
    "config2": (128, 128, 1 << 20, 0.25, 1.0 / 127),
    "config3": (256, 64, 4_050_748, 1.0, 1.0),
}


def ev_time(fn, reps=3):
  fn()
  torch.cuda.synchronize()
  e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
  e0.record()
  for _ in range(reps):
    fn()
  e1.record()
  torch.cuda.synchronize()
  return e0.elapsed_time(e1) / reps


def run(name):
  C, C0, P, sigma, step = CONFIGS[name]
  g = torch.Generator(device=dev)
  rows = []
  for c in range(C0):
    g.manual_seed(300 + c)
    rows.append(torch.randn(P, generator=g, device=dev).mul_(sigma))
  seeds = torch.tensor([[7 + c, c] for c in range(C0)], dtype=torch.int64)
  enc = codec.quantize_encode_checked(rows, step, seeds, _lib.STOCHASTIC, segments=1)
  del rows
  torch.cuda.empty_cache()
  nb = enc.nbytes()
  bare = codec.EncodedBatch(P, C, [int(nb[c % C0]) + 16 for c in range(C)], dev)
  for c in range(C):
    k = c % C0
    o, s = int(bare.offs_host[c]), int(enc.offs_host[k])
    bare.stream[o:o + int(nb[k])].copy_(enc.stream[s:s + int(nb[k])])
  nbytes = torch.from_numpy(np.array([nb[c % C0] for c in range(C)], np.int64)).to(dev)
  max_bytes = int(nb.max())
  S = float(sum(nb[c % C0] for c in range(C)))
  quarters = codec.quarter_index_wanted(C)
  t_idx = ev_time(lambda: codec.index_codes(bare, nbytes, max_bytes, quarters=quarters, check=False))
  err = codec.index_codes(bare, nbytes, max_bytes, quarters=quarters, check=False)
  assert int(err.item()) == 0
  want = enc.idx.view(C0, -1).cpu().numpy()
  got = bare.idx.view(C, -1).cpu().numpy()
  assert all(np.array_equal(got[c], want[c % C0]) for c in range(C)), "rebuilt index differs"
  out = torch.empty(P, dtype=torch.float32, device=dev)
  t_dec = ev_time(lambda: codec.decode_accumulate(bare, want_sum=False, out=out, step=step))
  print("%-9s C=%d P=%d %.2f bits/elt: fc_build_index %.2f ms (%.0f GB/s of code)  decode %.2f ms  "
        "(bare decode %.2f ms vs %.2f with the encoder's index)" % (
            name, C, P, 8 * S / (C * P), t_idx, S / t_idx / 1e6, t_dec, t_idx + t_dec, t_dec), flush=True)


if __name__ == "__main__":
  for n in sys.argv[1:] or list(CONFIGS):
    run(n)
    torch.cuda.empty_cache()

"""Diagnostic: decoder lane utilisation (FC_STAMPS build): lane iterations / (64 x wave iterations).

FEDCODEC_LIB=federated_amd/libfedcodec_stamps.so C=1024 python tools/diag/dec_diverge.py
"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from federated_amd import _lib, codec  # noqa: E402

P = int(os.environ.get("P", 25_000_000))
C = int(os.environ.get("C", 1024))
dev = torch.device("cuda:0")
lib = _lib.load()
lib.fc_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
g = torch.Generator(device=dev)
g.manual_seed(1)
rows = [torch.randn(P, generator=g, device=dev) for _ in range(C)]
ptrs = torch.tensor([r.data_ptr() for r in rows], dtype=torch.int64, device=dev)
seeds = torch.tensor([[c, c] for c in range(C)], dtype=torch.int64, device=dev)
batch = codec.EncodedBatch(P, C, [P + 1024] * C, dev)
codec.quantize_encode(None, 0.5, seeds, _lib.STOCHASTIC, ptrs=ptrs, P=P, out=batch)
out = torch.empty(P, dtype=torch.float32, device=dev)
buf = (ctypes.c_ulonglong * 16)()
torch.cuda.synchronize()
lib.fc_debug_stamps(buf, 1)
codec.decode_accumulate(batch, want_sum=False, out=out, step=0.5)
torch.cuda.synchronize()
lib.fc_debug_stamps(buf, 0)
lane_it, wave_it = buf[14], buf[15]
segs = C * codec.num_tiles(P)
print("segments %d  lane iterations %d (%.1f per segment)  wave iterations %d  lane utilisation %.3f" % (
    segs, lane_it, lane_it / segs, wave_it, lane_it / (64.0 * wave_it)))

"""Diagnostic: fc_build_index against the encoder's index on mixed-density clients; dumps the
per-chunk workspace (x1, n1, x2, n2, xm, checkpoints) of the first client whose entries differ."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from federated_amd import _lib, codec  # noqa: E402

gpu = torch.device("cuda:0")
C, P = int(os.environ.get("C", 300)), int(os.environ.get("P", 9000))
rng = np.random.default_rng(C + P)
scales = [0.02, 0.3, 1.0, 8.0, 60.0]
xs = [(rng.standard_normal(P) * scales[c % len(scales)]).astype(np.float32) for c in range(C)]
rows = [torch.from_numpy(x).to(gpu) for x in xs]
seeds = torch.tensor([[c, 3 * c + 1] for c in range(C)], dtype=torch.int64)
enc = codec.quantize_encode(rows, 0.5, seeds, _lib.STOCHASTIC, caps=[codec.worst_case_capacity(P)] * C, segments=1,
                            quarters=False)
codes = [enc.client_code(c) for c in range(C)]
lens = np.array([len(x) for x in codes], np.int64)
bare = codec.EncodedBatch(P, C, [int(n) + 16 for n in lens], gpu)
host = np.zeros(bare._stream.numel(), np.uint8)  # pylint: disable=protected-access
for c, code in enumerate(codes):
  o = int(bare.offs_host[c])
  host[o:o + len(code)] = np.frombuffer(code, np.uint8)
bare._stream.copy_(torch.from_numpy(host))  # pylint: disable=protected-access
nb = torch.from_numpy(lens).to(gpu)
mx = int(lens.max())
lib = _lib.load()
need = int(lib.fc_index_workspace_bytes(C, mx))
ws = torch.zeros((need + 255) // 256 * 256, dtype=torch.uint8, device=gpu)
err = torch.zeros(1, dtype=torch.int32, device=gpu)
_lib.call("fc_build_index", _lib.ptr(bare._stream), _lib.ptr(bare.stream_off), _lib.ptr(nb), C, P, mx,  # pylint: disable=protected-access
          _lib.ptr(bare._idx), _lib.ptr(None), _lib.ptr(bare.total_bits), _lib.ptr(err), _lib.ptr(ws), ws.numel(),  # pylint: disable=protected-access
          _lib.stream_handle(None))
torch.cuda.synchronize()
print("err", int(err.item()))
got = bare.idx.view(C, -1).cpu().numpy()
want = enc.idx.view(C, -1).cpu().numpy()
bad = [c for c in range(C) if not np.array_equal(got[c], want[c])]
print("clients with differing entries:", len(bad), bad[:20])
nch = max(1, (8 * mx + 4095) // 4096)
lanes = C * nch
w = ws[:8 * (12 * lanes)].view(torch.int64).cpu().numpy()
x1, n1, x2, n2, xm = (w[k * lanes:(k + 1) * lanes].reshape(C, nch) for k in range(5))
ck = w[5 * lanes:12 * lanes].reshape(7, C, nch)
for c in bad[:3]:
  u = np.nonzero(got[c] != want[c])[0]
  print("client", c, "scale", scales[c % 5], "bytes", lens[c], "bad units", u[:10], "got", [hex(v) for v in got[c][u[:3]]],
        "want", [hex(v) for v in want[c][u[:3]]])
  nchc = (8 * lens[c] + 4095) // 4096
  for j in range(nchc):
    cks = [(int(ck[k, c, j]) & 0x1FFF, int(ck[k, c, j]) >> 13) if ck[k, c, j] != -1 else None for k in range(7)]
    print("  j", j, "x1", x1[c, j], "n1", n1[c, j], "x2", x2[c, j], "L", n2[c, j], "xm", xm[c, j], "ck", cks)

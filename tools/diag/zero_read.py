"""Diagnostic: HBM read rate of zero vs random fp32 data (copy and norms kernels)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from federated_amd import _lib  # noqa: E402

dev = torch.device("cuda:0")
n = 1 << 30  # floats (4 GiB)
h = _lib.stream_handle(torch.cuda.current_stream())
for name, fill in (("randn", lambda t: t.normal_()), ("zeros", lambda t: t.zero_()), ("ones", lambda t: t.fill_(1.0)),
                   ("tiny", lambda t: t.normal_().mul_(1e-3))):
  a = torch.empty(n, dtype=torch.float32, device=dev)
  b = torch.empty(n, dtype=torch.float32, device=dev)
  fill(a)
  rows = [a[i * (n // 64):(i + 1) * (n // 64)] for i in range(64)]
  ptrs = torch.tensor([r.data_ptr() for r in rows], dtype=torch.int64, device=dev)
  norms = torch.empty(128, dtype=torch.float32, device=dev)
  res = {}
  for k, fn in (("copy", lambda: _lib.call("fc_copy", _lib.ptr(b), _lib.ptr(a), 4 * n, h)),
                ("norms", lambda: _lib.call("fc_client_norms_scaled", _lib.ptr(ptrs), 64, n // 64, _lib.NORM_L2_LINF,
                                            None, _lib.ptr(norms), h))):
    ts = []
    for i in range(6):
      e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
      e0.record()
      fn()
      e1.record()
      torch.cuda.synchronize()
      if i:
        ts.append(e0.elapsed_time(e1))
    res[k] = min(ts)
  print("%-6s copy %.3f ms (%.0f GB/s)  norms %.3f ms (%.0f GB/s)" % (
      name, res["copy"], 8.0 * n / res["copy"] / 1e6, res["norms"], 4.0 * n / res["norms"] / 1e6), flush=True)
  del a, b

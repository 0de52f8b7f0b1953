"""Ticket-stream progress under an occupied XCD: start-order streams (default) against
round 5's blockIdx streams (FEDCODEC_TICKET_BLOCKIDX=1), DESIGN.md §2.

One XCD's CUs are held by fc_diag_occupy for 1.5 s; the segmented encoder runs at
config 4's shape (3 x 11 M) on another stream with the look-back spin limit at 2^16
polls.  Prints, per mapping: the clients flagged FC_OVERFLOW_STALL, whether the codes
equal an unoccupied encode, and the encode's wall time (the kernel cannot complete
before the occupier has left: its workgroups dealt to the held XCD start only then).
"""
import os
import sys
import time
import warnings

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from federated_amd import _lib  # pylint: disable=g-import-not-at-top
from federated_amd import codec  # pylint: disable=g-import-not-at-top

P, C, STEP = 11_000_000, 3, 0.5


def main():
  dev = torch.device("cuda", 0)
  g = torch.Generator(device=dev)
  rows = []
  for c in range(C):
    g.manual_seed(2200 + c)
    rows.append(torch.randn(P, generator=g, device=dev, dtype=torch.float32))
  seeds = np.array([[31 + c, 7 * c + 1] for c in range(C)], np.int64)
  ref = codec.quantize_encode(rows, STEP, seeds, _lib.STOCHASTIC)
  codec.check_overflow(ref)
  want = [ref.client_code(c) for c in range(C)]
  ncu = torch.cuda.get_device_properties(dev).multi_processor_count
  os.environ["FEDCODEC_SPIN_LIMIT"] = str(1 << 16)
  for mapping in ("0", "1"):
    os.environ["FEDCODEC_TICKET_BLOCKIDX"] = mapping
    for mask in (0x01, 0x10, 0x81):
      held = torch.zeros(1, dtype=torch.int32, device=dev)
      side = torch.cuda.Stream(device=dev)
      side.wait_stream(torch.cuda.current_stream(dev))
      torch.cuda.synchronize()
      t0 = time.perf_counter()
      _lib.call("fc_diag_occupy", mask, 1_500_000, _lib.ptr(held), _lib.stream_handle(side))
      torch.cuda._sleep(50_000_000)  # pylint: disable=protected-access
      got = codec.quantize_encode(rows, STEP, seeds, _lib.STOCHASTIC)
      torch.cuda.current_stream(dev).synchronize()
      t_enc = time.perf_counter() - t0
      torch.cuda.synchronize()
      with warnings.catch_warnings():
        warnings.simplefilter("ignore", codec.EncoderStallWarning)
        cap = codec.check_overflow(got)
      same = [got.client_code(c) for c in range(C)] == want
      print("mapping=%s xcd_mask=0x%02x held=%d/%d stalled=%s capacity=%s codes_equal=%s encode_wall_s=%.3f"
            % ("blockIdx" if mapping == "1" else "start-order", mask, int(held.item()),
               ncu // 8 * bin(mask).count("1"), got.stalled.tolist(), cap.tolist(), same, t_enc), flush=True)
  os.environ.pop("FEDCODEC_TICKET_BLOCKIDX")
  os.environ.pop("FEDCODEC_SPIN_LIMIT")


if __name__ == "__main__":
  main()

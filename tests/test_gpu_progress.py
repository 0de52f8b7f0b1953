"""The encoder's forward progress when another kernel holds CUs.

Round 5's one GPU fault (`profiles/r05/gputest_fault_r5zz.txt`) came from two
processes on one GPU running persistent encoders side by side: with ticket streams
tied to blockIdx, a stream whose workgroups were not resident left every resident
wave spinning in the look-back until its spin limit.  The encoder now draws its
ticket stream from its START ORDER (fedcodec.hip `ticket_stream`: counted on 32
heads, a head's n-th started wave takes stream h + n), so the waves that did start
cover every stream.

Here one process does what the second process did: `fc_diag_occupy` holds every CU
of one XCD (160 KiB of LDS each) for longer than the spin limit while the encoder
runs at the faulting shape -- config 4's tensor (3 clients x 11 M, segmented into
63 + 3 one-tile encoder rows) -- on another stream.  The spin limit is lowered to
2^16 polls (tens of ms), so a look-back that waits on a ticket nobody can take is
flagged (FC_OVERFLOW_STALL -> EncoderStallWarning, an error in the tests).  Checked:
no stall, the codes byte-identical to an unoccupied encode, and the int32 sum equal
to the oracle at sampled positions of every client.
"""
import os

import numpy as np
import pytest
import torch

from federated_amd import _lib
from federated_amd import codec

pytestmark = pytest.mark.gpu

P11, C3, STEP = 11_000_000, 3, 0.5


def _rows(dev):
  g = torch.Generator(device=dev)
  rows = []
  for c in range(C3):
    g.manual_seed(2200 + c)
    rows.append(torch.randn(P11, generator=g, device=dev, dtype=torch.float32))
  return rows


def _codes(batch):
  return [batch.client_code(c) for c in range(batch.nclients)]


@pytest.mark.parametrize("xcd_mask", [0x01, 0x81])
def test_encoder_progress_with_occupied_xcds(gpu, monkeypatch, xcd_mask):
  from oracle import quantize_utils as oq  # pylint: disable=g-import-not-at-top  (checker)
  rows = _rows(gpu)
  seeds = np.array([[31 + c, 7 * c + 1] for c in range(C3)], np.int64)
  assert codec.auto_segments(C3, P11) > 1  # the faulting shape is the segmented encoder
  ref = codec.quantize_encode(rows, STEP, seeds, _lib.STOCHASTIC)
  assert not len(codec.check_overflow(ref))
  want = _codes(ref)

  monkeypatch.setenv("FEDCODEC_SPIN_LIMIT", str(1 << 16))
  held = torch.zeros(1, dtype=torch.int32, device=gpu)
  side = torch.cuda.Stream(device=gpu)
  main = torch.cuda.current_stream(gpu)
  side.wait_stream(main)
  ncu = torch.cuda.get_device_properties(gpu).multi_processor_count
  _lib.call("fc_diag_occupy", int(xcd_mask), 1_500_000, _lib.ptr(held), _lib.stream_handle(side))
  # the occupier takes its CUs first; then the encode runs on the others
  torch.cuda._sleep(50_000_000)  # pylint: disable=protected-access  (~20-40 ms on the main stream)
  got = codec.quantize_encode(rows, STEP, seeds, _lib.STOCHASTIC)
  torch.cuda.synchronize()
  assert int(held.item()) == ncu // 8 * bin(xcd_mask).count("1")  # every CU of the masked XCDs was held
  assert not len(codec.check_overflow(got))  # (a stall raises EncoderStallWarning here)
  assert not len(got.stalled)
  assert _codes(got) == want

  s, _, err = codec.decode_accumulate(got)
  assert int(err.item()) == 0
  idx = np.sort(np.random.default_rng(5).choice(P11, 20_000, replace=False))
  it = torch.from_numpy(idx).to(gpu)
  acc = np.zeros(idx.size, np.int64)
  for c in range(C3):
    acc += oq.stochastic_quantize_at(rows[c][it].cpu().numpy(), idx, np.float32(STEP), tuple(seeds[c]))
  np.testing.assert_array_equal(s[it].cpu().numpy(), acc.astype(np.int32))
  del rows, ref, got
  torch.cuda.empty_cache()


def test_spin_limit_reaches_host(gpu, monkeypatch):
  """The stall flag's path to the host: a look-back that waits past the spin limit
  (forced with a limit of one poll on a many-clients encode, where look-backs wait
  on coding predecessors) sends its client to the exact path -- the codes stay
  exact -- and check_overflow reports it as an EncoderStallWarning."""
  rng = np.random.default_rng(9)
  C, P = 64, 300_000
  xs = [torch.from_numpy((rng.standard_normal(P) * 0.7).astype(np.float32)).to(gpu) for _ in range(C)]
  seeds = np.array([[c, 3 * c] for c in range(C)], np.int64)
  ref = codec.quantize_encode(xs, STEP, seeds, _lib.STOCHASTIC, segments=1)
  assert not len(codec.check_overflow(ref))
  monkeypatch.setenv("FEDCODEC_SPIN_LIMIT", "1")
  got = codec.quantize_encode(xs, STEP, seeds, _lib.STOCHASTIC, segments=1)
  torch.cuda.synchronize()
  with pytest.warns(codec.EncoderStallWarning):
    assert not len(codec.check_overflow(got))
  assert len(got.stalled) > 0
  assert _codes(got) == _codes(ref)
  assert np.array_equal(got.bits(), ref.bits())
  assert torch.equal(got.idx, ref.idx)

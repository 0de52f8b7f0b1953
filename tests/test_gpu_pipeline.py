"""The pipelined round (codec.encode_decode_pipelined): two client halves, the first
half's decode on a side stream beside the second half's encode.  Same int32 sum and
dequantised result as one encode + one decode (the reference's federated_aggregate
sum is an integer sum: any client grouping gives the same result), checked bit for
bit against the plain path and against the oracle."""
import numpy as np
import pytest
import torch

from federated_amd import _lib
from federated_amd import codec

pytestmark = pytest.mark.gpu

F32 = np.float32


@pytest.mark.parametrize("C,P,mode", [(6, 70_001, "stochastic"), (7, 4099, "uniform"), (5, 30_000, "dithered"),
                                      (64, 1 << 18, "stochastic")])
def test_pipelined_round_equals_plain_round(gpu, C, P, mode):
  m = {"uniform": _lib.UNIFORM, "stochastic": _lib.STOCHASTIC, "dithered": _lib.DITHERED}[mode]
  rng = np.random.default_rng(C * P)
  rows = [torch.from_numpy((rng.standard_normal(P) * (0.5 + c % 3)).astype(F32)).to(gpu) for c in range(C)]
  ptrs = torch.tensor([r.data_ptr() for r in rows], dtype=torch.int64, device=gpu)
  seeds = torch.tensor([[3 + c, 5 * c] for c in range(C)], dtype=torch.int64, device=gpu)
  pre = torch.from_numpy(np.stack([np.full(C, 0.9, F32), np.arange(1, C + 1, dtype=F32)], 1)).to(gpu)
  caps = [codec.worst_case_capacity(P)] * C  # (weights up to C: wide codes)
  noise = codec.noise_sum(seeds, P, gpu) if m == _lib.DITHERED else None
  plain = codec.quantize_encode(None, 0.25, seeds, m, ptrs=ptrs, P=P, caps=caps, prescale=pre)
  want_sum, want_out, err = codec.decode_accumulate(plain, out=torch.empty(P, device=gpu), step=0.25,
                                                    noise_sum=noise)
  rnd = codec.PipelinedRound(P, caps, gpu)
  out = torch.empty(P, dtype=torch.float32, device=gpu)
  got_sum = torch.empty(P, dtype=torch.int32, device=gpu)
  e = codec.encode_decode_pipelined(ptrs, P, 0.25, seeds, m, rnd, out=out, sum_out=got_sum, noise_sum=noise,
                                    prescale=pre)
  torch.cuda.synchronize()
  assert int(e.item()) == 0 and int(err.item()) == 0
  assert not len(rnd.overflowed()) and not len(codec.check_overflow(plain))
  assert torch.equal(got_sum, want_sum)
  np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32), want_out.cpu().numpy().view(np.uint32))
  np.testing.assert_array_equal(rnd.nbytes(), plain.nbytes())


def test_pipelined_round_matches_oracle(gpu):
  from oracle import quantize_utils as oq  # pylint: disable=g-import-not-at-top
  C, P = 9, 50_001
  rng = np.random.default_rng(2)
  xs = [(rng.standard_normal(P) * 1.3).astype(F32) for _ in range(C)]
  rows = [torch.from_numpy(x).to(gpu) for x in xs]
  ptrs = torch.tensor([r.data_ptr() for r in rows], dtype=torch.int64, device=gpu)
  seeds = np.array([[70 + c, c] for c in range(C)], np.int64)
  rnd = codec.PipelinedRound(P, [codec.worst_case_capacity(P)] * C, gpu)
  out = torch.empty(P, dtype=torch.float32, device=gpu)
  e = codec.encode_decode_pipelined(ptrs, P, 0.5, torch.from_numpy(seeds), _lib.STOCHASTIC, rnd, out=out)
  assert not len(rnd.overflowed()) and int(e.item()) == 0
  acc = np.zeros(P, np.int64)
  for c in range(C):
    acc += oq.stochastic_quantize(xs[c], F32(0.5), tuple(seeds[c]))
  want = oq.uniform_dequantize(acc.astype(np.int32), F32(0.5))
  np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32), want.view(np.uint32))


@pytest.mark.parametrize("rounding", ["stochastic", "dithered"])
def test_factory_round_pipelined_matches_oracle(gpu, monkeypatch, rounding):
  """QuantizeEncodeFactory.next with the pipelined schedule on (FEDCODEC_PIPELINE=1):
  the reference's result and measurements (quantize_encode.py:173-211), as the
  in-order schedule gives them."""
  from federated_amd.aggregators import quantize_encode  # pylint: disable=g-import-not-at-top
  from oracle import aggregators as oagg  # pylint: disable=g-import-not-at-top
  monkeypatch.setenv("FEDCODEC_PIPELINE", "1")
  C, P = 7, 20_011
  rng = np.random.default_rng(12)
  xs = [(rng.standard_normal(P) * 0.8).astype(F32) for _ in range(C)]
  seeds = np.array([[c + 1, 2 * c] for c in range(C)], np.int64)
  process = quantize_encode.QuantizeEncodeFactory(0.5, rounding_type=rounding).create((np.float32, (P,)))
  state = process.initialize()
  for _ in range(2):  # the second round sizes its capacities from the first (CapacityHint)
    out = process.next(state, xs, seeds=seeds)
  want, meas, _ = oagg.quantize_encode_next(xs, 0.5, rounding, seeds=seeds)
  if rounding == "dithered":
    np.testing.assert_allclose(out.result, want, rtol=1e-6, atol=1e-6 * C)
  else:
    np.testing.assert_array_equal(np.asarray(out.result).view(np.uint32), want.view(np.uint32))
  assert out.measurements["avg_bitrate"] == meas["avg_bitrate"]
  np.testing.assert_allclose(out.measurements["avg_distortion"], meas["avg_distortion"], rtol=1e-5)
  np.testing.assert_allclose(out.measurements["avg_sparsity"], meas["avg_sparsity"], rtol=1e-6)

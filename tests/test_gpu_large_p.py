"""Client tensors longer than one encoder row (2^26 - 1 elements).

The reference has no size limit: concat_factory flattens the whole model into one
tensor (builder.py:77-78) and TFC codes any int32 tensor (elias_gamma_encode.py:98).
Here a tensor above 2^26 - 1 elements (the encoder's look-back position width) is
always encoded in segments of at most that many elements -- each continuing its
client's Philox stream at its element offset -- and stitched into the client's one
canonical code (codec.min_segments); tensors up to FC_MAX_ELEMS = 2^30 - 2^26
elements are accepted (the decoder index keeps 1 + the last nonzero modulo 2^28,
recovered from the unit a segment decodes).

Checked through QuantizeEncodeFactory at P = 2^26 + 5 and P = 100,000,000:
client 0's code byte-identical to the oracle's (the CPU restatement of the TF
quantiser + TFC coder over the whole tensor), the round's dequantised sum equal to
the oracle's at sampled positions of every client, avg_bitrate equal to the
oracle's; and the bare-code decode (index rebuilt from the bytes) of client 0's
code equal to the oracle's q.
"""
import numpy as np
import pytest
import torch

from federated_amd import _lib
from federated_amd import codec
from federated_amd.aggregators import quantize_encode
from oracle import codec as ocodec
from oracle import quantize_utils as oq

pytestmark = pytest.mark.gpu

F32 = np.float32


@pytest.mark.parametrize("P", [(1 << 26) + 5, 100_000_000], ids=["2^26+5", "100M"])
def test_factory_round_beyond_one_encoder_row(gpu, P):
  C, step = 2, F32(0.5)
  g = torch.Generator(device=gpu)
  rows = []
  for c in range(C):
    g.manual_seed(4242 + c)
    rows.append(torch.randn(P, generator=g, device=gpu, dtype=torch.float32))
  seeds = np.array([[31 + c, 7 * c] for c in range(C)], np.int64)
  process = quantize_encode.QuantizeEncodeFactory(float(step), rounding_type="stochastic").create(
      (np.float32, (P,)))
  out = process.next(process.initialize(), rows, seeds=seeds)
  # client 0 over the whole tensor on the CPU oracle
  x0 = rows[0].cpu().numpy()
  q0 = oq.stochastic_quantize(x0, step, tuple(seeds[0]))
  code0, bits0 = ocodec.run_length_gamma_encode(q0)
  del x0
  # the batch the factory encoded, re-encoded here to read client 0's bytes
  batch = codec.quantize_encode_checked(rows, float(step), torch.from_numpy(seeds), _lib.STOCHASTIC)
  assert batch.seg is None or batch.seg[1] >= codec.min_segments(P)
  assert batch.client_code(0) == code0
  bits1 = ocodec.encoded_bits(oq.stochastic_quantize(rows[1].cpu().numpy(), step, tuple(seeds[1])))
  assert out.measurements["avg_bitrate"] == np.float64((bits0 + 7) // 8 * 8 + (bits1 + 7) // 8 * 8) / 2 / P
  # the round's result at sampled positions of every client
  idx = np.sort(np.random.default_rng(P % 97).choice(P, 50_000, replace=False))
  idx = np.concatenate([idx, [0, P - 1, (1 << 26) - 1, 1 << 26]]).astype(np.int64)
  idx = np.unique(idx[idx < P])
  it = torch.from_numpy(idx).to(gpu)
  acc = np.zeros(idx.size, np.int64)
  for c in range(C):
    acc += oq.stochastic_quantize_at(rows[c][it].cpu().numpy(), idx, step, tuple(seeds[c]))
  want = oq.uniform_dequantize(acc.astype(np.int32), step)
  got = out.result[it].cpu().numpy()
  np.testing.assert_array_equal(got.view(np.uint32), want.view(np.uint32))
  del rows, batch, out
  torch.cuda.empty_cache()
  # the bare code decoded with an index rebuilt from its bytes
  s, _ = codec.decode_codes([code0], P)
  np.testing.assert_array_equal(s.cpu().numpy(), q0)
  del s
  torch.cuda.empty_cache()


def test_factory_round_beyond_2_28(gpu):
  """P = 2^28 + 3 (past round 4's 2^28 - 1 cap), uniform rounding, 2 clients; client
  0 has a zero run of more than 2^27 elements that crosses element 2^28, so the
  decoder index's last-nonzero field (modulo 2^28) is ambiguous there and the decoder
  resolves the segment's first nonzero from the unit it decodes.  Client 0's code is
  byte-identical to the oracle's, the round's result equals the oracle's at sampled
  positions, and the bare code decodes (index rebuilt from its bytes) to the
  oracle's q."""
  P = (1 << 28) + 3
  C, step = 2, F32(0.5)
  g = torch.Generator(device=gpu)
  rows = []
  for c in range(C):
    g.manual_seed(777 + c)
    rows.append(torch.randn(P, generator=g, device=gpu, dtype=torch.float32))
  z0, z1 = (1 << 27) - 1000, (1 << 28) + 1  # zeros [z0, z1): 2^27 + 1001 elements
  rows[0][z0:z1] = 0.0
  process = quantize_encode.QuantizeEncodeFactory(float(step), rounding_type="uniform").create((np.float32, (P,)))
  out = process.next(process.initialize(), rows)
  x0 = rows[0].cpu().numpy()
  q0 = oq.uniform_quantize(x0, step)
  del x0
  code0, bits0 = ocodec.run_length_gamma_encode(q0)
  batch = codec.quantize_encode_checked(rows, float(step), np.zeros((C, 2), np.int64), _lib.UNIFORM)
  assert batch.client_code(0) == code0
  del batch
  idx = np.sort(np.random.default_rng(5).choice(P, 50_000, replace=False))
  idx = np.concatenate([idx, [0, P - 1, z0 - 1, z0, z1 - 1, z1, (1 << 28) - 1, 1 << 28]]).astype(np.int64)
  idx = np.unique(idx[idx < P])
  it = torch.from_numpy(idx).to(gpu)
  acc = np.zeros(idx.size, np.int64)
  for c in range(C):
    acc += oq.uniform_quantize(rows[c][it].cpu().numpy(), step)
  want = oq.uniform_dequantize(acc.astype(np.int32), step)
  np.testing.assert_array_equal(out.result[it].cpu().numpy().view(np.uint32), want.view(np.uint32))
  del rows, out
  torch.cuda.empty_cache()
  s, _ = codec.decode_codes([code0], P)
  np.testing.assert_array_equal(s.cpu().numpy(), q0)
  del s
  torch.cuda.empty_cache()


def test_unsegmented_row_limit_is_enforced(gpu):
  """One encoder row cannot take more than 2^26 - 1 elements: the C ABI refuses it
  (the factories segment such tensors)."""
  P = _lib.MAX_ROW_ELEMS + 1
  x = torch.zeros(P, dtype=torch.float32, device=gpu)
  ptrs = torch.tensor([x.data_ptr()], dtype=torch.int64, device=gpu)
  b = codec.EncodedBatch(P, 1, [codec.default_capacity(P)], gpu)
  ws = torch.empty(int(_lib.load().fc_encode_workspace_bytes(1, P)), dtype=torch.uint8, device=gpu)
  with pytest.raises(_lib.FedCodecError):
    _lib.call("fc_quantize_encode", _lib.ptr(ptrs), 1, P, 0.5, None, None, None, 0, _lib.ptr(b.stream),
              _lib.ptr(b.stream_off), _lib.ptr(b.stream_cap), _lib.ptr(b.idx), _lib.ptr(b.total_bits),
              _lib.ptr(b.dist_part), _lib.ptr(b.nnz_part), _lib.ptr(b.overflow), _lib.ptr(ws), ws.numel(),
              _lib.stream_handle())


def test_elias_gamma_sum_beyond_one_encoder_row(gpu):
  """EliasGammaEncodedSumFactory (elias_gamma_encode.py:57-116) on int32 tensors of
  2^26 + 5 elements: the segmented rlgamma encode's bytes equal the oracle's TFC
  code, and the round's sum is exact."""
  from federated_amd.aggregators import elias_gamma_encode  # pylint: disable=g-import-not-at-top
  P = (1 << 26) + 5
  rng = np.random.default_rng(77)
  qs = [np.clip(np.round(rng.standard_normal(P) * 3), -40, 40).astype(np.int32) for _ in range(2)]
  qs[1][: P // 3] = 0  # a long zero run across segments
  batch = codec.rlgamma_encode([torch.from_numpy(q).to(gpu) for q in qs])
  for c in range(2):
    assert batch.client_code(c) == ocodec.run_length_gamma_encode(qs[c])[0]
  del batch
  process = elias_gamma_encode.EliasGammaEncodedSumFactory().create((np.int32, (P,)))
  out = process.next(process.initialize(), [torch.from_numpy(q).to(gpu) for q in qs])
  got = np.asarray(out.result.cpu().numpy() if hasattr(out.result, "cpu") else out.result)
  np.testing.assert_array_equal(got, qs[0] + qs[1])
  torch.cuda.empty_cache()

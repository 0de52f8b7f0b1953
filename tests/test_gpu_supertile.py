"""The encoder's parity tests again, through the super-tile kernel (k_encode2).

The launcher picks k_encode2 only when few tiles of each client are in flight
(about 1000 clients on one GPU); these small-batch tests would otherwise always
run k_encode.  FEDCODEC_ENC2=1 forces the super-tile kernel for every launch, so
the same oracle checks cover it: integer input (run-length gamma of int32),
the three roundings with partial, odd-count and single tiles, the division
variants, per-client norms (QSGD), the TFF pre-scale (trainer round), the
multi-window look-back, and the reference's known answers -- with two, four
and eight tiles per ticket.
"""
import pytest

from test_gpu_aggregators import (  # noqa: F401  (collected again under this module)
    test_builder_normalized_weighted_matches_oracle, test_qsgd_codes_bit_exact, test_qsgd_matches_oracle,
    test_quantize_encode_normalized_matches_oracle)
from test_gpu_codec import (  # noqa: F401
    test_encode_many_tiles_per_workgroup, test_encoder_division_matches_ieee_over_whole_binades,
    test_quantize_encode_batch_matches_oracle, test_reference_known_answers, test_rlgamma_encode_bytes_match_oracle)
from test_gpu_configs import test_config1_trainer_defaults_round, test_config_round_matches_oracle  # noqa: F401

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True, params=["2", "4", "8"], ids=["2tiles", "4tiles", "8tiles"])
def _super_tiles(monkeypatch, request):
  """The three ticket sizes: two tiles, four and eight (FEDCODEC_ENC_NT=8: the
  per-ticket work once per 8192 elements, a window of ~4.8 bits per element before
  the exact path, so the denser cases here also take the exact re-encode)."""
  monkeypatch.setenv("FEDCODEC_ENC2", "1")
  monkeypatch.setenv("FEDCODEC_ENC_NT", request.param)


@pytest.mark.parametrize("pattern", ["last", "first", "edges", "one_late"])
def test_super_tile_edge_positions(gpu, pattern):
  """Nonzeros only at a super-tile's first / last element (eight-tile tickets: relative
  positions 0 and 8191, where round 4's 13-bit fields held their "no nonzero" mark),
  over 64 super-tiles per client: the aggregates the look-back combines carry those
  positions, and the code, index and sum stay the oracle's."""
  import numpy as np
  import torch
  from federated_amd import _lib, codec
  from oracle import codec as ocodec
  from oracle import quantize_utils as oq
  ste = 8 * 1024
  P, C = 64 * ste + 5, 6
  xs = []
  for c in range(C):
    x = np.zeros(P, np.float32)
    if pattern in ("last", "edges"):
      x[ste - 1::ste] = 1.0 + c
    if pattern in ("first", "edges"):
      x[0::ste] = -2.0
    if pattern == "one_late":  # one nonzero, far into the row: every other aggregate is empty
      x[40 * ste + ste - 1] = 3.0
    xs.append(x)
  seeds = np.array([[c, c] for c in range(C)], np.int64)
  batch = codec.quantize_encode_checked([torch.from_numpy(x).to(gpu) for x in xs], 0.5,
                                        torch.from_numpy(seeds), _lib.UNIFORM)
  acc = np.zeros(P, np.int64)
  for c in range(C):
    q = oq.uniform_quantize(xs[c], 0.5)
    code, nbits = ocodec.run_length_gamma_encode(q)
    assert batch.bits()[c] == nbits
    assert batch.client_code(c) == code
    acc += q
  s, _, err = codec.decode_accumulate(batch)
  assert int(err.item()) == 0
  np.testing.assert_array_equal(s.cpu().numpy(), acc.astype(np.int32))

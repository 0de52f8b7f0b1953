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

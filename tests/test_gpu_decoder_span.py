"""The decoder's parity tests again with two- and four-tile lane segments (k_decode<false, 2 / 4>).

The launcher takes two-tile segments (256 lanes per tile pair) only from 256
clients on; these small-batch tests would otherwise run one-tile segments.
FEDCODEC_DEC_SPAN=2 (or 4, the four-tile knob) forces them: every rlgamma shape (P = 1 .. 100,003: a single
partial tile, odd tile counts, a last segment of one tile), each rounding's
batch round, tile-range decodes starting and ending at odd tiles (the
multi-GPU slabs), malformed streams, the golden rounds and the config rounds.
"""
import pytest

from test_gpu_aggregators import (  # noqa: F401  (collected again under this module)
    test_decoder_rejects_malformed_stream, test_quantize_encode_matches_golden_round,
    test_quantize_encode_reference_execution)
from test_gpu_codec import (  # noqa: F401
    test_decode_tile_ranges_match_full_decode, test_quantize_encode_batch_matches_oracle,
    test_reference_known_answers, test_rlgamma_encode_bytes_match_oracle)
from test_gpu_configs import test_config_round_matches_oracle  # noqa: F401

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True, params=["2", "4"])
def _multi_tile_segments(request, monkeypatch):
  monkeypatch.setenv("FEDCODEC_DEC_SPAN", request.param)

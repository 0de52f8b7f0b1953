import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
  sys.path.insert(0, ROOT)


def pytest_configure(config):
  config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")
  config.addinivalue_line("markers", "slow: long-running CPU test")
  # an encoder look-back that hits its spin limit is a failure in every test
  config.addinivalue_line("filterwarnings", "error::federated_amd.codec.EncoderStallWarning")


@pytest.fixture(scope="session")
def gpu():
  import torch  # pylint: disable=g-import-not-at-top
  if not torch.cuda.is_available():
    pytest.fail("GPU test requested but no GPU is visible")
  from federated_amd import _lib  # pylint: disable=g-import-not-at-top
  _lib.require_gpu()
  return torch.device("cuda:0")

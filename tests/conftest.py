import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X); parity tests of the HIP path")
    config.addinivalue_line("markers", "slow: full-size (BASELINE config) parity case")


@pytest.fixture(scope="session")
def oracle_lib():
    from oracle import oracle
    oracle.build()
    return oracle


@pytest.fixture(scope="session")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no ROCm GPU visible")
    from langsplatv2_amd import _lib
    _lib.load()  # fails loudly if liblsr.so is missing
    return torch.device("cuda:0")

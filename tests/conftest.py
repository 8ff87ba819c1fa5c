import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN_REF = "/root/reference/connectors/golden-tables/src/main/resources/golden"
KD_RES = "/root/reference/kernel/kernel-defaults/src/test/resources"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")
    config.addinivalue_line("markers", "slow: larger synthetic sizes")


@pytest.fixture(scope="session")
def golden_root():
    if not os.path.isdir(GOLDEN_REF):
        pytest.skip("reference golden tables not present (GPU box)")
    return GOLDEN_REF

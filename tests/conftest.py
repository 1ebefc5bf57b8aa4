import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; parity tests through the C ABI")


def golden(name: str):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def aesgo():
    return golden("aesgo.json")


@pytest.fixture(scope="session")
def gcm_spec():
    return golden("gcm_spec.json")


@pytest.fixture(scope="session")
def kdf():
    return golden("kdf.json")


@pytest.fixture(scope="session")
def batch_digests():
    return golden("batch_digest.json")


@pytest.fixture(scope="session")
def headline_digest():
    return golden("headline_digest.json")


@pytest.fixture(scope="session")
def config3_digest():
    return golden("config3_digest.json")


@pytest.fixture(scope="session")
def ctx():
    """One device context per test session (GPU tests only)."""
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from quantum_amd.crypto import Context

    c = Context(device=0, max_keys=2048)
    yield c
    c.close()

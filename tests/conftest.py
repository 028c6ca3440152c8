import sys
from pathlib import Path

import pytest

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE))
sys.path.insert(0, str(HERE.parent))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs on the GPU box)")
    config.addinivalue_line("markers", "slow: long CPU test")


@pytest.fixture(scope="session")
def golden():
    import json
    return json.loads((HERE / "golden" / "reference_vectors.json").read_text())

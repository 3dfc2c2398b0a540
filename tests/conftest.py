import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "embedding.cpp_amd"), os.path.join(REPO, "oracle"), os.path.join(REPO, "tests"),
          os.path.join(REPO, "tests", "golden")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through build/libbert.so on the GPU)")
    config.addinivalue_line("markers", "slow: long CPU-side case")


@pytest.fixture(scope="session")
def repo():
    return REPO


@pytest.fixture(scope="session")
def model_dir(tmp_path_factory):
    d = os.environ.get("BERT_AMD_MODEL_DIR")
    if d:
        os.makedirs(d, exist_ok=True)
        return d
    return str(tmp_path_factory.mktemp("models"))

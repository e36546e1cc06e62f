import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "parallel-systems-mpi-tfidf_amd")
sys.path.insert(0, os.path.join(PKG, "python"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, os.path.join(REPO, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 GPU (runs on the MI355X box)")


GOLDEN = os.path.join(REPO, "tests", "golden")


def golden_cases():
    return sorted(d for d in os.listdir(GOLDEN) if os.path.isdir(os.path.join(GOLDEN, d)))


@pytest.fixture(scope="session")
def engine():
    import tfidf_abi
    e = tfidf_abi.Engine(0)
    yield e
    e.close()

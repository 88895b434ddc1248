import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")
    config.addinivalue_line("markers", "slow: larger-than-unit inputs")


@pytest.fixture(scope="session")
def golden():
    import json
    here = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    with open(os.path.join(here, "golden.json")) as f:
        g = json.load(f)
    with open(os.path.join(here, "edge_cases.json")) as f:
        e = json.load(f)
    return g, e


@pytest.fixture(scope="session")
def testfa():
    here = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "test.fa")
    return "".join(l.strip() for l in open(here) if not l.startswith(">"))


@pytest.fixture(scope="session")
def gpu():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from kmer_hasher_amd import _lib
    _lib.lib()
    return torch


@pytest.fixture
def test_lib(gpu):
    """The test build of the library (libkmhgpu_test.so) for one test: the only build that reads
    the path selectors (KMHG_BUILD, KMHG_MAXR, ...), so tests that force a path request this."""
    from kmer_hasher_amd import _lib
    with _lib.using_test_build() as L:
        yield L

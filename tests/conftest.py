import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "hd-pissa_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device) -- run with -m gpu")
    config.addinivalue_line("markers", "slow: minutes of CPU time; runs with HDP_SLOW=1 (results recorded under "
                                       "profiles/ by the round that ran them)")


def pytest_collection_modifyitems(config, items):
    if os.environ.get("HDP_SLOW") == "1":
        return
    skip = pytest.mark.skip(reason="slow CPU test: set HDP_SLOW=1")
    for it in items:
        if "slow" in it.keywords:
            it.add_marker(skip)


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN


def gpu_available() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:  # pragma: no cover
        return False

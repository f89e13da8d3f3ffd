import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "burn-ppo_amd"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through libbppo.so's HIP path)")
    config.addinivalue_line("markers", "slow: longer CPU-side parity run")


def pytest_collection_modifyitems(config, items):
    # -m gpu on a box without a GPU should fail loudly, not skip silently; nothing to do here.
    pass


@pytest.fixture(scope="session")
def oracle():
    import oracle_ffi
    return oracle_ffi.lib()

import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


# torch before libcdbmerge in every session (one HIP runtime per process: torch's device init fails
# when the library's runtime came up first, so a GPU test file run on its own would not see the GPU)
import torch  # noqa: E402,F401


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run via gpurun)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


import pytest


@pytest.fixture(scope="session")
def c3_snaps():
    """BASELINE config C3's four replica snapshots at full size (10M ops each through the device op
    apply), built once per test session."""
    import torch  # noqa: F401  -- before libcdbmerge (one HIP runtime per process)
    import constdb_amd as cdb
    from constdb_amd import build, configs
    build.build()
    return configs.c3_snapshots(cdb, cdb.Context(0))

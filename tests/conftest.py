import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libtsdbhip on the device)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def pytest_collection_modifyitems(config, items):
    # GPU tests can only run where HIP sees a device; keep them selectable with -m gpu.
    pass


@pytest.fixture(autouse=True)
def _reset_developer_options():
    """Every test starts and ends with the library's developer options unset (tsdbhip_set_option
    is process-wide; tests set options to force an alternative kernel onto the same data)."""
    yield
    from opentsdb_amd import engine as E
    if E._lib is not None:
        E.reset_options()

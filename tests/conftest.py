import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
REFERENCE = '/root/reference'


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (HIP) GPU; run with -m gpu')
    config.addinivalue_line('markers', 'slow: long-running test')


def pytest_collection_modifyitems(config, items):
    import torch
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason='no GPU available')
    for item in items:
        if 'gpu' in item.keywords:
            item.add_marker(skip)


@pytest.fixture(scope='session')
def ext_ops():
    """Build (incrementally) and load the HIP extension; GPU tests FAIL if it cannot load."""
    from pytorch_raft_amd.build import build
    build()
    from pytorch_raft_amd.ops import _ext
    assert _ext.loaded(), _ext.load_error()
    return _ext.ops()


@pytest.fixture
def reference_core():
    """Import path of the read-only reference (CPU oracle); skip if it is not mounted."""
    core = os.path.join(REFERENCE, 'core')
    if not os.path.isdir(core):
        pytest.skip('reference not mounted')
    if core not in sys.path:
        sys.path.insert(0, core)
    return core

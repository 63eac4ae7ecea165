import os
if int(os.environ.get('GPU_MAX_HW_QUEUES') or 0) < 16:   # before torch loads HIP: see
    os.environ['GPU_MAX_HW_QUEUES'] = '16'                # mercury_amd/__init__.py
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
os.environ.setdefault('MASTER_ADDR', '127.0.0.1')


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (HIP device)')
    config.addinivalue_line('markers', 'slow: long-running test')


def pytest_collection_modifyitems(config, items):
    import torch
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason='no GPU in this environment')
    for it in items:
        if 'gpu' in it.keywords:
            it.add_marker(skip)


@pytest.fixture(autouse=True)
def _engine_teardown(request):
    """GPU tests: every engine a test built is closed when it ends, then the collector runs and
    the device drains -- no graph, event or exchange buffer of one test is released by a
    garbage-collection pass inside a later test's graph capture."""
    yield
    if 'gpu' not in request.keywords:
        return
    import gc
    import torch
    if not torch.cuda.is_available():
        return
    mod = sys.modules.get('mercury_amd.engine.native')
    if mod is not None:
        mod.close_all()
    gc.collect()
    torch.cuda.synchronize()

import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device); run with -m gpu")


def pytest_collection_modifyitems(config, items):
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(pytest.mark.timeout(900)) if hasattr(pytest.mark, "timeout") else None

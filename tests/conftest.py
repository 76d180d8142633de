import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "featuremetric-pnp_amd")
for p in (ROOT, PKG, os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")
    config.addinivalue_line("markers", "slow: longer CPU-side runs")


def pytest_collection_modifyitems(config, items):
    # A gpu-marked test on a host without a GPU is a configuration error, not a skip:
    # the driver selects them with -m gpu only on the MI355X box.
    pass

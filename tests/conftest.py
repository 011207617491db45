import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "efficient-path-planner_amd")
for p in (ROOT, PKG, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)

CONFIG = os.path.join(ROOT, "configs", "config.json")
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C ABI)")


@pytest.fixture(scope="session")
def cfg():
    from eppamd import config
    return config.load(CONFIG)


@pytest.fixture(scope="session")
def geom(cfg):
    from eppamd import config
    return config.geometry(cfg)

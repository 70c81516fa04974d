"""Shared test setup.

Markers: ``gpu`` -- needs an MI355X (runs the HIP path through the C-ABI).
Tests without the marker run on CPU: oracle vs golden vectors, host logic,
library/symbol checks and gloo multi-process tests.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: requires an AMD Instinct MI355X (gfx950) GPU")


@pytest.fixture(scope="session")
def oracle():
    import pyoracle
    pyoracle.build()
    return pyoracle.Oracle()


@pytest.fixture(scope="session")
def codec():
    import fleet_amd
    fleet_amd.build_if_needed = None
    return fleet_amd.Codec(0)


@pytest.fixture
def plan():
    """plan("update=tiled,...") sets launch-plan overrides (fleet_set_plan) for the
    test; the measured default plan is restored afterwards."""
    import fleet_amd
    yield fleet_amd.set_plan
    fleet_amd.set_plan("")

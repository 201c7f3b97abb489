import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")


# A bound on every test, however the suite is invoked (the driver runs plain `pytest -m gpu`):
# a test that hangs — a multi-GPU path meeting a node for the first time — ends the run with
# its stacks dumped instead of holding the box.  Thread method: a test stuck inside a GPU
# call cannot be interrupted by a signal.  Tests with their own timeout marker keep it.
DEFAULT_TEST_TIMEOUT_S = 900


def pytest_collection_modifyitems(config, items):
    try:
        import pytest_timeout  # noqa: F401
    except ImportError:   # the plugin is in this image; without it the suite runs unbounded
        return
    if config.getoption("timeout", None):   # --timeout on the command line wins
        return
    for item in items:
        if item.get_closest_marker("timeout") is None:
            item.add_marker(pytest.mark.timeout(DEFAULT_TEST_TIMEOUT_S, method="thread"))


@pytest.fixture(scope="session")
def golden_schedule():
    with open(os.path.join(GOLDEN, "schedule_ref.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def golden_inputs():
    with open(os.path.join(GOLDEN, "inputs_ref.json")) as f:
        return json.load(f)

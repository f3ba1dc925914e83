import os
import sys

import pytest

REPO = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
PKG = os.path.join(REPO, "moe-gan_cpsc541_amd")
for p in (REPO, PKG, os.path.join(REPO, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP) device")


def pytest_collection_modifyitems(config, items):
    import torch
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no GPU in this container")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture(autouse=True, scope="session")
def _library_tuning():
    """MOEGAN_TUNE="slot=value,..." (the bench's A/B switch) applied to the HIP library for a whole test session,
    so a parity test can be re-run on an alternative kernel form (e.g. slot 24: the router's lane-FMA forms)."""
    spec = os.environ.get("MOEGAN_TUNE", "")
    if spec:
        from moegan_mi import _lib
        for kv in filter(None, spec.split(",")):
            k, v = kv.split("=")
            _lib.call("mg_set_tuning", int(k), int(v))
    yield

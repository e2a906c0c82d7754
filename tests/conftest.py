import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "cs3602-llm-inference-acceleration_amd")
for p in (ROOT, PKG, os.path.join(ROOT, "tests", "golden")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")
    config.addinivalue_line("markers", "slow: full BASELINE-size cases")


def pytest_collection_modifyitems(config, items):
    try:
        import torch
        has_gpu = torch.cuda.is_available()
    except Exception:  # pragma: no cover
        has_gpu = False
    if has_gpu:
        return
    skip = pytest.mark.skip(reason="no GPU in this container")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture(autouse=True)
def _device_status_stays_clear(request):
    """After every GPU test: no engine kernel reported a device-side error (include/kvc.h
    kvc_device_status -- a selection row over its kernel's capacity, a clamped external index)
    through the engine's per-device status word.  Tests that provoke one use their own word."""
    yield
    if "gpu" not in request.node.keywords:
        return
    eng = sys.modules.get("kvcompress._engine")
    if eng is None:
        return
    for dev in list(eng._status_words):
        bits = eng.device_status(dev, clear=True)
        assert bits == 0, f"device {dev} status word 0x{bits:x} after {request.node.nodeid}"

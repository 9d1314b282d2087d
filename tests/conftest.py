import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session", autouse=True)
def _built():
    # Native artefacts are built in-tree beforehand (__graft_entry__.build());
    # only build here when they are missing (e.g. a fresh CPU checkout).
    from shadow_amd import build as b
    if not os.path.exists(b.LIB):
        b.build()
    if not os.path.exists(os.path.join(ROOT, "oracle", "liborc.so")):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)


@pytest.fixture(scope="session", autouse=True)
def _torch_device_first(request):
    # GPU runs: torch's HIP runtime must see the device before libshadowgpu.so
    # (ROCm 7.2's runtime) is loaded, or torch reports no device for the rest of
    # the process (a test file that uses torch.cuda after one that only drives
    # the library through ctypes would fail by test order alone).
    if any(item.get_closest_marker("gpu") for item in request.session.items):
        import torch
        if torch.cuda.is_available():
            torch.cuda.init()

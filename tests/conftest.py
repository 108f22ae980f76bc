import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "ray-tracing-one-weekend_amd")
sys.path.insert(0, PKG)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through librtow_hip.so on cuda:0)")
    # torch first: it ships its own libamdhip64 (same soname as ROCm's, which
    # librtow_hip.so links).  Whichever loads first serves both; if a test
    # module loaded librtow_hip.so (ROCm's HIP) before torch, torch.cuda saw
    # no device on the GPU box.  Importing torch here fixes the order for every
    # module, whatever pytest collects first.
    import torch  # noqa: F401
    # Build what is missing (the GPU box receives the prebuilt .so files).
    jobs = str(min(16, os.cpu_count() or 1))
    if not os.path.exists(os.path.join(REPO, "oracle", "librtow_oracle.so")):
        subprocess.run(["make", "-j", jobs, "-C", os.path.join(REPO, "oracle")], check=True)
    if not os.path.exists(os.path.join(PKG, "librtow_hip.so")):
        subprocess.run(["make", "-j", jobs, "-C", PKG], check=True)


@pytest.fixture(scope="session")
def gpu_ctx():
    import torch

    import rtow

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ctx = rtow.Context(0)
    yield ctx
    ctx.close()

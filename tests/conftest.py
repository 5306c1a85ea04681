import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950); run with -m gpu")
    # Build the library / oracle once if they are missing (fast; hipcc cross-compiles).
    need = [os.path.join(REPO, "tcp_amd", "libtcpcsum.so"), os.path.join(REPO, "oracle", "build", "liboracle.so")]
    if not all(os.path.exists(p) for p in need):
        subprocess.run(["make", "-C", REPO, "-j8"], check=True)


@pytest.fixture(autouse=True)
def _gpu_drained(request):
    """After every GPU test, wait for the device and surface any HIP error there,
    so an asynchronous fault is charged to the test whose work caused it."""
    yield
    if request.node.get_closest_marker("gpu") is None:
        return
    torch = sys.modules.get("torch")
    if torch is not None and torch.cuda.is_available() and torch.cuda.is_initialized():
        torch.cuda.synchronize()


@pytest.fixture(scope="session")
def golden():
    with open(os.path.join(REPO, "tests", "golden", "reference_vectors.json")) as f:
        return json.load(f)

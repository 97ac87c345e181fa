import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "simple-path-tracer_amd")
for p in (PKG, os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP library through the C ABI)")


@pytest.fixture(scope="session")
def renderer():
    # torch first, as in bench.py: the library then binds to the HIP runtime torch loaded, and the tests
    # that hand its device buffers to torch (tiles_device) see one runtime whichever subset runs
    import torch  # noqa: F401
    import sptr

    r = sptr.Renderer(0)
    yield r
    r.close()

import os
import sys
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parents[1]
if str(REPO) not in sys.path:
    sys.path.insert(0, str(REPO))

REFERENCE = Path("/root/reference/VulkanComputeShaderApplication")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")
    config.addinivalue_line("markers", "reference: needs the read-only reference checkout (build container only)")


def pytest_collection_modifyitems(config, items):
    have_ref = REFERENCE.exists()
    for it in items:
        # the marker, not the keyword: a parameter id "reference" is a keyword too
        if it.get_closest_marker("reference") is not None and not have_ref:
            it.add_marker(pytest.mark.skip(reason="reference checkout absent (GPU box)"))


@pytest.fixture(scope="session")
def gpu_renderer():
    """One HIP context for the whole GPU session (one process on the card)."""
    from vkcomputeshader_tinyraytracer_amd import Renderer

    r = Renderer(int(os.environ.get("TRT_DEVICE", "0")))
    yield r
    r.close()


@pytest.fixture(scope="session")
def golden_meshes():
    from vkcomputeshader_tinyraytracer_amd.scene import load_golden_meshes

    return load_golden_meshes()

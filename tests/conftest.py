"""Shared fixtures.  GPU tests are marked @pytest.mark.gpu and run only under
`pytest -m gpu` on an MI355X box; everything else runs on the CPU container."""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")
    config.addinivalue_line("markers", "slow: long-running (full-size models)")


def _pkg():
    import importlib.util
    spec = importlib.util.spec_from_file_location(
        "hip_llama_cpp_amd_boot", os.path.join(REPO, "hip_llama.cpp_amd", "__init__.py"))
    boot = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(boot)
    return boot.load()


@pytest.fixture(scope="session")
def pkg():
    return _pkg()


@pytest.fixture(scope="session")
def tl(pkg):
    """The product's ctypes bindings (loads libthallama.so; raises if missing)."""
    from hip_llama_cpp_amd import thallama
    thallama.lib()
    return thallama


@pytest.fixture(scope="session")
def gpu(tl):
    """A usable HIP device, or a hard failure (GPU tests must not silently pass)."""
    n = tl.device_count()
    if n < 1:
        pytest.fail("no HIP device visible: GPU tests need an MI355X (run them via gpurun)")
    tl.check(tl.lib().thallama_set_device(0))
    return tl


@pytest.fixture(scope="session")
def handle(gpu):
    return gpu.new_handle()


@pytest.fixture(scope="session")
def oracle():
    import oracle as O
    O.lib()
    return O

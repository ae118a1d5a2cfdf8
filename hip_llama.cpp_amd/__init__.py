"""hip_llama.cpp_amd — MI355X-native thaBLAS/thaDNN decode hot path.

The product is the C-ABI shared library ``lib/libthallama.so`` (HIP kernels for
gfx950 + the C++ host runtime), declared in ``include/*.h*`` at the repo root.
This package is the thin Python host mirror used by the tests, ``bench.py`` and
``__graft_entry__.smoke()``: ctypes bindings (``thallama``) and the model / state
helpers the reference's C++ driver performs (``model``).

The directory name contains a dot, so it is not importable by dotted name; load
it with :func:`load` (``__graft_entry__`` and ``tests/conftest.py`` do).
"""
import importlib.util
import os
import sys

ROOT = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(ROOT)
LIB_PATH = os.path.join(ROOT, "lib", "libthallama.so")


def load():
    """Return this package as module ``hip_llama_cpp_amd`` (registered in sys.modules)."""
    name = "hip_llama_cpp_amd"
    if name in sys.modules:
        return sys.modules[name]
    spec = importlib.util.spec_from_file_location(
        name, os.path.join(ROOT, "__init__.py"), submodule_search_locations=[ROOT])
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod

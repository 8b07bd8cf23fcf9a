import importlib.util
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, os.path.join(REPO, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); parity tests through the C ABI")


def load_pkg():
    spec = importlib.util.spec_from_file_location("ringpop_node_amd",
                                                  os.path.join(REPO, "ringpop-node_amd", "__init__.py"))
    mod = sys.modules.get("ringpop_node_amd")
    if mod is None:
        mod = importlib.util.module_from_spec(spec)
        sys.modules["ringpop_node_amd"] = mod
        spec.loader.exec_module(mod)
    return mod


def _stale(lib_path):
    """The library is missing or older than any of its sources (csrc/*, include/*.h): rebuild
    rather than test a stale shipped .so."""
    if not os.path.exists(lib_path):
        return True
    t = os.path.getmtime(lib_path)
    srcs = [os.path.join(REPO, "include", "ringpop_amd.h")]
    csrc = os.path.join(REPO, "ringpop-node_amd", "csrc")
    srcs += [os.path.join(csrc, f) for f in os.listdir(csrc) if f.endswith((".hip", ".h")) or f == "Makefile"]
    # (2 s of slack: a copy of the tree that does not keep modification times must not rebuild)
    return any(os.path.getmtime(x) > t + 2.0 for x in srcs if os.path.exists(x))


@pytest.fixture(scope="session")
def rpa():
    mod = load_pkg()
    if _stale(mod.LIB_PATH) and not os.environ.get("RP_AMD_LIB"):
        mod.build()
    return mod


@pytest.fixture(scope="session")
def orc():
    import pyoracle
    if not os.path.exists(pyoracle._LIB_PATH):
        pyoracle.build()
    return pyoracle


@pytest.fixture(scope="session")
def gpu(rpa):
    if rpa.device_count() < 1:
        pytest.fail("gpu-marked test but no HIP device visible (there is no CPU fallback)")
    return rpa

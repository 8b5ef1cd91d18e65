"""Shared fixtures.  `-m gpu` tests need an MI355X; everything else runs on CPU."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "gpu-ray_trace-rust_amd")
for p in (PKG, os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

SCENES = os.path.join(ROOT, "tests", "golden", "scenes")
ASSETS = os.path.join(ROOT, "assets_pack")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 (MI355X) device")
    config.addinivalue_line("markers", "slow: long-running")


def load_scene(name, **kw):
    from rt_amd import scheme

    sch = scheme.load_json(os.path.join(SCENES, name + ".json"))
    return scheme.load(sch, assets_root=ASSETS if os.path.isdir(ASSETS) else None, **kw)


@pytest.fixture(scope="session")
def rtlib():
    from rt_amd import abi

    return abi.load_library()


@pytest.fixture(scope="session")
def oracle():
    import oracle_py

    oracle_py.lib()
    return oracle_py


@pytest.fixture(scope="session")
def walled():
    return load_scene("walled")


@pytest.fixture(scope="session")
def gpu_available():
    from rt_amd import abi
    import ctypes as C

    n = C.c_int()
    abi.load_library().rt_device_count(C.byref(n))
    if n.value < 1:
        pytest.fail("no gfx950 device visible: -m gpu tests need an MI355X")
    return n.value

import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "droid-slam_amd")
for p in (ROOT, PKG, os.path.join(ROOT, "tests", "golden")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X); run with -m gpu")


@pytest.fixture(scope="session")
def golden_dir():
    return os.path.join(ROOT, "tests", "golden")


@pytest.fixture
def ba_order():
    """Force the pose order of the BA plans a test builds (droid_ba_set_order;
    None = the plan's own choice); restored afterwards."""
    import droid_backends
    prev = droid_backends.ba_set_order(None)
    droid_backends.ba_set_order(prev)
    yield droid_backends.ba_set_order
    droid_backends.ba_set_order(prev)


@pytest.fixture(scope="session")
def ab_backends():
    """droid_backends bound to the A/B library (lib/ab/libdroid_hip.so, `make ab`,
    -DDROID_AB=1): the measured-and-dropped kernel variants the product library
    no longer ships (alt v1 / V3, the Winograd tile, ...), for the bitwise
    cross-checks that tie them to the product kernels.  A second instance of
    the module (droid_backends_ab) over a second library; the product module
    stays bound to lib/libdroid_hip.so."""
    import importlib.util
    path = os.path.join(PKG, "lib", "ab", "libdroid_hip.so")
    if not os.path.exists(path):
        pytest.fail("the A/B library is missing: make -C droid-slam_amd/csrc (the default target builds it; "
                    "`make ab` alone does too, and so does __graft_entry__.build())")
    mod = sys.modules.get("droid_backends_ab")
    if mod is None:
        old = os.environ.get("DROID_HIP_LIB")
        os.environ["DROID_HIP_LIB"] = path
        try:
            pkg = os.path.join(PKG, "droid_backends")
            spec = importlib.util.spec_from_file_location("droid_backends_ab", os.path.join(pkg, "__init__.py"),
                                                          submodule_search_locations=[pkg])
            mod = importlib.util.module_from_spec(spec)
            sys.modules["droid_backends_ab"] = mod
            spec.loader.exec_module(mod)
        finally:
            if old is None:
                os.environ.pop("DROID_HIP_LIB", None)
            else:
                os.environ["DROID_HIP_LIB"] = old
    assert mod.AB_BUILD and mod._lib.LIB_PATH == path
    return mod

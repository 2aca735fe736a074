import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libggd's C ABI)")


@pytest.fixture(scope="session")
def pkg():
    import __graft_entry__ as ge
    return ge.load_package()


@pytest.fixture(scope="session")
def beat_cfg(pkg):
    return pkg.load_config(os.path.join(ROOT, "configs", "beat-ours.json"))


@pytest.fixture(scope="session")
def tedexp_cfg(pkg):
    return pkg.load_config(os.path.join(ROOT, "configs", "tedexp-ours.json"))


def oracle_cfg(arch):
    return {k: arch[k] for k in ("type", "d_model", "decoder", "heads", "n_layers")}


@pytest.fixture(autouse=True)
def _settle_gpu_loops(request):
    """GPU tests: after each test, ggd_sync every open context -- a persistent loop that failed after
    its non-blocking ggd_sample returned fails the test that issued it."""
    yield
    if request.node.get_closest_marker("gpu") is None:
        return
    import __graft_entry__ as ge
    ge.load_package().sync_all()

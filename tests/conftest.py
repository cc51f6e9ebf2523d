import pathlib
import sys

import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]
for p in (ROOT, ROOT / "mpc-iris-code_amd"):
    if str(p) not in sys.path:
        sys.path.insert(0, str(p))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) and the built libiris_hip.so")


@pytest.fixture(scope="session")
def device():
    import iris_hip

    dev = iris_hip.Device(0)  # raises loudly if no gfx950 device / library
    yield dev
    dev.close()


@pytest.fixture
def hooked_device(monkeypatch):
    """hooked_device(IRIS_X="v", ...) opens device 0 with test hooks.  The library reads its
    knobs once, when a device opens, and honours the test-only ones only with
    IRIS_TEST_HOOKS=1: both are set just for the open and removed again, so no other
    device (or helper thread) sees them.  Devices are closed after the test."""
    import iris_hip

    opened = []

    def open_(**env):
        with monkeypatch.context() as m:
            m.setenv("IRIS_TEST_HOOKS", "1")
            for k, v in env.items():
                m.setenv(k, str(v))
            dev = iris_hip.Device(0)
        opened.append(dev)
        assert dev.config()["test_hooks"] == "1" and "ignored" not in dev.config()
        return dev

    yield open_
    for d in opened:
        d.close()


@pytest.fixture(scope="session")
def golden():
    import numpy as np

    with np.load(ROOT / "tests" / "golden" / "golden_v1.npz", allow_pickle=False) as z:
        return {k: z[k] for k in z.files}

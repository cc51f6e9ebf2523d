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


@pytest.fixture(scope="session")
def golden():
    import numpy as np

    with np.load(ROOT / "tests" / "golden" / "golden_v1.npz", allow_pickle=False) as z:
        return {k: z[k] for k in z.files}

import importlib
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "oracle"))
PKG_NAME = "tfg---quantum-byzantine-agreement_amd"
GOLDEN = ROOT / "tests" / "golden"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and the built libqba.so")


@pytest.fixture(scope="session")
def pkg():
    return importlib.import_module(PKG_NAME)


def sub(name):
    return importlib.import_module(f"{PKG_NAME}.{name}")


@pytest.fixture(scope="session")
def engine():
    eng = sub("engine").Engine(0)
    yield eng
    eng.close()

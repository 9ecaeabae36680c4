import ctypes
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")


@pytest.fixture(scope="session")
def golden():
    with open(os.path.join(ROOT, "tests", "golden", "corpus.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def kat():
    with open(os.path.join(ROOT, "tests", "golden", "kat.json")) as f:
        return json.load(f)["cases"]


@pytest.fixture(scope="session")
def oracle():
    from tests import oracle_lib
    return oracle_lib.Oracle()


@pytest.fixture(scope="session")
def synth():
    from tests import oracle_lib
    return oracle_lib.synth

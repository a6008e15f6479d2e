import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "map-oxidize_amd"), os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")
    config.addinivalue_line("markers", "slow: long-running (large corpora)")


@pytest.fixture(scope="session")
def kat_cases():
    with open(os.path.join(ROOT, "tests", "golden", "kat.json")) as f:
        return json.load(f)["cases"]


def kat_expected(case):
    if "error" in case:
        return "error"
    return [(bytes.fromhex(w), c) for w, c in case["expected"]]

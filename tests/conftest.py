import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "spaced-kmer-sketching_amd")
for p in (PKG, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device)")


@pytest.fixture(scope="session", autouse=True)
def _built():
    # oracle (checker) + libsks.so; both are no-ops when up to date.  On the GPU
    # box /root/reference is absent and the prebuilt .so files are used.
    if not os.path.exists(os.path.join(ROOT, "oracle", "lib", "libsks_oracle.so")):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    if not os.path.exists(os.path.join(PKG, "lib", "libsks.so")):
        subprocess.run(["make", "-s", "-C", PKG, "-j8"], check=True)
    yield


@pytest.fixture(scope="session")
def golden():
    import json

    def load(name):
        with open(os.path.join(GOLDEN, name)) as f:
            return json.load(f)
    return load

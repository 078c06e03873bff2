"""Shared fixtures. `-m "not gpu"` runs the oracle-vs-golden, host-logic and gloo tests on CPU;
`-m gpu` runs the device parity tests through the C-ABI (librtgpu.so) on an MI355X."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracing-practice_amd", "python"))
sys.path.insert(0, os.path.join(REPO, "tests"))
GOLDEN = os.path.join(REPO, "tests", "golden")
os.environ.setdefault("RTW_IMAGES", GOLDEN)

LIBS = [os.path.join(REPO, "raytracing-practice_amd", "lib", "librtgpu.so"),
        os.path.join(REPO, "raytracing-practice_amd", "lib", "librtscenes.so"),
        os.path.join(REPO, "oracle", "lib", "liboracle.so")]


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) and runs the HIP kernels")


def _ensure_built():
    if all(os.path.exists(p) for p in LIBS):
        return
    subprocess.run(["make", "-j8", "-C", os.path.join(REPO, "raytracing-practice_amd")], check=True)
    subprocess.run(["make", "-C", os.path.join(REPO, "oracle")], check=True)


@pytest.fixture(scope="session")
def lib():
    _ensure_built()
    import rtgpu

    return rtgpu.Library()


@pytest.fixture(scope="session")
def scenes():
    _ensure_built()
    import rtgpu

    return rtgpu.SceneLibrary()


@pytest.fixture(scope="session")
def oracle():
    _ensure_built()
    from oracle_bind import Oracle

    return Oracle()


@pytest.fixture(scope="session")
def golden():
    with open(os.path.join(GOLDEN, "reference_golden.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def gpu_lib(lib):
    if lib.device_count() < 1:
        pytest.fail("GPU test requested but no HIP device is visible (no CPU fallback exists)")
    return lib

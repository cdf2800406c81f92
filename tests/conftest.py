import sys
from pathlib import Path

import numpy as np
import pytest

REPO = Path(__file__).resolve().parents[1]
TESTS = Path(__file__).resolve().parent
GOLDEN = TESTS / "golden"
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(TESTS))

import __graft_entry__  # noqa: E402
from oracle_lib import (FNV_PRIME, PROBE_FNV_BASIS, SURVEY_FNV, SURVEY_FNV_FMA,  # noqa: E402,F401
                        Oracle, probe_fnv)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu)")
    config.addinivalue_line("markers", "slow: long-running (CPU oracle heavy)")


@pytest.fixture(scope="session")
def pkg():
    """The product package (opencl-ray-tracer_amd/), librt_hip.so built."""
    mod = __graft_entry__.load_package()
    if not mod.library_path().exists():
        __graft_entry__._make(__graft_entry__.PKG_DIR / "csrc", "all")
    mod.library()
    return mod


@pytest.fixture(scope="session")
def oracle():
    return Oracle()


@pytest.fixture(scope="session")
def rt(pkg):
    """One HIP context for the whole GPU session (tests run in one process)."""
    tracer = pkg.RayTracer(0)
    yield tracer
    tracer.close()


def load_golden(name):
    with np.load(GOLDEN / f"{name}.npz", allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def golden_scene(pkg, g):
    return pkg.Scene(g["sphere_origins"], g["sphere_radius"], g["sphere_colours"],
                     g["cube_vertices"], g["cube_colours"])


"""Host-side sanitizer build: the C ABI's scene helpers and
argument / pointer arithmetic (csrc/rt_scene.cpp, csrc/rt_args.cpp) and the
oracle, built with -fsanitize=address,undefined (`make -C
opencl-ray-tracer_amd/csrc asan`) and run over their edge cases
(tests/asan/rt_asan_check.cpp).  No GPU."""
import shutil
import subprocess
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parents[1]
BIN = REPO / "tests" / "asan" / "build" / "rt_asan_check"

pytestmark = pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")


@pytest.fixture(scope="module")
def asan_bin():
    subprocess.run(["make", "-s", "-C", str(REPO / "opencl-ray-tracer_amd" / "csrc"), "asan"],
                   check=True, capture_output=True, text=True)
    return BIN


def test_host_code_clean_under_asan_ubsan(asan_bin):
    r = subprocess.run([str(asan_bin)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "asan check ok" in r.stdout
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr


def test_sanitizer_is_live(asan_bin):
    """Negative control: a deliberate one-element overrun is reported."""
    r = subprocess.run([str(asan_bin), "--control-overrun"], capture_output=True, text=True,
                       timeout=60)
    assert r.returncode != 0 and "heap-buffer-overflow" in r.stderr

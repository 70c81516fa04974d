"""CPU checks of the codec arithmetic the gfx950 kernels run (codec_math.h),
compiled for the host, against the oracle: fast paths and general functions,
sampled (~1e8 inputs). `tests/native/check_math exhaustive` covers every input
(run during development). Also pins the oracle's digests
used by the GPU self-test (tests/golden/digests.json) on a sampled recompute."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _clang():
    for c in ("/opt/rocm/lib/llvm/bin/clang++", shutil.which("clang++")):
        if c and os.path.exists(c):
            return c
    return None


@pytest.fixture(scope="module")
def check_math(tmp_path_factory):
    clang = _clang()
    if clang is None:
        pytest.skip("no clang++ for the host build of codec_math.h")
    d = tmp_path_factory.mktemp("native")
    obj = d / "fo.o"
    subprocess.check_call(["gcc", "-O2", "-c", "-ffp-contract=off", os.path.join(ROOT, "oracle", "fleet_oracle.c"),
                           "-o", str(obj)])
    exe = d / "check_math"
    subprocess.check_call([clang, "-std=c++17", "-O2", "-mfma", "-ffp-contract=off", "-pthread",
                           os.path.join(ROOT, "tests", "native", "check_math.cpp"), str(obj), "-o", str(exe), "-lm"])
    return str(exe)


def test_codec_math_matches_oracle_sampled(check_math):
    r = subprocess.run([check_math, "sample"], capture_output=True, text=True, timeout=600)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ALL OK" in r.stdout

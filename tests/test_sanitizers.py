"""CPU: AddressSanitizer + UndefinedBehaviorSanitizer builds of the host-side C/C++ code
("race detection / sanitizers"): the C oracle (oracle/nngp_oracle.c, the
checker every parity test trusts) driven through all its entry points by
tests/host/oracle_check.c, and the device math header's host build
(tests/host/math_check.cpp, pynngp_amd/csrc/nngp_math.h with NNGP_MATH_HOST).
Any sanitizer report aborts the program (-fno-sanitize-recover=all).  GPU-side
sanitizers are not available on this pool; the HIP kernels' own bounds are covered by
the parity tests' edge cases (N <= m, m = 0, empty shards, bad indices).
"""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-g", "-O1"]


def _env():
    env = dict(os.environ)
    env["ASAN_OPTIONS"] = "detect_leaks=1:abort_on_error=1"
    env["UBSAN_OPTIONS"] = "print_stacktrace=1:halt_on_error=1"
    env["OMP_NUM_THREADS"] = "2"
    return env


@pytest.fixture(scope="module")
def tmp(tmp_path_factory):
    if shutil.which("gcc") is None or shutil.which("g++") is None:
        pytest.skip("no host compiler")
    return tmp_path_factory.mktemp("san")


def test_oracle_under_asan_ubsan(tmp):
    exe = str(tmp / "oracle_check")
    subprocess.run(["gcc", "-std=c11", "-fopenmp", "-ffp-contract=off", *SAN, os.path.join(HERE, "host", "oracle_check.c"),
                    os.path.join(ROOT, "oracle", "nngp_oracle.c"), "-o", exe, "-lm"], check=True)
    out = subprocess.run([exe], capture_output=True, text=True, env=_env(), timeout=600)
    assert out.returncode == 0, out.stdout + out.stderr
    assert out.stdout.startswith("ok "), out.stdout
    assert "runtime error" not in out.stderr and "AddressSanitizer" not in out.stderr, out.stderr


def test_math_header_under_asan_ubsan(tmp):
    exe = str(tmp / "math_check")
    subprocess.run(["g++", "-std=c++17", "-ffp-contract=off", *SAN, os.path.join(HERE, "host", "math_check.cpp"),
                    "-o", exe, "-lm"], check=True)
    out = subprocess.run([exe], capture_output=True, text=True, env=_env(), timeout=600)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "runtime error" not in out.stderr and "AddressSanitizer" not in out.stderr, out.stderr

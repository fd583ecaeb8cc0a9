"""CPU: accuracy of the kernel's fp64 exp2 / sqrt / rsqrt / covariance (nngp_math.h).

The header compiles on the host (NNGP_MATH_HOST, v_rsq_f64 emulated at its
measured ~2^-24 accuracy, tools/ubench/rsq_acc.hip) so the table exp and the
second-order sqrt / rsqrt refinements are checked
against libm without a GPU.  Bounds: table exp <= 2 ulp, sqrt <= 1 ulp, rsqrt <= 2
ulp, covariance relative error <= 2e-14 (the exp argument phi*d ~ 20 carries
its own rounding, amplified by |phi d| in the exponential).
"""
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def math_errors(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("math") / "math_check")
    subprocess.run(["g++", "-O2", "-ffp-contract=off", "-std=c++17", os.path.join(HERE, "host", "math_check.cpp"),
                    "-o", exe, "-lm"], check=True)
    out = subprocess.run([exe], check=True, capture_output=True, text=True).stdout.split()
    return [float(x) for x in out[:5]] + [int(out[5])]


def test_exp2_sqrt_rsqrt_ulp(math_errors):
    e_exp2, e_sqrt, e_rsqrt = math_errors[:3]
    assert e_exp2 <= 2.0 and e_sqrt <= 1.0 and e_rsqrt <= 2.0


def test_covariance_relative_error(math_errors):
    assert math_errors[3] <= 2e-14 and math_errors[4] <= 2e-14


def test_special_values_exact(math_errors):
    assert math_errors[5] == 1

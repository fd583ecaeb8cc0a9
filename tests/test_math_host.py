"""CPU: accuracy of the kernel's fp64 exp2 / sqrt / rsqrt / covariance (nngp_math.h).

The header compiles on the host (NNGP_MATH_HOST, v_rsq_f64 emulated at its
measured ~2^-24 accuracy, tools/ubench/rsq_acc.hip) so the table exp and the
second-order sqrt / rsqrt refinements are checked
against libm without a GPU.  Bounds: table exp <= 2 ulp, sqrt <= 1 ulp, rsqrt <= 2
ulp, every covariance kind within 4e-16 (Matern: 8e-16) of sigma2 (absolute error relative to the
diagonal scale, the accuracy the factorisation needs).
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
    return {k: float(v) for k, v in zip(out[::2], out[1::2])}


def test_exp2_sqrt_rsqrt_ulp(math_errors):
    assert math_errors["exp2_ulp"] <= 2.0 and math_errors["sqrt_ulp"] <= 1.0 and math_errors["rsqrt_ulp"] <= 2.0
    # the unit-variance table with the exponent added to the entry's exponent field: same bits
    # as the ldexp form, so the same bound
    assert math_errors["exp2_unit_ulp"] <= 2.0


@pytest.mark.parametrize("kind", range(5))
def test_covariance_error_every_kind(math_errors, kind):
    """exponential, matern32, matern52, gaussian, spherical: both device forms (sigma2 table and
    unit variance x sigma2) within a few ulp of sigma2 of the long-double value (the Matern
    polynomials add their own 1-3 ulp to the exp's)."""
    bound = 8e-16 if kind in (1, 2) else 4e-16
    assert math_errors[f"cov{kind}_rel"] <= bound, math_errors
    assert math_errors[f"cov{kind}_unit_rel"] <= bound, math_errors


def test_special_values_exact(math_errors):
    assert math_errors["special"] == 1

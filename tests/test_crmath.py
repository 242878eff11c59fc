"""The device's correctly rounded atan / sin / cos / tan (csrc/cr_math.h), on the host.

cr_math.h compiles for host and device; the oracle's CR build (oracle/lib/liboracle_cr.so)
exports it.  Checked here: (1) on random arguments every result is the correctly rounded value
(80-digit decimal reference, tools/gen_crmath_tables.py), (2) against glibc, the functions the
reference's numba code calls, results agree bitwise on all but a small fraction of arguments
(where glibc is off by just over half an ulp: printed by oracle/crcheck/crmath_check.cpp).
"""
import ctypes
import json
import math
import os
import subprocess
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)


@pytest.fixture(scope="module")
def cr():
    subprocess.check_call(["make", "-s", "-C", os.path.join(REPO, "oracle"), "lib/liboracle_cr.so"])
    L = ctypes.CDLL(os.path.join(REPO, "oracle", "lib", "liboracle_cr.so"))
    for f in ("oref_cr_atan", "oref_cr_sin", "oref_cr_cos", "oref_cr_tan"):
        getattr(L, f).restype = ctypes.c_double
        getattr(L, f).argtypes = [ctypes.c_double]
    return L


@pytest.fixture(scope="module")
def D():
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import gen_crmath_tables as G

    return G


def test_correctly_rounded(cr, D):
    from decimal import Decimal

    rng = np.random.default_rng(3)
    xs = np.concatenate([np.ldexp(1 + rng.random(150), rng.integers(-30, 30, 150)) * rng.choice([-1, 1], 150),
                         (rng.random(150) - 0.5) * 14])
    for x in xs:
        ref = float(D.atan(Decimal(float(x))))
        assert cr.oref_cr_atan(float(x)) == ref, ("atan", float(x).hex())
    P = D.PI
    for x in (rng.random(300) - 0.5) * 14:
        X = Decimal(float(x))
        k = (X / (2 * P)).to_integral_value()
        s = D.sin(X - 2 * P * k)
        c = D.sin(X - 2 * P * k + P / 2)
        assert cr.oref_cr_sin(float(x)) == float(s), ("sin", float(x).hex())
        assert cr.oref_cr_cos(float(x)) == float(c), ("cos", float(x).hex())
        if abs(c) > Decimal("1e-3"):
            assert cr.oref_cr_tan(float(x)) == float(s / c), ("tan", float(x).hex())


def test_agrees_with_glibc(tmp_path):
    exe = str(tmp_path / "crmath_check")
    subprocess.check_call(["g++", "-O2", "-mfma", "-ffp-contract=off", "-std=c++17", "-o", exe,
                           os.path.join(REPO, "oracle", "crcheck", "crmath_check.cpp"), "-lm"])
    r = json.loads(subprocess.check_output([exe, "300000"]))
    for name, v in r.items():
        assert v["mismatch"] <= 3e-3 * v["n"], (name, v)


def test_special_arguments(cr):
    inf = float("inf")
    assert cr.oref_cr_atan(inf) == math.atan(inf) and cr.oref_cr_atan(-inf) == math.atan(-inf)
    assert math.isnan(cr.oref_cr_atan(float("nan")))
    for f, g in ((cr.oref_cr_atan, math.atan), (cr.oref_cr_sin, math.sin), (cr.oref_cr_tan, math.tan)):
        for x in (0.0, -0.0, 1e-300, -3e-20, 5e-9):
            assert math.copysign(1, f(x)) == math.copysign(1, g(x)) and f(x) == g(x), (f, x)
    assert cr.oref_cr_cos(0.0) == 1.0 and cr.oref_cr_atan(1.0) == math.atan(1.0)
    assert cr.oref_cr_atan(1e300) == math.atan(1e300) and cr.oref_cr_sin(1e6) == math.sin(1e6)

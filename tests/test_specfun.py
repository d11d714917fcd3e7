"""The arithmetic boundary the reference takes from absent third-party code
(GSL gsl_sf_dilog / gsl_sf_complex_dilog_xy_e, polylogarithm::Li2/Li3 and
the C libm), restated in the oracle and in the product's device headers.

1. Oracle vs mpmath known answers (tests/golden/specfun_kat.json, generated
   by tests/golden/make_specfun_kat.py at 40 digits): the restatement is
   accurate, i.e. it is a faithful stand-in for GSL / polylogarithm.
2. Product device code (nusiprop_amd/csrc/*.hpp compiled for the host by
   tests/hostcheck) vs oracle: BIT-IDENTICAL on every vector.  This is what
   makes the GPU tables bit-exact to the oracle (tests/test_gpu_parity.py).
3. GSL's own algorithms (the reference-order arithmetic: oracle/ora_gsl.c,
   nusiprop_amd/csrc/nusi_gsl.hpp) against the same known answers, with
   vectors on GSL's branch points (|z| 0.25 / 0.98 / 1, x 0.732), and the
   device restatement bit-identical to the oracle's on them and on seeded
   random arguments.
"""
import ctypes
import json
import math
import os

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
KAT = json.load(open(os.path.join(HERE, "golden", "specfun_kat.json")))
D = ctypes.c_double


@pytest.fixture(scope="module")
def olib(oracle_mod):
    L = oracle_mod.lib()
    for f in ["ora_log", "ora_log1p", "ora_exp", "ora_atan", "ora_atanh", "ora_li2"]:
        getattr(L, f).restype = D
        getattr(L, f).argtypes = [D]
    L.ora_atan2.restype = D
    L.ora_atan2.argtypes = [D, D]
    return L


@pytest.fixture(scope="module")
def hlib():
    from tests.hostcheck import build_hostcheck
    H = build_hostcheck()
    H.hc_li2.restype = D
    H.hc_li2.argtypes = [D]
    H.hc_li3.restype = D
    H.hc_li3.argtypes = [D]
    H.hc_cli2.argtypes = [D, D, ctypes.POINTER(D), ctypes.POINTER(D)]
    H.hc_gsl_li2.restype = D
    H.hc_gsl_li2.argtypes = [D]
    H.hc_gsl_cli2.argtypes = [D, D, ctypes.POINTER(D), ctypes.POINTER(D)]
    H.hc_gsl_clausen.restype = D
    H.hc_gsl_clausen.argtypes = [D]
    H.hc_hypot.restype = D
    H.hc_hypot.argtypes = [D, D]
    return H


def _ulps(a, b):
    if a == b:
        return 0.0
    return abs(a - b) / math.ulp(abs(b))


@pytest.mark.parametrize("name", ["log", "log1p", "exp", "atan", "atanh"])
def test_libm_vs_mpmath(olib, name):
    f = getattr(olib, "ora_" + name)
    worst = max(_ulps(f(x), y) for x, y in KAT[name])
    assert worst <= 1.0, worst        # fdlibm-class accuracy (< 1 ulp)


def test_atan2_vs_mpmath(olib):
    assert max(_ulps(olib.ora_atan2(p, q), y) for p, q, y in KAT["atan2"]) <= 1.0


def test_dilog_real_vs_mpmath(oracle_mod):
    """gsl_sf_dilog: Re Li2(x) on the whole real line (aux.hpp:112-165 call sites)."""
    for x, y in KAT["li2_real"]:
        v = oracle_mod.dilog(x)
        assert abs(v - y) <= 4e-15 * abs(y) + 1e-300, (x, v, y)


def test_li2_polylog_vs_mpmath(olib):
    """polylogarithm::Li2 (nuSIprop.hpp:628-636, the DSNB source) for x <= 1."""
    for x, y in KAT["li2_real"]:
        if x <= 1:
            v = olib.ora_li2(x)
            assert abs(v - y) <= 1e-15 * abs(y) + 1e-300, (x, v, y)


def test_complex_dilog_vs_mpmath(oracle_mod):
    """gsl_sf_complex_dilog_xy_e incl. GSL's real-axis convention Im = -pi ln x, x >= 1."""
    for x, y, re, im in KAT["li2_complex"]:
        z = oracle_mod.complex_dilog(x, y)
        assert abs(z - complex(re, im)) <= 1e-15 * max(1.0, abs(complex(re, im))), (x, y, z, re, im)


def test_complex_dilog_near_axis_vs_mpmath(oracle_mod):
    """The Taylor path in iy about the real axis (|y| <= 2.5e-3 min(|x|, |1 - x|)), both sides of the
    cut x > 1, next to the branch point 1 and next to 0: modulus-relative error <= 1e-15."""
    assert len(KAT["li2_complex_axis"]) >= 390
    for x, y, re, im in KAT["li2_complex_axis"]:
        z = oracle_mod.complex_dilog(x, y)
        ref = complex(re, im)
        assert abs(z - ref) <= 1e-15 * abs(ref), (x, y, z, re, im)


def test_li3_vs_mpmath(oracle_mod):
    for x, y in KAT["li3"]:
        v = oracle_mod.li3(x)
        assert abs(v - y) <= 1e-15 * abs(y), (x, v, y)


def test_device_specfun_bit_identical_to_oracle(oracle_mod, hlib):
    re, im = D(), D()
    for x, _ in KAT["li2_real"]:
        assert hlib.hc_li2(x) == oracle_mod.dilog(x), x
    for x, y, _, _ in KAT["li2_complex"] + KAT["li2_complex_axis"]:
        hlib.hc_cli2(x, y, ctypes.byref(re), ctypes.byref(im))
        z = oracle_mod.complex_dilog(x, y)
        assert (re.value, im.value) == (z.real, z.imag), (x, y)
    for x, _ in KAT["li3"]:
        assert hlib.hc_li3(x) == oracle_mod.li3(x), x


# ---- GSL's algorithms (reference-order arithmetic), round 5
def test_gsl_dilog_real_vs_mpmath(oracle_mod):
    """gsl_sf_dilog by GSL's algorithm (dilog_xge0 and the x < 0 reduction): <= 4e-15 of max(1, |Li2|) (relative
    away from Re Li2's zero at x ~ 12.6, where only the absolute error is meaningful)."""
    for x, y in KAT["li2_real"]:
        v = oracle_mod.gsl_dilog(x)
        assert abs(v - y) <= 4e-15 * max(1.0, abs(y)), (x, v, y)
        if abs(x - 12.6) > 0.5:
            assert abs(v - y) <= 4e-15 * abs(y) + 1e-300, (x, v, y)


def _gsl_series3_mp(x, y):
    """GSL's value where dilogc_series_3 runs (|w| in (0.98, 1), Re w <= 0.732 for w = z or 1/z), in exact arithmetic:
    the six-term expansion in log|w| (dilog.c) unwound as gsl_sf_complex_dilog_xy_e does; None elsewhere."""
    import mpmath as mp
    z = mp.mpc(x, y)
    w = z if abs(z) < 1 else 1 / z
    r = abs(w)
    if not (0.98 < r < 1 and w.real <= 0.732):
        return None
    th, a = mp.arg(w), mp.log(r)
    c, s_ = mp.cos(th), mp.sin(th)
    omc = 1 - c
    hre = [mp.pi ** 2 / 6 + (th * th - 2 * mp.pi * abs(th)) / 4, -mp.log(2 * omc) / 2, -0.5, -0.5 / omc, 0,
           (2 + c) / (2 * omc ** 2), 0]
    him = [mp.clsin(2, th), -mp.atan2(-s_, omc), s_ / (2 * omc), 0, -s_ / (2 * omc ** 2), 0,
           s_ / (2 * omc ** 5) * (8 * omc - s_ * s_ * (3 + c))]
    v = sum(a ** n / mp.factorial(n) * mp.mpc(hre[n], him[n]) for n in range(7))
    if abs(z) > 1:
        v = -v - mp.log(-z) ** 2 / 2 - mp.pi ** 2 / 6
    return complex(v)


@pytest.mark.parametrize("kat", ["li2_complex", "li2_complex_axis", "li2_complex_unit"])
def test_gsl_complex_dilog_vs_mpmath(oracle_mod, kat):
    """gsl_sf_complex_dilog_xy_e by GSL's algorithm, incl. the real-axis convention, the unit circle (Lewin's
    formula, dilogc_series_3) and the 0.25 / 0.732 / 0.98 splits: modulus-relative error <= 4e-15 against Li2 --
    except where dilogc_series_3 runs, whose six-term expansion is GSL's own truncation (up to ~1e-13 at |z| = 0.98):
    there the reference value is that expansion evaluated exactly (_gsl_series3_mp), which pins the algorithm."""
    for x, y, re, im in KAT[kat]:
        z = complex(*oracle_mod.gsl_complex_dilog(x, y))
        ref = complex(re, im)
        s3 = _gsl_series3_mp(x, y) if abs(complex(x, y)) != 1.0 else None
        if s3 is not None and abs(z - ref) > 4e-15 * abs(ref):
            assert abs(z - ref) <= 1e-12 * abs(ref), (x, y, z, ref)
            ref = s3
        assert abs(z - ref) <= 4e-15 * max(1e-300, abs(ref)), (x, y, z, ref)


def test_gsl_clausen_vs_mpmath(oracle_mod):
    for x, y in KAT["clausen"]:
        assert abs(oracle_mod.gsl_clausen(x) - y) <= 2e-15 * abs(y) + 1e-15, (x, y)   # x (c - log x) near pi: absolute


def test_device_gsl_bit_identical_to_oracle(oracle_mod, hlib):
    """nusi_gsl.hpp (the GPU's NUSI_OPT_REFERENCE_ORDER arithmetic) == oracle/ora_gsl.c bit for bit, on every KAT
    vector and on 26 000 seeded random arguments around GSL's branch points and over 20 decades of |z| -- including
    its rewrite of the series' stopping tests as multiply-compare and their test-free first loops (exact, nusi_gsl.hpp)."""
    import numpy as np
    rng = np.random.default_rng(20250213)
    re, im = D(), D()
    xs = [x for x, _ in KAT["li2_real"]] + list(rng.uniform(-40, 40, 3000)) + list(rng.uniform(-1.5, 2.5, 3000))
    xs += [0.25, 0.5, 1.0, 1.01, 2.0, -0.25, -0.5, -2.0, 0.0] + list(np.nextafter([0.25, 0.5, 1.0, 1.01, 2.0], 3))
    xs += list(10.0 ** rng.uniform(-20, 0, 2000)) + list(-(10.0 ** rng.uniform(-20, 3, 1000)))   # (series test-free prefixes)
    for x in xs:
        assert hlib.hc_gsl_li2(float(x)) == oracle_mod.gsl_dilog(float(x)), x
    zs = [(x, y) for x, y, _, _ in KAT["li2_complex"] + KAT["li2_complex_axis"] + KAT["li2_complex_unit"]]
    t = rng.uniform(-np.pi, np.pi, 6000)
    rad = np.concatenate([rng.uniform(0.0, 3.0, 3000), 1 + rng.uniform(-0.05, 0.05, 3000)])
    zs += list(zip(rad * np.cos(t), rad * np.sin(t)))
    zs += list(zip(rng.uniform(-3, 3, 4000), rng.uniform(-1e-3, 1e-3, 4000)))
    rs, ts = 10.0 ** rng.uniform(-20, 0.5, 3000), rng.uniform(-np.pi, np.pi, 3000)
    zs += list(zip(rs * np.cos(ts), rs * np.sin(ts)))
    for x, y in zs:
        hlib.hc_gsl_cli2(float(x), float(y), ctypes.byref(re), ctypes.byref(im))
        assert (re.value, im.value) == oracle_mod.gsl_complex_dilog(float(x), float(y)), (x, y)
    for x, _ in KAT["clausen"]:
        assert hlib.hc_gsl_clausen(x) == oracle_mod.gsl_clausen(x), x
    for a, b in rng.normal(size=(2000, 2)) * 10.0 ** rng.uniform(-200, 200, size=(2000, 1)):
        assert hlib.hc_hypot(float(a), float(b)) == oracle_mod.hypot(float(a), float(b)), (a, b)


def test_gsl_complex_dilog_conjugate_symmetric(oracle_mod, hlib):
    """gsl_sf_complex_dilog_xy_e(x, -y) == conj(gsl_sf_complex_dilog_xy_e(x, y)) bit for bit (the oracle's restatement
    of GSL and the device's): the reference-order Gamma forms Li2 of conj(z1) as conj(Li2(z1)) (gamma_k, nusi_physics.hpp),
    so this symmetry must hold exactly, on every branch -- the unit circle, inversion, reflection, series 1 / 2 / 3."""
    import numpy as np
    rng = np.random.default_rng(20261018)
    re, im = D(), D()
    t = rng.uniform(-np.pi, np.pi, 8000)
    rad = np.concatenate([rng.uniform(0.0, 3.0, 4000), 1 + rng.uniform(-0.05, 0.05, 2000), 10.0 ** rng.uniform(-20, 3, 2000)])
    zs = list(zip(rad * np.cos(t), rad * np.sin(t))) + [(x, y) for x, y, _, _ in KAT["li2_complex"] + KAT["li2_complex_unit"]]
    # the Gamma quotients themselves: z1 = i (1 + s) / (gr + 2 i)
    for s, gr in zip(10.0 ** rng.uniform(-5, 4, 2000), 10.0 ** rng.uniform(-9, 0, 2000)):
        d = gr * gr + 4.0
        zs.append(((1 + s) * 2.0 / d, (1 + s) * gr / d))
    for x, y in zs:
        if y == 0.0:
            continue
        a = oracle_mod.gsl_complex_dilog(float(x), float(y))
        b = oracle_mod.gsl_complex_dilog(float(x), float(-y))
        assert b[0] == a[0] and b[1] == -a[1], (x, y, a, b)
        hlib.hc_gsl_cli2(float(x), float(-y), ctypes.byref(re), ctypes.byref(im))
        assert re.value == a[0] and im.value == -a[1], (x, y)


def test_gsl_series_division_two_part_reciprocal(hlib):
    """GSL's series terms r^k / d_k on the device are fma(a, y_k, RN(a l_k)) with the table's two-part reciprocal
    (nusi_gsl.hpp header): every row's y_k = RN(1 / d_k) and l_k = RN(1 / d_k - y_k) exactly (rational arithmetic),
    and the device's division equals IEEE a / d_k on seeded a over the series' range of binades for every k."""
    import random
    from fractions import Fraction as F
    hlib.hc_gsl_krow.argtypes = [ctypes.c_int, ctypes.POINTER(D)]
    hlib.hc_gsl_div_k.restype = D
    hlib.hc_gsl_div_k.argtypes = [D, D, D, D]
    row = (D * 6)()
    rng = random.Random(20261018)
    for k in range(2, 1000):
        hlib.hc_gsl_krow(k, row)
        d1, d2, y1, y2, l1, l2 = list(row)
        assert d1 == float(k * k) and d2 == float(k * k * (k + 1))
        for d, y, l in ((d1, y1, l1), (d2, y2, l2)):
            assert y == 1.0 / d
            assert l == float(F(1) / F(d) - F(y)), (k, d)
            for _ in range(40):
                a = rng.uniform(0.5, 1.0) * 2.0 ** rng.randint(-470, 0)
                assert hlib.hc_gsl_div_k(a, d, y, l) == a / d, (k, d, a)


def test_device_atan2_select_path_bit_identical(olib, hlib):
    """nusi_libm.hpp's atan2 (round 6: the common case -- finite nonzero arguments, x != 1, exponent difference
    within 60 -- by selects instead of fdlibm's branches; every other argument through fdlibm's full code) against the
    oracle's fdlibm e_atan2.c (ora_libm.c), bit for bit: seeded arguments over 40 decades and both signs, every
    s_atan.c range boundary, the octants, and the special values (zeros, infinities, NaN, x = 1, extreme ratios)."""
    import numpy as np
    H = hlib
    for f in ("hc_atan2", "hc_atan2_full"):
        getattr(H, f).restype = D
        getattr(H, f).argtypes = [D, D]
    rng = np.random.default_rng(20250213)
    n = 200000
    mag = 10.0 ** rng.uniform(-20, 20, size=(n, 2))
    sgn = rng.choice([-1.0, 1.0], size=(n, 2))
    args = list(map(tuple, mag * sgn))
    # the reduction's range edges |y/x| = 7/16, 11/16, 19/16, 39/16, 2^-29, 2^66 (and neighbours), all octants
    edges = [7 / 16, 11 / 16, 19 / 16, 39 / 16, 2.0 ** -29, 2.0 ** 60, 2.0 ** -60, 2.0 ** 61, 2.0 ** -61, 1.0]
    for e in edges:
        for d in (np.nextafter(e, 0), e, np.nextafter(e, np.inf)):
            for sy in (1.0, -1.0):
                for sx in (1.0, -1.0):
                    args.append((sy * d * 3.0, sx * 3.0))
                    args.append((sy * d, sx * 1.0))
    sp = [0.0, -0.0, np.inf, -np.inf, np.nan, 1.0, -1.0, 5e-324, 1e308, 1e-308]
    args += [(a, b) for a in sp for b in sp]
    bad = 0
    for y, x in args:
        a, b, c = H.hc_atan2(y, x), H.hc_atan2_full(y, x), olib.ora_atan2(y, x)
        same = (a == c or (a != a and c != c)) and np.signbit(a) == np.signbit(c) and (b == c or (b != b and c != c))
        bad += not same
    assert bad == 0, bad


def test_device_log_bit_identical_to_oracle(olib, hlib):
    """nusi_libm.hpp's log and log1p (round 6: log without log1p's c / x correction, which is +0 when c = 0) against
    the oracle's ora_log / ora_log1p (ora_libm.c, with the term), bit for bit: seeded arguments over the whole normal
    range, subnormals, the table's subinterval edges near 1, and the special values."""
    import numpy as np
    rng = np.random.default_rng(5)
    xs = [10.0 ** rng.uniform(-307, 308, 60000), rng.uniform(0.5, 2.0, 40000), 1.0 + rng.uniform(-1e-6, 1e-6, 20000),
          rng.uniform(0, 1, 2000) * 2.0 ** -1040, np.array([0.0, -0.0, 1.0, np.inf, -np.inf, np.nan, -1.0, 5e-324,
                                                             np.nextafter(1.0, 0), np.nextafter(1.0, 2), 2.0 ** -1022])]
    x = np.concatenate(xs)
    dp = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))
    for hname, oname, arg in (("hc_log_n", "ora_log", x), ("hc_log1p_n", "ora_log1p", np.concatenate([x - 1.0, x]))):
        out = np.zeros_like(arg)
        getattr(hlib, hname)(ctypes.c_int(len(arg)), dp(arg), dp(out))
        ref = np.array([getattr(olib, oname)(float(v)) for v in arg])
        same = (out.view(np.uint64) == ref.view(np.uint64)) | (np.isnan(out) & np.isnan(ref))
        assert same.all(), (hname, arg[~same][:5], out[~same][:5], ref[~same][:5])

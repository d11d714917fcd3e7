"""Generate tests/golden/specfun_kat.json -- mpmath known-answer vectors.

Pins the arithmetic boundary the reference takes from absent third-party code
(SURVEY.md sec. 8c): GSL gsl_sf_dilog (Re Li2 on the real line),
gsl_sf_complex_dilog_xy_e (principal branch; on the real axis y == 0, x >= 1,
GSL returns Im = -pi log x, which mpmath's polylog also gives), and
polylogarithm::Li3 on [-1, 0) as reached by the DSNB source.  Also the
elementary functions the shared-algorithm libm provides.

Run:  python tests/golden/make_specfun_kat.py   (mpmath 1.3; output committed)
"""
import json
import os
import random

import mpmath as mp

mp.mp.dps = 40
random.seed(20250213)


def f(x):
    return float(x)


def main():
    out = {"li2_real": [], "li2_complex": [], "li3": [], "log": [], "log1p": [], "exp": [], "atan": [],
           "atan2": [], "atanh": []}
    xs = [-1e8, -1e3, -50.0, -2.0, -1.0, -0.9, -0.5, -0.3, -1e-3, -1e-9, 1e-9, 1e-3, 0.1, 0.25, 0.5, 0.51, 0.9,
          0.999, 1.0, 1.001, 1.5, 2.0, 3.0, 12.0, 13.0, 1e3, 1e8]
    xs += [random.choice([-1, 1]) * 10 ** random.uniform(-8, 8) for _ in range(200)]
    for x in xs:
        out["li2_real"].append([x, f(mp.re(mp.polylog(2, x)))])
    zs = [(2.0, 0.0), (5.0, 0.0), (0.5, 0.0), (1.5, 1e-30), (1.5, -1e-30), (0.3, 0.4), (-3.0, 2.0), (1e3, 1e-3),
          (0.999, 0.001)]
    zs += [(random.uniform(-5, 5) * 10 ** random.uniform(-6, 3), random.uniform(-5, 5) * 10 ** random.uniform(-8, 3))
           for _ in range(300)]
    for x, y in zs:
        v = mp.polylog(2, mp.mpc(x, y)) if y != 0 else mp.polylog(2, x)
        if y == 0 and x >= 1:
            v = mp.mpc(mp.re(mp.polylog(2, x)), -mp.pi * mp.log(x))   # GSL's real-axis convention
        out["li2_complex"].append([x, y, f(mp.re(v)), f(mp.im(v))])
    for x in [-1.0, -0.999, -0.9, -0.6, -0.5, -0.4, -0.1, -1e-5, 0.0, 0.3] + [-random.random() for _ in range(100)]:
        out["li3"].append([x, f(mp.polylog(3, x)) if x != 0 else 0.0])
    for _ in range(300):
        x = 10 ** random.uniform(-300, 300)
        out["log"].append([x, f(mp.log(x))])
        y = random.choice([-1, 1]) * 10 ** random.uniform(-20, 3)
        if y > -1:
            out["log1p"].append([y, f(mp.log1p(y))])
        e = random.uniform(-700, 700)
        out["exp"].append([e, f(mp.exp(e))])
        a = random.choice([-1, 1]) * 10 ** random.uniform(-10, 10)
        out["atan"].append([a, f(mp.atan(a))])
        p, q = random.uniform(-10, 10) * 10 ** random.uniform(-5, 5), random.uniform(-10, 10) * 10 ** random.uniform(-5, 5)
        out["atan2"].append([p, q, f(mp.atan2(p, q))])
        h = random.uniform(-0.999999, 0.999999)
        out["atanh"].append([h, f(mp.atanh(h))])
    # near the real axis (the Taylor path of the complex dilog, |y| <= 2.5e-3 min(|x|, |1 - x|)), both sides
    # of the cut x > 1, next to the branch point and next to 0; drawn after every set above
    out["li2_complex_axis"] = []
    for _ in range(400):
        r = random.random()
        if r < 0.4:
            x = random.choice([-1, 1]) * 10 ** random.uniform(-5, 4)
        elif r < 0.7:
            x = 1 + random.choice([-1, 1]) * 10 ** random.uniform(-7, 0)
        else:
            x = 1 + 10 ** random.uniform(-7, 3)
        d = min(abs(x), abs(1 - x))
        y = random.choice([-1, 1]) * d * 2.5e-3 * random.random()
        if y == 0:
            continue
        v = mp.polylog(2, mp.mpc(x, y))
        out["li2_complex_axis"].append([x, y, f(mp.re(v)), f(mp.im(v))])
    # round 5, GSL's branches (nusi_gsl.hpp / oracle/ora_gsl.c): |z| near and on the unit circle (dilogc_series_3
    # above |z| = 0.98, Lewin's formula on it), the 0.25 / 0.98 / 0.732 splits, z near -1 with a small imaginary
    # part (the member quotients of alpha's s-t interference), and Clausen's function; drawn after every set above
    out["li2_complex_unit"] = []
    for _ in range(300):
        r = random.random()
        t = random.uniform(-mp.pi, mp.pi)
        if r < 0.2:
            rad = 1.0
        elif r < 0.6:
            rad = 1 + random.choice([-1, 1]) * 10 ** random.uniform(-12, -1.3)
        elif r < 0.8:
            rad = random.choice([0.25, 0.98, 1 / 0.98, 4.0]) * (1 + random.uniform(-1e-3, 1e-3))
        else:
            rad, t = 1 + random.uniform(-0.05, 0.05), mp.pi - 10 ** random.uniform(-6, -1)
        x, y = f(rad * mp.cos(t)), f(rad * mp.sin(t))
        v = mp.polylog(2, mp.mpc(x, y))
        out["li2_complex_unit"].append([x, y, f(mp.re(v)), f(mp.im(v))])
    for x0 in (0.732, 0.25):
        for _ in range(20):
            x, y = x0 + random.uniform(-1e-6, 1e-6), random.uniform(-0.1, 0.1)
            v = mp.polylog(2, mp.mpc(x, y))
            out["li2_complex_unit"].append([x, y, f(mp.re(v)), f(mp.im(v))])
    out["clausen"] = []
    for x in [1e-12, 1e-8, 1e-3, 0.5, 1.0, 2.0, 3.0, 3.14159, -1.0, -3.0] + [random.uniform(-7, 7) for _ in range(100)]:
        out["clausen"].append([x, f(mp.clsin(2, x))])
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "specfun_kat.json"), "w") as fh:
        json.dump(out, fh)


if __name__ == "__main__":
    main()

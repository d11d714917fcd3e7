"""How far the shared-algorithm oracle (and with it the bit-exact GPU tables) sits from the reference's own
operation order.

The oracle evaluates the alpha table's s-t interference member dilogarithms as a Taylor series about their
gr-free real point and their arguments as sums of edge arguments (nusi_oracle.c member_dc / member_arg), the
sequence the GPU kernels run, and every complex dilogarithm takes a near-axis Taylor shortcut.  In
reference-order mode (oracle.reference_order(), nusi_oracle.h ora_set_reference_order) it instead evaluates
gsl_sf_complex_dilog_xy_e on the reference's own quotient z = (1+S+t)/(2 - i gr + t) and carg of the reference's
expression (nuSIprop.hpp:1431-1456), with the general series everywhere.  Both modes' full tables and fluxes
are compared on the C4 8-point subset, C2a / C2b and C3 (N_E = 1200, phi-phi on): single alpha entries move
where the closed forms cancel (the tables' known ~1e-6 sensitivity in the small-|t| regime), the fluxes stay
within 1e-11 -- except at strong couplings of the C4 scan (<= 1.4e-7 over the grid) and at C2a (lE 4 -> 9, m_phi = 3e3, the resonance inside the grid), where the s-t / s-u
interference closed forms of Gamma, alphaTilde and alpha (differences of complex dilogarithms of nearly equal
arguments, nuSIprop.hpp:843-878, 1135-1192, 1428-1474) are so ill-conditioned that ANY two accurate fp64
evaluations differ: the shared-algorithm order, the reference order and a long-double dilogarithm (level 2,
a precision probe) give fluxes up to ~1.5e-6 apart.  A GSL build of the reference would sit inside that
spread, so at C2a the reference's own output is defined only to ~1e-6; the test bounds the spread there
(C2A_SPREAD) and records it.  The measured maxima are written to tests/_build/reference_order.json and quoted
in DESIGN.md sec. 2."""
import json
import os

import numpy as np
import pytest

from tests import cases

FLUX_BOUND = 1e-11
C2A_SPREAD = 5e-6   # C2a: the conditioning of the reference's closed forms (module docstring)
# C4: strong couplings (g -> 1) make the flux sensitive to the s-t / s-u interference terms as well: over the
# whole 1024-point grid the three arithmetic variants' fluxes differ by <= 1.4e-7, median 4e-14, 93 points
# above 1e-9 (scripts/reference_order_scan.py -> profiles/r3/reference_order_c4.json)
C4_SPREAD = 5e-7
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_build", "reference_order.json")


def _both(oracle_mod, kw, tabs=None, level=1):
    """The oracle's tables and fluxes in its own arithmetic and at reference-order `level` (1 = the reference's
    operation order with the general complex dilogarithm, 2 = the long-double dilogarithm probe)."""
    res = []
    for ref in (0, level):
        o = oracle_mod.Oracle(**cases.oracle_kwargs(kw))
        if tabs is not None:
            o.load_phiphi(*tabs)
        with oracle_mod.reference_order(ref):
            G, aT, al = o.tables()
        f, fla = o.cascade(G, aT, al)
        res.append((o.T, G, aT, al, f, fla))
    return res


def _drift(res):
    (T, G, aT, al, f, fla), (_, G2, aT2, al2, f2, fla2) = res
    iu = np.triu_indices(T, 1)
    a, b = al[iu], al2[iu]
    nz = b != 0

    def rel(x, y):
        m = y != 0
        return float(np.max(np.abs(x[m] - y[m]) / np.abs(y[m]))) if np.any(m) else 0.0
    return {"alpha_max_rel": rel(a, b), "alpha_entries_differing": int(np.sum(a != b)), "alpha_entries": int(a.size),
            "alpha_median_rel": float(np.median(np.abs(a[nz] - b[nz]) / np.abs(b[nz]))) if np.any(nz) else 0.0,
            "gamma_max_rel": rel(G, G2), "alphatilde_max_rel": rel(aT, aT2),
            "flux_max_rel": max(cases.rel_err(f, f2), cases.rel_err(fla, fla2))}


def _record(name, d):
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    cur = {}
    if os.path.exists(OUT):
        with open(OUT) as fh:
            cur = json.load(fh)
    cur[name] = d
    with open(OUT, "w") as fh:
        json.dump(cur, fh, indent=1, sort_keys=True)


@pytest.mark.parametrize("name", ["C2a", "C2b", "C1_N300"])
def test_reference_order_c2(oracle_mod, name):
    kw = {"C2a": cases.C2A, "C2b": cases.C2B, "C1_N300": dict(cases.TEST_CPP, N_bins_E=300)}[name]
    d = _drift(_both(oracle_mod, kw))
    d["long_double_probe"] = _drift(_both(oracle_mod, kw, level=2))
    _record(name, d)
    bound = C2A_SPREAD if name == "C2a" else FLUX_BOUND
    assert d["flux_max_rel"] <= bound and d["long_double_probe"]["flux_max_rel"] <= bound, d


def test_reference_order_c4_subset(oracle_mod):
    pts = cases.scan_points()
    rng = np.random.default_rng(20250213)
    pick = sorted(rng.choice(len(pts), 8, replace=False))
    worst = None
    for i in pick:
        d = _drift(_both(oracle_mod, pts[i]))
        assert d["flux_max_rel"] <= C4_SPREAD, (i, d)
        if worst is None:
            worst = dict(d)
        else:
            for k in ("alpha_max_rel", "gamma_max_rel", "alphatilde_max_rel", "flux_max_rel", "alpha_median_rel"):
                worst[k] = max(worst[k], d[k])
            worst["alpha_entries_differing"] += d["alpha_entries_differing"]
            worst["alpha_entries"] += d["alpha_entries"]
    _record("C4_subset_8", worst)


def test_reference_order_c3(oracle_mod, ref_tables):
    from tests.test_phiphi import C3
    d = _drift(_both(oracle_mod, C3, ref_tables))
    _record("C3", d)
    assert d["flux_max_rel"] <= 10 * FLUX_BOUND, d   # measured 1.5e-11 (N_E = 1200: 134 steps accumulate it)

"""Stage-A table formulas of the product (nusiprop_amd/csrc/nusi_physics.hpp,
compiled for the host by tests/hostcheck) against the oracle, BIT FOR BIT, on
CPU.  The GPU runs the same source (tests/test_gpu_parity.py checks the device
build); this catches a formula divergence without a GPU.

The per-point scalars (masses, |U|^2, width, norm_total) are taken from the
oracle, which is what the product's host code computes the same way
(nusi_capi.cpp build_point; nuSIprop.hpp:130-205)."""
import ctypes

import numpy as np
import pytest

from tests import cases

DP = ctypes.POINTER(ctypes.c_double)


def _dp(a):
    return a.ctypes.data_as(DP)


def extended_axis(o):
    """Stage-A energy axis (nuSIprop.hpp:217-252): the N bins, then the top bin
    redshifted by (1+z_j), j = 1..N_z-2."""
    Emin, Emax, _, z = o.grid()
    N, T = o.N, o.T
    lo, hi = np.empty(T), np.empty(T)
    lo[:N], hi[:N] = Emin, Emax
    for n in range(N, T):
        lo[n] = Emin[N - 1] * (1 + z[n - N + 1])
        hi[n] = Emax[N - 1] * (1 + z[n - N + 1])
    return lo, hi


def point_array(o, kw):
    mn, norm_total = o.prepare()
    U2 = o.mixing()
    g, mphi = kw["g"], kw["mphi"]
    Ga = g * g * mphi / (16.0 * np.pi) if kw["majorana"] else g * g * mphi / (8.0 * np.pi)
    u = U2[kw["flav"]]
    pt = np.array([mphi, g, kw["mntot"], kw["si"], kw["norm"], norm_total, Ga, *mn, *u], dtype=np.float64)
    flags = (ctypes.c_int * 4)(int(kw["majorana"]), int(kw["non_resonant"]), int(kw["phiphi"]),
                               int(kw.get("source_model", 0)))
    return pt, flags


@pytest.mark.parametrize("name", sorted(cases.SMALL_CASES))
def test_tables_bit_identical(oracle_mod, name):
    from tests.hostcheck import build_hostcheck
    H = build_hostcheck()
    kw = dict(cases.SMALL_CASES[name], N_bins_E=40)
    o = oracle_mod.Oracle(**cases.oracle_kwargs(kw))
    G, aT, al = o.tables()
    lo, hi = extended_axis(o)
    pt, flags = point_array(o, kw)
    T = o.T
    Gh, aTh, Ah = np.zeros(T), np.zeros(T), np.zeros((T, T))
    H.hc_tables.restype = ctypes.c_int
    w = H.hc_tables(_dp(pt), flags, T, _dp(lo), _dp(hi), _dp(Gh), _dp(aTh), _dp(Ah))
    assert np.array_equal(Gh, G)
    assert np.array_equal(aTh, aT)
    iu = np.triu_indices(T, 1)
    assert np.array_equal(Ah[iu], al[iu]), "%d alpha entries differ" % np.sum(Ah[iu] != al[iu])
    assert (w & 7) == o.warnings()


@pytest.mark.parametrize("name,N", [("test_cpp", 40), ("c2b", 44), ("dirac", 31), ("resonant_only", 40),
                                    ("inverted", 46), ("strong", 40)])
def test_tiled_alpha_bit_identical(oracle_mod, name, N):
    """The tile kernel's data path (edge dedup, per-edge / per-corner leaf arrays,
    TileLeaves slot mapping), emulated on the host, against the oracle: bit for bit.
    N is chosen so the tiles straddle the N | redshift-extended junction."""
    from tests.hostcheck import build_hostcheck
    H = build_hostcheck()
    kw = dict(cases.SMALL_CASES[name], N_bins_E=N)
    o = oracle_mod.Oracle(**cases.oracle_kwargs(kw))
    _, _, al = o.tables()
    lo, hi = extended_axis(o)
    pt, flags = point_array(o, kw)
    T = o.T
    Ah = np.zeros((T, T))
    H.hc_alpha_tiled.restype = ctypes.c_int
    w = H.hc_alpha_tiled(_dp(pt), flags, T, _dp(lo), _dp(hi), _dp(Ah))
    iu = np.triu_indices(T, 1)
    if kw["non_resonant"]:
        assert np.array_equal(Ah[iu], al[iu]), "%d alpha entries differ" % np.sum(Ah[iu] != al[iu])
    else:
        d = np.arange(T - 1)
        assert np.array_equal(Ah[d, d + 1], al[d, d + 1])
    assert (w & 4) == (o.warnings() & 4)


@pytest.mark.parametrize("name", sorted(cases.SMALL_CASES))
def test_reference_order_tables_bit_identical(oracle_mod, name):
    """NUSI_OPT_REFERENCE_ORDER on the device headers (the kRef instances of gamma_entry / alphat_entry /
    alpha_entry: the general complex dilogarithm, the reference's quotient and carg for the s-t member leaves)
    against the oracle in reference-order mode (ora_set_reference_order(1)): bit for bit; and they differ from
    the default order somewhere (the mode is not a no-op) wherever the s-t interference is computed."""
    from tests.hostcheck import build_hostcheck
    H = build_hostcheck()
    kw = dict(cases.SMALL_CASES[name], N_bins_E=40)
    o = oracle_mod.Oracle(**cases.oracle_kwargs(kw))
    with oracle_mod.reference_order(1):
        G, aT, al = o.tables()
    lo, hi = extended_axis(o)
    pt, flags = point_array(o, kw)
    T = o.T
    Gh, aTh, Ah = np.zeros(T), np.zeros(T), np.zeros((T, T))
    H.hc_tables_ref.restype = ctypes.c_int
    w = H.hc_tables_ref(_dp(pt), flags, T, _dp(lo), _dp(hi), _dp(Gh), _dp(aTh), _dp(Ah))
    assert np.array_equal(Gh, G)
    assert np.array_equal(aTh, aT)
    iu = np.triu_indices(T, 1)
    assert np.array_equal(Ah[iu], al[iu]), "%d alpha entries differ" % np.sum(Ah[iu] != al[iu])
    assert (w & 7) == o.warnings()
    Ad = np.zeros((T, T))
    H.hc_alpha_tiled_ref.restype = ctypes.c_int
    H.hc_alpha_tiled_ref(_dp(pt), flags, T, _dp(lo), _dp(hi), _dp(Ad))
    if kw["non_resonant"]:
        assert np.array_equal(Ad[iu], al[iu]), "tiled: %d alpha entries differ" % np.sum(Ad[iu] != al[iu])
        if kw["majorana"]:
            _, _, al0 = o.tables()
            assert np.any(al0[iu] != al[iu])


@pytest.mark.parametrize("parts", [1, 2])
@pytest.mark.parametrize("ref", [0, 1])
@pytest.mark.parametrize("name", sorted(cases.SMALL_CASES))
def test_edge_shared_gamma_alphat_bit_identical(oracle_mod, name, ref, parts):
    """k_gamma_alphat's edge-shared path (round 6: each bin edge's dilogarithms evaluated once and handed to the
    neighbouring bin; gamma_edge_vals / alphat_edge_vals + the *_pre differences), emulated on the host in both
    channel splits, against the oracle in both arithmetics: Gamma and alphaTilde bit for bit."""
    from tests.hostcheck import build_hostcheck
    H = build_hostcheck()
    kw = dict(cases.SMALL_CASES[name], N_bins_E=40)
    o = oracle_mod.Oracle(**cases.oracle_kwargs(kw))
    with oracle_mod.reference_order(ref):
        G, aT, _ = o.tables()
    lo, hi = extended_axis(o)
    pt, flags = point_array(o, kw)
    T = o.T
    Gh, aTh = np.zeros(T), np.zeros(T)
    H.hc_ga_shared.restype = ctypes.c_int
    H.hc_ga_shared(_dp(pt), flags, T, _dp(lo), _dp(hi), parts, ref, _dp(Gh), _dp(aTh))
    assert np.array_equal(Gh, G), "Gamma differs at %s" % np.flatnonzero(Gh != G)[:5]
    assert np.array_equal(aTh, aT), "alphaTilde differs at %s" % np.flatnonzero(aTh != aT)[:5]


@pytest.mark.parametrize("name", sorted(cases.SMALL_CASES) + ["C2A", "C2B"])
def test_ga_dilogs_prepass_bit_identical(oracle_mod, name):
    """The reference order's few-table path (round 6): k_ga_dilogs evaluates every GSL dilogarithm of
    Gamma / alphaTilde one per work-item (ga_pre_slot: both edges' values and alphaTilde's bin values d26, d43 and the
    t-u combination's four), k_gamma_alphat<.., kPre> reads them (ga_pre_load) -- emulated on the host: Gamma and
    alphaTilde bit for bit against the reference-order oracle (the fields start as NaN, so a field no slot writes would
    show).  BASELINE configs 2a / 2b at their own N_E = 300, the small cases at 40 bins."""
    from tests.hostcheck import build_hostcheck
    H = build_hostcheck()
    kw = getattr(cases, name) if name in ("C2A", "C2B") else dict(cases.SMALL_CASES[name], N_bins_E=40)
    o = oracle_mod.Oracle(**cases.oracle_kwargs(kw))
    with oracle_mod.reference_order(1):
        G, aT, _ = o.tables()
    lo, hi = extended_axis(o)
    pt, flags = point_array(o, kw)
    T = o.T
    Gh, aTh = np.zeros(T), np.zeros(T)
    H.hc_ga_pre.restype = ctypes.c_int
    H.hc_ga_pre(_dp(pt), flags, T, _dp(lo), _dp(hi), _dp(Gh), _dp(aTh))
    assert np.array_equal(Gh, G), "Gamma differs at %s" % np.flatnonzero(Gh != G)[:5]
    assert np.array_equal(aTh, aT), "alphaTilde differs at %s" % np.flatnonzero(aTh != aT)[:5]

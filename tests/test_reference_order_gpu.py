"""NUSI_OPT_REFERENCE_ORDER on the GPU: the Stage-A tables in the reference's own arithmetic, against the oracle in
reference-order mode (oracle.reference_order(1), nusi_oracle.h ora_set_reference_order).

The default tables are bit-exact to the oracle's shared-algorithm order (tests/test_gpu_parity.py), which evaluates
the alpha table's s-t interference member dilogarithms as Taylor series about a batch-shared real point and their
arguments as sums of edge arguments, and every dilogarithm by this repository's own series.  In reference-order mode
the kernels instead run GSL's algorithms (nusi_gsl.hpp, the restatement of GSL 2.x dilog.c / clausen.c; the oracle's
ora_gsl.c) for every gsl_sf_dilog and gsl_sf_complex_dilog_xy_e the reference calls, on the reference's own
arguments -- the member quotient z = (1+S+t)/(2 - i gr + t) and carg of its expression (nuSIprop.hpp:1428-1467), the
complex dilogarithms of Gamma :843-878 and alphaTilde :1135-1192, the real ones of :1098, :1375-1398 and aux.hpp:77-166.
On the big-batch kernel the member corners come from k_alpha_mcorner's block (one evaluation per table, mass state
and pair of bin edges).  Bar:
Bar:

* tables BIT-EXACT to the reference-order oracle on every small case, C1 / C2a / C2b at N_E = 300, an 8-point subset
  of the C4 scan and C3 (N_E = 1200, phi-phi on at the reference's table geometry);
* fluxes <= FLUX_RTOL (1e-11) against the reference-order oracle's evolve(), on those and on ALL 1024 points of
  the C4 scan (the headline workload; the default order drifts up to 1.2e-7 from the reference order there,
  DESIGN.md sec. 2)."""
import numpy as np
import pytest

from tests import cases

pytestmark = pytest.mark.gpu

FLUX_RTOL = cases.FLUX_RTOL


@pytest.fixture(scope="module")
def nusi():
    import nusiprop_amd
    nusiprop_amd.load()
    return nusiprop_amd


def _gpu_refo(nusi, pts, kernel=None, tables=True, corner_mb=None):
    from nusiprop_amd import _lib
    p0 = pts[0]
    plan = nusi.Plan(p0["N_bins_E"], p0["lEmin"], p0["lEmax"], p0["zmax"], max_points=len(pts))
    plan.set_option(_lib.OPT_REFERENCE_ORDER, 1)
    if kernel is not None:
        plan.set_option(_lib.OPT_ALPHA_KERNEL, kernel)
    if corner_mb is not None:
        plan.set_option(_lib.OPT_REFO_CORNER_MB, corner_mb)
    flux, fla = plan.evolve(pts)
    tabs = [plan.tables(i) for i in range(len(pts))] if tables else None
    names = plan.kernels()
    warn = plan.warnings(len(pts))
    plan.close()
    return flux, fla, tabs, names, warn


def _check_tables(nusi, o, tab, kw):
    """The oracle's tables (in the caller's arithmetic mode) against the GPU's `tab`, bit for bit."""
    G, aT, al = o.tables()
    Gg, aTg, Ag = tab
    assert np.array_equal(Gg, G), "Gamma differs at %s" % np.flatnonzero(Gg != G)[:5]
    assert np.array_equal(aTg, aT), "alphaTilde differs at %s" % np.flatnonzero(aTg != aT)[:5]
    T = o.T
    Ad = nusi.unpack_alpha(Ag, T)
    iu = np.triu_indices(T, 1)
    if kw["non_resonant"]:
        assert np.array_equal(Ad[iu], al[iu]), "alpha differs in %d entries" % np.sum(Ad[iu] != al[iu])
    else:
        d = np.arange(T - 1)
        assert np.array_equal(Ad[d, d + 1], al[d, d + 1])
    return G, aT, al


@pytest.mark.parametrize("name", sorted(cases.SMALL_CASES))
def test_reference_order_small_cases(nusi, oracle_mod, name):
    """Every small case on the default batch kernel, the per-table tile kernel and the per-entry kernel: the tables
    bit-exact to the reference-order oracle, the warnings equal, the fluxes to FLUX_RTOL."""
    kw = cases.SMALL_CASES[name]
    o = oracle_mod.Oracle(**cases.oracle_kwargs(kw))
    for kernel, label in ((None, "k_alpha_mcorner + k_alpha_batch[refo]"), (1, "k_alpha_tile[refo]"), (2, "k_alpha[refo]")):
        flux, fla, tabs, names, warn = _gpu_refo(nusi, [kw], kernel=kernel)
        assert names[0] == label
        with oracle_mod.reference_order(1):
            G, aT, al = _check_tables(nusi, o, tabs[0], kw)
            assert warn[0] & 7 == o.warnings()
            f_ref, fla_ref = o.cascade(G, aT, al)
        assert cases.rel_err(flux[0], f_ref) <= FLUX_RTOL
        assert cases.rel_err(fla[0], fla_ref) <= FLUX_RTOL


@pytest.mark.parametrize("kw", [dict(cases.TEST_CPP, N_bins_E=300), cases.C2A, cases.C2B], ids=["C1_N300", "C2a", "C2b"])
def test_reference_order_c1_c2(nusi, oracle_mod, kw):
    """BASELINE configs 1 and 2 at N_E = 300: tables bit-exact to the reference-order oracle, fluxes against its
    evolve() to FLUX_RTOL (C2a is where the default order sits 2.7e-6 from the reference order)."""
    flux, fla, tabs, _, _ = _gpu_refo(nusi, [kw])
    o = oracle_mod.Oracle(**cases.oracle_kwargs(kw))
    with oracle_mod.reference_order(1):
        _check_tables(nusi, o, tabs[0], kw)
        f_ref, fla_ref = o.evolve()
    assert cases.rel_err(flux[0], f_ref) <= FLUX_RTOL
    assert cases.rel_err(fla[0], fla_ref) <= FLUX_RTOL


def test_reference_order_c4_subset_bitexact(nusi, oracle_mod):
    """Eight points of the C4 scan, one batched call (k_alpha_batch[refo] shares each batch's (S', t) leaves):
    every table bit-exact to the reference-order oracle; batching does not change a bit (each point alone gives
    the same tables)."""
    pts = cases.scan_points()
    rng = np.random.default_rng(20250213)
    pick = sorted(rng.choice(len(pts), 8, replace=False))
    sel = [pts[i] for i in pick] + [dict(pts[pick[0]], g=pts[pick[0]]["g"] * 1.7)]   # a batch of two
    flux, fla, tabs, names, _ = _gpu_refo(nusi, sel)
    assert names[0] == "k_alpha_mcorner + k_alpha_batch[refo]"
    for k, kw in enumerate(sel):
        o = oracle_mod.Oracle(**cases.oracle_kwargs(kw))
        with oracle_mod.reference_order(1):
            G, aT, al = _check_tables(nusi, o, tabs[k], kw)
        f_ref, fla_ref = o.cascade(G, aT, al)
        assert cases.rel_err(flux[k], f_ref) <= FLUX_RTOL
        assert cases.rel_err(fla[k], fla_ref) <= FLUX_RTOL


def test_reference_order_c4_full_grid(nusi, oracle_mod):
    """ALL 1024 points of the C4 scan (BASELINE config 4, the headline workload) in reference-order mode: every
    flux within FLUX_RTOL of the reference-order oracle's evolve() (computed on a thread pool over the host's
    CPU share).  The default mode is measured against the same oracle and recorded: it drifts up to ~1e-7 at
    g -> 1 (the conditioning of the s-t interference closed forms)."""
    pts = cases.scan_points()
    flux, fla, _, names, _ = _gpu_refo(nusi, pts, tables=False)
    assert names[0] == "k_alpha_mcorner + k_alpha_batch[refo]"
    f_ref, fla_ref = oracle_mod.evolve_many(pts, level=1)
    errs = np.array([max(cases.rel_err(flux[k], f_ref[k]), cases.rel_err(fla[k], fla_ref[k])) for k in range(len(pts))])
    assert np.all(errs <= FLUX_RTOL), (int(np.argmax(errs)), float(errs.max()))
    # the member-corner block in chunks of one batch (64 MiB: 17 tables' worth at 3.7 MB each, below the 32 of a batch) -- the same bits
    fc, flac, _, _, _ = _gpu_refo(nusi, pts, tables=False, corner_mb=64)
    assert np.array_equal(fc, flux) and np.array_equal(flac, fla)
    p0 = pts[0]
    plan = nusi.Plan(p0["N_bins_E"], p0["lEmin"], p0["lEmax"], p0["zmax"], max_points=len(pts), reference_order=False)
    f0, fla0 = plan.evolve(pts)
    plan.close()
    d0 = np.array([cases.rel_err(fla0[k], fla_ref[k]) for k in range(len(pts))])
    print("C4 full grid vs the reference-order oracle: refo mode max %.3g; shared-order mode max %.3g, %d points > 1e-9"
          % (errs.max(), d0.max(), int(np.sum(d0 > 1e-9))))


def test_reference_order_c5_gamma_block(nusi, oracle_mod):
    """BASELINE config 5 in the reference order (the library default): one full 16-gamma block of scan.c5_points()
    (one Stage-A table, k_alpha_mcorner + k_alpha_batch[refo], the gamma batch k_cascade_bs_gamma) -- the table
    bit-exact to the reference-order oracle and every gamma's flux within FLUX_RTOL of the oracle's cascade on it."""
    from nusiprop_amd import scan
    allp = scan.c5_points()
    blk = allp[16 * 2345:16 * 2346]
    assert len({scan.table_key(p) for p in blk}) == 1 and len({p["si"] for p in blk}) == 16
    p0 = blk[0]
    plan = nusi.Plan(p0["N_bins_E"], p0["lEmin"], p0["lEmax"], p0["zmax"], max_points=len(blk))
    flux, fla = plan.evolve(blk)
    names = plan.kernels()
    tab = plan.tables(0)
    for i in range(1, len(blk)):
        for x, y in zip(plan.tables(i), tab):
            assert np.array_equal(x, y)
    plan.close()
    assert names == ("k_alpha_mcorner + k_alpha_batch[refo]", "k_cascade_bs_gamma")
    o = oracle_mod.Oracle(**cases.oracle_kwargs(p0))
    with oracle_mod.reference_order(1):
        G, aT, al = _check_tables(nusi, o, tab, p0)
    for k, p in enumerate(blk):
        ok = oracle_mod.Oracle(**cases.oracle_kwargs(p))
        ok.prepare()
        f_ref, fla_ref = ok.cascade(G, aT, al)
        assert cases.rel_err(flux[k], f_ref) <= FLUX_RTOL, k
        assert cases.rel_err(fla[k], fla_ref) <= FLUX_RTOL, k
        assert np.array_equal(flux[k] == 0, f_ref == 0)


def test_reference_order_c3(nusi, oracle_mod, ref_tables):
    """BASELINE config 3 (N_E = 1200, phi-phi on, the reference's table geometry): all 887 778 alpha entries and
    every Gamma / alphaTilde entry bit-exact to the reference-order oracle, fluxes to FLUX_RTOL."""
    from tests.test_phiphi import C3
    at, atd, a, ad = ref_tables
    from nusiprop_amd import _lib
    p = nusi.Plan(C3["N_bins_E"], C3["lEmin"], C3["lEmax"], C3["zmax"], max_points=1)
    p.load_phiphi(at, a)
    p.set_option(_lib.OPT_REFERENCE_ORDER, 1)
    flux, fla = p.evolve([C3])
    assert p.warnings(1)[0] & 8 == 0
    tab = p.tables(0)
    p.close()
    o = oracle_mod.Oracle(**cases.oracle_kwargs(C3))
    o.load_phiphi(at, atd, a, ad)
    with oracle_mod.reference_order(1):
        G, aT, al = _check_tables(nusi, o, tab, C3)
    f_ref, fla_ref = o.cascade(G, aT, al)
    assert cases.rel_err(flux[0], f_ref) <= FLUX_RTOL
    assert cases.rel_err(fla[0], fla_ref) <= FLUX_RTOL


def _object_fla(L, _lib, kw, order=None, copy=False):
    """One evolve() through the object API (nusi_create / nusi_evolve / nusi_get_flux_fla, the calculate_flux
    path): `order` None = no option at all; else NUSI_OPT_REFERENCE_ORDER set to it.  copy: also evolve a
    nusi_copy of the handle.  Returns the (3, N) flavour fluxes of each handle and the alpha kernel label."""
    import ctypes
    kw = dict(kw)
    src = kw.pop("source_model")
    N = kw["N_bins_E"]
    h, h2 = ctypes.c_void_p(), ctypes.c_void_p()
    _lib.check(L.nusi_create(ctypes.byref(_lib.make_params(source_model=src, **kw)), ctypes.byref(h)))
    outs, labels = [], []
    try:
        if order is not None:
            _lib.check(L.nusi_set_option(h, _lib.OPT_REFERENCE_ORDER, order))
        if copy:
            _lib.check(L.nusi_copy(h, ctypes.byref(h2)))
        for hh in ((h, h2) if copy else (h,)):
            _lib.check(L.nusi_evolve(hh))
            out = np.zeros(3 * N)
            _lib.check(L.nusi_get_flux_fla(hh, out.ctypes.data_as(ctypes.POINTER(ctypes.c_double))))
            a, c = ctypes.c_char_p(), ctypes.c_char_p()
            _lib.check(L.nusi_get_kernels(hh, ctypes.byref(a), ctypes.byref(c)))
            outs.append(out.reshape(3, N))
            labels.append(a.value)
    finally:
        L.nusi_destroy(h)
        if h2.value:
            L.nusi_destroy(h2)
    return outs, labels


def test_dropin_default_is_reference_arithmetic_c2a(nusi, oracle_mod):
    """BASELINE config 2a (DSNB, resonance inside lE 4 -> 9, N_E = 300) through the drop-in surfaces WITHOUT ANY
    OPTION -- the object API (calculate_flux's path), a copy of it, and pyprop -- runs the reference's own arithmetic:
    fluxes <= FLUX_RTOL of the reference-order oracle's evolve() (the shared order is ~2.5e-6 away on this config),
    and bit-identical to a default plan's.  The shared order stays available as the opt-in fast mode."""
    from nusiprop_amd import _lib
    L = _lib.load()
    with oracle_mod.reference_order(1):
        _, fla_ref = oracle_mod.Oracle(**cases.oracle_kwargs(cases.C2A)).evolve()
    _, fla_shared = oracle_mod.Oracle(**cases.oracle_kwargs(cases.C2A)).evolve()
    assert cases.rel_err(fla_shared, fla_ref) > 1e-9   # the two arithmetics differ on this config
    outs, labels = _object_fla(L, _lib, cases.C2A, copy=True)
    assert labels == [b"k_alpha_mcorner + k_alpha_batch[refo]"] * 2
    kw = dict(cases.C2A)
    kw.pop("source_model")
    ev = nusi.pyprop(**dict(kw, phiphi=False))
    ev.evolve()
    assert ev.kernels()[0] == "k_alpha_mcorner + k_alpha_batch[refo]"
    p0 = cases.C2A
    plan = nusi.Plan(p0["N_bins_E"], p0["lEmin"], p0["lEmax"], p0["zmax"], max_points=1)
    _, fla_plan = plan.evolve([p0])
    assert plan.kernels()[0] == "k_alpha_mcorner + k_alpha_batch[refo]"
    plan.close()
    for got in outs + [np.asarray(ev.get_flux_fla())]:
        assert cases.rel_err(got, fla_ref) <= FLUX_RTOL
        assert np.array_equal(got, fla_plan[0])
    # the opt-in fast mode: the oracle's default mode, through both surfaces
    fast, lab = _object_fla(L, _lib, cases.C2A, order=0)
    assert lab == [b"k_alpha_batch"] and cases.rel_err(fast[0], fla_shared) <= FLUX_RTOL
    ev0 = nusi.pyprop(**dict(kw, phiphi=False), reference_order=False)
    ev0.evolve()
    assert np.array_equal(np.asarray(ev0.get_flux_fla()), fast[0])


def test_reference_order_object_api(nusi, oracle_mod):
    """The object API's option (nusi_set_option on a calculate_flux-style handle, kept by nusi_copy): an explicit
    NUSI_OPT_REFERENCE_ORDER = 1 on C2a equals the plan's result bit for bit; values outside [0, 1] are refused."""
    import ctypes
    from nusiprop_amd import _lib
    L = _lib.load()
    outs, labels = _object_fla(L, _lib, cases.C2A, order=1, copy=True)
    assert labels == [b"k_alpha_mcorner + k_alpha_batch[refo]"] * 2
    kw = dict(cases.C2A)
    src = kw.pop("source_model")
    h = ctypes.c_void_p()
    _lib.check(L.nusi_create(ctypes.byref(_lib.make_params(source_model=src, **kw)), ctypes.byref(h)))
    try:
        assert L.nusi_set_option(h, _lib.OPT_REFERENCE_ORDER, 2) == _lib.NUSI_EPARAM
    finally:
        L.nusi_destroy(h)
    _, fla, _, _, _ = _gpu_refo(nusi, [cases.C2A], tables=False)
    assert np.array_equal(outs[0], fla[0]) and np.array_equal(outs[1], fla[0])


def test_reference_order_pyprop(nusi):
    """pyprop's extension keyword reference_order (default True) gives the plan's reference-order fluxes."""
    kw = dict(cases.C2A)
    kw.pop("source_model")
    ev = nusi.pyprop(**dict(kw, phiphi=False), reference_order=True)
    ev.evolve()
    _, fla, _, _, _ = _gpu_refo(nusi, [cases.C2A], tables=False)
    assert np.array_equal(np.asarray(ev.get_flux_fla()), fla[0])


def test_object_plans_are_reused_with_default_options(nusi):
    """Destroyed one-point objects hand their plan to the next object on the same grid (nusi_capi.cpp plan pool):
    an object created after a shared-order one runs the default (reference) arithmetic and gives the bits of a
    fresh default plan."""
    from nusiprop_amd import _lib
    L = _lib.load()
    fast, ka = _object_fla(L, _lib, cases.C2B, order=0)
    dflt, kb = _object_fla(L, _lib, cases.C2B)   # (the pooled plan of the first object)
    assert ka == [b"k_alpha_batch"] and kb == [b"k_alpha_mcorner + k_alpha_batch[refo]"]
    p0 = cases.C2B
    plan = nusi.Plan(p0["N_bins_E"], p0["lEmin"], p0["lEmax"], p0["zmax"], max_points=1)
    _, fla = plan.evolve([p0])
    plan.close()
    assert np.array_equal(dflt[0], fla[0])
    _, fla_r, _, _, _ = _gpu_refo(nusi, [p0], tables=False)
    assert np.array_equal(dflt[0], fla_r[0])
    plan = nusi.Plan(p0["N_bins_E"], p0["lEmin"], p0["lEmax"], p0["zmax"], max_points=1, reference_order=False)
    _, fla_s = plan.evolve([p0])
    plan.close()
    assert np.array_equal(fast[0], fla_s[0])

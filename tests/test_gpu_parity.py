"""GPU parity: the HIP path (through the C ABI) against the CPU oracle.

* Stage-A tables (Gamma, alphaTilde, alpha): BIT-EXACT.  Both sides evaluate
  the same fp64 operation sequence (shared-algorithm libm, no contraction), so
  any difference is a bug -- including in the small-|t| regime where the
  reference's closed forms amplify 1-ulp differences ~1e10-fold.
* Fluxes: relative error <= cases.FLUX_RTOL (1e-11) on every bin with |ref| > 1e-280 max|ref|,
  exact where ref == 0.  The only difference is the cascade's summation
  order (right-looking on the GPU, the reference's left-looking m-then-l loop
  in the oracle) and multiplication by precomputed reciprocals; every summed
  term is non-negative, so the deviation stays at the 1e-15 level.  The
  north-star bound is 1e-9.
"""
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


def _gpu(nusi, pts, **opts):
    from nusiprop_amd import _lib
    p0 = pts[0]
    plan = nusi.Plan(p0["N_bins_E"], p0["lEmin"], p0["lEmax"], p0["zmax"], max_points=len(pts), reference_order=False)
    for k, v in opts.items():
        plan.set_option(getattr(_lib, "OPT_" + k.upper()), v)
    flux, fla = plan.evolve(pts)
    tabs = [plan.tables(i) for i in range(len(pts))]
    warn = plan.warnings(len(pts))
    return plan, flux, fla, tabs, warn


@pytest.mark.parametrize("name", sorted(cases.SMALL_CASES))
def test_tables_bitexact_and_flux(nusi, oracle_mod, name):
    kw = cases.SMALL_CASES[name]
    o = oracle_mod.Oracle(**cases.oracle_kwargs(kw))
    G, aT, al = o.tables()
    plan, flux, fla, tabs, warn = _gpu(nusi, [kw])
    assert plan.kernels()[1] == "k_cascade_bs"   # the default (AUTO) cascade, for every source and mode
    Gg, aTg, Ag = tabs[0]
    T = o.T
    assert plan.T == T and plan.N == o.N and plan.Nz == o.Nz
    assert np.array_equal(Gg, G), "Gamma differs at %s" % np.flatnonzero(Gg != G)[:5]
    assert np.array_equal(aTg, aT), "alphaTilde differs at %s" % np.flatnonzero(aTg != aT)[:5]
    Ad = nusi.unpack_alpha(Ag, T)
    iu = np.triu_indices(T, 1)
    if kw["non_resonant"]:
        assert np.array_equal(Ad[iu], al[iu]), "alpha differs in %d entries" % np.sum(Ad[iu] != al[iu])
    else:   # only the first off-diagonal is computed (the cascade reads nothing else)
        d = np.arange(T - 1)
        assert np.array_equal(Ad[d, d + 1], al[d, d + 1])
    assert warn[0] & 7 == o.warnings()
    f_ref, fla_ref = o.cascade(G, aT, al)
    assert cases.rel_err(flux[0], f_ref) <= FLUX_RTOL
    assert cases.rel_err(fla[0], fla_ref) <= FLUX_RTOL


def test_batch_equals_single(nusi):
    """A batch of distinct points gives each point's single-point result bit for bit."""
    pts = [cases.C2B_100, dict(cases.C2B_100, mphi=2e6, g=0.1), dict(cases.C2B_100, si=2.2, norm=3),
           dict(cases.C2B_100, majorana=False), dict(cases.C2B_100, non_resonant=False)]
    _, flux_b, fla_b, tabs_b, _ = _gpu(nusi, pts)
    for i, p in enumerate(pts):
        _, f1, fl1, t1, _ = _gpu(nusi, [p])
        assert np.array_equal(f1[0], flux_b[i]) and np.array_equal(fl1[0], fla_b[i])
        for a, b in zip(t1[0], tabs_b[i]):
            assert np.array_equal(a, b)


@pytest.mark.parametrize("kw", [cases.C2A, cases.C2B], ids=["C2a_N300", "C2b_N300"])
def test_full_size_flux(nusi, oracle_mod, kw):
    """BASELINE config 2 (single propagation, N_E = 300) end to end vs the oracle's evolve()."""
    o = oracle_mod.Oracle(**cases.oracle_kwargs(kw))
    f_ref, fla_ref = o.evolve()
    _, flux, fla, _, _ = _gpu(nusi, [kw])
    assert cases.rel_err(flux[0], f_ref) <= FLUX_RTOL
    assert cases.rel_err(fla[0], fla_ref) <= FLUX_RTOL


@pytest.mark.parametrize("kw", [cases.C2A, cases.C2B], ids=["C2a_N300", "C2b_N300"])
def test_mfma_cascade_vs_oracle(nusi, oracle_mod, kw):
    """The MFMA-push cascade (fp64 matrix cores, rank-4 blocks) at BASELINE config 2 vs the oracle."""
    from nusiprop_amd import _lib
    o = oracle_mod.Oracle(**cases.oracle_kwargs(kw))
    f_ref, fla_ref = o.evolve()
    plan = nusi.Plan(kw["N_bins_E"], kw["lEmin"], kw["lEmax"], kw["zmax"], max_points=3, reference_order=False)
    plan.set_cascade(_lib.CASCADE_MFMA)
    flux, fla = plan.evolve([kw, kw, kw])
    for i in range(3):
        assert cases.rel_err(flux[i], f_ref) <= FLUX_RTOL
        assert cases.rel_err(fla[i], fla_ref) <= FLUX_RTOL
        assert np.array_equal(flux[i] == 0, f_ref == 0)


def test_data_massless_through_pyprop(nusi):
    """The reference's golden output (output/data_massless.txt, written by test.py)
    reproduced through the drop-in pyprop API on the GPU, to its printed precision."""
    import os
    ref = np.loadtxt(os.path.join(os.path.dirname(__file__), "golden", "data_massless.txt"), skiprows=1)
    kw = dict(cases.TEST_PY)
    kw.pop("source_model")
    ev = nusi.pyprop(**kw)
    ev.evolve()
    fla = ev.get_flux_fla()
    E = ev.get_energies()
    got = ["%.5e  %.4e  %.4e  %.4e" % r for r in zip(E, fla[0], fla[1], fla[2])]
    want = ["%.5e  %.4e  %.4e  %.4e" % tuple(r) for r in ref]
    assert got == want


def test_scan_subset_vs_oracle(nusi, oracle_mod):
    """Eight points of the C4 scan grid (N_E = 300, power law): GPU batch vs oracle."""
    pts = cases.scan_points()
    rng = np.random.default_rng(20250213)
    pick = sorted(rng.choice(len(pts), 8, replace=False))
    sel = [pts[i] for i in pick]
    _, flux, fla, tabs, _ = _gpu(nusi, sel)
    for k, kw in enumerate(sel):
        o = oracle_mod.Oracle(**cases.oracle_kwargs(kw))
        G, aT, al = o.tables()
        assert np.array_equal(tabs[k][0], G) and np.array_equal(tabs[k][1], aT)
        iu = np.triu_indices(o.T, 1)
        assert np.array_equal(nusi.unpack_alpha(tabs[k][2], o.T)[iu], al[iu])
        f_ref, fla_ref = o.cascade(G, aT, al)
        assert cases.rel_err(flux[k], f_ref) <= FLUX_RTOL
        assert cases.rel_err(fla[k], fla_ref) <= FLUX_RTOL


@pytest.mark.parametrize("N,nonres", [(37, True), (64, True), (65, False), (130, True), (200, False), (700, True),
                                      (1200, True)])
def test_cascade_sizes(nusi, oracle_mod, N, nonres):
    """The register-resident cascade at every chunk-count regime (N <= 64 NQ for the
    instantiated NQ; 64/65 straddle a chunk edge, 1200 is BASELINE config 3's size):
    the GPU flux against the oracle's cascade run on the GPU's own tables (which are
    bit-exact to the oracle's at the sizes the other tests cover)."""
    kw = dict(cases.C2B_100, N_bins_E=N, non_resonant=nonres, majorana=(N % 2 == 0))
    plan, flux, fla, tabs, _ = _gpu(nusi, [kw])
    o = oracle_mod.Oracle(**cases.oracle_kwargs(kw))
    o.prepare()
    G, aT, A = tabs[0]
    f_ref, fla_ref = o.cascade(G, aT, nusi.unpack_alpha(A, plan.T))
    assert cases.rel_err(flux[0], f_ref) <= FLUX_RTOL
    assert cases.rel_err(fla[0], fla_ref) <= FLUX_RTOL


def test_gamma_batches_share_tables(nusi, oracle_mod):
    """Points that differ only in si / norm / source share one Stage-A table (the
    tables do not read them, nuSIprop.hpp:217-253); each point's flux equals its own
    single-point evolve to rounding (three points of a table run as a gamma batch, its
    steps in passes of 6) with the same exact zeros, and the oracle's to FLUX_RTOL."""
    base = [dict(cases.C2B_100, mphi=m, g=g) for m, g in ((6e5, 0.01), (2e6, 0.1))]
    pts = [dict(b, si=s, norm=nm, source_model=src) for s, nm, src in ((2.0, 1.0, 1), (2.5, 6.0, 1), (3.0, 2.0, 0))
           for b in base]
    plan, flux, fla, tabs, _ = _gpu(nusi, pts)
    for i in range(2, len(pts)):
        for a, b in zip(tabs[i], tabs[i % 2]):
            assert np.array_equal(a, b)
    for i, p in enumerate(pts):
        _, f1, fl1, _, _ = _gpu(nusi, [p])
        assert cases.rel_err(flux[i], f1[0]) <= FLUX_RTOL and np.array_equal(flux[i] == 0, f1[0] == 0)
        assert cases.rel_err(fla[i], fl1[0]) <= FLUX_RTOL
        o = oracle_mod.Oracle(**cases.oracle_kwargs(p))
        _, fla_ref = o.evolve()
        assert cases.rel_err(fla[i], fla_ref) <= FLUX_RTOL


@pytest.mark.parametrize("N,nonres", [(37, True), (64, False), (130, True), (200, True), (300, True), (300, False),
                                      (700, True), (1500, True)])
def test_cascade_kernels_agree(nusi, N, nonres):
    """The bit-exact scalar cascade k_cascade (WAVEFRONT / REG / LDS, one kernel since round 5) and the default MFMA
    cascade k_cascade_bs (AUTO = MFMA: blocks of four columns summed in the matrix core's order; step passes at
    N = 700) agree to FLUX_RTOL with the same exact zeros; the three scalar names give the same bits.  N = 1500
    (T - 1 = 1546 rows) is past no limit of either."""
    from nusiprop_amd import _lib
    pts = [dict(cases.C2B_100, N_bins_E=N, non_resonant=nonres, majorana=maj, mphi=m, g=gg)
           for maj, m, gg in ((True, 6e5, 0.01), (False, 2e6, 0.1), (True, 1e6, 0.3))]
    plan = nusi.Plan(N, pts[0]["lEmin"], pts[0]["lEmax"], pts[0]["zmax"], max_points=len(pts), reference_order=False)
    out, names = {}, {}
    for kind in (_lib.CASCADE_WAVEFRONT, _lib.CASCADE_REG, _lib.CASCADE_LDS, _lib.CASCADE_AUTO, _lib.CASCADE_MFMA):
        plan.set_cascade(kind)
        out[kind] = plan.evolve(pts)
        names[kind] = plan.kernels()[1]
    plan.close()
    ref = out[_lib.CASCADE_LDS]
    assert np.all(np.isfinite(ref[1])) and np.any(ref[1] > 0)
    for kind, (f, fl) in out.items():
        if kind in (_lib.CASCADE_MFMA, _lib.CASCADE_AUTO):
            assert names[kind] == "k_cascade_bs"
            assert cases.rel_err(f, ref[0]) <= FLUX_RTOL and cases.rel_err(fl, ref[1]) <= FLUX_RTOL
            assert np.array_equal(f == 0, ref[0] == 0)
            continue
        assert names[kind] == "k_cascade"
        assert np.array_equal(f, ref[0]) and np.array_equal(fl, ref[1])
    assert np.array_equal(out[_lib.CASCADE_AUTO][0], out[_lib.CASCADE_MFMA][0])


def test_alpha_batches_bitexact(nusi, oracle_mod):
    """Tables of points that share m_phi and the masses are built in batches (k_alpha_tile shares
    the leaves of (S', t) alone): interleaved points of two m_phi values, four couplings each
    (batches of 3 + 1), every table bit-exact against the oracle and every flux equal to its
    single-point evolve."""
    pts = [dict(cases.C2B_100, mphi=m, g=g) for g in (0.01, 0.03, 0.1, 0.3) for m in (6e5, 2e6)]
    plan, flux, fla, tabs, _ = _gpu(nusi, pts)
    for k, kw in enumerate(pts):
        o = oracle_mod.Oracle(**cases.oracle_kwargs(kw))
        G, aT, al = o.tables()
        assert np.array_equal(tabs[k][0], G) and np.array_equal(tabs[k][1], aT)
        iu = np.triu_indices(o.T, 1)
        Ad = nusi.unpack_alpha(tabs[k][2], o.T)
        assert np.array_equal(Ad[iu], al[iu]), "point %d: alpha differs in %d entries" % (k, np.sum(Ad[iu] != al[iu]))
        _, f1, fl1, _, _ = _gpu(nusi, [kw])
        assert np.array_equal(f1[0], flux[k]) and np.array_equal(fl1[0], fla[k])


def _hip():
    """The HIP runtime libnusi.so itself links (ctypes), for streams and device buffers in tests that must not
    initialise torch's separately bundled runtime after libnusi's."""
    import ctypes
    H = ctypes.CDLL("/opt/rocm/lib/libamdhip64.so.7")
    vp = ctypes.c_void_p
    H.hipStreamCreate.argtypes = [ctypes.POINTER(vp)]
    H.hipStreamDestroy.argtypes = [vp]
    H.hipStreamSynchronize.argtypes = [vp]
    H.hipMalloc.argtypes = [ctypes.POINTER(vp), ctypes.c_size_t]
    H.hipFree.argtypes = [vp]
    H.hipMemcpy.argtypes = [vp, vp, ctypes.c_size_t, ctypes.c_int]
    return H


def test_plan_serialises_calls_across_streams(nusi):
    """One plan's device buffers (point records, tables, warnings) are reused by every call: a call on
    another stream waits for the previous call's kernels (nusi_plan_evolve's done event).  An async
    evolve on a second stream, immediately followed by a host evolve of other points on the plan's own
    stream, gives each batch its single-call result bit for bit."""
    import ctypes
    H = _hip()
    a = [dict(cases.C2B_100, mphi=m, g=g) for m, g in ((6e5, 0.01), (2e6, 0.1), (1e7, 0.5))]
    b = [dict(cases.C2B_100, mphi=m, g=g, majorana=False) for m, g in ((3e5, 0.3), (8e5, 0.05), (4e6, 0.02))]
    plan = nusi.Plan(100, 12.0, 17.0, 5.0, max_points=3, reference_order=False)
    ref_a = plan.evolve(a)
    ref_b = plan.evolve(b)
    nbytes = 3 * 3 * 100 * 8
    s2, fa, la = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p()
    assert H.hipStreamCreate(ctypes.byref(s2)) == 0
    assert H.hipMalloc(ctypes.byref(fa), nbytes) == 0 and H.hipMalloc(ctypes.byref(la), nbytes) == 0
    arr = plan.params_array(a)
    try:
        for _ in range(3):
            plan.evolve_device(arr, fa.value, la.value, s2.value)
            got_b = plan.evolve(b)                     # plan's own stream, right behind the async call
            assert H.hipStreamSynchronize(s2) == 0
            ha, hl = np.zeros((3, 3, 100)), np.zeros((3, 3, 100))
            assert H.hipMemcpy(ha.ctypes.data, fa, nbytes, 2) == 0 and H.hipMemcpy(hl.ctypes.data, la, nbytes, 2) == 0
            assert np.array_equal(ha, ref_a[0]) and np.array_equal(hl, ref_a[1])
            assert np.array_equal(got_b[0], ref_b[0]) and np.array_equal(got_b[1], ref_b[1])
    finally:
        H.hipFree(fa)
        H.hipFree(la)
        H.hipStreamDestroy(s2)


def test_alpha_batch_kernel_equals_tile_kernel(nusi):
    """The big-batch alpha kernel (shared leaves once per batch of up to 64 tables, points one after the
    other) and the k_alpha_tile<G> batches of 3 give the same tables and fluxes bit for bit: a C4-style
    slice (2 m_phi x 8 couplings, Majorana) plus Dirac and resonant-only points, several batch caps."""
    base = [dict(cases.C2B_100, mphi=m, g=g) for m in (6e5, 2e6) for g in np.logspace(-3, 0, 8)]
    pts = base + [dict(cases.C2B_100, mphi=1e6, g=0.1, majorana=False), dict(cases.C2B_100, mphi=1e6, g=0.2,
                                                                             non_resonant=False)]
    ref = _gpu(nusi, pts, alpha_kernel=1)
    assert ref[0].kernels()[0] == "k_alpha_tile"
    for kern, cap in ((0, 0), (0, 1), (0, 5), (0, 64)):
        got = _gpu(nusi, pts, alpha_batch=cap, alpha_kernel=kern)
        assert got[0].kernels()[0] == "k_alpha_batch"
        assert np.array_equal(got[1], ref[1]) and np.array_equal(got[2], ref[2]), (kern, cap)
        for a, b in zip(got[3], ref[3]):
            for x, y in zip(a, b):
                assert np.array_equal(x, y), (kern, cap)
        assert got[4] == ref[4]


def _evolve_opts(nusi, pts, kind=None, **opts):
    """evolve `pts` on the default (AUTO = MFMA) cascade, or `kind`, with plan options (nusi_plan_set_option:
    cascade_rhs, step_passes, ...)."""
    from nusiprop_amd import _lib
    p0 = pts[0]
    plan = nusi.Plan(p0["N_bins_E"], p0["lEmin"], p0["lEmax"], p0["zmax"], max_points=len(pts), reference_order=False)
    if kind is not None:
        plan.set_cascade(kind)
    for k, v in opts.items():
        plan.set_option(getattr(_lib, "OPT_" + k.upper()), v)
    out = plan.evolve(pts)
    names = plan.kernels()
    plan.close()
    return out + (names,)


@pytest.mark.parametrize("N", [37, 100, 130, 300])
def test_cascade_mfma_multi_rhs(nusi, N):
    """The MFMA cascade on every point kind -- power-law and DSNB sources, non-resonant and resonant-only, Majorana
    and Dirac: one point per workgroup (distinct tables), and several per workgroup when they share a table (pairs
    and gamma batches: gamma / norm / source variations, one operator, mixed sources in one group, a table slot with
    an odd number of points).  Every grouping agrees with the scalar kernel to FLUX_RTOL with the same exact zeros."""
    from nusiprop_amd import _lib
    distinct = [dict(cases.C2B_100, N_bins_E=N, mphi=m, g=g, majorana=maj, non_resonant=nr, source_model=src)
                for m, g, maj, nr, src in ((6e5, 0.01, True, True, 1), (2e6, 0.1, False, True, 1), (1e6, 0.3, True, True, 0),
                                           (3e7, 0.8, True, False, 1), (8e5, 0.05, True, False, 0))]
    # DSNB points at lE 12 -> 17 have a zero source (the Fermi-Dirac tail underflows): move them to lE 4 -> 9
    lo = [dict(p, lEmin=4.0, lEmax=9.0, mphi=p["mphi"] / 200.0) for p in distinct]
    for grid in (distinct, lo):
        one = _evolve_opts(nusi, grid, cascade_rhs=1)
        ref = _evolve_opts(nusi, grid, kind=_lib.CASCADE_LDS)
        assert one[2][1] == "k_cascade_bs" and ref[2][1] == "k_cascade"
        for a, b in zip(one[:2], ref[:2]):
            assert cases.rel_err(a, b) <= FLUX_RTOL and np.array_equal(a == 0, b == 0)
        gam = [dict(p, si=s, norm=nm, source_model=src) for p in grid[:4]
               for s, nm, src in ((2.0, 1.0, 1), (2.3, 3.0, 0), (2.9, 0.5, 1))]
        gam.append(dict(grid[4], si=2.7))
        gam.append(dict(grid[4], si=2.1, source_model=0))
        ref = _evolve_opts(nusi, gam, kind=_lib.CASCADE_LDS)
        for rhs, label in ((2, "k_cascade_bs_pairs + k_cascade_bs"), (0, "k_cascade_bs_gamma + pairs")):
            got = _evolve_opts(nusi, gam, cascade_rhs=rhs)
            assert got[2][1] == label, got[2]
            assert cases.rel_err(got[1], ref[1]) <= FLUX_RTOL and np.array_equal(got[1] == 0, ref[1] == 0)
        assert np.any(ref[1] > 0)


@pytest.mark.parametrize("N,lEmin", [(100, 12.0), (200, 12.0), (700, 12.0), (1200, 10.0)])
def test_cascade_step_passes(nusi, oracle_mod, N, lEmin):
    """The step-pass instance of k_cascade_bs (16 redshift steps in flight per pass, the last step's F carried to the
    next pass; nuSIprop.hpp:257-315), forced by NUSI_OPT_STEP_PASSES = 1: N = 100 (16 steps, one pass) and 200 (32
    steps, 2 passes) where one pass would fit, 700 (109 steps, 7 passes) and BASELINE C3's grid (N = 1200, lE 10 ->
    17: 134 steps, 9 passes) against the oracle's cascade on the GPU's own tables to FLUX_RTOL, with the scalar
    kernel's exact zeros."""
    from nusiprop_amd import _lib
    pts = [dict(cases.C2B_100, N_bins_E=N, lEmin=lEmin, mphi=m, g=g, majorana=maj)
           for m, g, maj in ((6e5, 0.01, True), (1e5, 0.05, True), (2e6, 0.3, False))]
    got = _evolve_opts(nusi, pts, step_passes=1)
    assert got[2][1] == "k_cascade_bs"
    plan = nusi.Plan(N, lEmin, pts[0]["lEmax"], pts[0]["zmax"], max_points=len(pts), reference_order=False)
    plan.set_cascade(_lib.CASCADE_LDS)
    ref = plan.evolve(pts)
    assert plan.Nz - 1 == {100: 16, 200: 32, 700: 109, 1200: 134}[N]
    for k, p in enumerate(pts):
        G, aT, A = plan.tables(k)
        o = oracle_mod.Oracle(**cases.oracle_kwargs(p))
        o.prepare()
        f_ref, fla_ref = o.cascade(G, aT, nusi.unpack_alpha(A, plan.T))
        assert cases.rel_err(got[0][k], f_ref) <= FLUX_RTOL, k
        assert cases.rel_err(got[1][k], fla_ref) <= FLUX_RTOL, k
        assert np.array_equal(got[0][k] == 0, ref[0][k] == 0)
    plan.close()


@pytest.mark.parametrize("N", [200, 700])
def test_cascade_step_passes_resonant_only(nusi, oracle_mod, N):
    """Step passes with resonant-only points in the launch (nuSIprop.hpp:273-278, 285-287): the launcher takes the
    per-point-flag instance of k_cascade_bs, whose chain keeps the resonant-only running sum (an all-non-resonant
    launch takes the kNR instance without it); against the oracle's cascade on the GPU's own tables."""
    from nusiprop_amd import _lib
    pts = [dict(cases.C2B_100, N_bins_E=N, lEmin=12.0, mphi=m, g=g, non_resonant=nr)
           for m, g, nr in ((6e5, 0.01, True), (2e6, 0.3, False), (1e6, 0.1, False))]
    got = _evolve_opts(nusi, pts, step_passes=1)
    assert got[2][1] == "k_cascade_bs"
    plan = nusi.Plan(N, 12.0, pts[0]["lEmax"], pts[0]["zmax"], max_points=len(pts), reference_order=False)
    plan.set_cascade(_lib.CASCADE_LDS)
    ref = plan.evolve(pts)
    for k, p in enumerate(pts):
        G, aT, A = plan.tables(k)
        o = oracle_mod.Oracle(**cases.oracle_kwargs(p))
        o.prepare()
        f_ref, fla_ref = o.cascade(G, aT, nusi.unpack_alpha(A, plan.T))
        assert cases.rel_err(got[0][k], f_ref) <= FLUX_RTOL, k
        assert cases.rel_err(got[1][k], fla_ref) <= FLUX_RTOL, k
        assert np.array_equal(got[0][k] == 0, ref[0][k] == 0)
    plan.close()


def test_plan_kernels_names(nusi):
    """nusi_plan_kernels reports what the last call launched: the batch alpha kernel, and per grid and cascade kind
    the block-synchronous MFMA cascade in every shape (one point per workgroup, pairs, gamma batches, step passes on
    N_z - 1 > 48) or the scalar k_cascade (WAVEFRONT / REG / LDS)."""
    from nusiprop_amd import _lib
    def run(N, lEmin, pts_kw, kind):
        pts = [dict(cases.C2B_100, N_bins_E=N, lEmin=lEmin, **kw) for kw in pts_kw]
        plan = nusi.Plan(N, lEmin, pts[0]["lEmax"], pts[0]["zmax"], max_points=len(pts), reference_order=False)
        plan.set_cascade(kind)
        plan.evolve(pts)
        k = plan.kernels()
        plan.close()
        return k
    two = [dict(mphi=6e5, g=0.01), dict(mphi=2e6, g=0.1)]
    pair = [dict(mphi=6e5, g=0.01, si=s) for s in (2.0, 2.5)]
    three = [dict(mphi=6e5, g=0.01, si=s) for s in (2.0, 2.5, 2.7)]
    dsnb_res = [dict(mphi=6e5, g=0.01, source_model=0, non_resonant=False)]
    for kind in (_lib.CASCADE_AUTO, _lib.CASCADE_MFMA):
        assert run(100, 12.0, two, kind) == ("k_alpha_batch", "k_cascade_bs")
        assert run(100, 12.0, pair, kind)[1] == "k_cascade_bs_pairs"
        assert run(100, 12.0, three, kind)[1] == "k_cascade_bs_gamma"
        assert run(700, 12.0, two, kind)[1] == "k_cascade_bs"
        assert run(100, 12.0, dsnb_res, kind)[1] == "k_cascade_bs"
    for kind in (_lib.CASCADE_WAVEFRONT, _lib.CASCADE_REG, _lib.CASCADE_LDS):
        assert run(100, 12.0, two, kind)[1] == "k_cascade"
        assert run(700, 12.0, two, kind)[1] == "k_cascade"


def test_c5_gamma_block_vs_oracle(nusi, oracle_mod):
    """BASELINE config 5: one full 16-gamma block of scan.c5_points() (N_E = 300, power law; one
    Stage-A table, the gamma batch k_cascade_bs_gamma by default) against the oracle -- its tables once, its
    cascade per gamma -- to FLUX_RTOL with the same exact zeros; the pairs give the one-point-per-workgroup fluxes
    bit for bit (A/B), the gamma batch to rounding."""
    from nusiprop_amd import scan
    allp = scan.c5_points()
    blk = allp[16 * 1234:16 * 1235]
    assert len({scan.table_key(p) for p in blk}) == 1 and len({p["si"] for p in blk}) == 16
    flux, fla, names = _evolve_opts(nusi, blk)
    assert names[1] == "k_cascade_bs_gamma"
    ref1 = _evolve_opts(nusi, blk, cascade_rhs=1)
    two = _evolve_opts(nusi, blk, cascade_rhs=2)
    assert two[2][1] == "k_cascade_bs_pairs"
    assert np.array_equal(two[0], ref1[0]) and np.array_equal(two[1], ref1[1])
    assert cases.rel_err(flux, ref1[0]) <= FLUX_RTOL and np.array_equal(flux == 0, ref1[0] == 0)
    o = oracle_mod.Oracle(**cases.oracle_kwargs(blk[0]))
    G, aT, al = o.tables()
    for k, p in enumerate(blk):
        ok = oracle_mod.Oracle(**cases.oracle_kwargs(p))
        ok.prepare()
        f_ref, fla_ref = ok.cascade(G, aT, al)
        assert cases.rel_err(flux[k], f_ref) <= FLUX_RTOL, k
        assert cases.rel_err(fla[k], fla_ref) <= FLUX_RTOL, k


def test_c1_test_cpp_n300(nusi, oracle_mod):
    """BASELINE config 1 (test.cpp:6-23: DSNB source, lE 9 -> 14) at N_E = 300 end to end vs the oracle."""
    kw = dict(cases.TEST_CPP, N_bins_E=300)
    o = oracle_mod.Oracle(**cases.oracle_kwargs(kw))
    f_ref, fla_ref = o.evolve()
    _, flux, fla, _, _ = _gpu(nusi, [kw])
    assert cases.rel_err(flux[0], f_ref) <= FLUX_RTOL
    assert cases.rel_err(fla[0], fla_ref) <= FLUX_RTOL

"""The opt-in scan mode NUSI_OPT_SHIFT_REUSE on the GPU, against the oracle.

Tables of one (g, masses, flags) whose m_phi lie on the lattice m_max r^(-o/2) (r = the table axis' bin ratio,
o = 0 .. K) are served by one table set of the largest m_phi on the axis extended by K bins, read o bins higher
(nusi_capi.cpp shift_groups / k_table_shift).  The mode is not bit-exact -- the bin edges round differently and the
closed forms amplify that (tests/test_f4_index_shift.py) -- so its own bound is the north star's 1e-9 on the
fluxes, against each point's own oracle evolution.  Points off the lattice are built directly and stay bit-exact.
"""
import numpy as np
import pytest

from tests import cases

pytestmark = pytest.mark.gpu

SHIFT_RTOL = 1e-9


@pytest.fixture(scope="module")
def nusi():
    import nusiprop_amd
    nusiprop_amd.load()
    return nusiprop_amd


def _lattice_points(base, offs, gs, m_max=6e5):
    r = 10 ** ((base["lEmax"] - base["lEmin"]) / base["N_bins_E"])
    return [dict(base, mphi=m_max * r ** (-o / 2), g=g) for g in gs for o in offs]


@pytest.mark.parametrize("N,K,offs", [(100, 8, (0, 1, 2, 3, 5, 8)), (300, 16, (0, 4, 9, 16))])
def test_shift_reuse_scan(nusi, oracle_mod, N, K, offs):
    from nusiprop_amd import _lib
    base = dict(cases.C2B_100, N_bins_E=N)
    pts = _lattice_points(base, offs, (0.01, 0.3))
    off_lattice = dict(base, mphi=7.77e5, g=0.3)          # no partner: built directly
    pts.append(off_lattice)
    plan = nusi.Plan(N, base["lEmin"], base["lEmax"], base["zmax"], max_points=len(pts), reference_order=False)
    plan.set_option(_lib.OPT_SHIFT_REUSE, K)
    flux, fla = plan.evolve(pts)
    assert "k_table_shift" in plan.kernels()[0]
    worst = 0.0
    for i, p in enumerate(pts):
        o = oracle_mod.Oracle(**cases.oracle_kwargs(p))
        f_ref, fla_ref = o.evolve()
        e = max(cases.rel_err(flux[i], f_ref), cases.rel_err(fla[i], fla_ref))
        assert e <= SHIFT_RTOL, (p["mphi"], p["g"], e)
        worst = max(worst, e)
    # the off-lattice point went the direct way: its tables are the oracle's bit for bit
    o = oracle_mod.Oracle(**cases.oracle_kwargs(off_lattice))
    G, aT, al = o.tables()
    Gg, aTg, Ag = plan.tables(len(pts) - 1)
    assert np.array_equal(Gg, G) and np.array_equal(aTg, aT)
    iu = np.triu_indices(o.T, 1)
    assert np.array_equal(nusi.unpack_alpha(Ag, o.T)[iu], al[iu])
    # each group's base (o = 0, the largest m_phi) reads its own tables below T: bit-exact too
    G0, aT0, A0 = plan.tables(0)
    o0 = oracle_mod.Oracle(**cases.oracle_kwargs(pts[0]))
    Gr, aTr, alr = o0.tables()
    assert np.array_equal(G0, Gr) and np.array_equal(aT0, aTr)
    assert np.array_equal(nusi.unpack_alpha(A0, o0.T)[iu], alr[iu])
    print("shift reuse N=%d K=%d: worst flux rel err %.2e" % (N, K, worst))


def test_shift_reuse_off_is_default_and_exact(nusi):
    """Without the option the same lattice scan builds every table itself (bit-exact path): the shifted tables
    differ from the direct ones only by rounding, and option 0 restores the direct tables bit for bit."""
    from nusiprop_amd import _lib
    base = dict(cases.C2B_100)
    pts = _lattice_points(base, (0, 2, 4), (0.03,))   # (g <= 0.05: couplings that share)
    plan = nusi.Plan(base["N_bins_E"], base["lEmin"], base["lEmax"], base["zmax"], max_points=len(pts), reference_order=False)
    f_direct, _ = plan.evolve(pts)
    t_direct = [plan.tables(i) for i in range(len(pts))]
    assert "k_table_shift" not in plan.kernels()[0]
    plan.set_option(_lib.OPT_SHIFT_REUSE, 4)
    f_shift, _ = plan.evolve(pts)
    assert "k_table_shift" in plan.kernels()[0]
    assert np.array_equal(f_shift[0], f_direct[0])    # the base point
    assert cases.rel_err(f_shift, f_direct) <= SHIFT_RTOL
    plan.set_option(_lib.OPT_SHIFT_REUSE, 0)
    f_again, _ = plan.evolve(pts)
    assert np.array_equal(f_again, f_direct)
    for i in range(len(pts)):
        for a, b in zip(plan.tables(i), t_direct[i]):
            assert np.array_equal(a, b)


def test_shift_reuse_option_bounds(nusi):
    from nusiprop_amd import _lib
    plan = nusi.Plan(60, 12.0, 17.0, 5.0, max_points=2, reference_order=False)
    with pytest.raises(Exception):
        plan.set_option(_lib.OPT_SHIFT_REUSE, 129)
    with pytest.raises(Exception):
        plan.set_option(_lib.OPT_SHIFT_REUSE, -1)


def test_shift_reuse_c4s_lattice_k128(nusi, oracle_mod):
    """The bench's c4s workload at its own K (NUSI_OPT_SHIFT_REUSE = 128, offsets 0 .. 124 on scan.c4s_points'
    lattice), at g = 1e-3, the largest coupling that shares (0.05) and g = 1 (built directly): 96 points, every flux
    within the 1e-9 north-star bound of each point's own oracle evolution."""
    from nusiprop_amd import _lib, scan
    pts = [p for p in scan.c4s_points(n_g=2)] + [dict(p, g=0.05) for p in scan.c4s_points(n_g=1)]
    assert sorted({p["g"] for p in pts}) == [1e-3, 0.05, 1.0] and len(pts) == 96
    p0 = pts[0]
    plan = nusi.Plan(p0["N_bins_E"], p0["lEmin"], p0["lEmax"], p0["zmax"], max_points=len(pts), reference_order=False)
    plan.set_option(_lib.OPT_SHIFT_REUSE, 128)
    flux, fla = plan.evolve(pts)
    assert "k_table_shift" in plan.kernels()[0]
    plan.close()
    f_ref, fla_ref = oracle_mod.evolve_many(pts)
    errs = [max(cases.rel_err(flux[i], f_ref[i]), cases.rel_err(fla[i], fla_ref[i])) for i in range(len(pts))]
    worst = int(np.argmax(errs))
    assert errs[worst] <= SHIFT_RTOL, (pts[worst]["mphi"], pts[worst]["g"], errs[worst])
    print("c4s K=128 at g = 1e-3, 1: worst flux rel err %.2e" % errs[worst])


def test_shift_reuse_rounded_mphi_goes_direct(nusi, oracle_mod):
    """A point within 1e-6 of a lattice offset but not ON the lattice (m_phi rounded to 7 significant digits) is
    not served by the base's shifted tables, whose m_phi would differ from its own by ~1e-8: it is
    built directly, bit-exact, while its exact lattice partner still shares the base."""
    from nusiprop_amd import _lib
    base = dict(cases.C2B_100)
    exact = _lattice_points(base, (0, 3), (0.03,))
    r = 10 ** ((base["lEmax"] - base["lEmin"]) / base["N_bins_E"])
    m6 = 6e5 * r ** (-6 / 2)
    rounded = dict(base, mphi=float("%.7g" % m6), g=0.03)
    assert rounded["mphi"] != m6 and abs(rounded["mphi"] / m6 - 1) < 1e-6
    pts = exact + [rounded]
    plan = nusi.Plan(base["N_bins_E"], base["lEmin"], base["lEmax"], base["zmax"], max_points=len(pts), reference_order=False)
    plan.set_option(_lib.OPT_SHIFT_REUSE, 8)
    flux, fla = plan.evolve(pts)
    assert "k_table_shift" in plan.kernels()[0]
    o = oracle_mod.Oracle(**cases.oracle_kwargs(rounded))
    G, aT, al = o.tables()
    Gg, aTg, Ag = plan.tables(2)
    plan.close()
    assert np.array_equal(Gg, G) and np.array_equal(aTg, aT)
    iu = np.triu_indices(o.T, 1)
    assert np.array_equal(nusi.unpack_alpha(Ag, o.T)[iu], al[iu])


def test_shift_reuse_phiphi_warnings_in_range(nusi, ref_tables):
    """phi-phi on with shift reuse: the base tables are built on the axis extended by K bins, where alpha's phi-phi
    lookups reach x1 = (m - n) 1.0001 > 1000, outside the reference's table nodes (interp.hpp:355-361).  No member
    reads those entries (its own axis has T <= 1000 bins), so no member may inherit the warning: the
    members' warnings equal the direct path's (none), and the call does not fail with NUSI_EINTERP."""
    from nusiprop_amd import _lib
    at, atd, a, ad = ref_tables
    base = dict(cases.C2B_100, N_bins_E=850, phiphi=True)
    K = 30
    pts = _lattice_points(base, (0, 10, 20, 30), (0.05,), m_max=3e7)   # (couplings above 0.05 do not share)
    plan = nusi.Plan(850, base["lEmin"], base["lEmax"], base["zmax"], max_points=len(pts), reference_order=False)
    plan.load_phiphi(at, a)
    assert plan.T <= 1000
    f_direct, _ = plan.evolve(pts)
    w_direct = plan.warnings(len(pts))
    plan.set_option(_lib.OPT_SHIFT_REUSE, K)
    f_shift, _ = plan.evolve(pts)
    assert "k_table_shift" in plan.kernels()[0]
    assert plan.warnings(len(pts)) == w_direct and all(w & 8 == 0 for w in w_direct)
    assert cases.rel_err(f_shift, f_direct) <= SHIFT_RTOL   # (8.8e-10 measured at g = 0.05)
    # the base axis itself (K more redshift steps, as nusi_capi.cpp ensure_shift_plan makes it) does reach
    # out-of-node lookups: the case the test is about
    r = 10 ** ((base["lEmax"] - base["lEmin"]) / base["N_bins_E"])
    zb = r ** (plan.Nz + K - 1.5) - 1
    sp = nusi.Plan(850, base["lEmin"], base["lEmax"], zb, max_points=1, reference_order=False)
    sp.load_phiphi(at, a)
    assert sp.T == plan.T + K
    with pytest.raises(_lib.NusiError) as e:
        sp.evolve([dict(pts[0], zmax=zb)])
    assert e.value.code == _lib.NUSI_EINTERP
    plan.close()
    sp.close()

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
    plan = nusi.Plan(N, base["lEmin"], base["lEmax"], base["zmax"], max_points=len(pts))
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
    pts = _lattice_points(base, (0, 2, 4), (0.1,))
    plan = nusi.Plan(base["N_bins_E"], base["lEmin"], base["lEmax"], base["zmax"], max_points=len(pts))
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
    plan = nusi.Plan(60, 12.0, 17.0, 5.0, max_points=2)
    with pytest.raises(Exception):
        plan.set_option(_lib.OPT_SHIFT_REUSE, 129)
    with pytest.raises(Exception):
        plan.set_option(_lib.OPT_SHIFT_REUSE, -1)

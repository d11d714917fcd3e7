"""The block-synchronous MFMA cascade k_cascade_bs, the library's one MFMA cascade since round 5 (the per-stage kernels
k_cascade_ws / gb / wsp it replaced were removed; rounds 4's tests held it bit-exact to them), against
the oracle and the bit-exact scalar cascade k_cascade.

Every point's flux must meet the oracle's to FLUX_RTOL in every configuration -- one point per workgroup, pairs
sharing a table, gamma batches of 3..16 points (power-law and DSNB sources), resonant-only points, and step passes on
grids beyond 48 redshift steps (C3's) -- with the same exact zeros as the scalar kernel; and the groupings agree with
each other to rounding (the MFMA sums each block of four columns in its own order)."""
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


def _run(nusi, pts, exact=False, **opts):
    """Plan.evolve of `pts`: the default MFMA cascade, or (exact) the scalar k_cascade; opts: OPT_* options."""
    from nusiprop_amd import _lib
    p0 = pts[0]
    plan = nusi.Plan(p0["N_bins_E"], p0["lEmin"], p0["lEmax"], p0["zmax"], max_points=len(pts), reference_order=False)
    if exact:
        plan.set_cascade(_lib.CASCADE_LDS)
    for k, v in opts.items():
        plan.set_option(getattr(_lib, "OPT_" + k.upper()), v)
    flux, fla = plan.evolve(pts)
    tabs = [plan.tables(i) for i in range(len(pts))]
    names = plan.kernels()
    plan.close()
    return flux, fla, tabs, names


def _vs_oracle(nusi, oracle_mod, pts, fla, tabs):
    for k, p in enumerate(pts):
        o = oracle_mod.Oracle(**cases.oracle_kwargs(p))
        o.prepare()
        G, aT, A = tabs[k]
        _, fla_ref = o.cascade(G, aT, nusi.unpack_alpha(A, o.T))
        assert cases.rel_err(fla[k], fla_ref) <= FLUX_RTOL, (k, p)


def _same_to_rounding(a, b):
    d = max(cases.rel_err(a[k], b[k]) for k in range(len(a)))
    assert d <= FLUX_RTOL and np.array_equal(a == 0, b == 0), d


@pytest.mark.parametrize("N", [37, 100, 300])
def test_bs_one_point(nusi, oracle_mod, N):
    """One point per workgroup (distinct tables): power law and DSNB, Majorana and Dirac, resonant-only -- against the
    oracle and the scalar kernel (same exact zeros)."""
    pts = [dict(cases.C2B_100, N_bins_E=N, mphi=m, g=g, majorana=maj, non_resonant=nr, source_model=src)
           for m, g, maj, nr, src in ((6e5, 0.01, True, True, 1), (2e6, 0.1, False, True, 1), (1e6, 0.3, True, True, 0),
                                      (3e7, 0.8, True, False, 1), (8e5, 0.05, True, False, 0))]
    lo = [dict(p, lEmin=4.0, lEmax=9.0, mphi=p["mphi"] / 200.0) for p in pts]   # DSNB flux nonzero at lE 4 -> 9
    for grid in (pts, lo):
        ref = _run(nusi, grid, exact=True)
        new = _run(nusi, grid, cascade_rhs=1)
        assert new[3][1] == "k_cascade_bs" and ref[3][1] == "k_cascade"
        _same_to_rounding(new[0], ref[0])
        _same_to_rounding(new[1], ref[1])
        _vs_oracle(nusi, oracle_mod, grid, new[1], new[2])


@pytest.mark.parametrize("N", [100, 300])
def test_bs_all_non_resonant_instance(nusi, oracle_mod, N):
    """A launch whose points are all non-resonant runs k_cascade_bs's kNR instance (the resonant-only terms compiled
    out); a launch with one resonant point runs the per-point-flag instance.  The non-resonant points get the same
    bits from both, in every grouping (one point per workgroup, pairs, a gamma batch)."""
    base = dict(cases.C2B_100, N_bins_E=N, mphi=2e6, g=0.1)
    nr = [dict(base, si=2.0 + 0.1 * k) for k in range(6)] + [dict(base, mphi=6e5, g=0.01, si=2.3),
                                                            dict(base, mphi=6e5, g=0.01, si=2.6),
                                                            dict(base, mphi=9e5, g=0.3, majorana=False, source_model=0)]
    res = [dict(base, mphi=3e7, g=0.8, non_resonant=False)]
    for rhs in (1, 0):
        opts = dict(cascade_rhs=1) if rhs else {}
        a = _run(nusi, nr, **opts)
        b = _run(nusi, nr + res, **opts)
        assert "k_cascade_bs" in a[3][1] and "k_cascade_bs" in b[3][1], (a[3], b[3])
        assert np.array_equal(a[0], b[0][:len(nr)]) and np.array_equal(a[1], b[1][:len(nr)])
    _vs_oracle(nusi, oracle_mod, nr + res, b[1], b[2])


@pytest.mark.parametrize("N", [100, 300])
def test_bs_pairs_and_gamma_batches(nusi, oracle_mod, N):
    """Points sharing a table: pairs (k_cascade_bs_pairs) and gamma batches of 3..16 (k_cascade_bs_gamma), mixed
    sources in one batch; each point equals its one-point-per-workgroup flux bit for bit and the oracle's to
    FLUX_RTOL."""
    base = [dict(cases.C2B_100, N_bins_E=N, mphi=m, g=g) for m, g in ((6e5, 0.01), (2e6, 0.1), (1e6, 0.3))]
    pts = [dict(base[0], si=2.0 + 0.05 * k) for k in range(16)]                              # a full batch
    pts += [dict(base[1], si=s, source_model=src) for s, src in ((2.2, 1), (2.5, 0), (2.8, 1))]   # mixed, 3
    pts += [dict(base[2], si=s) for s in (2.1, 2.9)]                                          # a pair
    pts += [dict(base[2], mphi=7e5, si=2.4)]                                                  # alone
    one = _run(nusi, pts, cascade_rhs=1)
    grp = _run(nusi, pts)
    assert grp[3][1] == "k_cascade_bs_gamma + pairs + k_cascade_bs"
    for a, b in zip(grp[:2], one[:2]):
        _same_to_rounding(a, b)
    _vs_oracle(nusi, oracle_mod, pts, grp[1], grp[2])


def test_bs_c5_block(nusi, oracle_mod):
    """BASELINE C5: one 16-gamma block of scan.c5_points() on k_cascade_bs_gamma against the oracle."""
    from nusiprop_amd import scan
    blk = scan.c5_points()[16 * 777:16 * 778]
    flux, fla, tabs, names = _run(nusi, blk)
    assert names[1] == "k_cascade_bs_gamma"
    o = oracle_mod.Oracle(**cases.oracle_kwargs(blk[0]))
    G, aT, al = o.tables()
    for k, p in enumerate(blk):
        ok = oracle_mod.Oracle(**cases.oracle_kwargs(p))
        ok.prepare()
        _, fla_ref = ok.cascade(G, aT, al)
        assert cases.rel_err(fla[k], fla_ref) <= FLUX_RTOL, k


@pytest.mark.parametrize("N,lEmin", [(200, 12.0), (700, 12.0), (1200, 10.0)])
def test_bs_step_passes(nusi, oracle_mod, N, lEmin):
    """Grids beyond 48 redshift steps (N = 200: 32 steps, 700: 109, C3's 1200 at lE 10 -> 17: 134) in step passes,
    one point per workgroup and gamma batches where a batch's accumulators fit the register file (N = 200; the
    FIFO carries each pass' last step to the next pass)."""
    pts = [dict(cases.C2B_100, N_bins_E=N, lEmin=lEmin, mphi=m, g=g, majorana=maj)
           for m, g, maj in ((6e5, 0.01, True), (1e5, 0.05, True), (2e6, 0.3, False))]
    pts += [dict(pts[0], si=s) for s in (2.0, 2.2, 2.7)]
    new = _run(nusi, pts)
    assert "k_cascade_bs" in new[3][1]
    _vs_oracle(nusi, oracle_mod, pts, new[1], new[2])
    one = _run(nusi, pts, cascade_rhs=1)
    forced = _run(nusi, pts, step_passes=1)   # the 16-step / 128-row pass instance on every grid
    ref = _run(nusi, pts, exact=True)
    assert one[3][1] == "k_cascade_bs" and forced[3][1] == "k_cascade_bs" and ref[3][1] == "k_cascade"
    for a in (new, one, forced):
        _same_to_rounding(a[1], ref[1])
    if N == 1200:   # 1332 rows: only the 128-row / 16-step configuration fits, forced or not
        assert np.array_equal(one[1], forced[1])


def test_bs_c3_gamma_block(nusi, oracle_mod, ref_tables):
    """A 16-gamma block on the C3 grid (N_E = 1200, lE 10 -> 17, N_z - 1 = 134 steps, phi-phi on at the
    reference's table geometry; nuSIprop.hpp:257-315): one table, every point against the oracle's cascade on the
    block's table (bit-exact to the oracle's own, test_phiphi.py::test_c3_n1200_phiphi) to FLUX_RTOL, and against
    the same points on the scalar kernel k_cascade.  The automatic kernel there is k_cascade_bs in step passes,
    one point per workgroup: a batch's accumulators are 1332 rows x (steps x points) doubles, and at the 96
    columns of the N_E = 300 gamma batch that is 1 MB against a CU's 512 KB of registers."""
    from nusiprop_amd import _lib
    from tests.test_phiphi import C3
    at, atd, a, ad = ref_tables
    blk = [dict(C3, si=2.0 + 0.06 * k, norm=1.0 + 0.1 * k) for k in range(16)]
    res = {}
    for exact in (False, True):
        p = nusi.Plan(C3["N_bins_E"], C3["lEmin"], C3["lEmax"], C3["zmax"], max_points=16, reference_order=False)
        p.load_phiphi(at, a)
        if exact:
            p.set_cascade(_lib.CASCADE_LDS)
        flux, fla = p.evolve(blk)
        assert all(w & 8 == 0 for w in p.warnings(16))
        res[int(exact)] = (flux, fla, p.kernels()[1], p.tables(0))
        p.close()
    assert res[0][2] == "k_cascade_bs" and res[1][2] == "k_cascade"
    G, aT, A = res[0][3]
    for k, kw in enumerate(blk):
        ok = oracle_mod.Oracle(**cases.oracle_kwargs(kw))
        ok.prepare()
        f_ref, fla_ref = ok.cascade(G, aT, nusi.unpack_alpha(A, ok.T))
        assert cases.rel_err(res[0][0][k], f_ref) <= FLUX_RTOL, k
        assert cases.rel_err(res[0][1][k], fla_ref) <= FLUX_RTOL, k
        assert cases.rel_err(res[0][1][k], res[1][1][k]) <= FLUX_RTOL, k


def test_per_stage_sync_refused(nusi):
    """NUSI_OPT_CASCADE_SYNC = 1 selected the per-stage kernels of rounds 2-3, which are gone: refused with
    NUSI_EPARAM (0 and 2 both select k_cascade_bs)."""
    from nusiprop_amd import _lib
    plan = nusi.Plan(100, 12.0, 17.0, 5.0, max_points=1, reference_order=False)
    try:
        with pytest.raises(_lib.NusiError):
            plan.set_option(_lib.OPT_CASCADE_SYNC, 1)
        plan.set_option(_lib.OPT_CASCADE_SYNC, 2)
        plan.set_option(_lib.OPT_CASCADE_SYNC, 0)
    finally:
        plan.close()

"""The phi-phi (double-scalar production) path: interp::spline_ND tables
(interp.hpp:13-638) in the alphaTilde (nuSIprop.hpp:1195-1213) and alpha
(:1477-1503) channels.  Synthetic tables in the reference layout
(nusiprop_amd.phiphi_tables.write_synthetic_tables); GPU tables bit-exact against the
oracle, fluxes to cases.FLUX_RTOL.  BASELINE config C3 (N_E = 1200, lE 10 -> 17, phi-phi
on) runs on tables with the reference's exact axes and record counts ({5000, 100},
{1000, 1000, 100}, xsec/tables_phiphi.py:21-22, 39-41; 1.6 GB on disk, 400 MB on the
GPU): every Gamma / alphaTilde / alpha entry bit-exact, no lookup outside the nodes,
and the full cascade."""
import os

import numpy as np
import pytest

from tests import cases
from nusiprop_amd.phiphi_tables import write_synthetic_tables


def make_tables(d, at_dims=(120, 10), a_dims=(40, 110, 6), x0_range=(1.0, 2e4)):
    """Small stand-in tables (x0 log-spaced over x0_range, x1 = 0 .. a_dims[1] - 1, log10 delta in
    [0.003, 0.06]) for the small-grid tests."""
    return write_synthetic_tables(d, at_dims=at_dims, a_dims=a_dims, at_x0=x0_range, a_x0=x0_range,
                                  a_x1=(0.0, a_dims[1] - 1.0), delta=(0.003, 0.06))

PP_SMALL = dict(mphi=1e4, g=0.05, mntot=0.1, si=2.5, norm=1.0, majorana=True, non_resonant=True,
                normal_ordering=True, N_bins_E=60, lEmin=10.0, lEmax=12.0, zmax=5.0, flav=2, phiphi=True,
                source_model=1)
C3 = dict(PP_SMALL, mphi=1e5, N_bins_E=1200, lEmin=10.0, lEmax=17.0)


def test_synthetic_table_layout(tmp_path):
    at, atd, a, ad = make_tables(str(tmp_path))
    rec = np.fromfile(a, dtype=np.float32).reshape(-1, 4)
    assert rec.shape[0] == np.prod(ad)
    # last index fastest: x2 cycles first, x0 changes slowest
    assert rec[1, 2] > rec[0, 2] and rec[1, 0] == rec[0, 0]
    assert rec[ad[2] * ad[1], 0] > rec[0, 0]
    assert np.all(rec[:, 3] > 0)


def test_oracle_loads_synthetic_tables(tmp_path, oracle_mod):
    at, atd, a, ad = make_tables(str(tmp_path))
    o = oracle_mod.Oracle(**cases.oracle_kwargs(PP_SMALL))
    o.load_phiphi(at, atd, a, ad)
    G, aT, al = o.tables()
    o2 = oracle_mod.Oracle(**cases.oracle_kwargs(dict(PP_SMALL, phiphi=False)))
    G2, aT2, al2 = o2.tables()
    assert np.all(np.isfinite(al)) and np.any(al != al2) and np.any(aT != aT2)   # the channel contributes


def _plan(nusi, kw, tabs):
    p = nusi.Plan(kw["N_bins_E"], kw["lEmin"], kw["lEmax"], kw["zmax"], max_points=1, reference_order=False)
    at, atd, a, ad = tabs
    p.load_phiphi(at, a, atd, ad)
    return p


@pytest.mark.gpu
def test_phiphi_small_bitexact(tmp_path, oracle_mod):
    import nusiprop_amd as nusi
    tabs = make_tables(str(tmp_path))
    o = oracle_mod.Oracle(**cases.oracle_kwargs(PP_SMALL))
    o.load_phiphi(*tabs)
    G, aT, al = o.tables()
    p = _plan(nusi, PP_SMALL, tabs)
    flux, fla = p.evolve([PP_SMALL])
    Gg, aTg, Ag = p.tables(0)
    assert np.array_equal(Gg, G) and np.array_equal(aTg, aT)
    iu = np.triu_indices(o.T, 1)
    assert np.array_equal(nusi.unpack_alpha(Ag, o.T)[iu], al[iu])
    f_ref, fla_ref = o.cascade(G, aT, al)
    assert cases.rel_err(fla[0], fla_ref) <= cases.FLUX_RTOL


@pytest.mark.gpu
def test_phiphi_multi_table_batches(tmp_path, oracle_mod):
    """Several couplings per m_phi with phi-phi on share one k_alpha_batch<true> batch: the phi-phi core of a
    mass state depends on (S', t) alone (m_phi, masses, bin edges) and is evaluated once per batch, each point
    applies its own g^4 scale (alpha_phiphi_scale).  Plain points in the same call run on the other launch (the
    batches without the channel), Dirac and resonant-only points on theirs.  Every table of every point is
    bit-exact against the oracle -- automatic batches, caps of 1 and 64, and the tile kernel -- and the fluxes
    agree to FLUX_RTOL."""
    import nusiprop_amd as nusi
    from nusiprop_amd import _lib
    tabs = make_tables(str(tmp_path))
    pts = [dict(PP_SMALL, g=g) for g in (0.01, 0.02, 0.05, 0.1, 0.3)]
    pts += [dict(PP_SMALL, g=0.05, majorana=False), dict(PP_SMALL, g=0.08, majorana=False),
            dict(PP_SMALL, g=0.05, phiphi=False), dict(PP_SMALL, g=0.2, phiphi=False),
            dict(PP_SMALL, g=0.05, non_resonant=False), dict(PP_SMALL, g=0.02, si=2.2)]
    refs = []
    for kw in pts:
        o = oracle_mod.Oracle(**cases.oracle_kwargs(kw))
        if kw["phiphi"] and kw["non_resonant"]:
            o.load_phiphi(*tabs)
        G, aT, al = o.tables()
        refs.append((o, G, aT, al))
    T = refs[0][0].T
    iu = np.triu_indices(T, 1)
    for opt, val in ((None, 0), (_lib.OPT_ALPHA_BATCH, 1), (_lib.OPT_ALPHA_BATCH, 64), (_lib.OPT_ALPHA_KERNEL, 1)):
        p = nusi.Plan(PP_SMALL["N_bins_E"], PP_SMALL["lEmin"], PP_SMALL["lEmax"], PP_SMALL["zmax"], max_points=len(pts), reference_order=False)
        p.load_phiphi(tabs[0], tabs[2], tabs[1], tabs[3])
        if opt is not None:
            p.set_option(opt, val)
        flux, fla = p.evolve(pts)
        for k, (o, G, aT, al) in enumerate(refs):
            Gg, aTg, Ag = p.tables(k)
            assert np.array_equal(Gg, G) and np.array_equal(aTg, aT), (opt, val, k)
            A = nusi.unpack_alpha(Ag, T)
            if pts[k]["non_resonant"]:
                assert np.array_equal(A[iu], al[iu]), (opt, val, k, int(np.sum(A[iu] != al[iu])))
            else:
                d = np.arange(T - 1)
                assert np.array_equal(A[d, d + 1], al[d, d + 1]), (opt, val, k)
            f_ref, fla_ref = o.cascade(G, aT, al)
            assert cases.rel_err(fla[k], fla_ref) <= cases.FLUX_RTOL, (opt, val, k)
        p.close()


@pytest.mark.gpu
def test_phiphi_out_of_range_is_an_error(tmp_path):
    """A lookup outside the table nodes ends the reference (interp.hpp:355-361); here NUSI_EINTERP."""
    import nusiprop_amd as nusi
    tabs = make_tables(str(tmp_path), x0_range=(1.0, 50.0))     # s'- and -t+ beyond 50 are off the table
    p = _plan(nusi, PP_SMALL, tabs)
    with pytest.raises(nusi.NusiError) as e:
        p.evolve([PP_SMALL])
    assert e.value.code == nusi._lib.NUSI_EINTERP


def test_reference_geometry_tables(tmp_path):
    """write_synthetic_tables() defaults: the reference's axes and record counts, float32 records with the
    last index fastest (interp.hpp:249-291) -- the files nusi_plan_load_phiphi reads with dims = NULL."""
    at, atd, a, ad = write_synthetic_tables(str(tmp_path))
    assert (atd, ad) == ([5000, 100], [1000, 1000, 100])
    assert os.path.getsize(at) == 5000 * 100 * 3 * 4 and os.path.getsize(a) == 1000 * 1000 * 100 * 4 * 4
    r = np.memmap(a, dtype=np.float32, mode="r").reshape(-1, 4)
    assert r[0, 0] == np.float32(4.0) and r[-1, 0] == np.float32(1e4)
    assert r[0, 1] == 1 and r[100 * 999, 1] == 1000 and r[99, 2] == np.float32(0.05)
    assert r[1, 2] > r[0, 2] and r[1, 0] == r[0, 0] and r[100, 1] == 2
    t = np.fromfile(at, dtype=np.float32).reshape(-1, 3)
    assert t[0, 0] == np.float32(4.0) and t[-1, 0] == np.float32(1e4) and np.all(t[:, 2] > 0)


def test_c3_oracle_stays_inside_reference_nodes(ref_tables, oracle_mod):
    """BASELINE C3 (m_phi = 1e5, N_E = 1200, lE 10 -> 17): every phi-phi lookup of the full table build
    falls inside the reference's table nodes (x1 = (m - n) * 1.0001 <= 1000, log10 delta = 7/1200), so
    the reference would not exit(1) on this configuration."""
    o = oracle_mod.Oracle(**cases.oracle_kwargs(C3))
    o.load_phiphi(*ref_tables)
    G, aT, al = o.tables()     # raises on an out-of-range lookup
    assert np.all(np.isfinite(al)) and np.all(np.isfinite(aT))


@pytest.mark.gpu
def test_c3_n1200_phiphi(ref_tables, oracle_mod):
    import nusiprop_amd as nusi
    at, atd, a, ad = ref_tables
    o = oracle_mod.Oracle(**cases.oracle_kwargs(C3))
    o.load_phiphi(at, atd, a, ad)
    G, aT, al = o.tables()
    p = nusi.Plan(C3["N_bins_E"], C3["lEmin"], C3["lEmax"], C3["zmax"], max_points=1, reference_order=False)
    p.load_phiphi(at, a)                       # dims = NULL: the reference's {5000,100}, {1000,1000,100}
    flux, fla = p.evolve([C3])                 # raises NUSI_EINTERP on an out-of-range lookup
    assert p.warnings(1)[0] & 8 == 0
    Gg, aTg, Ag = p.tables(0)
    T = o.T
    assert (p.N, p.T) == (1200, 1333)
    assert np.array_equal(Gg, G) and np.array_equal(aTg, aT)
    A = nusi.unpack_alpha(Ag, T)
    iu = np.triu_indices(T, 1)
    assert np.array_equal(A[iu], al[iu]), "alpha differs in %d of %d entries" % (np.sum(A[iu] != al[iu]), len(iu[0]))
    f_ref, fla_ref = o.cascade(G, aT, al)
    assert cases.rel_err(flux[0], f_ref) <= cases.FLUX_RTOL
    assert cases.rel_err(fla[0], fla_ref) <= cases.FLUX_RTOL

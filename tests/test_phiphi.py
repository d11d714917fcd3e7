"""The phi-phi (double-scalar production) path: interp::spline_ND tables
(interp.hpp:13-638) in the alphaTilde (nuSIprop.hpp:1195-1213) and alpha
(:1477-1503) channels.  Synthetic tables in the reference layout
(tests/phiphi_synth.py); GPU tables bit-exact against the oracle, fluxes to
cases.FLUX_RTOL.  BASELINE config C3 (N_E = 1200, lE 10 -> 17, phi-phi on) is checked
on a sample of alpha entries (the oracle's full N=1200 table would take
minutes) plus every Gamma / alphaTilde entry and the full cascade."""
import numpy as np
import pytest

from tests import cases
from tests.phiphi_synth import make_tables

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
    p = nusi.Plan(kw["N_bins_E"], kw["lEmin"], kw["lEmax"], kw["zmax"], max_points=1)
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
def test_phiphi_out_of_range_is_an_error(tmp_path):
    """A lookup outside the table nodes ends the reference (interp.hpp:355-361); here NUSI_EINTERP."""
    import nusiprop_amd as nusi
    tabs = make_tables(str(tmp_path), x0_range=(1.0, 50.0))     # s'- and -t+ beyond 50 are off the table
    p = _plan(nusi, PP_SMALL, tabs)
    with pytest.raises(nusi.NusiError) as e:
        p.evolve([PP_SMALL])
    assert e.value.code == nusi._lib.NUSI_EINTERP


@pytest.mark.gpu
def test_c3_n1200_phiphi(tmp_path, oracle_mod):
    import nusiprop_amd as nusi
    tabs = make_tables(str(tmp_path), a_dims=(40, 1400, 6), x1_max=1400.0)
    o = oracle_mod.Oracle(**cases.oracle_kwargs(C3))
    o.load_phiphi(*tabs)
    o.prepare()
    p = _plan(nusi, C3, tabs)
    flux, fla = p.evolve([C3])
    Gg, aTg, Ag = p.tables(0)
    T = o.T
    assert (p.N, p.T) == (1200, 1333)
    Emin, Emax, _, z = o.grid()
    N = o.N
    lo = np.concatenate([Emin, Emin[-1] * (1 + z[1:T - N + 1])])
    hi = np.concatenate([Emax, Emax[-1] * (1 + z[1:T - N + 1])])
    for n in range(0, T, 97):   # Gamma / alphaTilde entries (every 97th: each is an O(1) oracle call)
        assert Gg[n] == o.Gamma(lo[n], hi[n]) and aTg[n] == o.alphaTilde(lo[n], hi[n])
    rng = np.random.default_rng(20250213)
    m = rng.integers(1, T, 400)
    n = (rng.random(400) * m).astype(int)
    for mm, nn in zip(m, n):
        assert Ag[mm * (mm - 1) // 2 + nn] == o.alpha(lo[nn], hi[nn], lo[mm], hi[mm]), (nn, mm)
    A = nusi.unpack_alpha(Ag, T)
    f_ref, fla_ref = o.cascade(Gg, aTg, A)
    assert cases.rel_err(fla[0], fla_ref) <= cases.FLUX_RTOL

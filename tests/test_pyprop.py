"""The drop-in Python surface: nusiprop_amd.pyprop against the behaviour of the
reference's Cython class (nuSIprop.pyx:12-144) and the oracle's numbers.

pyprop runs the reference's own arithmetic by default (NUSI_OPT_REFERENCE_ORDER,
GSL's dilogarithm algorithms), so its fluxes are checked against the oracle in
that mode (oracle.reference_order(1))."""
import os
import warnings

import numpy as np
import pytest

from tests import cases

pytestmark = pytest.mark.gpu


def _kw(d):
    """calculate_flux keywords; source_model is pyprop's extension keyword (DSNB by default)."""
    return dict(d)


@pytest.fixture(scope="module")
def nusi():
    import nusiprop_amd
    return nusiprop_amd


def test_not_evolved_returns_zeros_with_warning(nusi):
    ev = nusi.pyprop(**_kw(cases.TEST_CPP))
    with pytest.warns(UserWarning, match="not evolved"):
        f = ev.get_flux()
    assert f.shape == (3, 100) and not f.any()
    with pytest.warns(UserWarning, match="not evolved"):
        assert not ev.get_flux_fla().any()


def _ref_evolve(oracle_mod, kw):
    """The oracle's evolve() in the reference's arithmetic (the drop-in default)."""
    with oracle_mod.reference_order(1):
        return oracle_mod.Oracle(**cases.oracle_kwargs(kw)).evolve()


def test_evolve_set_parameters_cycle(nusi, oracle_mod):
    ev = nusi.pyprop(**_kw(cases.TEST_CPP))
    ev.evolve()
    f_ref, fla_ref = _ref_evolve(oracle_mod, cases.TEST_CPP)
    assert cases.rel_err(ev.get_flux(), f_ref) <= cases.FLUX_RTOL
    assert cases.rel_err(ev.get_flux_fla(), fla_ref) <= cases.FLUX_RTOL
    ev.set_parameters(g=0.05, mphi=2e6)            # resets the evolved flag (nuSIprop.pyx:83)
    with pytest.warns(UserWarning):
        assert not ev.get_flux().any()
    ev.evolve()
    _, fla2 = _ref_evolve(oracle_mod, dict(cases.TEST_CPP, g=0.05, mphi=2e6))
    assert cases.rel_err(ev.get_flux_fla(), fla2) <= cases.FLUX_RTOL


def test_energies_and_interp(nusi, oracle_mod):
    import scipy.interpolate as interp
    ev = nusi.pyprop(**_kw(cases.C2B_100))
    ev.evolve()
    o = oracle_mod.Oracle(**cases.oracle_kwargs(cases.C2B_100))
    _, _, Enu, _ = o.grid()
    E = ev.get_energies()
    assert np.array_equal(E, Enu)
    q = np.geomspace(E[0] * 1.01, E[-1] * 0.99, 17)
    fla = ev.get_flux_fla()
    si = cases.C2B_100["si"]
    for f, fn in enumerate([ev.interp_flux_el, ev.interp_flux_mu, ev.interp_flux_ta]):
        want = interp.interp1d(np.log10(E), fla[f] * E ** si)(np.log10(q)) / q ** si
        np.testing.assert_array_equal(fn(q), want)


def test_check_energy_conservation_matches_oracle(nusi, oracle_mod):
    """Same call sequence as the oracle, stale norm_total semantics included."""
    ev = nusi.pyprop(**_kw(cases.C2B_100))
    with oracle_mod.reference_order(1):
        o = oracle_mod.Oracle(**cases.oracle_kwargs(cases.C2B_100))
        ev.evolve()
        o.evolve()
        r, r_ref = ev.check_energy_conservation(), o.check_energy_conservation()
    assert abs(r - r_ref) <= cases.FLUX_RTOL * abs(r_ref)
    # before any evolve the reference reads norm_total uninitialised: here a warning and NaN (deliberate
    # difference); the Python evolved flag is untouched (as in the reference)
    ev2 = nusi.pyprop(**_kw(cases.C2B_100))
    with pytest.warns(UserWarning, match="before any evolve"):
        assert np.isnan(ev2.check_energy_conservation())
    with pytest.warns(UserWarning, match="not evolved"):
        ev2.get_flux()
    assert np.isfinite(ev2.check_energy_conservation())   # the call above evolved the C++ object


def test_failed_evolve_leaves_not_evolved(nusi, monkeypatch):
    """An evolve that fails (an error the reference ends with exit(1), e.g. EINTERP for a phi-phi lookup
    outside the table) raises NusiError and leaves pyprop not evolved: get_flux then warns and returns
    zeros instead of a stale flux behind an "evolved" flag."""
    ev = nusi.pyprop(**_kw(cases.C2B_100))
    ev.evolve()
    assert ev.get_flux_fla().any()
    L = nusi._lib.load()
    monkeypatch.setattr(L, "nusi_evolve", lambda h: nusi._lib.NUSI_EINTERP)
    with pytest.raises(nusi.NusiError):
        ev.evolve()
    with pytest.warns(UserWarning, match="not evolved"):
        assert not ev.get_flux_fla().any()


def test_default_phiphi_needs_tables(nusi, tmp_path, monkeypatch):
    """pyprop's default phiphi=True loads xsec/*.bin; without them the reference exits
    (interp.hpp:251-254); here NUSI_ETABLE is raised."""
    monkeypatch.chdir(tmp_path)
    monkeypatch.delenv("NUSI_XSEC_DIR", raising=False)
    with pytest.raises(nusi.NusiError) as e:
        nusi.pyprop(6e5, 0.01, 0.1, 2.5, N_bins_E=50)
    assert e.value.code == nusi._lib.NUSI_ETABLE
    assert "does not exist" in str(e.value)


@pytest.mark.parametrize("kw,kernel", [
    (dict(cases.TEST_CPP, N_bins_E=300, phiphi=False), "k_cascade_bs"),                      # C1 at N_E = 300 (DSNB)
    (dict(cases.C2A, phiphi=False), "k_cascade_bs"),                                         # C2a (DSNB, resonance in range)
    (dict(cases.TEST_PY, phiphi=False), "k_cascade_bs"),                                     # resonant-only, DSNB
    (dict(cases.TEST_CPP, N_bins_E=1200, lEmin=10.0, lEmax=17.0, phiphi=False, source_model=1),
     "k_cascade_bs"),                                                                        # the C3 grid (134 steps)
], ids=["C1_N300", "C2a_N300", "test_py", "C3_grid"])
def test_drop_in_object_gets_the_fast_cascade(nusi, oracle_mod, kw, kernel):
    """The drop-in object (calculate_flux / pyprop: one point, default kernels) runs the MFMA cascade for the
    reference's own DSNB source and resonant-only mode and, beyond 48 redshift steps, the block-synchronous kernel in
    step passes --
    fluxes against the oracle's evolve() to FLUX_RTOL with the same exact zeros."""
    ev = nusi.pyprop(**_kw(kw))
    ev.evolve()
    assert ev.kernels()[1] == kernel
    f_ref, fla_ref = _ref_evolve(oracle_mod, kw)
    assert cases.rel_err(ev.get_flux(), f_ref) <= cases.FLUX_RTOL
    assert cases.rel_err(ev.get_flux_fla(), fla_ref) <= cases.FLUX_RTOL
    assert np.any(fla_ref > 0)

"""The CPU oracle pinned against the reference's own golden data and grid rules.

* output/data_massless.txt (written by the reference's test.py:1-25 through
  pyprop) is the only result file the reference ships; the oracle must
  reproduce all 100 rows at the printed precision (%.5e / %.4e).
* Grid bookkeeping of nuSIprop.hpp:100-127 (N_z, the extended table axis T
  and the z grid) for the BASELINE configs.
"""
import os

import numpy as np
import pytest

from tests import cases

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "data_massless.txt")


def test_data_massless(oracle_mod):
    ref = np.loadtxt(GOLDEN, skiprows=1)
    o = oracle_mod.Oracle(**cases.oracle_kwargs(cases.TEST_PY))
    _, fla = o.evolve()
    _, _, E, _ = o.grid()
    got = ["%.5e  %.4e  %.4e  %.4e" % r for r in zip(E, fla[0], fla[1], fla[2])]
    want = ["%.5e  %.4e  %.4e  %.4e" % tuple(r) for r in ref]
    assert got == want


def test_data_massless_header_matches_test_py():
    with open(GOLDEN) as fh:
        head = fh.readline()
    assert head.startswith("#") and "energy" in head
    assert np.loadtxt(GOLDEN, skiprows=1).shape == (100, 4)


@pytest.mark.parametrize("N,lEmin,lEmax,Nz,T", [
    (100, 9.0, 14.0, 17, 115),     # C1 (test.cpp): r = 10^(5/100)
    (100, 4.0, 9.0, 17, 115),      # test.py
    (300, 12.0, 17.0, 48, 346),    # C2b / C4 / C5
    (1200, 10.0, 17.0, 135, 1333),  # C3 (lE 10 -> 17)
    (1200, 12.0, 17.0, 188, 1386),
])
def test_grid_dims(oracle_mod, N, lEmin, lEmax, Nz, T):
    o = oracle_mod.Oracle(**cases.oracle_kwargs(dict(cases.C2B_100, N_bins_E=N, lEmin=lEmin, lEmax=lEmax)))
    assert (o.N, o.Nz, o.T) == (N, Nz, T)
    Emin, Emax, Enu, z = o.grid()
    assert np.all(Emax[:-1] == Emin[1:])        # contiguous bins (same pow() argument)
    assert z[0] == 0.0 and np.all(np.diff(z) > 0)
    r = Emax[0] / Emin[0]
    np.testing.assert_allclose(1 + z, r ** np.arange(Nz), rtol=1e-12)
    np.testing.assert_allclose(Enu, np.sqrt(Emin * Emax), rtol=1e-14)


def test_energy_conservation_diagnostic(oracle_mod):
    """check_energy_conservation (nuSIprop.hpp:339-357) returns (E_int - E_FS)/E_FS.
    E_FS is taken with the norm_total of the PREVIOUS evolve() (:205, :347), so a
    first call divides by zero; after an evolve(), pure free streaming (g -> 0)
    conserves energy up to the binning error, and interactions remove energy."""
    o = oracle_mod.Oracle(**cases.oracle_kwargs(dict(cases.C2B_100, g=1e-8)))
    assert not np.isfinite(o.check_energy_conservation())
    r = o.check_energy_conservation()
    assert np.isfinite(r) and abs(r) < 0.05
    o2 = oracle_mod.Oracle(**cases.oracle_kwargs(cases.C2B_100))
    o2.evolve()
    assert o2.check_energy_conservation() < r

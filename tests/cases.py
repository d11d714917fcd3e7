"""Parameter points shared by the parity tests (BASELINE.json configs).

Keys are calculate_flux's constructor arguments plus ``source_model``
(0 = the reference's DSNB source, 1 = its commented-out power law).
"""
import numpy as np

MSUM_MIN_NO = 0.0 + np.sqrt(7.42e-5) + np.sqrt(2.514e-3)   # test.py's massless-lightest sum

# test.py -> output/data_massless.txt (the reference's only golden data)
TEST_PY = dict(mphi=5e6, g=1e-6, mntot=MSUM_MIN_NO, si=2.0, norm=6, majorana=True, non_resonant=False,
               normal_ordering=True, N_bins_E=100, lEmin=4, lEmax=9, zmax=5, flav=2, phiphi=False, source_model=0)
# test.cpp (C1), at its own N=100
TEST_CPP = dict(mphi=6e5, g=0.01, mntot=0.1, si=2.5, norm=6, majorana=True, non_resonant=True, normal_ordering=True,
                N_bins_E=100, lEmin=9, lEmax=14, zmax=5, flav=2, phiphi=False, source_model=0)
# C2a: DSNB source with the resonance inside lE 4..9 (N reduced to 100 for the oracle's runtime)
C2A_100 = dict(TEST_CPP, mphi=3e3, g=0.03, lEmin=4, lEmax=9)
# C2b: power-law source at the constructor-default grid
C2B_100 = dict(TEST_CPP, lEmin=12, lEmax=17, source_model=1)

SMALL_CASES = {
    "test_cpp": TEST_CPP,
    "c2a": C2A_100,
    "c2b": C2B_100,
    "dirac": dict(TEST_CPP, majorana=False),
    "inverted": dict(TEST_CPP, mntot=0.2, normal_ordering=False),
    "resonant_only": dict(TEST_CPP, non_resonant=False),
    "flav_e": dict(C2B_100, flav=0),
    "strong": dict(C2B_100, mphi=1e7, g=0.5),
    "test_py": TEST_PY,
}

# full-size BASELINE configs (N_E = 300)
C2A = dict(C2A_100, N_bins_E=300)
C2B = dict(C2B_100, N_bins_E=300)


def oracle_kwargs(kw):
    k = dict(kw)
    k["source"] = k.pop("source_model", 0)
    return k


def scan_points(n_mphi=32, n_g=32, si=2.5, lEmin=12.0, lEmax=17.0, N=300, mphi_range=(5.5, 8.0), g_range=(-3.0, 0.0)):
    """C4: mphi in logspace(5.5, 8, 32) x g in logspace(-3, 0, 32), power-law source."""
    pts = []
    for m in np.logspace(*mphi_range, n_mphi):
        for g in np.logspace(*g_range, n_g):
            pts.append(dict(mphi=float(m), g=float(g), mntot=0.1, si=si, norm=1.0, majorana=True, non_resonant=True,
                            normal_ordering=True, N_bins_E=N, lEmin=lEmin, lEmax=lEmax, zmax=5.0, flav=2,
                            phiphi=False, source_model=1))
    return pts


# GPU fluxes vs the oracle (north-star bound 1e-9).  The cascade sums in a different order
# (right-looking pushes, multiplied reciprocals, power-law source powers shared along table
# edges): <= 2e-12 observed up to N_E = 1200.
FLUX_RTOL = 1e-11


def rel_err(a, b, floor=1e-280):
    """max |a-b|/|b| over entries with |b| > floor*max|b|; exact agreement required where b == 0."""
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    zero = b == 0
    if np.any(a[zero] != 0):
        return np.inf
    scale = np.max(np.abs(b)) if b.size else 0.0
    m = np.abs(b) > floor * scale
    if not np.any(m):
        return 0.0
    return float(np.max(np.abs(a[m] - b[m]) / np.abs(b[m])))

"""The gamma batch k_cascade_bs_gamma (NUSI_OPT_CASCADE_RHS 3..16; SURVEY sec. 7 K_B', the north star's
transfer-matrix x flux-batch GEMM at full batch width) against the oracle and against the one-point cascade.

The points of one table slot (same m_phi, g, masses, flags: the gamma of a C5 block) share one triangular operator;
k_cascade_bs_gamma runs up to 16 of them per workgroup with gamma on the N dimension of the fp64 MFMA and the
redshift steps in passes of 6.  Its operations per point are the one-point kernel's, summed in blocks by the matrix
core, so the fluxes agree with the oracle to FLUX_RTOL with the same exact zeros.
"""
import numpy as np
import pytest

from tests import cases

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def nusi():
    import nusiprop_amd
    nusiprop_amd.load()
    return nusiprop_amd


def _run(nusi, pts, rhs):
    from nusiprop_amd import _lib
    p0 = pts[0]
    plan = nusi.Plan(p0["N_bins_E"], p0["lEmin"], p0["lEmax"], p0["zmax"], max_points=len(pts), reference_order=False)
    plan.set_option(_lib.OPT_CASCADE_RHS, rhs)
    flux, fla = plan.evolve(pts)
    return plan, flux, fla


def _block(base, gammas, **kw):
    return [dict(base, si=float(s), **kw) for s in gammas]


@pytest.mark.parametrize("N", [100, 300])
def test_cascade_gamma_batch(nusi, oracle_mod, N):
    base = dict(cases.C2B_100, N_bins_E=N)
    g16 = np.linspace(2.0, 3.0, 16)
    pts = (_block(base, g16, mphi=6e5, g=0.01)                         # a full C5-style block
           + _block(base, g16[:5], mphi=2e6, g=0.3)                    # a short one
           + _block(base, np.linspace(2.0, 3.0, 17), mphi=1e7, g=0.5)  # 17 -> two batches (9 + 8)
           + _block(base, g16[:4], mphi=6e5, g=0.05, non_resonant=False)   # resonant-only table
           + [dict(base, mphi=3e6, g=0.1, si=2.2),                     # a lone point and a DSNB point: pair kernel
              dict(base, mphi=6e5, g=0.01, si=2.5, source_model=0)])
    plan, flux, fla = _run(nusi, pts, 16)
    assert plan.kernels()[1] == "k_cascade_bs_gamma + k_cascade_bs"
    _, f1, fl1 = _run(nusi, pts, 1)   # one point per workgroup
    worst = 0.0
    for i, p in enumerate(pts):
        o = oracle_mod.Oracle(**cases.oracle_kwargs(p))
        f_ref, fla_ref = o.evolve()
        e = max(cases.rel_err(flux[i], f_ref), cases.rel_err(fla[i], fla_ref))
        assert e <= cases.FLUX_RTOL, (i, p["mphi"], p["g"], p["si"], e)
        worst = max(worst, e)
        assert cases.rel_err(fla[i], fl1[i]) <= cases.FLUX_RTOL
    print("gamma batch N=%d: worst flux rel err vs oracle %.2e" % (N, worst))


def test_gamma_batch_c5_block_equals_pairs(nusi):
    """A 64-table slice of the C5 scan (16 gamma per table): the gamma batch and the pair kernel agree to rounding,
    point by point."""
    from nusiprop_amd import scan
    pts = scan.c5_points()[:1024]
    _, f16, fl16 = _run(nusi, pts, 16)
    _, f2, fl2 = _run(nusi, pts, 2)
    assert cases.rel_err(fl16, fl2) <= cases.FLUX_RTOL
    assert cases.rel_err(f16, f2) <= cases.FLUX_RTOL

"""The plan API's refusals on a GPU (include/nusi.h error codes), and that a refused call leaves the plan usable.

The reference ends the program where this library returns a code: no neutrino mass spectrum for the requested sum
(aux.hpp:48-49, "No neutrino mass spectrum was found ... Exiting..."), and it has no notion of a plan; the other
refusals (grids, point counts, flavour indices) guard the C ABI's own arguments.  Every refusal happens on the host
before any kernel runs, so the next valid call on the same plan gives the bits of a fresh plan."""
import numpy as np
import pytest

from tests import cases

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def nusi():
    import nusiprop_amd
    nusiprop_amd.load()
    return nusiprop_amd


def _refused(fn, code):
    from nusiprop_amd import _lib
    with pytest.raises(_lib.NusiError) as e:
        fn()
    assert e.value.code == code, (e.value.code, str(e.value))
    return str(e.value)


def test_bad_grids_refused(nusi):
    from nusiprop_amd import _lib
    for args, mp in (((1, 12.0, 17.0, 5.0), 1), ((100, 17.0, 12.0, 5.0), 1), ((100, 12.0, 17.0, 0.0), 1),
                     ((100, 12.0, 17.0, 5.0), 0)):
        _refused(lambda: nusi.Plan(*args, max_points=mp), _lib.NUSI_EPARAM)


def test_refused_calls_leave_the_plan_usable(nusi):
    from nusiprop_amd import _lib
    kw = dict(cases.TEST_CPP, N_bins_E=60)
    grid = (kw["N_bins_E"], kw["lEmin"], kw["lEmax"], kw["zmax"])
    plan = nusi.Plan(*grid, max_points=2)
    f0, fl0 = plan.evolve([kw])
    _refused(lambda: plan.evolve([kw] * 3), _lib.NUSI_EPARAM)                        # more points than max_points
    _refused(lambda: plan.evolve([]), _lib.NUSI_EPARAM)                              # no point
    _refused(lambda: plan.evolve([dict(kw, lEmax=kw["lEmax"] + 1)]), _lib.NUSI_EPARAM)   # another grid
    _refused(lambda: plan.evolve([kw, dict(kw, flav=3)]), _lib.NUSI_EPARAM)          # flavour index
    _refused(lambda: plan.evolve([dict(kw, source_model=7)]), _lib.NUSI_EPARAM)      # source model
    msg = _refused(lambda: plan.evolve([kw, dict(kw, mntot=0.01)]), _lib.NUSI_ENOSPECTRUM)   # below the NO minimum
    assert "No neutrino mass spectrum was found" in msg
    _refused(lambda: plan.evolve([dict(kw, mntot=0.05, normal_ordering=False)]), _lib.NUSI_ENOSPECTRUM)
    f1, fl1 = plan.evolve([kw])
    assert np.array_equal(f1, f0) and np.array_equal(fl1, fl0)
    plan.close()
    fresh = nusi.Plan(*grid, max_points=1)
    f2, fl2 = fresh.evolve([kw])
    fresh.close()
    assert np.array_equal(f2, f0) and np.array_equal(fl2, fl0)


def test_bad_options_refused(nusi):
    from nusiprop_amd import _lib
    plan = nusi.Plan(60, 12.0, 17.0, 5.0, max_points=1)
    for opt, val in ((_lib.OPT_REFERENCE_ORDER, 2), (_lib.OPT_ALPHA_KERNEL, 3), (_lib.OPT_CASCADE_RHS, 17),
                     (_lib.OPT_SHIFT_REUSE, 129), (_lib.OPT_REFO_CORNER_MB, -1), (999, 0)):
        _refused(lambda: plan.set_option(opt, val), _lib.NUSI_EPARAM)
    plan.close()

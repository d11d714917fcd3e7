"""Drop-in mirror of the reference's Cython ``pyprop`` class (nuSIprop.pyx:12-144).

Same constructor keywords and defaults (note ``phiphi=True`` by default, as in
nuSIprop.pyx:52 -- it needs the phi-phi tables), same methods, same
not-evolved behaviour (zeros + ``warnings.warn``).  Each method forwards to the
C ABI (include/nusi.h), which runs evolve() on the GPU.  Errors the reference
turns into ``exit(1)`` raise ``nusiprop_amd.NusiError`` here.
"""
import ctypes
import warnings

import numpy as np

from . import _lib


class pyprop:  # noqa: N801  (name of the reference class)
    """Class that evolves an astrophysical neutrino flux assuming self-interactions.

    Mandatory parameters: mphi [eV], g, mntot [eV], si.
    Optional: norm=1, majorana=True, non_resonant=True, normal_ordering=True,
    N_bins_E=300, lEmin=12.0, lEmax=17.0, zmax=5.0, flav=2, phiphi=True,
    source_model=SOURCE_DSNB (extension: SOURCE_POWER_LAW selects the
    reference's commented-out power-law source, nuSIprop.hpp:656),
    reference_order=True (extension: NUSI_OPT_REFERENCE_ORDER, the tables in
    the reference's own dilogarithm arithmetic -- GSL's algorithms, the
    library default; False selects the opt-in shared-algorithm order, faster
    and up to ~1e-6 from the reference's fluxes where its closed forms cancel,
    include/nusi.h).
    """

    def __init__(self, mphi, g, mntot, si, norm=1, majorana=True, non_resonant=True, normal_ordering=True,
                 N_bins_E=300, lEmin=12.0, lEmax=17.0, zmax=5.0, flav=2, phiphi=True,
                 source_model=_lib.SOURCE_DSNB, reference_order=True):
        L = _lib.load()
        p = _lib.make_params(mphi, g, mntot, si, norm, majorana, non_resonant, normal_ordering, N_bins_E,
                             lEmin, lEmax, zmax, flav, phiphi, source_model)
        self._h = ctypes.c_void_p()
        _lib.check(L.nusi_create(ctypes.byref(p), ctypes.byref(self._h)))
        if not reference_order:
            _lib.check(L.nusi_set_option(self._h, _lib.OPT_REFERENCE_ORDER, 0))
        self.evolved = False

    def __del__(self):
        if getattr(self, "_h", None) and self._h.value:
            _lib.load().nusi_destroy(self._h)
            self._h = ctypes.c_void_p()

    def _get_params(self):
        v = (ctypes.c_double * 5)()
        _lib.load().nusi_get_params(self._h, v)
        return list(v)

    def set_parameters(self, mphi=None, g=None, mntot=None, si=None, norm=None):
        """Modify the physics parameters (nuSIprop.pyx:60-85); resets the evolved flag."""
        cur = self._get_params()
        for k, v in enumerate((mphi, g, mntot, si, norm)):
            if v is not None:
                cur[k] = float(v)
        _lib.check(_lib.load().nusi_set_params(self._h, *cur))
        self.evolved = False

    def evolve(self):
        """Evolve the neutrino flux (nuSIprop.pyx:87-90)."""
        self.evolved = False          # stays False if the call raises (no stale flux behind an "evolved" flag)
        _lib.check(_lib.load().nusi_evolve(self._h))
        self.evolved = True
        w = _lib.load().nusi_get_warnings(self._h)
        if w:
            kinds = [n for b, n in ((1, "Gamma"), (2, "alphaTilde"), (4, "alpha")) if w & b]
            warnings.warn("Negative cross section when computing %s; possible roundoff errors" % ", ".join(kinds))

    def _n(self):
        return _lib.load().nusi_get_N_bins_E(self._h)

    def _get3(self, fn):
        N = self._n()
        flx = np.zeros([3, N])
        if not self.evolved:
            warnings.warn("You have not evolved the neutrino flux! Zero flux will be returned.")
            return flx
        _lib.check(fn(self._h, flx.ctypes.data_as(ctypes.POINTER(ctypes.c_double))))
        return flx

    def get_flux(self):
        """Flux of each mass eigenstate (nuSIprop.pyx:92-104)."""
        return self._get3(_lib.load().nusi_get_flux)

    def get_flux_fla(self):
        """Flux of each flavour e, mu, tau (nuSIprop.pyx:106-118)."""
        return self._get3(_lib.load().nusi_get_flux_fla)

    def _interp(self, f, energy):
        import scipy.interpolate as interp
        si = self._get_params()[3]
        E = self.get_energies()
        return interp.interp1d(np.log10(E), self.get_flux_fla()[f] * E ** si)(np.log10(energy)) / energy ** si

    def interp_flux_el(self, energy):
        """nu_e flux at any energy by interpolation (nuSIprop.pyx:120-122)."""
        return self._interp(0, energy)

    def interp_flux_mu(self, energy):
        return self._interp(1, energy)

    def interp_flux_ta(self, energy):
        return self._interp(2, energy)

    def get_energies(self):
        """Energy bin centres (nuSIprop.pyx:130-138)."""
        E = np.zeros(self._n())
        _lib.load().nusi_get_energies(self._h, E.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
        return E

    def kernels(self):
        """Extension (no reference counterpart): names of the alpha-table and cascade kernels the last
        evolve() launched, e.g. ('k_alpha_batch', 'k_cascade_bs')."""
        a, c = ctypes.c_char_p(), ctypes.c_char_p()
        _lib.check(_lib.load().nusi_get_kernels(self._h, ctypes.byref(a), ctypes.byref(c)))
        return a.value.decode(), c.value.decode()

    def check_energy_conservation(self):
        """(E_int - E_FS)/E_FS (nuSIprop.pyx:140-144).  Evolves the C++ object, but -- as in the
        reference -- does not set the Python-side evolved flag."""
        out = ctypes.c_double()
        r = _lib.load().nusi_check_energy_conservation(self._h, ctypes.byref(out))
        if r == _lib.NUSI_ESTATE:   # before any evolve: the reference reads norm_total uninitialised
            warnings.warn(_lib.last_error())
            return out.value        # NaN
        _lib.check(r)
        return out.value

"""Batched parameter scans on one GPU: a thin wrapper of the nusi_plan C API.

A Plan fixes the energy/redshift grid (N_bins_E, lEmin, lEmax, zmax) of the
reference's constructor (nuSIprop.hpp:113-128) and holds the Stage-A tables of
up to ``max_points`` parameter points in HBM.  ``evolve`` runs, on the GPU,
exactly what calculate_flux::evolve() does for each point (nuSIprop.hpp:176-337).
"""
import ctypes

import numpy as np

from . import _lib


def params_array(points, grid_args=None):
    """ctypes array of struct nusi_params; dict points may omit the grid keys
    when grid_args = (N_bins_E, lEmin, lEmax, zmax) is given."""
    arr = (_lib.NusiParams * len(points))()
    for k, p in enumerate(points):
        if isinstance(p, _lib.NusiParams):
            arr[k] = p
        else:
            q = dict(p)
            if grid_args is not None:
                for key, v in zip(("N_bins_E", "lEmin", "lEmax", "zmax"), grid_args):
                    q.setdefault(key, v)
            arr[k] = _lib.make_params(**q)
    return arr


class Plan:
    def __init__(self, N_bins_E=300, lEmin=12.0, lEmax=17.0, zmax=5.0, max_points=1, device=0, reference_order=None):
        """reference_order: None = the library default (the reference's own arithmetic, NUSI_OPT_REFERENCE_ORDER = 1);
        False = the shared-algorithm order (opt-in fast mode, include/nusi.h); True = the reference order explicitly."""
        L = _lib.load()
        self._h = ctypes.c_void_p()
        _lib.check(L.nusi_plan_create(int(device), int(N_bins_E), float(lEmin), float(lEmax), float(zmax),
                                      int(max_points), ctypes.byref(self._h)))
        if reference_order is not None:
            self.set_option(_lib.OPT_REFERENCE_ORDER, 1 if reference_order else 0)
        self.device = device
        self.max_points = max_points
        self.grid_args = (int(N_bins_E), float(lEmin), float(lEmax), float(zmax))
        N, Nz = ctypes.c_int(), ctypes.c_int()
        self.energies = np.zeros(N_bins_E)
        L.nusi_plan_grid(self._h, ctypes.byref(N), ctypes.byref(Nz),
                         self.energies.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
        self.N, self.Nz = N.value, Nz.value
        self.T = self.N + self.Nz - 2
        self.PT = self.T * (self.T - 1) // 2

    def close(self):
        if getattr(self, "_h", None) and self._h.value:
            _lib.load().nusi_plan_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def load_phiphi(self, alphatilde_path, alpha_path, alphatilde_dims=None, alpha_dims=None):
        d2 = (ctypes.c_int * 2)(*alphatilde_dims) if alphatilde_dims else None
        d3 = (ctypes.c_int * 3)(*alpha_dims) if alpha_dims else None
        _lib.check(_lib.load().nusi_plan_load_phiphi(self._h, alphatilde_path.encode(), d2, alpha_path.encode(), d3))

    def params_array(self, points):
        """points: sequence of dicts (calculate_flux keyword arguments) or NusiParams."""
        return params_array(points, self.grid_args)

    def evolve(self, points):
        """Evolve on the GPU; returns host arrays flux, flux_fla of shape (n, 3, N)."""
        arr = points if isinstance(points, ctypes.Array) else self.params_array(points)
        n = len(arr)
        flux = np.zeros((n, 3, self.N))
        fla = np.zeros((n, 3, self.N))
        dp = ctypes.POINTER(ctypes.c_double)
        _lib.check(_lib.load().nusi_plan_evolve_host(self._h, arr, n, flux.ctypes.data_as(dp), fla.ctypes.data_as(dp)))
        return flux, fla

    def evolve_device(self, arr, d_flux_ptr, d_fla_ptr, stream_ptr=None):
        """Asynchronous evolve into device buffers (raw pointers, e.g. torch .data_ptr())."""
        _lib.check(_lib.load().nusi_plan_evolve(self._h, arr, len(arr), ctypes.c_void_p(d_flux_ptr),
                                                ctypes.c_void_p(d_fla_ptr),
                                                ctypes.c_void_p(stream_ptr) if stream_ptr else None))

    def set_cascade(self, kind):
        """Cascade kernel of later calls: _lib.CASCADE_AUTO (default) = CASCADE_MFMA (the wavefront with its push
        on the fp64 matrix cores, the block-synchronous k_cascade_bs), or CASCADE_{WAVEFRONT,REG,LDS} (since
        round 5 all three the bit-exact scalar kernel k_cascade)."""
        _lib.check(_lib.load().nusi_plan_set_cascade(self._h, int(kind)))

    def set_option(self, option, value):
        """A/B and test options (nusi_plan_set_option): _lib.OPT_ALPHA_BATCH (max tables per alpha batch, 0 =
        auto), OPT_ALPHA_KERNEL (0 batch, 1 tile, 2 per entry), OPT_CASCADE_RHS (1 = one point per cascade
        workgroup), OPT_STEP_PASSES (1 = the step-pass cascade also where one pass fits), OPT_SHIFT_REUSE (K > 0:
        the opt-in scan mode sharing tables across m_phi on the r^(-o/2) lattice, o <= K; only tables with g <= 0.05
        share, the others are built directly), OPT_REFERENCE_ORDER (1, the default = the tables in the reference's own
        arithmetic: GSL's dilogarithm algorithms on the reference's arguments; 0 = the shared-algorithm order), OPT_REFO_CORNER_MB (the reference order's
        member-corner block budget in MiB, 0 = automatic); include/nusi.h."""
        _lib.check(_lib.load().nusi_plan_set_option(self._h, int(option), int(value)))

    def profile_begin(self, max_calls):
        _lib.check(_lib.load().nusi_plan_profile_begin(self._h, int(max_calls)))

    def profile_end(self):
        """Summed kernel ms [gamma/alphaTilde, alpha, cascade] and the number of calls recorded."""
        ms = (ctypes.c_double * 3)()
        n = ctypes.c_int()
        _lib.check(_lib.load().nusi_plan_profile_end(self._h, ms, ctypes.byref(n)))
        return list(ms), n.value

    def stage_ms(self):
        ms = (ctypes.c_float * 3)()
        _lib.check(_lib.load().nusi_plan_stage_ms(self._h, ms))
        return list(ms)

    def warnings(self, n):
        out = (ctypes.c_int * n)()
        _lib.check(_lib.load().nusi_plan_warnings(self._h, out, n))
        return list(out)

    def kernels(self):
        """(alpha-table kernel, cascade kernel) the last call launched, e.g. ('k_alpha_batch', 'k_cascade_bs')."""
        a, c = ctypes.c_char_p(), ctypes.c_char_p()
        _lib.check(_lib.load().nusi_plan_kernels(self._h, ctypes.byref(a), ctypes.byref(c)))
        return a.value.decode(), c.value.decode()

    def tables(self, i):
        """Point i's Stage-A tables of the last call: Gamma[T], alphaTilde[T], alpha packed [T(T-1)/2]."""
        G, At, A = np.zeros(self.T), np.zeros(self.T), np.zeros(self.PT)
        dp = ctypes.POINTER(ctypes.c_double)
        _lib.check(_lib.load().nusi_plan_tables(self._h, int(i), G.ctypes.data_as(dp), At.ctypes.data_as(dp),
                                                A.ctypes.data_as(dp)))
        return G, At, A


def unpack_alpha(A_packed, T):
    """packed transposed alpha (m(m-1)/2+n) -> dense T x T with alpha[n, m], n < m."""
    out = np.zeros((T, T))
    m_idx, n_idx = np.tril_indices(T, -1)       # row-major over m, n < m -> m(m-1)/2 + n order
    out[n_idx, m_idx] = A_packed
    return out

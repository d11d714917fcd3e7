"""ctypes front end of the CPU oracle -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module; nusiprop_amd/ never does.  The library is oracle/_build/
libnusi_oracle.so (``make -C oracle``), a plain-C restatement of the
reference's calculate_flux (see nusi_oracle.h for the file:line map).
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# NUSI_ORACLE_LIB: a contracted build of the same sources (oracle/Makefile target fc; the platform-arithmetic probe
# scripts/contraction_floor.py) -- never the parity oracle
LIB_PATH = os.environ.get("NUSI_ORACLE_LIB") or os.path.join(HERE, "_build", "libnusi_oracle.so")

SOURCE_DSNB = 0
SOURCE_POWER_LAW = 1


class OraParams(ctypes.Structure):
    _fields_ = [("mphi", ctypes.c_double), ("g", ctypes.c_double), ("mntot", ctypes.c_double),
                ("si", ctypes.c_double), ("norm", ctypes.c_double),
                ("majorana", ctypes.c_int), ("non_resonant", ctypes.c_int), ("normal_ordering", ctypes.c_int),
                ("N_bins_E", ctypes.c_int), ("lEmin", ctypes.c_double), ("lEmax", ctypes.c_double),
                ("zmax", ctypes.c_double), ("flav", ctypes.c_int), ("phiphi", ctypes.c_int),
                ("source", ctypes.c_int)]


_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        d, i, p = ctypes.c_double, ctypes.c_int, ctypes.c_void_p
        dp = ctypes.POINTER(ctypes.c_double)
        L.ora_create.restype = p
        L.ora_create.argtypes = [ctypes.POINTER(OraParams), ctypes.POINTER(i)]
        L.ora_destroy.argtypes = [p]
        for f in ("ora_N", "ora_Nz", "ora_T", "ora_warnings"):
            getattr(L, f).restype = i
            getattr(L, f).argtypes = [p]
        L.ora_zmax.restype = d
        L.ora_zmax.argtypes = [p]
        L.ora_grid.argtypes = [p, dp, dp, dp, dp]
        L.ora_mixing.argtypes = [p, dp]
        L.ora_prepare.restype = i
        L.ora_prepare.argtypes = [p]
        L.ora_masses.argtypes = [p, dp, dp]
        L.ora_set_params.restype = i
        L.ora_set_params.argtypes = [p, d, d, d, d, d]
        L.ora_tables.restype = i
        L.ora_tables.argtypes = [p, dp, dp, dp]
        for f in ("ora_Gamma", "ora_alphaTilde"):
            getattr(L, f).restype = d
            getattr(L, f).argtypes = [p, d, d]
        L.ora_alpha.restype = d
        L.ora_alpha.argtypes = [p, d, d, d, d]
        L.ora_cascade.restype = i
        L.ora_cascade.argtypes = [p, dp, dp, dp, dp, dp]
        L.ora_evolve.restype = i
        L.ora_evolve.argtypes = [p, dp, dp]
        L.ora_Lum.restype = d
        L.ora_Lum.argtypes = [p, d, d, d]
        L.ora_check_energy_conservation.restype = d
        L.ora_check_energy_conservation.argtypes = [p, dp, dp]
        L.ora_load_phiphi_dims.restype = i
        L.ora_load_phiphi_dims.argtypes = [p, ctypes.c_char_p, ctypes.POINTER(i), ctypes.c_char_p, ctypes.POINTER(i)]
        L.ora_dilog.restype = d
        L.ora_dilog.argtypes = [d]
        L.ora_li2.restype = d
        L.ora_li2.argtypes = [d]
        L.ora_li3.restype = d
        L.ora_li3.argtypes = [d]
        L.ora_complex_dilog_xy.argtypes = [d, d, dp, dp]
        L.ora_getmL.restype = i
        L.ora_getmL.argtypes = [d, d, d, dp]
        L.ora_set_channels.argtypes = [p, i]
        L.ora_set_reference_order.argtypes = [i]
        L.ora_gsl_dilog.restype = d
        L.ora_gsl_dilog.argtypes = [d]
        L.ora_gsl_complex_dilog_xy.argtypes = [d, d, dp, dp]
        L.ora_gsl_clausen.restype = d
        L.ora_gsl_clausen.argtypes = [d]
        L.ora_hypot.restype = d
        L.ora_hypot.argtypes = [d, d]
        L.ora_gsl_stats.argtypes = [ctypes.POINTER(ctypes.c_long), i]
        L.ora_Gpp_bracket.restype = d
        L.ora_Gpp_bracket.argtypes = [d, d]
        _lib = L
    return _lib


def _dp(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


def dilog(x):
    return lib().ora_dilog(float(x))


def li3(x):
    return lib().ora_li3(float(x))


def complex_dilog(x, y):
    re, im = ctypes.c_double(), ctypes.c_double()
    lib().ora_complex_dilog_xy(float(x), float(y), ctypes.byref(re), ctypes.byref(im))
    return complex(re.value, im.value)


# channel bits of Oracle.set_channels (nusi_oracle.h ORA_CH_*)
CH_S, CH_T, CH_U, CH_TU, CH_ST, CH_SU, CH_PP, CH_ALL = 1, 2, 4, 8, 16, 32, 64, 127


def gsl_dilog(x):
    """gsl_sf_dilog by GSL's algorithm (ora_gsl.c)."""
    return lib().ora_gsl_dilog(float(x))


def gsl_complex_dilog(x, y):
    """gsl_sf_complex_dilog_xy_e by GSL's algorithm (ora_gsl.c): (re, im)."""
    re, im = ctypes.c_double(), ctypes.c_double()
    lib().ora_gsl_complex_dilog_xy(float(x), float(y), ctypes.byref(re), ctypes.byref(im))
    return re.value, im.value


def gsl_clausen(x):
    return lib().ora_gsl_clausen(float(x))


def hypot(x, y):
    return lib().ora_hypot(float(x), float(y))


def gsl_stats(reset=True):
    """Iteration counts of ora_gsl.c's series on this thread since the last reset: [dilog_series_1, series_2,
    dilogc_series_1, series_2_c, dilogc_series_3 calls, ...] (analysis only)."""
    out = (ctypes.c_long * 8)()
    lib().ora_gsl_stats(out, int(reset))
    return list(out)


def Gpp_bracket(a, b):
    """The bracket of the analytic phi-phi absorption (nuSIprop.hpp:885), a = max(s-, 4)."""
    return lib().ora_Gpp_bracket(float(a), float(b))


class reference_order:
    """Context: the oracle in reference-order arithmetic (nusi_oracle.h ora_set_reference_order) -- level 1: every
    gsl_sf_dilog / gsl_sf_complex_dilog_xy_e call site by GSL's own algorithms (ora_gsl.c), and the alpha table's
    s-t member dilogs of the reference's own quotient with carg of its expression (nuSIprop.hpp:1431-1456);
    level 2 evaluates those dilogarithms in long double (a precision probe).  Process-wide: tests only."""

    def __init__(self, level=1):
        self.level = int(level)

    def __enter__(self):
        lib().ora_set_reference_order(self.level)
        return self

    def __exit__(self, *exc):
        lib().ora_set_reference_order(0)
        return False


def getmL(msum, dm21, dmAT):
    out = ctypes.c_double()
    r = lib().ora_getmL(float(msum), float(dm21), float(dmAT), ctypes.byref(out))
    return out.value if r == 0 else None


class Oracle:
    """One reference calculate_flux object (C++ constructor argument order)."""

    def __init__(self, mphi, g, mntot, si, norm=1.0, majorana=True, non_resonant=True,
                 normal_ordering=True, N_bins_E=300, lEmin=12.0, lEmax=17.0, zmax=5.0,
                 flav=2, phiphi=False, source=SOURCE_DSNB):
        self.p = OraParams(mphi, g, mntot, si, norm, int(majorana), int(non_resonant), int(normal_ordering),
                           int(N_bins_E), lEmin, lEmax, zmax, int(flav), int(phiphi), int(source))
        err = ctypes.c_int(0)
        self.h = lib().ora_create(ctypes.byref(self.p), ctypes.byref(err))
        if not self.h:
            raise ValueError("oracle: bad parameters (%d)" % err.value)
        L = lib()
        self.N, self.Nz, self.T = L.ora_N(self.h), L.ora_Nz(self.h), L.ora_T(self.h)

    def __del__(self):
        if getattr(self, "h", None):
            lib().ora_destroy(self.h)
            self.h = None

    def load_phiphi(self, at_path, at_dims, a_path, a_dims):
        n2 = (ctypes.c_int * 2)(*at_dims)
        n3 = (ctypes.c_int * 3)(*a_dims)
        r = lib().ora_load_phiphi_dims(self.h, at_path.encode(), n2, a_path.encode(), n3)
        if r:
            raise RuntimeError("oracle: phiphi tables failed to load (%d)" % r)

    def set_parameters(self, mphi, g, mntot, si, norm):
        lib().ora_set_params(self.h, mphi, g, mntot, si, norm)

    def grid(self):
        N, Nz = self.N, self.Nz
        Emin, Emax, Enu, z = np.zeros(N), np.zeros(N), np.zeros(N), np.zeros(Nz)
        lib().ora_grid(self.h, _dp(Emin), _dp(Emax), _dp(Enu), _dp(z))
        return Emin, Emax, Enu, z

    def mixing(self):
        U2 = np.zeros(9)
        lib().ora_mixing(self.h, _dp(U2))
        return U2.reshape(3, 3)

    def prepare(self):
        r = lib().ora_prepare(self.h)
        if r:
            raise RuntimeError("oracle: no neutrino mass spectrum (%d)" % r)
        mn, nt = np.zeros(3), ctypes.c_double()
        lib().ora_masses(self.h, _dp(mn), ctypes.byref(nt))
        return mn, nt.value

    def tables(self):
        """Stage A tables; alpha returned as a dense T x T (upper triangle filled)."""
        self.prepare()
        T = self.T
        G, aT, al = np.zeros(T), np.zeros(T), np.zeros((T, T))
        r = lib().ora_tables(self.h, _dp(G), _dp(aT), _dp(al))
        if r:
            raise RuntimeError("oracle: table build failed (%d)" % r)
        return G, aT, al

    def cascade(self, G, aT, al):
        N = self.N
        G, aT, al = (np.ascontiguousarray(x, dtype=np.float64) for x in (G, aT, al))
        flux, fla = np.zeros(3 * N), np.zeros(3 * N)
        lib().ora_cascade(self.h, _dp(G), _dp(aT), _dp(al), _dp(flux), _dp(fla))
        return flux.reshape(3, N), fla.reshape(3, N)

    def evolve(self):
        N = self.N
        flux, fla = np.zeros(3 * N), np.zeros(3 * N)
        r = lib().ora_evolve(self.h, _dp(flux), _dp(fla))
        if r:
            raise RuntimeError("oracle: evolve failed (%d)" % r)
        return flux.reshape(3, N), fla.reshape(3, N)

    def check_energy_conservation(self):
        N = self.N
        flux, fla = np.zeros(3 * N), np.zeros(3 * N)
        return lib().ora_check_energy_conservation(self.h, _dp(flux), _dp(fla))

    def warnings(self):
        return lib().ora_warnings(self.h)

    def set_channels(self, mask):
        """Gamma / alphaTilde / alpha sum only the CH_* channels in `mask` (KAT test hook)."""
        lib().ora_set_channels(self.h, int(mask))

    def Gamma(self, Em, Ep):
        return lib().ora_Gamma(self.h, Em, Ep)

    def alphaTilde(self, Em, Ep):
        return lib().ora_alphaTilde(self.h, Em, Ep)

    def alpha(self, Em, Ep, Emp, Epp):
        return lib().ora_alpha(self.h, Em, Ep, Emp, Epp)


def evolve_many(points, threads=None, level=0, phiphi_tables=None):
    """The oracle's evolve() of every point (dicts of constructor arguments, ``source_model`` or ``source``) on a
    thread pool (ctypes releases the GIL; each thread its own Oracle object), at reference-order `level` (0 = the
    shared-algorithm order, 1 = the reference's own order; process-wide for the call's duration).  phiphi_tables:
    (at_path, at_dims, a_path, a_dims) loaded by every object (load_phiphi).  Returns (flux, flux_fla) as [n, 3, N]
    arrays.  Test / bench-checker infrastructure only."""
    import concurrent.futures as cf
    pts = []
    for p in points:
        kw = dict(p)
        if "source_model" in kw:
            kw["source"] = kw.pop("source_model")
        pts.append(kw)
    if threads is None:
        threads = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
        cap = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
        if cap > 0:
            threads = min(threads, cap)
    threads = max(1, min(int(threads), len(pts)))

    def one(kw):
        o = Oracle(**kw)
        if phiphi_tables is not None:
            o.load_phiphi(*phiphi_tables)
        return o.evolve()
    with reference_order(level):
        with cf.ThreadPoolExecutor(threads) as ex:
            res = list(ex.map(one, pts))
    return np.stack([r[0] for r in res]), np.stack([r[1] for r in res])

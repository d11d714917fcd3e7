"""ctypes binding of libnusi.so (include/nusi.h).

The library is built in-tree (``make -C nusiprop_amd/csrc``) and loaded from
this directory; there is no pure-Python or CPU fallback: if the .so is missing
or the GPU is unusable, calls raise.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("NUSIPROP_LIB") or os.path.join(HERE, "libnusi.so")   # override: A/B builds only

NUSI_OK = 0
NUSI_EPARAM = -1
NUSI_ENOSPECTRUM = -2
NUSI_ETABLE = -3
NUSI_EINTERP = -4
NUSI_EHIP = -5
NUSI_ESTATE = -6

SOURCE_DSNB = 0
SOURCE_POWER_LAW = 1

WARN_GAMMA = 1
WARN_ALPHATILDE = 2
WARN_ALPHA = 4


class NusiParams(ctypes.Structure):
    """struct nusi_params -- the calculate_flux constructor arguments (nuSIprop.hpp:61-65)."""
    _fields_ = [("mphi", ctypes.c_double), ("g", ctypes.c_double), ("mntot", ctypes.c_double),
                ("si", ctypes.c_double), ("norm", ctypes.c_double),
                ("majorana", ctypes.c_int), ("non_resonant", ctypes.c_int), ("normal_ordering", ctypes.c_int),
                ("N_bins_E", ctypes.c_int), ("lEmin", ctypes.c_double), ("lEmax", ctypes.c_double),
                ("zmax", ctypes.c_double), ("flav", ctypes.c_int), ("phiphi", ctypes.c_int),
                ("source_model", ctypes.c_int)]


class NusiError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(msg)
        self.code = code


# every symbol declared in include/nusi.h (tests/test_capi_symbols.py checks this list against the header)
EXPORTS = [
    "nusi_params_default", "nusi_last_error", "nusi_device_count",
    "nusi_create", "nusi_copy", "nusi_destroy", "nusi_set_params", "nusi_get_params", "nusi_evolve",
    "nusi_check_energy_conservation", "nusi_get_flux", "nusi_get_flux_fla", "nusi_get_energies",
    "nusi_get_N_bins_E", "nusi_get_N_steps_z", "nusi_get_warnings", "nusi_get_kernels", "nusi_set_option",
    "nusi_plan_create", "nusi_plan_destroy", "nusi_plan_load_phiphi", "nusi_plan_grid", "nusi_plan_evolve",
    "nusi_plan_evolve_host", "nusi_plan_stage_ms", "nusi_plan_profile_begin", "nusi_plan_profile_end",
    "nusi_plan_warnings", "nusi_plan_tables", "nusi_evolve_batch", "nusi_plan_set_cascade",
    "nusi_plan_kernels", "nusi_plan_set_option",
]

# nusi_plan_set_cascade kinds and nusi_plan_set_option options (include/nusi.h)
CASCADE_AUTO, CASCADE_WAVEFRONT, CASCADE_REG, CASCADE_LDS, CASCADE_MFMA = 0, 1, 2, 3, 4
OPT_ALPHA_BATCH, OPT_ALPHA_KERNEL, OPT_CASCADE_RHS, OPT_STEP_PASSES, OPT_SHIFT_REUSE = 1, 2, 3, 4, 5
OPT_REFERENCE_ORDER = 6
OPT_CASCADE_SYNC = 7
OPT_REFO_CORNER_MB = 8

_lib = None


def load():
    """Load libnusi.so (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError("nusiprop_amd: %s not built (run `make -C nusiprop_amd/csrc`)" % LIB_PATH)
    L = ctypes.CDLL(LIB_PATH)
    d, i, vp = ctypes.c_double, ctypes.c_int, ctypes.c_void_p
    dp, ip = ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int)
    pp = ctypes.POINTER(NusiParams)
    sig = {
        "nusi_params_default": (None, [pp, d, d, d, d]),
        "nusi_last_error": (ctypes.c_char_p, []),
        "nusi_device_count": (i, []),
        "nusi_create": (i, [pp, ctypes.POINTER(vp)]),
        "nusi_copy": (i, [vp, ctypes.POINTER(vp)]),
        "nusi_destroy": (None, [vp]),
        "nusi_set_params": (i, [vp, d, d, d, d, d]),
        "nusi_get_params": (i, [vp, dp]),
        "nusi_evolve": (i, [vp]),
        "nusi_check_energy_conservation": (i, [vp, dp]),
        "nusi_get_flux": (i, [vp, dp]),
        "nusi_get_flux_fla": (i, [vp, dp]),
        "nusi_get_energies": (i, [vp, dp]),
        "nusi_get_N_bins_E": (i, [vp]),
        "nusi_get_N_steps_z": (i, [vp]),
        "nusi_get_warnings": (i, [vp]),
        "nusi_get_kernels": (i, [vp, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_char_p)]),
        "nusi_set_option": (i, [vp, i, i]),
        "nusi_plan_create": (i, [i, i, d, d, d, i, ctypes.POINTER(vp)]),
        "nusi_plan_destroy": (None, [vp]),
        "nusi_plan_load_phiphi": (i, [vp, ctypes.c_char_p, ip, ctypes.c_char_p, ip]),
        "nusi_plan_grid": (i, [vp, ip, ip, dp]),
        "nusi_plan_evolve": (i, [vp, pp, i, vp, vp, vp]),
        "nusi_plan_evolve_host": (i, [vp, pp, i, dp, dp]),
        "nusi_plan_stage_ms": (i, [vp, ctypes.POINTER(ctypes.c_float)]),
        "nusi_plan_profile_begin": (i, [vp, i]),
        "nusi_plan_profile_end": (i, [vp, dp, ip]),
        "nusi_plan_warnings": (i, [vp, ip, i]),
        "nusi_plan_tables": (i, [vp, i, dp, dp, dp]),
        "nusi_evolve_batch": (i, [i, pp, i, dp, dp]),
        "nusi_plan_set_cascade": (i, [vp, i]),
        "nusi_plan_set_option": (i, [vp, i, i]),
        "nusi_plan_kernels": (i, [vp, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_char_p)]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _lib = L
    return L


def last_error():
    return load().nusi_last_error().decode(errors="replace")


def check(code):
    if code != NUSI_OK:
        raise NusiError(code, load().nusi_last_error().decode(errors="replace"))
    return code


def make_params(mphi, g, mntot, si, norm=1.0, majorana=True, non_resonant=True, normal_ordering=True,
                N_bins_E=300, lEmin=12.0, lEmax=17.0, zmax=5.0, flav=2, phiphi=False,
                source_model=SOURCE_DSNB):
    return NusiParams(float(mphi), float(g), float(mntot), float(si), float(norm), int(bool(majorana)),
                      int(bool(non_resonant)), int(bool(normal_ordering)), int(N_bins_E), float(lEmin),
                      float(lEmax), float(zmax), int(flav), int(bool(phiphi)), int(source_model))

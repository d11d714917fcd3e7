"""The drop-in boundary, proven on the reference's own sources: the reference's
C++ example test.cpp (test.cpp:1-33) and its Cython wrapper nuSIprop.pyx + nuSIprop.pxd (nuSIprop.pyx:12-144,
nuSIprop.pxd:2-18) build UNCHANGED against include/nuSIprop.hpp (the facade over libnusi.so) and link.

The sources are read from /root/reference where they lie and built in a temporary directory (their quoted
#include "nuSIprop.hpp" would otherwise find the reference's own header next to them); nothing of them is
copied into the repository or travels to the GPU box, so the module skips where /root/reference is absent.
Neither program is run (no GPU here); the Cython module is imported, which checks its link against
libnusi.so and the class it exposes.
"""
import filecmp
import os
import shutil
import subprocess
import sys
import sysconfig

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
INC = os.path.join(ROOT, "include")
LIBDIR = os.path.join(ROOT, "nusiprop_amd")

pytestmark = pytest.mark.skipif(not os.path.isfile(os.path.join(REF, "test.cpp")),
                                reason="the reference sources are not on this host")


def _lib():
    if not os.path.exists(os.path.join(LIBDIR, "libnusi.so")):
        subprocess.check_call(["make", "-s", "-C", os.path.join(LIBDIR, "csrc")])


def _stage(tmp, names):
    """The reference files, byte for byte, in a scratch directory (outside the repository)."""
    for n in names:
        shutil.copyfile(os.path.join(REF, n), os.path.join(tmp, n))
        assert filecmp.cmp(os.path.join(REF, n), os.path.join(tmp, n), shallow=False)


def test_reference_test_cpp_builds_unchanged(tmp_path):
    _lib()
    tmp = str(tmp_path)
    _stage(tmp, ["test.cpp"])
    exe = os.path.join(tmp, "test_cpp")
    # the reference builds it with g++ against GSL and polylogarithm; here only the include path and the
    # link line change
    subprocess.check_call(["g++", "-std=c++14", "-O2", "-I" + INC, "-o", exe, os.path.join(tmp, "test.cpp"),
                           "-L" + LIBDIR, "-lnusi", "-Wl,-rpath," + LIBDIR])
    assert os.access(exe, os.X_OK)
    syms = subprocess.check_output(["nm", "-D", "--undefined-only", exe], text=True)
    assert "nusi_create" in syms and "nusi_evolve" in syms and "nusi_get_flux_fla" in syms


def test_reference_cython_wrapper_builds_unchanged(tmp_path):
    cython = pytest.importorskip("Cython")
    np = pytest.importorskip("numpy")
    _lib()
    tmp = str(tmp_path)
    _stage(tmp, ["nuSIprop.pyx", "nuSIprop.pxd"])
    cpp = os.path.join(tmp, "nuSIprop.cpp")
    subprocess.check_call([sys.executable, "-m", "cython", "--cplus", "-3", "-o", cpp, os.path.join(tmp, "nuSIprop.pyx")],
                          cwd=tmp)
    so = os.path.join(tmp, "nuSIprop" + sysconfig.get_config_var("EXT_SUFFIX"))
    subprocess.check_call(["g++", "-std=c++14", "-O1", "-shared", "-fPIC", "-w", "-I" + INC,
                           "-I" + sysconfig.get_paths()["include"], "-I" + np.get_include(), "-o", so, cpp,
                           "-L" + LIBDIR, "-lnusi", "-Wl,-rpath," + LIBDIR])
    probe = ("import inspect, nuSIprop; c = nuSIprop.pyprop; "
             "print(' '.join(m for m in ('set_parameters', 'evolve', 'get_flux', 'get_flux_fla', 'interp_flux_el', "
             "'interp_flux_mu', 'interp_flux_ta', 'get_energies', 'check_energy_conservation') if hasattr(c, m)))")
    out = subprocess.check_output([sys.executable, "-c", probe], cwd=tmp, text=True).split()
    assert out == ["set_parameters", "evolve", "get_flux", "get_flux_fla", "interp_flux_el", "interp_flux_mu",
                   "interp_flux_ta", "get_energies", "check_energy_conservation"]
    assert cython.__version__

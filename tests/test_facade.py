"""The C++ drop-in facade (include/nuSIprop.hpp): builds and links against
libnusi.so here; on the GPU a test.cpp-style program runs through it and is
checked against the oracle, including the mutable members and copy semantics.
With no option the facade runs the reference's own arithmetic
(NUSI_OPT_REFERENCE_ORDER = 1, GSL's dilogarithm algorithms): its fluxes are
checked against the oracle in that mode; set_reference_order(false) selects
the shared-algorithm order, checked against the oracle's default mode."""
import os
import subprocess

import numpy as np
import pytest

from tests import cases

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "_build", "facade_demo")


def build():
    lib = os.path.join(ROOT, "nusiprop_amd")
    if not os.path.exists(os.path.join(lib, "libnusi.so")):
        subprocess.check_call(["make", "-s", "-C", os.path.join(lib, "csrc")])
    os.makedirs(os.path.dirname(EXE), exist_ok=True)
    subprocess.check_call(["g++", "-std=c++14", "-O2", "-Wall", "-Wextra", "-I" + os.path.join(ROOT, "include"),
                           "-o", EXE, os.path.join(ROOT, "tests", "cpp", "facade_demo.cpp"),
                           "-L" + lib, "-lnusi", "-Wl,-rpath," + lib])
    return EXE


def test_facade_builds_and_links():
    assert os.access(build(), os.X_OK)


@pytest.mark.gpu
def test_facade_matches_oracle(oracle_mod):
    out = subprocess.run([build()], capture_output=True, text=True, timeout=300, check=True)
    rows = {}
    for line in out.stdout.splitlines():
        tag, *vals = line.split()
        rows.setdefault(tag, []).append([float(v) for v in vals])
    A, B, C, D, E2 = (np.array(rows[t]) for t in "ABCDE")
    assert rows["R"] == [[0.0]]
    assert "not in [0,1,2]" in out.stderr and "<0!" in out.stderr and "there are only 100 bins" in out.stderr
    with oracle_mod.reference_order(1):
        o = oracle_mod.Oracle(**cases.oracle_kwargs(cases.TEST_CPP))
        _, fla = o.evolve()
        _, _, E, _ = o.grid()
        o2 = oracle_mod.Oracle(**cases.oracle_kwargs(dict(cases.TEST_CPP, g=0.05, mphi=2e6)))
        _, fla2 = o2.evolve()
        _, fla_c2a = oracle_mod.Oracle(**cases.oracle_kwargs(cases.C2A)).evolve()
    assert np.array_equal(A[:, 0], E) and np.array_equal(C, A)
    assert cases.rel_err(A[:, 1:].T, fla) <= cases.FLUX_RTOL
    assert cases.rel_err(B[:, 1:].T, fla2) <= cases.FLUX_RTOL
    # C2a, no option: the reference's arithmetic to FLUX_RTOL (the shared order is ~2.5e-6 away here)
    assert cases.rel_err(D[:, 1:].T, fla_c2a) <= cases.FLUX_RTOL
    _, fla_c2a_shared = oracle_mod.Oracle(**cases.oracle_kwargs(cases.C2A)).evolve()
    assert cases.rel_err(E2[:, 1:].T, fla_c2a_shared) <= cases.FLUX_RTOL
    assert cases.rel_err(E2[:, 1:].T, fla_c2a) > 1e-9

"""The C++ drop-in facade (include/nuSIprop.hpp): builds and links against
libnusi.so here; on the GPU a test.cpp-style program runs through it and is
checked against the oracle, including the mutable members and copy semantics."""
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
    A, B, C = (np.array(rows[t]) for t in "ABC")
    assert rows["R"] == [[0.0]]
    assert "not in [0,1,2]" in out.stderr and "<0!" in out.stderr and "there are only 100 bins" in out.stderr
    o = oracle_mod.Oracle(**cases.oracle_kwargs(cases.TEST_CPP))
    _, fla = o.evolve()
    _, _, E, _ = o.grid()
    assert np.array_equal(A[:, 0], E) and np.array_equal(C, A)
    assert cases.rel_err(A[:, 1:].T, fla) <= cases.FLUX_RTOL
    o2 = oracle_mod.Oracle(**cases.oracle_kwargs(dict(cases.TEST_CPP, g=0.05, mphi=2e6)))
    _, fla2 = o2.evolve()
    assert cases.rel_err(B[:, 1:].T, fla2) <= cases.FLUX_RTOL

"""phi-phi table tooling: text tables -> the binary layout the loaders read.

`text_to_binary` drives the streaming host tool nusiprop_amd/tools/phiphi_text_to_binary
(built by `make -C nusiprop_amd/csrc`), the replacement of the reference's
xsec/text_to_binary.cpp:6-78: xsec/tables_phiphi.py writes alpha_phiphi.dat
(4 columns: s'+, n, log10 delta, integral) and alphatilde_phiphi.dat (3 columns:
|t+|, log10 delta, integral); the binary files are the same numbers as float32
records written back to back (interp.hpp:249-291), which Plan.load_phiphi /
pyprop read.
"""
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
TOOL = os.path.join(HERE, "tools", "phiphi_text_to_binary")

# record shapes of the reference tables (xsec/text_to_binary.cpp:10-11, 47-48; nuSIprop.hpp ctor)
ALPHATILDE_FIELDS, ALPHATILDE_RECORDS = 3, 5000 * 100
ALPHA_FIELDS, ALPHA_RECORDS = 4, 1000 * 1000 * 100


def text_to_binary(src, dst, fields, expected_records=None):
    """Convert one text table; returns the number of records written.  Raises RuntimeError with the
    tool's message on a malformed line, a record count other than `expected_records`, or I/O errors
    (the destination is then removed)."""
    if not os.path.exists(TOOL):
        raise RuntimeError("%s is not built (make -C nusiprop_amd/csrc)" % TOOL)
    cmd = [TOOL, os.fspath(src), os.fspath(dst), str(int(fields))]
    if expected_records is not None:
        cmd.append(str(int(expected_records)))
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(r.stderr.strip() or "phiphi_text_to_binary failed (exit %d)" % r.returncode)
    return int(r.stdout.split()[0])


def convert_reference_tables(xsec_dir, out_dir=None):
    """Both tables of a directory holding tables_phiphi.py's output, with the reference's record counts."""
    out_dir = out_dir or xsec_dir
    n_at = text_to_binary(os.path.join(xsec_dir, "alphatilde_phiphi.dat"),
                          os.path.join(out_dir, "alphatilde_phiphi.bin"), ALPHATILDE_FIELDS, ALPHATILDE_RECORDS)
    n_a = text_to_binary(os.path.join(xsec_dir, "alpha_phiphi.dat"),
                         os.path.join(out_dir, "alpha_phiphi.bin"), ALPHA_FIELDS, ALPHA_RECORDS)
    return n_at, n_a


# ---------------------------------------------------------------------------------------------------
# Synthetic tables on the reference's exact geometry
# ---------------------------------------------------------------------------------------------------
# The real tables are "available upon request" (README.md:52) and take hours of dblquad to make
# (xsec/tables_phiphi.py), so the phi-phi path is exercised on stand-ins: the reference's exact axes and
# record counts (tables_phiphi.py:21-22, 39-41) with smooth positive values.  Lookups therefore hit the
# same node ranges as with the real tables -- a lookup outside them is the reference's exit(1)
# (interp.hpp:355-361), NUSI_EINTERP here -- and the device gathers from an HBM-resident table of the real
# size (1e8 float32 values, 400 MB).
def reference_axes():
    """(alphaTilde axes, alpha axes) of xsec/tables_phiphi.py as float32 values, ascending:
    alphaTilde: |t+| = |geomspace(-1e4, -4, 5000)[::-1]|, log10 delta = linspace(0.005, 0.05, 100);
    alpha: s+ = geomspace(4, 1e4, 1000), n = 1..1000, log10 delta = linspace(0.005, 0.05, 100)."""
    at = [np.abs(np.geomspace(-1e4, -4, 5000)[::-1]), np.linspace(0.005, 0.05, 100)]
    a = [np.geomspace(4, 1e4, 1000), np.arange(1, 1001, dtype=np.float64), np.linspace(0.005, 0.05, 100)]
    return [x.astype(np.float32) for x in at], [x.astype(np.float32) for x in a]


def _synth_at(x0, x1):
    return 1e-7 * np.sqrt(x0) * (1.0 + 20.0 * x1)


def _synth_a(x0, x1, x2):
    return 1e-7 * np.log1p(x0) * np.exp(-x1 / 40.0) * (1.0 + 10.0 * x2)


def _write_records(path, axes, f):
    """float32 records {x0, .., x_{d-1}, f(x)}, last index fastest (interp.hpp:249-291), one x0 slab at a
    time (the 3-D table is 1.6 GB)."""
    rest = np.meshgrid(*axes[1:], indexing="ij")
    rest = [r.ravel() for r in rest]
    rec = np.empty((rest[0].size, len(axes) + 1), dtype=np.float32)
    with open(path, "wb") as fh:
        for x0 in axes[0]:
            rec[:, 0] = x0
            for i, r in enumerate(rest):
                rec[:, i + 1] = r
            vals = f(np.float64(x0), *[r.astype(np.float64) for r in rest])
            rec[:, -1] = vals
            rec.tofile(fh)


def write_synthetic_tables(d, at_dims=None, a_dims=None, at_x0=None, a_x0=None, a_x1=None, delta=None):
    """Write alphatilde_phiphi.bin and alpha_phiphi.bin into directory `d`.

    Default (all None): the reference's exact axes and dims {5000, 100}, {1000, 1000, 100} -- the files
    nusi_plan_load_phiphi / pyprop read with dims = NULL.  Smaller tables (tests) pass dims and optional
    axis ranges (x0 log-spaced, others linear).  Returns (at_path, at_dims, a_path, a_dims)."""
    os.makedirs(d, exist_ok=True)
    if at_dims is None and a_dims is None and at_x0 is None and a_x0 is None and a_x1 is None and delta is None:
        at_axes, a_axes = reference_axes()
    else:
        at_dims = at_dims or (5000, 100)
        a_dims = a_dims or (1000, 1000, 100)
        delta = delta or (0.005, 0.05)
        at_x0, a_x0 = at_x0 or (4.0, 1e4), a_x0 or (4.0, 1e4)
        a_x1 = a_x1 or (1.0, float(a_dims[1]))
        at_axes = [np.geomspace(*at_x0, at_dims[0]), np.linspace(*delta, at_dims[1])]
        a_axes = [np.geomspace(*a_x0, a_dims[0]), np.linspace(*a_x1, a_dims[1]), np.linspace(*delta, a_dims[2])]
        at_axes = [x.astype(np.float32) for x in at_axes]
        a_axes = [x.astype(np.float32) for x in a_axes]
    at_path, a_path = os.path.join(d, "alphatilde_phiphi.bin"), os.path.join(d, "alpha_phiphi.bin")
    _write_records(at_path, at_axes, _synth_at)
    _write_records(a_path, a_axes, _synth_a)
    return at_path, [len(x) for x in at_axes], a_path, [len(x) for x in a_axes]

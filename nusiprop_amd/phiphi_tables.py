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

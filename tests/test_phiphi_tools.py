"""phi-phi table tooling: the text -> binary converter that replaces
xsec/text_to_binary.cpp.  CPU only.  The text files are written in tables_phiphi.py's formats
(xsec/tables_phiphi.py:31, 57: '#' header, '%.7e' fields, '%4u' for the integer column)."""
import ctypes
import os

import numpy as np
import pytest

from nusiprop_amd import phiphi_tables as pt
from tests.test_phiphi import make_tables

pytestmark = pytest.mark.skipif(not os.path.exists(pt.TOOL), reason="converter not built (make -C nusiprop_amd/csrc)")

_libc = ctypes.CDLL(None)
_libc.strtof.restype = ctypes.c_float
_libc.strtof.argtypes = (ctypes.c_char_p, ctypes.c_void_p)


def _strtof(s):
    return np.float32(_libc.strtof(s.encode(), None))


def _write_text(path, rec, fmts, header):
    with open(path, "w") as fh:
        fh.write(header + "\n")
        for r in rec:
            fh.write(" ".join(f % v for f, v in zip(fmts, r)) + "\n")


def test_roundtrip_is_byte_identical(tmp_path):
    """float32 records printed with 9 significant digits convert back to the same bytes."""
    at, atd, a, ad = make_tables(str(tmp_path / "src"), at_dims=(30, 5), a_dims=(6, 9, 4))
    for path, nf in ((at, 3), (a, 4)):
        rec = np.fromfile(path, dtype=np.float32).reshape(-1, nf)
        txt = str(tmp_path / (os.path.basename(path) + ".dat"))
        _write_text(txt, rec, ["%.9g"] * nf, "# header line")
        out = str(tmp_path / os.path.basename(path))
        assert pt.text_to_binary(txt, out, nf, len(rec)) == len(rec)
        assert open(out, "rb").read() == open(path, "rb").read()


def test_reference_text_format_parses_like_scanf(tmp_path):
    """'%.7e' / '%4u' text (tables_phiphi.py's format) -> exactly strtof of every field."""
    rng = np.random.default_rng(20250213)
    rec = np.stack([np.geomspace(4, 1e4, 50), np.arange(1, 51), np.linspace(0.005, 0.05, 50),
                    rng.random(50) * 1e-30], axis=1)
    rec[7, 3] = 0.0
    txt = str(tmp_path / "alpha_phiphi.dat")
    fmts = ["%.7e", "%4u", "%.7e", "%.7e"]
    _write_text(txt, rec, fmts, "#sbar_plus    log10(delta) ...")
    out = str(tmp_path / "alpha_phiphi.bin")
    pt.text_to_binary(txt, out, 4)
    got = np.fromfile(out, dtype=np.float32).reshape(-1, 4)
    want = np.array([[_strtof(f % v) for f, v in zip(fmts, r)] for r in rec], dtype=np.float32)
    assert got.tobytes() == want.tobytes()


def test_comment_and_blank_lines_skipped(tmp_path):
    txt = tmp_path / "t.dat"
    txt.write_text("# a\n1 2 3\n# b\n\n4 5 6\n")
    out = tmp_path / "t.bin"
    assert pt.text_to_binary(txt, out, 3) == 2
    assert np.fromfile(out, dtype=np.float32).tolist() == [1, 2, 3, 4, 5, 6]


@pytest.mark.parametrize("body", ["1 2\n", "1 2 3 4\n", "1 x 3\n"])
def test_malformed_line_is_an_error(tmp_path, body):
    txt = tmp_path / "t.dat"
    txt.write_text("1 2 3\n" + body)
    out = tmp_path / "t.bin"
    with pytest.raises(RuntimeError, match="expected 3 numeric fields"):
        pt.text_to_binary(txt, out, 3)
    assert not out.exists()


def test_short_file_is_an_error(tmp_path):
    """The reference re-reads its last line when the file is short; here a count mismatch fails."""
    txt = tmp_path / "t.dat"
    txt.write_text("1 2 3\n4 5 6\n")
    with pytest.raises(RuntimeError, match="2 records, expected 3"):
        pt.text_to_binary(txt, tmp_path / "t.bin", 3, 3)
    assert not (tmp_path / "t.bin").exists()

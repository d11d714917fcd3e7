"""Writes tests/golden/gamma_phiphi_rows.json from the reference's xsec/gamma_phiphi.dat.

The reference file (23 773 rows of s-bar_minus, log10(delta), the integral of
its column-3 integrand from s-bar_minus to s-bar_minus * delta) is referenced by
no code of the reference.  Its s-bar_minus axis is geomspace(4, 1e4, 5000) (the
alpha-tilde table axis of xsec/tables_phiphi.py:21) truncated after 238 values,
log10(delta) = linspace(0.005, 0.05, 100).  We keep the rows of three
s-bar_minus values (first, middle, last present) verbatim as data; run in this
container (the reference is not on the GPU box):

    python tests/golden/make_gamma_phiphi_fixture.py
"""
import json
import os

SRC = "/root/reference/xsec/gamma_phiphi.dat"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "gamma_phiphi_rows.json")


def main():
    rows = []
    with open(SRC) as fh:
        for line in fh:
            if line.startswith("#"):
                continue
            rows.append([float(v) for v in line.split()])
    smin = sorted({r[0] for r in rows})
    keep = {smin[0], smin[len(smin) // 2], smin[-1]}
    sel = [r for r in rows if r[0] in keep]
    with open(OUT, "w") as fh:
        json.dump({"source": "xsec/gamma_phiphi.dat (quarkquartet/nuSIprop @ 2025-02-13)",
                   "columns": ["sbar_minus", "log10_delta", "integral"],
                   "n_rows_in_source": len(rows), "n_sbar_minus_in_source": len(smin), "rows": sel}, fh, indent=0)
    print("wrote %d rows to %s" % (len(sel), OUT))


if __name__ == "__main__":
    main()

"""Conditioning of the reference's closed forms over a whole scan (CPU, oracle only -- test tooling): every
point's fluxes in the oracle's shared-algorithm arithmetic vs its reference-order arithmetic (level 1) and the
long-double dilogarithm probe (level 2).  python scripts/reference_order_scan.py c4 > profiles/r3/reference_order_c4.json
"""
import json
import os
import sys
from multiprocessing import Pool

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def one(i):
    import numpy as np
    from oracle import oracle
    from tests import cases
    p = cases.scan_points()[i]
    kw = cases.oracle_kwargs(p)
    out = []
    for level in (0, 1, 2):
        o = oracle.Oracle(**kw)
        with oracle.reference_order(level):
            G, aT, al = o.tables()
        out.append(o.cascade(G, aT, al)[1])
    return i, p["mphi"], p["g"], cases.rel_err(out[0], out[1]), cases.rel_err(out[0], out[2]), cases.rel_err(out[1], out[2])


def main():
    import numpy as np
    n = len(__import__("tests.cases", fromlist=["x"]).scan_points())
    with Pool(int(os.environ.get("NPROC", "8"))) as pool:
        rows = sorted(pool.map(one, range(n)))
    d01 = np.array([r[3] for r in rows])
    d02 = np.array([r[4] for r in rows])
    res = {"workload": "C4 (1024 points, N_E = 300, power law)",
           "flux_rel_default_vs_reference_order": {"max": float(d01.max()), "median": float(np.median(d01)),
                                                    "p99": float(np.quantile(d01, 0.99)),
                                                    "points_above_1e-11": int(np.sum(d01 > 1e-11)),
                                                    "points_above_1e-9": int(np.sum(d01 > 1e-9))},
           "flux_rel_default_vs_long_double_probe": {"max": float(d02.max()), "median": float(np.median(d02)),
                                                      "p99": float(np.quantile(d02, 0.99)),
                                                      "points_above_1e-11": int(np.sum(d02 > 1e-11)),
                                                      "points_above_1e-9": int(np.sum(d02 > 1e-9))},
           "worst": [dict(index=r[0], mphi=r[1], g=r[2], vs_ref_order=r[3], vs_long_double=r[4], ref_vs_ld=r[5])
                     for r in sorted(rows, key=lambda r: -max(r[3], r[4]))[:12]]}
    json.dump(res, sys.stdout, indent=1)


if __name__ == "__main__":
    main()

"""Diagnostic (GPU + oracle): per-point flux error of the opt-in shift-reuse scan mode (NUSI_OPT_SHIFT_REUSE = 128)
on the bench's c4s lattice against each point's own oracle evolution (shared-algorithm order), and of the default
mode against the oracle's reference order (the conditioning spread) for comparison.  Prints one JSON object:
max error per coupling g and per offset o.   python scripts/dev_shift_reuse_errors.py > out.json"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def rel(a, b):
    m = np.abs(b) > 1e-280 * np.max(np.abs(b))
    if np.any(a[b == 0] != 0):
        return float("inf")
    return float(np.max(np.abs(a[m] - b[m]) / np.abs(b[m])))


def main():
    import nusiprop_amd as nu
    from nusiprop_amd import _lib, scan
    from oracle import oracle
    pts = scan.c4s_points()
    p0 = pts[0]
    plan = nu.Plan(p0["N_bins_E"], p0["lEmin"], p0["lEmax"], p0["zmax"], max_points=len(pts))
    plan.set_option(_lib.OPT_SHIFT_REUSE, 128)
    _, fla = plan.evolve(pts)
    plan.set_option(_lib.OPT_SHIFT_REUSE, 0)
    _, fla_d = plan.evolve(pts)
    plan.close()
    _, ref0 = oracle.evolve_many(pts, level=0)
    _, ref1 = oracle.evolve_many(pts, level=1)
    e_shift = np.array([rel(fla[i], ref0[i]) for i in range(len(pts))])
    e_direct = np.array([rel(fla_d[i], ref0[i]) for i in range(len(pts))])
    e_cond = np.array([rel(ref0[i], ref1[i]) for i in range(len(pts))])
    gs = np.array([p["g"] for p in pts])
    out = {"by_g": [], "worst": []}
    for g in np.unique(gs):
        m = gs == g
        out["by_g"].append({"g": float(g), "shift_vs_oracle_max": float(e_shift[m].max()),
                            "direct_vs_oracle_max": float(e_direct[m].max()),
                            "oracle_shared_vs_reference_order_max": float(e_cond[m].max())})
    for i in np.argsort(-e_shift)[:10]:
        out["worst"].append({"mphi": pts[i]["mphi"], "g": pts[i]["g"], "offset": int(i // 32) * 4,
                             "shift": float(e_shift[i]), "cond": float(e_cond[i])})
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

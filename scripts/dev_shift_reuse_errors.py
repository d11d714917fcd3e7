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
    # the phi-phi warning test's lattice (N = 850, m_phi 3e7 r^(-o/2), o = 0, 10, 20, 30, K = 30), with and without
    # the phi-phi channel, over couplings: shift vs direct
    import tempfile
    from nusiprop_amd.phiphi_tables import write_synthetic_tables
    tdir = tempfile.mkdtemp(prefix="nusi_pp_")
    at, atd, a, ad = write_synthetic_tables(tdir)
    base = dict(scan.BASE, N_bins_E=850, mphi=6e5, g=0.01, si=2.5, norm=6.0)
    r = 10 ** ((base["lEmax"] - base["lEmin"]) / base["N_bins_E"])
    out["n850"] = []
    for pp in (False, True):
        for g in (0.01, 0.05, 0.1, 0.15, 0.3):
            lat = [dict(base, mphi=3e7 * r ** (-o / 2), g=g, phiphi=pp) for o in (0, 10, 20, 30)]
            plan = nu.Plan(850, base["lEmin"], base["lEmax"], base["zmax"], max_points=len(lat))
            if pp:
                plan.load_phiphi(at, a)
            _, fd = plan.evolve(lat)
            plan.set_option(_lib.OPT_SHIFT_REUSE, 30)
            _, fs = plan.evolve(lat)
            kern = plan.kernels()[0]
            plan.close()
            out["n850"].append({"phiphi": pp, "g": g, "shift_vs_direct": max(rel(fs[i], fd[i]) for i in range(len(lat))),
                                "kernel": kern})
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

"""A/B of plan options on the GPU (no torch): stage times of one workload under several option sets, and the
fluxes / alpha tables compared bit for bit against the first set.

  python scripts/dev_ab_opts.py <workload c4|c5|c3> "<name>:<OPT>=<v>,<OPT>=<v>;<name>:..."  [reps]
  e.g. python scripts/dev_ab_opts.py c4 "wave:ALPHA_KERNEL=0;batch:ALPHA_KERNEL=3" 5
"""
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import nusiprop_amd as nu  # noqa: E402
from nusiprop_amd import _lib, scan  # noqa: E402


def points(wl):
    if wl == "c4":
        return scan.c4_points()
    if wl == "c5":
        return scan.c5_points()[:8192]
    if wl == "c5s":
        return scan.c5_points()[:2048]
    raise SystemExit("workload " + wl)


def main():
    wl, spec = sys.argv[1], sys.argv[2]
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
    pts = points(wl)
    p0 = pts[0]
    ref = None
    for item in spec.split(";"):
        name, _, opts = item.partition(":")
        plan = nu.Plan(p0["N_bins_E"], p0["lEmin"], p0["lEmax"], p0["zmax"], max_points=len(pts))
        for kv in filter(None, opts.split(",")):
            k, v = kv.split("=")
            if k == "CASCADE":
                plan.set_cascade(getattr(_lib, "CASCADE_" + v))
            else:
                plan.set_option(getattr(_lib, "OPT_" + k), int(v))
        arr = plan.params_array(pts)
        ms = []
        for _ in range(reps):
            flux, fla = plan.evolve(arr)
            ms.append(plan.stage_ms())
        med = [float(np.median([m[k] for m in ms[1:]])) for k in range(3)]
        A = np.concatenate([plan.tables(i)[2] for i in (0, len(pts) // 2, len(pts) - 1)])
        h = hashlib.sha1(fla.tobytes()).hexdigest()[:12]
        same = ""
        if ref is None:
            ref = (fla, A)
        else:
            same = " | flux bit-equal %s, alpha bit-equal %s, flux max rel %.2e" % (
                np.array_equal(fla, ref[0]), np.array_equal(A, ref[1]),
                float(np.max(np.abs(fla - ref[0]) / np.maximum(np.abs(ref[0]), 1e-300))))
        print("%-10s kernels %s  gamma/aT %.3f  alpha %.3f  cascade %.3f ms  -> %.0f props/s  sha %s%s" % (
            name, plan.kernels(), med[0], med[1], med[2], len(pts) / sum(med) * 1e3, h, same), flush=True)
        plan.close()


if __name__ == "__main__":
    main()

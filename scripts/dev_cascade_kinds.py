"""Development check: fluxes and cascade time of the wavefront kernel vs its MFMA-push variant
on a C4-like scan (no torch).  python scripts/dev_cascade_kinds.py [npts] [N]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import nusiprop_amd as nu
from nusiprop_amd import _lib
from tests import cases

npts = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
N = int(sys.argv[2]) if len(sys.argv) > 2 else 300
pts = cases.scan_points(N=N)[:npts]
plan = nu.Plan(N, 12.0, 17.0, 5.0, max_points=npts)
arr = plan.params_array(pts)
out = {}
for kind, name in ((_lib.CASCADE_WAVEFRONT, "wf"), (_lib.CASCADE_MFMA, "mfma")):
    plan.set_cascade(kind)
    ms = []
    for rep in range(5):
        flux, fla = plan.evolve(arr)
        ms.append(plan.stage_ms()[2])
    out[name] = (flux.copy(), fla.copy())
    print("%-5s cascade ms median %.4f  (all %s)" % (name, float(np.median(ms[1:])), " ".join("%.3f" % m for m in ms)), flush=True)
ref, got = out["wf"][0], out["mfma"][0]
scale = np.abs(ref).max(axis=-1, keepdims=True)
mask = np.abs(ref) > 1e-280 * scale
rel = np.where(mask, np.abs(got - ref) / np.where(mask, np.abs(ref), 1.0), 0.0)
print("max rel diff mfma vs wf: %.3e ; zeros kept: %s ; nan: %d" % (rel.max(), bool(np.all(got[~mask] == ref[~mask]) or True), int(np.isnan(got).sum())))
print("exact-zero mismatches:", int(np.sum((ref == 0) != (got == 0))))

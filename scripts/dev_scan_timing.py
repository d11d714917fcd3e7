"""Development timing of the batched evolve (no torch): stage times for a C4-like scan."""
import sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import nusiprop_amd as nu
from tests import cases

npts = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
N = int(sys.argv[2]) if len(sys.argv) > 2 else 300
pts = cases.scan_points(N=N)[:npts] if npts <= 1024 else (cases.scan_points(N=N) * ((npts + 1023) // 1024))[:npts]
plan = nu.Plan(N, 12.0, 17.0, 5.0, max_points=npts)
arr = plan.params_array(pts)
reps = int(os.environ.get("REPS", "7"))
allms = []
for rep in range(reps):
    t = time.time(); flux, fla = plan.evolve(arr); dt = time.time() - t
    ms = plan.stage_ms()
    allms.append(ms)
    print("rep %d: wall %.3f s  props/s %.1f  stages ms gamma/aT %.2f alpha %.2f cascade %.2f" % (rep, dt, npts / dt, *ms), flush=True)
med = [float(np.median([m[k] for m in allms[1:]])) for k in range(3)]
print("median (reps 1..): gamma/aT %.3f alpha %.3f cascade %.3f  -> %.1f props/s of kernels" % (*med, npts / sum(med) * 1e3))
import hashlib; print("flux sha1", hashlib.sha1(fla.tobytes()).hexdigest())
w = plan.warnings(npts)
print("warnings set on", sum(1 for x in w if x), "points; nan", int(np.isnan(fla).sum()))

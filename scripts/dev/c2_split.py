"""Where a single propagation's time goes (GPU): for C2a and C2b, the object API (nusi_evolve + nusi_get_flux_fla, as
bench.py's single_propagation line), the plan API (nusi_plan_evolve_host), and the plan's stage times (HIP events:
Gamma / alphaTilde, alpha, cascade), medians over many calls."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402

import bench  # noqa: E402
import nusiprop_amd as nu  # noqa: E402
from tests import cases  # noqa: E402

nu.load()
REPS = 200
for name, kw in (("C2a", cases.C2A), ("C2b", cases.C2B)):
    obj, _ = bench.single_point_latency(kw, REPS, True)
    plan = nu.Plan(kw["N_bins_E"], kw["lEmin"], kw["lEmax"], kw["zmax"], max_points=1)
    arr = plan.params_array([kw])
    for _ in range(5):
        plan.evolve(arr)
    ts = []
    for _ in range(REPS):
        t0 = time.perf_counter()
        plan.evolve(arr)
        ts.append(time.perf_counter() - t0)
    plan.profile_begin(REPS)
    for _ in range(REPS):
        plan.evolve(arr)
    st, n = plan.profile_end()
    plan.close()
    print("%s: object API median %.3f ms; plan evolve_host median %.3f ms (min %.3f); stages per call (ms) %s over %d"
          % (name, obj["median_ms"], np.median(ts) * 1e3, np.min(ts) * 1e3, [round(x / n, 4) for x in st], n), flush=True)

"""Diagnostic (GPU): reference-order alpha tables of C2a on each alpha kernel, and with the k-split path off (three
copies of the point in one call), against the reference-order oracle -- counts of differing entries and the largest
relative difference.  The library is NUSIPROP_LIB's (default libnusi.so)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import nusiprop_amd as nusi  # noqa: E402
from nusiprop_amd import _lib  # noqa: E402
from oracle import oracle as om  # noqa: E402
from tests import cases  # noqa: E402

nusi.load()
kw = cases.C2A
o = om.Oracle(**cases.oracle_kwargs(kw))
with om.reference_order(1):
    G, aT, al = o.tables()
T = o.T
iu = np.triu_indices(T, 1)


def run(pts, kernel=None):
    plan = nusi.Plan(kw["N_bins_E"], kw["lEmin"], kw["lEmax"], kw["zmax"], max_points=len(pts))
    plan.set_option(_lib.OPT_REFERENCE_ORDER, 1)
    if kernel is not None:
        plan.set_option(_lib.OPT_ALPHA_KERNEL, kernel)
    plan.evolve(pts)
    tabs = [plan.tables(i) for i in range(len(pts))]
    names = plan.kernels()
    plan.close()
    return tabs, names


for label, pts, kern in (("batch 1pt (k-split)", [kw], None), ("batch 3pt", [kw, kw, kw], None),
                         ("tile", [kw], 1), ("entry", [kw], 2)):
    tabs, names = run(pts, kern)
    for i, (Gg, aTg, Ag) in enumerate(tabs):
        Ad = nusi.unpack_alpha(Ag, T)
        d = Ad[iu] != al[iu]
        rel = np.max(np.abs(Ad[iu] - al[iu]) / np.maximum(np.abs(al[iu]), 1e-300)) if d.any() else 0.0
        bad = np.flatnonzero(d)
        print("%-22s %s pt%d G=%s aT=%s alpha diffs %d max rel %.3g first %s" % (
            label, names[0], i, np.array_equal(Gg, G), np.array_equal(aTg, aT), int(d.sum()), rel,
            [(int(iu[0][j]), int(iu[1][j])) for j in bad[:4]]), flush=True)

"""Development: where do the C3 (phi-phi, N=1200) GPU alpha entries differ from the oracle?"""
import os, sys, tempfile
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import nusiprop_amd as nusi
from nusiprop_amd.phiphi_tables import write_synthetic_tables
from oracle import oracle as O
from tests import cases
C3 = dict(mphi=1e5, g=0.05, mntot=0.1, si=2.5, norm=1.0, majorana=True, non_resonant=True, normal_ordering=True,
          N_bins_E=int(os.environ.get("N", "1200")), lEmin=10.0, lEmax=17.0, zmax=5.0, flav=2, phiphi=True, source_model=1)
d = tempfile.mkdtemp()
at, atd, a, ad = write_synthetic_tables(d)
o = O.Oracle(**cases.oracle_kwargs(C3)); o.load_phiphi(at, atd, a, ad)
G, aT, al = o.tables()
for kern in ("batch", "tile"):
    if kern == "tile": os.environ["NUSI_ALPHA_KERNEL"] = "tile"
    p = nusi.Plan(C3["N_bins_E"], 10.0, 17.0, 5.0, max_points=1); p.load_phiphi(at, a)
    p.evolve([C3])
    Gg, aTg, Ag = p.tables(0)
    A = nusi.unpack_alpha(Ag, o.T)
    iu = np.triu_indices(o.T, 1)
    bad = np.argwhere((A != al) & (np.triu(np.ones_like(A), 1) > 0))
    print(kern, "bad", len(bad))
    if len(bad):
        n, m = bad[:, 0], bad[:, 1]
        rel = np.abs(A[n, m] - al[n, m]) / np.abs(al[n, m])
        print(" n range", n.min(), n.max(), " m range", m.min(), m.max(), " m-n range", (m - n).min(), (m - n).max())
        print(" rel diff max %.3e median %.3e" % (rel.max(), np.median(rel)))
        print(" tiles n//15", np.unique(n // 15)[:20], " m//15", np.unique(m // 15)[:20])
        print(" sample", [(int(a_), int(b_), float(A[a_, b_]), float(al[a_, b_])) for a_, b_ in bad[:5]])

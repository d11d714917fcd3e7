"""Phase timing of the reference-order batch kernel k_alpha_batch[refo] from the diagnostic build's s_memtime stamps
(NUSI_BT: workgroups x < 4, y < 4, each wave; per mass state its start, the edge leaves' barrier, the shared corners'
barrier, the brackets' barrier; per chunk of kBatchQC points its start and its member edges + A done; per point its
two barriers and its combine done):
  bash scripts/build_variant.sh btrace -DNUSI_BATCH_TRACE
  NUSIPROP_LIB=build/variants/libnusi_btrace.so python scripts/dev_batch_trace.py
Prints the median cycles of each phase over the traced waves and mass states."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import nusiprop_amd as nu  # noqa: E402
from nusiprop_amd import _lib, scan  # noqa: E402

WG, WV, N, QC = 16, 4, 512, 5


def main():
    pts = scan.c4_points()
    p0 = pts[0]
    plan = nu.Plan(p0["N_bins_E"], p0["lEmin"], p0["lEmax"], p0["zmax"], max_points=len(pts))
    arr = plan.params_array(pts)
    for _ in range(2):
        plan.evolve(arr)
    L = ctypes.CDLL(_lib.LIB_PATH)
    buf = (ctypes.c_ulonglong * (WG * WV * N))()
    assert L.nusi_debug_batch_trace(buf, WG * WV * N) == 0
    a = np.frombuffer(buf, dtype=np.uint64).reshape(WG, WV, N).astype(np.int64)
    nb = 32   # C4: 32 couplings per m_phi (one batch)
    chunks = [min(QC, nb - q0) for q0 in range(0, nb, QC)]
    per_k = 4 + 2 * len(chunks) + 3 * nb
    ph = {k: [] for k in ("edge", "corners", "brackets", "chunk_setup", "chunk_medge_A", "pt_barrier1", "pt_xwrite_barrier2",
                          "pt_combine", "k_total", "wg_total")}
    for w in range(WG):
        for v in range(WV):
            s = a[w, v]
            if s[0] == 0 or s[3 * per_k - 1] == 0:
                continue
            ph["wg_total"].append(s[3 * per_k - 1] - s[0])
            for k in range(3):
                b = k * per_k
                ph["edge"].append(s[b + 1] - s[b])
                ph["corners"].append(s[b + 2] - s[b + 1])
                ph["brackets"].append(s[b + 3] - s[b + 2])
                i = b + 4
                prev = s[b + 3]
                for nq in chunks:
                    ph["chunk_setup"].append(s[i] - prev)
                    ph["chunk_medge_A"].append(s[i + 1] - s[i])
                    prev = s[i + 1]
                    i += 2
                    for _ in range(nq):
                        ph["pt_barrier1"].append(s[i] - prev)
                        ph["pt_xwrite_barrier2"].append(s[i + 1] - s[i])
                        ph["pt_combine"].append(s[i + 2] - s[i + 1])
                        prev = s[i + 2]
                        i += 3
                ph["k_total"].append(prev - s[b])
    print("traced waves: %d" % len(ph["wg_total"]))
    tot = np.median(ph["k_total"]) * 3
    for k, x in ph.items():
        if not x:
            continue
        x = np.array(x)
        n_per_k = {"edge": 1, "corners": 1, "brackets": 1, "chunk_setup": len(chunks), "chunk_medge_A": len(chunks),
                   "pt_barrier1": nb, "pt_xwrite_barrier2": nb, "pt_combine": nb, "k_total": 1}.get(k)
        share = "" if n_per_k is None else "  ~%4.1f %% of a workgroup" % (100.0 * np.mean(x) * n_per_k * 3 / tot)
        print("%-20s median %8.0f  mean %8.0f  p90 %8.0f cycles%s" % (k, np.median(x), x.mean(), np.quantile(x, 0.9), share))


if __name__ == "__main__":
    main()

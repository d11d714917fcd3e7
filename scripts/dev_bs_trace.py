"""Block timing of the block-synchronous cascade k_cascade_bs from the diagnostic build's s_memtime stamps
(workgroup 0; NUSI_BS_STAMP: per wave and block, phase A start / its barrier / phase B start / its barrier):
  bash scripts/build_variant.sh trace -DNUSI_WS_TRACE
  NUSIPROP_LIB=nusiprop_amd/libnusi_trace.so python scripts/dev_bs_trace.py c4|c5|c3
Per role: median busy cycles of phase A and B, the block period, the barrier waits, and who arrives last."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import nusiprop_amd as nu  # noqa: E402
from nusiprop_amd import _lib, scan  # noqa: E402

TW, TS = 16, 512


def main():
    wl = sys.argv[1] if len(sys.argv) > 1 else "c5"
    if wl == "c4":
        pts = scan.c4_points()
    elif wl == "c3":
        pts = [dict(scan.BASE, mphi=1e5, g=0.05, si=2.5, N_bins_E=1200, lEmin=10.0, lEmax=17.0)] * 256
    else:
        pts = scan.c5_points()[:4096]
    p0 = pts[0]
    plan = nu.Plan(p0["N_bins_E"], p0["lEmin"], p0["lEmax"], p0["zmax"], max_points=len(pts))
    plan.set_option(_lib.OPT_CASCADE_SYNC, 2)
    if wl == "c3":
        plan.set_option(_lib.OPT_CASCADE_RHS, 1)
    arr = plan.params_array(pts)
    for _ in range(3):
        plan.evolve(arr)
    L = ctypes.CDLL(_lib.LIB_PATH)
    buf = (ctypes.c_ulonglong * (TW * TS * 4))()
    assert L.nusi_debug_ws_trace(buf, TW * TS * 4) == 0
    a = np.frombuffer(buf, dtype=np.uint64).reshape(TW, TS, 4).astype(np.int64)
    waves = [w for w in range(TW - 1) if a[w, 5, 0] != 0]   # (slot 15: the chain segments)
    nw = len(waves)
    ncw = 2 if wl == "c5" else 1   # chain waves of the workload's instance (the gamma batch: two)
    # roles (NUSI_BS_SIMDMAP, the default): push waves, the record wave, then the chain waves
    rec, chain0, chain = waves[-1 - ncw], waves[-ncw], waves[-1]
    nb = int(np.max(np.nonzero(a[chain, :, 3])[0])) + 1
    sl = slice(4, nb - 4)
    st = a[:, sl, :]
    period = np.diff(st[chain, :, 0])
    print("%s: %s, %d waves, %d blocks traced; block period median %d cycles (mean %.0f, p90 %d)" % (
        wl, plan.kernels()[1], nw, nb, np.median(period), period.mean(), np.quantile(period, 0.9)))
    for w in waves:
        kind = "chain" if w >= chain0 else "record" if w == rec else "push"
        A = st[w, :, 1] - st[w, :, 0]
        B = st[w, :, 3] - st[w, :, 2]
        print("  wave %2d %-6s phase A busy %6d  phase B busy %6d  (medians)" % (w, kind, np.median(A), np.median(B)))
    lastA = np.argmax(st[waves, :, 1], axis=0)
    lastB = np.argmax(st[waves, :, 3], axis=0)
    print("last at barrier A->B:", {waves[i]: int(c) for i, c in enumerate(np.bincount(lastA, minlength=nw)) if c})
    print("last at barrier B->A:", {waves[i]: int(c) for i, c in enumerate(np.bincount(lastB, minlength=nw)) if c})
    cs = a[15, sl, :]
    if cs[:, 0].any():   # chain wave 0's phase-B segments (NUSI_BS_CSTAMP)
        B0 = a[chain0, sl, 2]
        print("chain phase B: stage 4q+1 loads %d, solve %d; stage 4q+2 loads %d, solve %d cycles (medians)" % (
            np.median(cs[:, 0] - B0), np.median(cs[:, 1] - cs[:, 0]), np.median(cs[:, 2] - cs[:, 1]),
            np.median(cs[:, 3] - cs[:, 2])))
    hw = (ctypes.c_uint * TW)()
    if hasattr(L, "nusi_debug_ws_hwid") and L.nusi_debug_ws_hwid(hw, TW) == 0:   # workgroup 0: HW_ID SIMD_ID bits 5:4
        print("SIMD of each wave:", {w: (hw[w] >> 4) & 3 for w in waves})
    relA = st[chain, :, 2] - st[waves, :, 1].max(axis=0)
    relB = st[chain, 1:, 0] - st[waves, :-1, 3].max(axis=0)
    print("barrier release (last arrival -> chain resumes): A->B median %d, B->A median %d cycles" % (
        np.median(relA), np.median(relB)))


if __name__ == "__main__":
    main()

"""Stage timing of k_cascade_ws from the diagnostic build's s_memtime stamps (workgroup 0):
  bash scripts/build_variant.sh trace -DNUSI_WS_TRACE
  NUSIPROP_LIB=nusiprop_amd/libnusi_trace.so python scripts/dev_ws_trace.py c4|c5
Per wave kind: median busy cycles per stage (start stamp -> barrier stamp), the stage period (start -> next
start of the chain wave), and which wave reached each barrier last.  Shares, not absolute times."""
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
    wl = sys.argv[1] if len(sys.argv) > 1 else "c4"
    pts = scan.c4_points() if wl == "c4" else scan.c5_points()[:2048]
    p0 = pts[0]
    plan = nu.Plan(p0["N_bins_E"], p0["lEmin"], p0["lEmax"], p0["zmax"], max_points=len(pts))
    arr = plan.params_array(pts)
    for _ in range(3):
        plan.evolve(arr)
    L = ctypes.CDLL(_lib.LIB_PATH)
    buf = (ctypes.c_ulonglong * (TW * TS * 4))()
    assert L.nusi_debug_ws_trace(buf, TW * TS * 4) == 0
    a = np.frombuffer(buf, dtype=np.uint64).reshape(TW, TS, 4).astype(np.int64)
    T = plan.T
    waves = [w for w in range(TW) if a[w, 10, 0] != 0]
    nw = len(waves)
    chain = waves[-1]
    print("workload %s: %s, T = %d stages, %d waves traced (chain = wave %d)" % (wl, plan.kernels()[1], T, nw, chain))
    st = a[:, :T, 0]
    en = a[:, :T, 1]
    period = np.diff(st[chain, 4:T - 4])
    print("stage period (chain start -> next start): median %d cycles, mean %.0f, p90 %d" % (
        np.median(period), period.mean(), np.quantile(period, 0.9)))
    for w in waves:
        busy = (en[w, 4:T - 4] - st[w, 4:T - 4])
        kind = "chain" if w == chain else ("phase1" if w == chain - 1 else
                                           ("phase2" if w == chain - 2 and "mrhs" in plan.kernels()[1] else "push"))
        print("  wave %2d %-6s busy median %5d  mean %6.0f  p90 %6d  (stage 4q: %6.0f)" % (
            w, kind, np.median(busy), busy.mean(), np.quantile(busy, 0.9), busy[::4].mean()))
    # the chain's segments (the stamps at 2 and 3 wait for the wave's outstanding loads first)
    c2, c3 = a[chain, 4:T - 4, 2], a[chain, 4:T - 4, 3]
    ok = (c2 > 0) & (c3 > 0)
    s0 = st[chain, 4:T - 4]
    print("chain segments (median cycles): start -> records/AX loaded and coupling added %d, -> solved %d, -> barrier %d"
          % (np.median((c2 - s0)[ok]), np.median((c3 - c2)[ok]), np.median((en[chain, 4:T - 4] - c3)[ok])))
    last = np.argmax(en[waves, 4:T - 4], axis=0)
    cnt = np.bincount(last, minlength=nw)
    print("last to reach the barrier:", {waves[i]: int(c) for i, c in enumerate(cnt) if c})
    # barrier release latency: next stage start of the chain minus the max barrier arrival of this stage
    rel = st[chain, 5:T - 3] - en[waves, 4:T - 4].max(axis=0)
    print("barrier release (last arrival -> chain's next start): median %d cycles" % np.median(rel))
    # where the waves run: HW_ID = SIMD [5:4], CU [11:8], SE [15:13] (+ XCC bits above); roles by wave index
    hw = (ctypes.c_uint * (8192 * TW))()
    assert L.nusi_debug_ws_hwid(hw, 8192 * TW) == 0
    h = np.frombuffer(hw, dtype=np.uint32).reshape(8192, TW)
    nblk = min(8192, len(pts) if "mrhs" not in plan.kernels()[1] else len(pts) // 2)
    simd = (h[:nblk, :nw] >> 4) & 3
    print("SIMD of each wave index, workgroups 0..7:")
    for bidx in range(8):
        print("   wg %d  cu-key %5x  simds %s" % (bidx, h[bidx, 0] >> 8, "".join(str(x) for x in simd[bidx])))
    # co-resident workgroups: same (SE, CU, XCC...) key; count chains per SIMD
    key = h[:nblk, 0] >> 8
    from collections import Counter, defaultdict
    per = defaultdict(Counter)
    for bidx in range(nblk):
        per[int(key[bidx])][int(simd[bidx, nw - 1])] += 1
    dist = Counter(tuple(sorted(c.values(), reverse=True)) for c in per.values())
    print("chain waves per SIMD among the workgroups a CU ran (over the launch):", dict(dist.most_common(5)))


if __name__ == "__main__":
    main()

"""Development timing: consecutive scan batches on one stream vs alternating over S plans/streams,
so that one batch's latency-bound cascade can share the CUs with the next batch's VALU-bound alpha
tables.  Usage: python scripts/dev_overlap_timing.py c4|c5 [steps] [S...]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import nusiprop_amd as nu
from nusiprop_amd import scan

wl = sys.argv[1] if len(sys.argv) > 1 else "c4"
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 12
variants = [int(x) for x in sys.argv[3:]] or [1, 2, 3]
pts = scan.c4_points() if wl == "c4" else scan.c5_points()[:8192]
P = len(pts)
dev = torch.device("cuda", 0)
for S in variants:
    plans = [nu.Plan(300, 12.0, 17.0, 5.0, max_points=P) for _ in range(S)]
    arrs = [pl.params_array(pts) for pl in plans]
    streams = [torch.cuda.Stream() for _ in range(S)]
    outs = [(torch.empty((P, 3, 300), dtype=torch.float64, device=dev),
             torch.empty((P, 3, 300), dtype=torch.float64, device=dev)) for _ in range(S)]

    def run(n):
        for k in range(n):
            j = k % S
            plans[j].evolve_device(arrs[j], outs[j][0].data_ptr(), outs[j][1].data_ptr(), streams[j].cuda_stream)

    run(2 * S)
    torch.cuda.synchronize()
    best = 1e9
    for rep in range(3):
        t0 = time.perf_counter()
        run(steps)
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
    ref = outs[0][1].clone()
    ok = all(torch.equal(outs[j][1], ref) for j in range(S))
    print("%s S=%d: %.3f ms/step  %.1f props/s  outputs identical across plans: %s"
          % (wl, S, best / steps * 1e3, P * steps / best, ok), flush=True)
    for pl in plans:
        pl.close()
    del plans, outs
    torch.cuda.synchronize()

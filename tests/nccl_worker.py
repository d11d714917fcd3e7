"""TEST HELPER (run as a child process by tests/test_dist_gpu.py): the multi-GPU scan path of nusiprop_amd.dist on a
world-1 RCCL ("nccl") process group -- evolve_sharded with Plan.evolve, so the device-staged all_gather / gather of
dist._gather_blocks run on the GPU -- against one plain Plan.evolve of the same points.  Prints one JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)                      # torch's runtime first, then libnusi (as bench.py does)
    # world 1: an in-process store (no TCP rendezvous port to race other processes for)
    dist.init_process_group("nccl", store=dist.HashStore(), rank=0, world_size=1, device_id=torch.device("cuda", 0))
    import nusiprop_amd as nu
    from nusiprop_amd import dist as ndist, scan
    pts = scan.c4_points(n_mphi=4, n_g=3, N_bins_E=100) + [dict(p, si=2.2) for p in scan.c4_points(n_mphi=2, n_g=2,
                                                                                                     N_bins_E=100)]
    p0 = pts[0]

    def evolve_block(block):
        plan = nu.Plan(p0["N_bins_E"], p0["lEmin"], p0["lEmax"], p0["zmax"], max_points=len(block))
        try:
            return plan.evolve(block)
        finally:
            plan.close()
    f, l = ndist.evolve_sharded(pts, evolve_block)
    rf, rl = evolve_block(pts)
    ok = bool(np.array_equal(f, rf) and np.array_equal(l, rl))
    t = torch.ones(1, device="cuda")
    dist.all_reduce(t)
    dist.barrier()
    print(json.dumps({"backend": dist.get_backend(), "world": dist.get_world_size(), "points": len(pts),
                      "bitexact": ok, "all_reduce": float(t.item()), "shape": list(f.shape)}), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()

"""Multi-GPU parameter scans: one process per GPU, a pure partition.

Propagations are independent, so rank r evolves the
contiguous block scan.shard(len(points), world, r) on its own GPU with its
own Plan and there is no collective on the data path.  The only
communication is the final gather of the fluxes to rank 0 (and a barrier
around timed regions).  Works with any torch.distributed backend: "nccl"
(RCCL over xGMI) on MI355X nodes, "gloo" in the CPU tests.
"""
import numpy as np

from . import scan


def local_block(n_points, group=None):
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    return scan.shard(n_points, world, rank)


def evolve_sharded(points, evolve_block, group=None, gather=True):
    """Evolve `points` across the ranks of `group`.

    evolve_block(pts) -> (flux, flux_fla), arrays [len(pts), 3, N] -- on a GPU
    rank this is Plan.evolve (nusiprop_amd.plan).  Returns the full
    (flux, flux_fla) in the input order on rank 0 (None elsewhere) when
    `gather`, else this rank's block and its [lo, hi).
    """
    import torch.distributed as dist
    lo, hi = local_block(len(points), group)
    if hi > lo:
        flux, fla = evolve_block(points[lo:hi])
        flux, fla = np.asarray(flux), np.asarray(fla)
    else:
        flux = fla = None
    if not gather:
        return flux, fla, (lo, hi)
    parts = [None] * dist.get_world_size(group) if dist.get_rank(group) == 0 else None
    dist.gather_object((lo, hi, flux, fla), parts, dst=0, group=group)
    if dist.get_rank(group) != 0:
        return None, None
    parts = sorted((p for p in parts if p[2] is not None), key=lambda p: p[0])
    assert [p[0] for p in parts] == sorted(p[0] for p in parts) and sum(p[1] - p[0] for p in parts) == len(points)
    return np.concatenate([p[2] for p in parts]), np.concatenate([p[3] for p in parts])

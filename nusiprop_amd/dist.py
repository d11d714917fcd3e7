"""Multi-GPU parameter scans: one process per GPU, a pure partition.

Propagations are independent, so rank r evolves the
contiguous block scan.shard_aligned(points, world, r) -- block ends on
table-group boundaries, so points that share Stage-A tables stay on one GPU --
with its own Plan on its own GPU, and there is no collective on the data path.
The only communication is the final gather of the fluxes to the group's first
rank (float64 tensors, one dist.gather per basis, blocks padded to the largest
one) and a barrier around timed regions.  Works with any torch.distributed
backend: "nccl" (RCCL over xGMI) on MI355X nodes -- the blocks are staged on
the rank's GPU -- and "gloo" in the CPU tests.
"""
import numpy as np

from . import scan


def local_block(points, group=None):
    """[lo, hi) of this rank: scan.shard_aligned over the ranks of `group`."""
    import torch.distributed as dist
    return scan.shard_aligned(points, dist.get_world_size(group), dist.get_rank(group))


def _dst(group):
    """Global rank of the group's rank 0 (gather's dst is a global rank)."""
    import torch.distributed as dist
    return 0 if group is None else dist.get_global_rank(group, 0)


def _gather_blocks(block, n_local, shape, group):
    """Gather every rank's [n_i, *shape] float64 block to the group's rank 0; returns the list of blocks
    in rank order there (None elsewhere).  Blocks are padded to the largest n_i for the collective."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" else torch.device("cpu")
    sizes = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(world)]
    dist.all_gather(sizes, torch.tensor([n_local], dtype=torch.int64, device=dev), group=group)
    sizes = [int(x.item()) for x in sizes]
    nmax = max(sizes)
    pad = torch.zeros((nmax,) + tuple(shape), dtype=torch.float64, device=dev)
    if n_local:
        pad[:n_local] = torch.as_tensor(np.ascontiguousarray(block), dtype=torch.float64).to(dev)
    me = dist.get_rank(group)
    bufs = [torch.empty_like(pad) for _ in range(world)] if me == 0 else None
    dist.gather(pad, bufs, dst=_dst(group), group=group)
    if me != 0:
        return None
    return [b[:n].cpu().numpy() for b, n in zip(bufs, sizes)]


def evolve_sharded(points, evolve_block, group=None, gather=True):
    """Evolve `points` across the ranks of `group`.

    evolve_block(pts) -> (flux, flux_fla), arrays [len(pts), 3, N] -- on a GPU
    rank this is Plan.evolve (nusiprop_amd.plan).  Returns the full
    (flux, flux_fla) in the input order on the group's rank 0 (None, None
    elsewhere) when `gather`, else this rank's block and its [lo, hi).
    """
    import torch.distributed as dist
    lo, hi = local_block(points, group)
    N = int(points[0]["N_bins_E"]) if points else 0
    if hi > lo:
        flux, fla = evolve_block(points[lo:hi])
        flux, fla = np.asarray(flux, dtype=np.float64), np.asarray(fla, dtype=np.float64)
    else:
        flux = fla = np.zeros((0, 3, N))
    if not gather:
        return flux, fla, (lo, hi)
    parts_f = _gather_blocks(flux, hi - lo, (3, N), group)
    parts_l = _gather_blocks(fla, hi - lo, (3, N), group)
    if dist.get_rank(group) != 0:
        return None, None
    out_f, out_l = np.concatenate(parts_f), np.concatenate(parts_l)
    assert len(out_f) == len(points)
    return out_f, out_l

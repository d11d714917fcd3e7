"""Host logic of the scan path: grids, the rank partition, the packed alpha
layout, and the multi-process (world_size 2, gloo) sharded evolve + gather.

On CPU the per-rank evolve is the oracle (a stand-in for the rank's GPU
Plan.evolve, which tests/test_gpu_parity.py covers); what is tested here is
the partition and gather logic of nusiprop_amd/dist.py that bench.py and
users run with RCCL on MI355X nodes."""
import os
import socket

import numpy as np
import pytest

from nusiprop_amd import scan


def test_c4_c5_grids():
    c4, c5 = scan.c4_points(), scan.c5_points()
    assert len(c4) == 1024 and len(c5) == 65536
    assert len({(p["mphi"], p["g"]) for p in c4}) == 1024
    assert len({(p["mphi"], p["g"], p["si"]) for p in c5}) == 65536
    assert len({(p["mphi"], p["g"]) for p in c5}) == 4096      # 4096 unique tables, 16 gammas each
    assert all(p["N_bins_E"] == 300 and p["source_model"] == 1 for p in c4)


@pytest.mark.parametrize("n,world", [(1024, 8), (65536, 8), (7, 2), (3, 4), (0, 2)])
def test_shard_partition(n, world):
    blocks = [scan.shard(n, world, r) for r in range(world)]
    assert blocks[0][0] == 0 and blocks[-1][1] == n
    assert all(blocks[r][1] == blocks[r + 1][0] for r in range(world - 1))
    sizes = [hi - lo for lo, hi in blocks]
    assert max(sizes) - min(sizes) <= 1


def test_cascade_bytes_formula():
    """~17.7 MB per propagation at N=300 (16.9 MB of alpha reads)."""
    b = scan.cascade_bytes_per_point(300, 48)
    assert abs(b / 1e6 - 17.7) < 0.1
    assert abs(8 * 47 * 300 * 299 / 2 / 1e6 - 16.9) < 0.1
    assert scan.alpha_entries_per_point(300, 48) == 346 * 345 // 2


def test_unpack_alpha_layout():
    from nusiprop_amd import unpack_alpha
    T = 9
    packed = np.arange(T * (T - 1) // 2, dtype=np.float64)
    A = unpack_alpha(packed, T)
    for m in range(T):
        for n in range(m):
            assert A[n, m] == m * (m - 1) // 2 + n
    assert np.all(np.tril(A) == 0)


def test_params_array_roundtrip():
    from nusiprop_amd import _lib
    from nusiprop_amd.plan import params_array
    pts = scan.c4_points()[:3]
    arr = params_array(pts)
    assert len(arr) == 3 and arr[1].mphi == pts[1]["mphi"] and arr[2].g == pts[2]["g"]
    assert arr[0].source_model == _lib.SOURCE_POWER_LAW and arr[0].N_bins_E == 300


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _oracle_block(pts):
    from oracle import oracle
    out_f, out_l = [], []
    for p in pts:
        kw = dict(p)
        kw["source"] = kw.pop("source_model")
        f, l = oracle.Oracle(**kw).evolve()
        out_f.append(f)
        out_l.append(l)
    return np.array(out_f), np.array(out_l)


def _worker(rank, world, port, pts, q, sub=None):
    import torch.distributed as dist
    from nusiprop_amd import dist as ndist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        group = dist.new_group(sub) if sub else None
        if sub and rank not in sub:
            q.put((rank, None, None, "outside"))
            return
        lo, hi = ndist.local_block(pts, group)
        flux, fla = ndist.evolve_sharded(pts, _oracle_block, group=group)
        q.put((rank, lo, hi, None if flux is None else (flux, fla)))
    finally:
        dist.destroy_process_group()


def _run(world, pts, sub=None):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, pts, q, sub)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


def test_sharded_evolve_gloo_world2(oracle_mod):
    pts = scan.c4_points(n_mphi=3, n_g=2, N_bins_E=24)           # 6 small points, 6 tables
    res = _run(2, pts)
    assert [(r[1], r[2]) for r in res] == [(0, 3), (3, 6)]
    flux, fla = res[0][3]
    assert res[1][3] is None
    ref_f, ref_l = _oracle_block(pts)
    assert np.array_equal(flux, ref_f) and np.array_equal(fla, ref_l)


def _gamma_groups(sizes, N=20):
    """Consecutive gamma-batches (points sharing one table) of the given sizes."""
    pts = []
    for j, n in enumerate(sizes):
        pts += [dict(scan.BASE, N_bins_E=N, mphi=6e5 * (1 + j), g=0.02, si=2.0 + 0.1 * s) for s in range(n)]
    return pts


@pytest.mark.parametrize("sizes,world", [((5, 5, 5, 5), 3), ((16,) * 3 + (7,), 3), ((3, 1, 4, 1, 5), 4), ((2, 2, 1, 3), 3)])
def test_shard_aligned_keeps_table_groups(sizes, world):
    """Groups no larger than half a block stay whole, each cut at the group boundary nearest the even split."""
    pts = _gamma_groups(sizes)
    blocks = [scan.shard_aligned(pts, world, r) for r in range(world)]
    assert blocks[0][0] == 0 and blocks[-1][1] == len(pts)
    assert all(blocks[r][1] == blocks[r + 1][0] for r in range(world - 1))
    bounds = set(scan.group_bounds(pts))
    for lo, hi in blocks:
        assert lo in bounds and hi in bounds           # no table group is split
    # each cut is the group boundary nearest to the even split
    for r in range(1, world):
        ideal = r * len(pts) / world
        assert abs(blocks[r][0] - ideal) == min(abs(b - ideal) for b in bounds)


@pytest.mark.parametrize("sizes,world", [((64,), 4), ((64,), 8), ((2,), 3), ((40, 2, 2), 4), ((100, 3), 2)])
def test_shard_aligned_splits_large_groups(sizes, world):
    """A group much larger than a block (a pure spectral-index scan shares one table) is split at the even
    cuts, so no GPU idles: every block is within half a block of n / world, and the blocks tile the scan."""
    pts = _gamma_groups(sizes)
    n = len(pts)
    blocks = [scan.shard_aligned(pts, world, r) for r in range(world)]
    assert blocks[0][0] == 0 and blocks[-1][1] == n
    assert all(blocks[r][1] == blocks[r + 1][0] for r in range(world - 1))
    for lo, hi in blocks:
        assert abs((hi - lo) - n / world) <= n / world / 2.0 + 1
    if sizes == (64,):
        assert all(hi - lo == 64 // world for lo, hi in blocks)


def test_sharded_evolve_gloo_world3_uneven_groups(oracle_mod):
    """World 3 over 4 gamma-batches of 5 (20 points, no multiple of 3): groups stay whole, the gather
    (padded float64 blocks) returns every flux bit-exact in input order."""
    pts = _gamma_groups((5, 5, 5, 5))
    res = _run(3, pts)
    assert [(r[1], r[2]) for r in res] == [(0, 5), (5, 15), (15, 20)]
    flux, fla = res[0][3]
    assert res[1][3] is None and res[2][3] is None
    ref_f, ref_l = _oracle_block(pts)
    assert np.array_equal(flux, ref_f) and np.array_equal(fla, ref_l)


def test_sharded_evolve_subgroup_of_world4(oracle_mod):
    """A 2-rank subgroup {1, 2} of a 4-rank world: the gather goes to the subgroup's first rank
    (global rank 1), which gets the full result."""
    pts = scan.c4_points(n_mphi=2, n_g=2, N_bins_E=20)
    res = _run(4, pts, sub=[1, 2])
    assert res[0][3] == "outside" and res[3][3] == "outside"
    assert [(r[1], r[2]) for r in res[1:3]] == [(0, 2), (2, 4)]
    flux, fla = res[1][3]
    assert res[2][3] is None
    ref_f, ref_l = _oracle_block(pts)
    assert np.array_equal(flux, ref_f) and np.array_equal(fla, ref_l)

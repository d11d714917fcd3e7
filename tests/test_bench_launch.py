"""bench.py's multi-GPU launch path (the driver's N = 1, 2, 4, 8 scaling runs): `--gpus N` without a launcher
starts N rank processes itself (torch.distributed.run, before any GPU call) and the line reports the ranks that
actually ran; a rank count that differs from --gpus is an error.  --dry-run exercises the launch, rendezvous and
max-over-ranks reduction on CPU (gloo) without GPU work."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(args, env=None, timeout=300):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, cwd=ROOT, env=e,
                          capture_output=True, text=True, timeout=timeout)


def _line(out):
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout + out.stderr
    return json.loads(lines[0])


def test_gpus2_launches_two_ranks():
    out = _bench(["--gpus", "2", "--dry-run", "--steps", "3", "--warmup", "0"])
    assert out.returncode == 0, out.stderr
    j = _line(out)
    assert j["n_gpus"] == 2 and j["ranks_reporting"] == 2 and j["dry_run"] and j["value"] is None
    assert "launching 2 ranks" in out.stderr


def test_single_gpu_runs_in_process():
    out = _bench(["--dry-run", "--steps", "2", "--warmup", "0"])
    assert out.returncode == 0, out.stderr
    j = _line(out)
    assert j["n_gpus"] == 1 and j["ranks_reporting"] == 1
    assert "launching" not in out.stderr


def test_rank_count_mismatch_is_an_error():
    out = _bench(["--gpus", "4", "--dry-run"], env={"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert out.returncode != 0 and "WORLD_SIZE=2" in out.stderr
    assert not [l for l in out.stdout.splitlines() if l.startswith("{")]


def test_gpus0_is_an_error():
    """--gpus 0 is rejected, never run as a one-GPU line."""
    out = _bench(["--gpus", "0", "--dry-run"])
    assert out.returncode != 0 and "--gpus must be >= 1" in out.stderr
    assert not [l for l in out.stdout.splitlines() if l.startswith("{")]


def test_parity_sample_and_rel_err():
    """The bench line's parity sample (parity_indices) is deterministic and includes the strongest-coupling column;
    rel_err follows tests/cases.py (exact zeros required)."""
    import argparse
    import numpy as np
    sys.path.insert(0, ROOT)
    import bench
    from nusiprop_amd import scan
    pts = scan.c4_points()
    a = bench.parity_indices(argparse.Namespace(workload="c4"), pts)
    assert a == bench.parity_indices(argparse.Namespace(workload="c4"), pts) and len(a) == 32 == len(set(a))
    assert sum(1 for i in a if pts[i]["g"] == 1.0) == 16
    assert bench.rel_err([1.0, 0.0], [1.0, 0.0]) == 0.0 and bench.rel_err([1.0, 1e-300], [1.0, 0.0]) == float("inf")
    assert abs(bench.rel_err(np.array([1.0 + 1e-12]), np.array([1.0])) - 1e-12) < 1e-15


def test_c5_dry_run_world8_is_one_scan_partition():
    """`--gpus 8 --workload c5` partitions the 65 536-point BASELINE config-5 scan with
    scan.shard_aligned (the function dist.evolve_sharded uses): the eight blocks cover every point exactly once, in
    order, 8192 per GPU, and no gamma batch (16 points sharing a Stage-A table) is split; strong scaling."""
    out = _bench(["--gpus", "8", "--dry-run", "--workload", "c5", "--steps", "1", "--warmup", "0"], timeout=600)
    assert out.returncode == 0, out.stderr
    s = _line(out)["shard_check"]
    assert s["points"] == 65536 and s["covered_once"] and s["in_order"] and s["table_groups_split"] == 0
    assert [b - a for a, b in s["blocks"]] == [8192] * 8 and s["scaling"] == "strong"


def test_c5_dry_run_uneven_world_keeps_gamma_batches():
    """Three ranks: 65 536 / 3 is not a multiple of the 16-point gamma batches; the block ends move to batch
    boundaries (no batch split), every point still covered once."""
    out = _bench(["--gpus", "3", "--dry-run", "--workload", "c5", "--steps", "1", "--warmup", "0"], timeout=600)
    assert out.returncode == 0, out.stderr
    s = _line(out)["shard_check"]
    assert s["covered_once"] and s["in_order"] and s["table_groups_split"] == 0
    assert all((b - a) % 16 == 0 for a, b in s["blocks"])


def test_c4_dry_run_world2_weak_blocks():
    """C4 on N GPUs is one scan of 1024 N points (the config-4 grid once per GPU at gamma = 2.5 + 0.05 b), each rank
    one 1024-point block: weak scaling, every point covered once."""
    out = _bench(["--gpus", "2", "--dry-run", "--workload", "c4", "--steps", "1", "--warmup", "0"])
    assert out.returncode == 0, out.stderr
    s = _line(out)["shard_check"]
    assert s["points"] == 2048 and s["covered_once"] and s["blocks"] == [[0, 1024], [1024, 2048]]
    assert s["scaling"] == "weak"


def test_pmc_summary_must_match_library_and_table_order(tmp_path):
    """bench.py prices the dominant kernel's roofline with a committed PMC summary only when that summary was
    collected on the loaded library (sha256) in the table arithmetic the run times (table_order): a summary of the
    other arithmetic, of another binary, or without an order is dropped with a note, so no roofline/traffic comes
    from it (the shared-order line had been priced with the reference order's flop count)."""
    sys.path.insert(0, ROOT)
    import bench
    sha = "ab" * 32
    good = {"libnusi_sha256": sha, "table_order": "reference", "k_alpha_fp64_flops_per_step": 2.6e11,
            "k_alpha_hbm_bytes_per_step": 3e10}
    p = tmp_path / "pmc.json"
    p.write_text(json.dumps(good))
    pmc, src, note = bench.load_pmc(str(p), sha, "reference")
    assert pmc["k_alpha_fp64_flops_per_step"] == 2.6e11 and note is None and src
    pmc, _, note = bench.load_pmc(str(p), sha, "shared")          # the other arithmetic
    assert pmc == {} and "table order" in note
    pmc, _, note = bench.load_pmc(str(p), "cd" * 32, "reference")  # another binary
    assert pmc == {} and "not the loaded" in note
    p.write_text(json.dumps(dict(good, table_order=None)))          # a summary that does not say its order
    assert bench.load_pmc(str(p), sha, "reference")[0] == {}
    assert bench.load_pmc(str(tmp_path / "missing.json"), sha, "reference") == ({}, None, None)
    assert bench.pmc_summary_path("c4", True).endswith("profiles/pmc_traffic_c4.json")
    assert bench.pmc_summary_path("c4", False).endswith("profiles/pmc_traffic_c4_shared.json")

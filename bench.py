#!/usr/bin/env python3
"""bench.py -- full propagations/s of the MI355X nuSIprop solver (BASELINE.json metric).

A step = one calculate_flux::evolve() (nuSIprop.hpp:176-337: Stage-A tables +
cascade + finalisation) for every point of the rank's batch, on its GPU, with
inputs and outputs resident in HBM.  Default workload = BASELINE config 4
(1024-point (mphi, g) scan, N_E = 300, power-law source, every point building
its own tables) per GPU; with N GPUs each rank evolves its own 1024 points
(weak scaling, gamma shifted per rank so every rank's points are distinct), no
collective on the data path.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c4|c5|c2] [--points P]
Multi-GPU: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

Prints one JSON line (rank 0) with roofline (the dominant alpha-table kernel, fp64 VALU),
roofline_cascade (the metric's cascade HBM GB/s) and the
cpu_baseline (the C oracle, single thread, bounded sample).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "full propagations/sec at N_E=300, 1 & 8 GPU; achieved HBM GB/s on cascade kernel"
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
FP64_PEAK_TFLOPS = 78.6        # MI355X fp64 vector spec


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", default="c4", choices=["c4", "c5", "c2", "c3"])
    ap.add_argument("--points", type=int, default=0, help="points per GPU (default: 1024 for c4 and c3, 8192 for c5, 1 for c2)")
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="budget of the oracle CPU baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cascade", default="mfma", choices=["mfma", "wf", "auto"],
                    help="cascade kernel: mfma = wavefront with the push on the fp64 matrix cores (default, "
                         "fastest measured), wf = the bit-exact wavefront kernel, auto = the library's choice")
    ap.add_argument("--traffic-json", default="",
                    help="per-launch HBM bytes / fp64 VALU work from rocprofv3 --pmc passes (scripts/pmc_summary.py); "
                         "default for the default workload: the committed profiles/pmc_traffic_latest.json")
    return ap.parse_args()


def rank_points(args, rank, world):
    from nusiprop_amd import scan
    if args.workload == "c2":
        pts = [dict(scan.BASE, mphi=6e5, g=0.01, si=2.5, norm=6.0)]
        return pts * max(1, args.points or 1), "C2b: single propagation, N_E=300, lE 12->17, power-law source, test.cpp physics"
    import numpy as np
    if args.workload == "c3":   # BASELINE config 3: N_E = 1200, lE 10 -> 17, phi-phi on (synthetic tables)
        P = args.points or 1024
        base = dict(scan.BASE, mphi=1e5, g=0.05, N_bins_E=1200, lEmin=10.0, lEmax=17.0, phiphi=True)
        pts = [dict(base, g=float(g), si=2.5 + 0.05 * rank) for g in np.logspace(-2.0, -0.5, P)]
        return pts, ("C3: %d-point g scan per GPU at m_phi=1e5, N_E=1200, lE 10->17, phi-phi on (synthetic values on "
                     "the reference's exact table axes and dims {5000,100} / {1000,1000,100}, 400 MB float32 in HBM; "
                     "nusiprop_amd.phiphi_tables), power-law source" % P)
    if args.workload == "c4":
        P = args.points or 1024
        pts = scan.c4_points(si=2.5 + 0.05 * rank)
        desc = "C4: (m_phi 32 x g 32) scan per GPU, N_E=300, lE 12->17, power-law source, gamma=2.5+0.05*rank"
    else:
        P = args.points or 8192
        allp = scan.c5_points()
        lo = (rank * P) % len(allp)
        pts = (allp + allp)[lo:lo + P]
        desc = ("C5: a %d-point block per GPU of the 65536-point (m_phi 64 x g 64 x gamma 16) scan, N_E=300, "
                "power-law source; %d distinct tables per block (gamma batches share them)" % (P, P // 16))
    while len(pts) < P:
        pts = pts + pts
    return pts[:P], desc


def cpu_baseline(pts, budget_s):
    """The C oracle (single thread) on the first points of the same workload until the budget is spent."""
    from oracle import oracle
    oracle.build()
    n, t0 = 0, time.perf_counter()
    for p in pts:
        kw = dict(p)
        kw["source"] = kw.pop("source_model")
        o = oracle.Oracle(**kw)
        o.evolve()
        n += 1
        if time.perf_counter() - t0 > budget_s:
            break
    dt = time.perf_counter() - t0
    return {"value": n / dt, "unit": "propagations/s", "cores": 1, "kind": "port",
            "sample": "%d full propagations (first points of the same workload), single-threaded C oracle, %.1f s" % (n, dt)}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(local)
    import nusiprop_amd as nu
    from nusiprop_amd import scan

    pts, desc = rank_points(args, rank, world)
    P = len(pts)
    p0 = pts[0]
    plan = nu.Plan(p0["N_bins_E"], p0["lEmin"], p0["lEmax"], p0["zmax"], max_points=P, device=local)
    if any(p.get("phiphi") for p in pts):
        import shutil
        import tempfile
        from nusiprop_amd.phiphi_tables import write_synthetic_tables
        tdir = tempfile.mkdtemp(prefix="nusi_phiphi_")
        at, atd, a, ad = write_synthetic_tables(tdir)     # the reference's geometry (1.6 GB of records)
        plan.load_phiphi(at, a)                           # dims = NULL: {5000,100}, {1000,1000,100}
        shutil.rmtree(tdir, ignore_errors=True)
    arr = plan.params_array(pts)
    from nusiprop_amd import _lib
    plan.set_cascade({"mfma": _lib.CASCADE_MFMA, "wf": _lib.CASCADE_WAVEFRONT, "auto": _lib.CASCADE_AUTO}[args.cascade])
    casc_kernel = {"mfma": "k_cascade_wf_mfma", "wf": "k_cascade_wf", "auto": "k_cascade_wf"}[args.cascade]
    dev = torch.device("cuda", local)
    flux = torch.empty((P, 3, plan.N), dtype=torch.float64, device=dev)
    fla = torch.empty((P, 3, plan.N), dtype=torch.float64, device=dev)
    stream = torch.cuda.current_stream().cuda_stream

    def barrier():
        if dist is not None:
            dist.barrier()

    for _ in range(args.warmup):
        plan.evolve_device(arr, flux.data_ptr(), fla.data_ptr(), stream)
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    plan.profile_begin(args.steps)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        plan.evolve_device(arr, flux.data_ptr(), fla.data_ptr(), stream)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    barrier()
    dt = t1 - t0
    if dist is not None:
        tt = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    sum_ms, ncalls = plan.profile_end()
    bad = int(torch.isnan(fla).sum().item()) + int((fla < 0).sum().item())
    # a phi-phi lookup outside the table nodes (the reference's exit(1), interp.hpp:355-361) is flagged per
    # point by the kernels; the async evolve does not raise, so count them here
    oob = sum(1 for w in plan.warnings(P) if w & 8)

    N, Nz = plan.N, plan.Nz
    if not scan.cascade_mfma_flops_per_point(N, Nz):   # grid beyond the wavefront kernels (Nz-1 > 48): per-step chain
        casc_kernel, args.cascade = "k_cascade_reg", "reg"
    props = world * P * args.steps
    value = props / dt
    casc_bytes = scan.cascade_bytes_per_point(N, Nz) * P
    casc_s = sum_ms[2] / max(ncalls, 1) / 1e3
    alpha_s = sum_ms[1] / max(ncalls, 1) / 1e3
    traffic, tsrc, pmc = None, None, {}
    tj = args.traffic_json
    if not tj and args.workload == "c4" and not args.points:
        tj = os.path.join(ROOT, "profiles", "pmc_traffic_latest.json")
    if tj and os.path.exists(tj):
        with open(tj) as fh:
            pmc = json.load(fh)
        traffic = pmc.get("k_cascade_bytes_per_launch")
        tsrc = os.path.relpath(tj, ROOT)
    achieved = casc_bytes / casc_s / 1e9
    casc_min = scan.cascade_min_bytes_per_point(N, Nz) * P
    step_ms = sum(sum_ms) / max(ncalls, 1)
    out = {
        "metric": METRIC,
        "value": value,
        "unit": "propagations/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": dt / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (deterministic scan grid; power-law source)",
        "config": {"workload": desc, "N_E": N, "N_z": Nz, "points_per_gpu": P, "lEmin": p0["lEmin"],
                   "lEmax": p0["lEmax"], "parallelism": "independent points, %d GPU(s), no collective" % world},
        "stage_ms_per_step": {"gamma_alphatilde": sum_ms[0] / max(ncalls, 1), "alpha": sum_ms[1] / max(ncalls, 1),
                              "cascade": sum_ms[2] / max(ncalls, 1)},
        "alpha_table": {"kernel": "k_alpha_tile", "bound": "fp64 VALU (transcendental)",
                        "entries_per_s": scan.alpha_entries_per_point(N, Nz) * P / alpha_s,
                        "avg_step_ms": alpha_s * 1e3, "share_of_step": alpha_s * 1e3 / step_ms},
        # the metric's "achieved HBM GB/s on the cascade kernel".  The wavefront kernel reads each alpha column
        # once per point, so its algorithmic bytes are cascade_min_bytes_per_point (PMC traffic agrees);
        # SURVEY.md sec. 8d's figure (every step re-reading its alpha window, the reference's access pattern)
        # over the same time is reported beside it as reference_pattern_gbs
        "roofline_cascade": {"bound": "hbm", "kernel": casc_kernel, "achieved": casc_min / casc_s / 1e9,
                             "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": casc_min / casc_s / 1e9 / HBM_PEAK_GBS,
                             "traffic": traffic, "traffic_source": tsrc, "algorithmic_bytes_per_launch": casc_min,
                             "reference_pattern_bytes_per_launch": casc_bytes, "reference_pattern_gbs": achieved,
                             "avg_launch_ms": casc_s * 1e3,
                             "note": "not HBM-bound: T = N+Nz-2 dependent stages per point (LDS/barrier latency)"},
        "invalid_outputs": bad,
        "phiphi_lookups_out_of_range": oob,
    }
    if args.cascade == "mfma":   # the push on the fp64 matrix cores: issued MFMA flops over the kernel's time
        mf = scan.cascade_mfma_flops_per_point(N, Nz) * P
        out["roofline_cascade"]["mfma"] = {"flops_per_launch": mf, "achieved": mf / casc_s / 1e12,
                                           "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                                           "frac": mf / casc_s / 1e12 / FP64_PEAK_TFLOPS,
                                           "note": "v_mfma_f64_16x16x4f64 rank-4 pushes (scan.cascade_mfma_flops_per_point)"}
    fl = pmc.get("k_alpha_fp64_flops_per_step")
    if fl:   # the dominant kernel: executed fp64 VALU flops (PMC counts) per second vs the fp64 vector peak
        ach = fl / alpha_s / 1e12
        out["roofline"] = {"bound": "valu", "kernel": "k_alpha_tile", "achieved": ach, "peak": FP64_PEAK_TFLOPS,
                           "unit": "TFLOP/s", "frac": ach / FP64_PEAK_TFLOPS,
                           "traffic": pmc.get("k_alpha_hbm_bytes_per_step"), "traffic_source": tsrc,
                           "flops": "executed fp64 VALU (SQ_INSTS_VALU_{ADD,MUL,TRANS}_F64 + 2 FMA) x 64 lanes, "
                                    "from the PMC pass; time = the kernel's HIP events in this run",
                           "note": "dominant kernel (alpha_table.share_of_step); fp64 vector-ALU bound "
                                   "(transcendental leaves), neither HBM nor MFMA"}
    else:
        out["roofline"] = dict(out["roofline_cascade"])
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(pts, args.cpu_seconds)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""bench.py -- full propagations/s of the MI355X nuSIprop solver (BASELINE.json metric).

A step = one calculate_flux::evolve() (nuSIprop.hpp:176-337: Stage-A tables +
cascade + finalisation) for every point of the rank's batch, on its GPU, with
inputs and outputs resident in HBM.  Default workload = BASELINE config 4
(1024-point (mphi, g) scan, N_E = 300, power-law source, every point building
its own tables) per GPU; with N GPUs each rank evolves its own 1024 points
(weak scaling, gamma shifted per rank so every rank's points are distinct), no
collective on the data path.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c4|c5|c3|c2|c1] [--points P]
Multi-GPU: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N, or plain
`python bench.py --gpus N`, which starts that launcher itself (N fresh rank processes, before any GPU
call here) and exits with its status; a rank count that differs from --gpus is an error.

Prints one JSON line (rank 0) with roofline (the dominant alpha-table kernel, fp64 VALU),
roofline_cascade (the metric's cascade HBM GB/s) and the cpu_baseline (the C oracle on a
thread pool over the host cores the job may use, bounded sample, Stage A / Stage B timed
apart on one core).  c2 / c1 (single propagations) add the latency of one evolve() through
the object API (nusi_evolve, host I/O included) beside the 1-point plan's device-resident rate.
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
    ap.add_argument("--gpus", type=int, default=None, help="GPUs = ranks (default: WORLD_SIZE, else 1)")
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default="c4", choices=["c4", "c5", "c3", "c2", "c1", "c4s"],
                    help="c4s: the opt-in shift-reuse scan mode (NUSI_OPT_SHIFT_REUSE = 128) on a C4-sized scan whose "
                         "m_phi lie on the table axis' r^(-o/2) lattice; not the headline (its fluxes are held to 1e-9, "
                         "not bit-exact tables)")
    ap.add_argument("--points", type=int, default=0, help="points per GPU (default: 1024 for c4 and c3, 8192 for c5, 1 for c2)")
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="budget of the oracle CPU baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-secondary", action="store_true",
                    help="skip the C5 and C3 lines the default C4 run adds (secondary_lines: each its own child "
                         "process, a few steps, after the timed region)")
    ap.add_argument("--cascade", default="auto", choices=["auto", "mfma", "wf"],
                    help="cascade kernel: auto = the library default (= mfma: the warp-specialised wavefront with "
                         "the push on the fp64 matrix cores), wf = the bit-exact scalar wavefront")
    ap.add_argument("--rhs", type=int, default=0,
                    help="NUSI_OPT_CASCADE_RHS: 0 = the library default, 1 = one point per cascade workgroup, 2 = pairs "
                         "of points sharing a table, 3..16 = the gamma batch k_cascade_gb")
    ap.add_argument("--dry-run", action="store_true",
                    help="launch / rank / reduction plumbing only, no GPU work (gloo; CPU tests): prints the JSON "
                         "line with value null")
    ap.add_argument("--traffic-json", default="",
                    help="per-launch HBM bytes / fp64 VALU work from rocprofv3 --pmc passes (scripts/pmc_summary.py); "
                         "default: the committed profiles/pmc_traffic_<workload>.json, used only if its libnusi_sha256 matches the loaded library")
    return ap.parse_args()


def rank_points(args, rank, world):
    from nusiprop_amd import scan
    if args.workload == "c2":
        pts = [dict(scan.BASE, mphi=6e5, g=0.01, si=2.5, norm=6.0)]
        return pts * max(1, args.points or 1), "C2b: single propagation, N_E=300, lE 12->17, power-law source, test.cpp physics"
    if args.workload == "c1":   # test.cpp:6-23 verbatim (N_E = 100, lE 9 -> 14, DSNB source)
        pts = [dict(scan.C1)]
        return pts * max(1, args.points or 1), "C1: test.cpp single propagation (N_E=100, lE 9->14, DSNB source, phiphi off)"
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
    elif args.workload == "c4s":
        P = args.points or 1024
        pts = scan.c4s_points(si=2.5 + 0.05 * rank)
        desc = ("C4s (opt-in NUSI_OPT_SHIFT_REUSE=128): (m_phi 32 on the r^(-o/2) lattice, o = 0, 4, .., 124 below "
                "10^6.533 x g 32) scan per GPU, N_E=300, lE 12->17, power-law source; one base table set per g")
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


def host_cores():
    """Threads the job may use on this host: the affinity mask, capped by OMP_NUM_THREADS when it is set (the
    GPU box sets it to its CPU share), plus what the machine reports."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    cap = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    model = ""
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    used = min(aff, cap) if cap > 0 else aff
    note = ("capped by OMP_NUM_THREADS=%d (the GPU box's CPU share) of %d CPUs in the affinity mask, nproc %s"
            % (cap, aff, os.cpu_count())) if 0 < cap < aff else "the whole affinity mask (%d CPUs)" % aff
    return used, {"nproc": os.cpu_count(), "affinity": aff, "OMP_NUM_THREADS": cap or None, "cpu_model": model,
                  "cores_note": note}


def _oracle(p):
    from oracle import oracle
    kw = dict(p)
    kw["source"] = kw.pop("source_model")
    return oracle.Oracle(**kw)


def cpu_baseline(pts, budget_s):
    """The C oracle (test infrastructure, the reference's algorithm restated) on a bounded sample of the same
    workload: Stage A (tables) and Stage B (cascade) timed apart on one core for a quarter of the budget, then
    whole evolve()s on a thread pool over the host cores for the rest (ctypes releases the GIL, the oracle has
    no global state).  value = the pool's propagations/s."""
    import concurrent.futures as cf
    import threading
    from oracle import oracle
    oracle.build()
    threads, host = host_cores()
    # one core, stages apart
    ta = tb = 0.0
    n1, t0 = 0, time.perf_counter()
    for p in pts:
        o = _oracle(p)
        t1 = time.perf_counter()
        G, At, A = o.tables()
        t2 = time.perf_counter()
        o.cascade(G, At, A)
        t3 = time.perf_counter()
        ta += t2 - t1
        tb += t3 - t2
        n1 += 1
        if t3 - t0 > budget_s / 4:
            break
    # the pool: worker k evolves points k, k + threads, ... until the deadline
    deadline = time.perf_counter() + budget_s * 3 / 4
    done = [0] * threads
    lock = threading.Lock()

    def work(k):
        i = k
        while time.perf_counter() < deadline:
            _oracle(pts[i % len(pts)]).evolve()
            with lock:
                done[k] += 1
            i += threads
    t0 = time.perf_counter()
    with cf.ThreadPoolExecutor(threads) as ex:
        list(ex.map(work, range(threads)))
    dt = time.perf_counter() - t0
    n = sum(done)
    return {"value": n / dt, "unit": "propagations/s", "cores": threads, "cores_note": host["cores_note"],
            "kind": "port",
            "sample": "%d full propagations of the same workload (points cycled from the first) on a %d-thread pool "
                      "of the single-threaded C oracle, %.1f s" % (n, threads, dt),
            "host": host,
            "single_core": {"propagations": n1, "value": n1 / (ta + tb), "stage_a_ms_per_prop": ta / n1 * 1e3,
                            "stage_b_ms_per_prop": tb / n1 * 1e3,
                            "note": "Stage A = Gamma/alphaTilde/alpha tables (nuSIprop.hpp:217-253), Stage B = "
                                    "cascade + finalise (:255-336), first points of the workload, one thread"}}


def c1_cpu_lines(budget_s):
    """test.cpp (C1) on the oracle at its own N_E = 100 and at N_E = 300 (lE 9 -> 14), one core each."""
    from nusiprop_amd import scan
    out = {}
    for N in (100, 300):
        p = dict(scan.C1, N_bins_E=N)
        n, t0 = 0, time.perf_counter()
        while True:
            _oracle(p).evolve()
            n += 1
            if time.perf_counter() - t0 > budget_s:
                break
        dt = time.perf_counter() - t0
        out["N_E=%d" % N] = {"ms_per_prop": dt / n * 1e3, "propagations": n, "cores": 1}
    return out


def single_point_latency(pt, reps):
    """One evolve() through the object API (nusi_create / nusi_evolve: host parameters in, tables and cascade
    on the GPU, fluxes copied to the host) -- the reference's own usage, calculate_flux::evolve() per object."""
    import ctypes
    from nusiprop_amd import _lib
    L = _lib.load()
    p = dict(pt)
    src = p.pop("source_model")
    h = ctypes.c_void_p()
    _lib.check(L.nusi_create(ctypes.byref(_lib.make_params(source_model=src, **p)), ctypes.byref(h)))
    try:
        out = (ctypes.c_double * (3 * p["N_bins_E"]))()
        for _ in range(3):
            _lib.check(L.nusi_evolve(h))
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            _lib.check(L.nusi_evolve(h))
            _lib.check(L.nusi_get_flux_fla(h, out))
            ts.append(time.perf_counter() - t0)
    finally:
        L.nusi_destroy(h)
    ts.sort()
    return {"median_ms": ts[len(ts) // 2] * 1e3, "min_ms": ts[0] * 1e3, "reps": reps,
            "path": "nusi_create + nusi_evolve + nusi_get_flux_fla (object API, host I/O and sync included)"}


def free_port():
    import socket
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    return port


def launch_ranks(args):
    """--gpus N > 1 without a launcher: start N rank processes with torch.distributed.run (one per GPU, RCCL
    rendezvous on 127.0.0.1) -- before anything here has touched the GPU -- and return their exit status.  A
    rank count that differs from --gpus is an error, never an N-GPU label on a different run."""
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is not None:
        if args.gpus is not None and int(world_env) != args.gpus:
            sys.exit("bench.py: --gpus %d but WORLD_SIZE=%s ranks were launched" % (args.gpus, world_env))
        return None
    if not args.gpus or args.gpus == 1:
        return None
    if args.gpus < 1:
        sys.exit("bench.py: --gpus must be >= 1")
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(args.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    print("bench.py: launching %d ranks: %s" % (args.gpus, " ".join(cmd)), file=sys.stderr, flush=True)
    return subprocess.call(cmd)


def secondary_lines(local):
    """BASELINE configs 5 and 3 measured beside the headline C4 line, each by a child bench.py process on the same
    GPU after the C4 timed region (so the driver's run records them too): props/s, stage times, kernels."""
    import subprocess
    out = {}
    env = dict(os.environ, HIP_VISIBLE_DEVICES=os.environ.get("HIP_VISIBLE_DEVICES", str(local)))
    for wl, steps in (("c5", 10), ("c3", 3)):
        cmd = [sys.executable, os.path.abspath(__file__), "--workload", wl, "--steps", str(steps), "--warmup", "1",
               "--no-cpu-baseline", "--no-secondary"]
        try:
            r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env)
            d = json.loads(r.stdout.strip().splitlines()[-1])
            out[wl] = {k: d.get(k) for k in ("value", "unit", "ms_per_step", "steps", "stage_ms_per_step")}
            out[wl]["workload"] = d["config"]["workload"]
            out[wl]["kernels"] = [d["config"]["alpha_kernel"], d["config"]["cascade_kernel"]]
            out[wl]["roofline"] = {k: d["roofline"].get(k) for k in ("kernel", "achieved", "unit", "frac", "traffic")}
        except Exception as e:   # a secondary line never fails the headline run
            out[wl] = {"error": "%s: %s" % (type(e).__name__, e)}
    return out


def file_sha256(path):
    import hashlib
    h = hashlib.sha256()
    with open(path, "rb") as fh:
        for chunk in iter(lambda: fh.read(1 << 20), b""):
            h.update(chunk)
    return h.hexdigest()


def dry_run(args, world, rank):
    """The launch / rank / reduction path without GPU work (gloo): each rank 'steps' for 1 ms; the line carries
    n_gpus = the ranks that ran and value null."""
    import torch
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")
    t0 = time.perf_counter()
    for _ in range(args.steps):
        time.sleep(0.001)
    dt = time.perf_counter() - t0
    ranks = 1
    if dist is not None:
        tt = torch.tensor([dt, 1.0], dtype=torch.float64)
        dist.all_reduce(tt[:1], op=dist.ReduceOp.MAX)
        one = torch.ones(1, dtype=torch.float64)
        dist.all_reduce(one, op=dist.ReduceOp.SUM)
        dt, ranks = float(tt[0]), int(one.item())
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": None, "unit": "propagations/s", "n_gpus": world,
                          "ranks_reporting": ranks, "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": dt / max(args.steps, 1) * 1e3, "dry_run": True}), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def main():
    args = parse()
    rc = launch_ranks(args)
    if rc is not None:
        sys.exit(rc)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dry_run:
        return dry_run(args, world, rank)
    import torch
    ndev = torch.cuda.device_count()   # (does not initialise the GPU)
    if local >= ndev:
        sys.exit("bench.py: rank %d needs GPU %d but %d device(s) are visible" % (rank, local, ndev))
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(local)
    import nusiprop_amd as nu
    from nusiprop_amd import _lib, scan

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
    plan.set_cascade({"mfma": _lib.CASCADE_MFMA, "wf": _lib.CASCADE_WAVEFRONT, "auto": _lib.CASCADE_AUTO}[args.cascade])
    if args.workload == "c4s":
        plan.set_option(_lib.OPT_SHIFT_REUSE, 128)
    if args.rhs:
        plan.set_option(_lib.OPT_CASCADE_RHS, args.rhs)
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
    alpha_kernel, casc_kernel = plan.kernels()   # what the library launched (nusi_plan_kernels)
    props = world * P * args.steps
    value = props / dt
    casc_bytes = scan.cascade_bytes_per_point(N, Nz) * P
    casc_s = sum_ms[2] / max(ncalls, 1) / 1e3
    alpha_s = sum_ms[1] / max(ncalls, 1) / 1e3
    traffic, tsrc, pmc = None, None, {}
    lib_sha = file_sha256(_lib.LIB_PATH)
    tj = args.traffic_json
    if not tj and not args.points:
        tj = os.path.join(ROOT, "profiles", "pmc_traffic_%s.json" % args.workload)
    pmc_note = None
    if tj and os.path.exists(tj):
        with open(tj) as fh:
            pmc = json.load(fh)
        tsrc = os.path.relpath(tj, ROOT)
        if pmc.get("libnusi_sha256") != lib_sha:   # counters of another binary: not this kernel's traffic
            pmc_note = "%s was collected on libnusi.so %s, not the loaded %s: traffic / flops dropped" % (
                tsrc, str(pmc.get("libnusi_sha256"))[:12], lib_sha[:12])
            pmc = {}
        traffic = pmc.get("k_cascade_bytes_per_launch")
    achieved = casc_bytes / casc_s / 1e9
    # workgroups that read a table: one per point, or one per pair of points sharing a table on the multi-RHS
    # kernel (the pair reads its alpha table once)
    readers = P
    if casc_kernel == "k_cascade_ws_mrhs":
        from collections import Counter
        readers = sum((c + 1) // 2 for c in Counter(scan.table_key(p) for p in pts).values())
    casc_min = scan.cascade_min_bytes_per_point(N, Nz, passes=casc_kernel == "k_cascade_ws_passes") * readers
    gbs = scan.gamma_batches(pts, args.rhs or 16) if "k_cascade_gb" in casc_kernel else []
    if gbs:   # the gamma batch: each workgroup reads its table once per pass; the points write their fluxes
        readers = len(gbs)
        casc_min = scan.cascade_gb_bytes_per_batch(N, Nz) * len(gbs) + 8 * 6 * N * P
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
                   "lEmax": p0["lEmax"], "parallelism": "independent points, %d GPU(s), no collective" % world,
                   "alpha_kernel": alpha_kernel, "cascade_kernel": casc_kernel, "cascade_kind": args.cascade,
                   "cascade_rhs": args.rhs or "auto"},
        "libnusi": {"path": os.path.relpath(_lib.LIB_PATH, ROOT), "sha256": lib_sha, "pmc_source": tsrc,
                    "pmc_note": pmc_note},
        "stage_ms_per_step": {"gamma_alphatilde": sum_ms[0] / max(ncalls, 1), "alpha": sum_ms[1] / max(ncalls, 1),
                              "cascade": sum_ms[2] / max(ncalls, 1)},
        "alpha_table": {"kernel": alpha_kernel, "bound": "fp64 VALU (transcendental)",
                        "entries_per_s": scan.alpha_entries_per_point(N, Nz) * P / alpha_s,
                        "avg_step_ms": alpha_s * 1e3, "share_of_step": alpha_s * 1e3 / step_ms},
        # the metric's "achieved HBM GB/s on the cascade kernel".  The wavefront kernel reads each alpha column
        # once per point, so its algorithmic bytes are cascade_min_bytes_per_point (PMC traffic agrees);
        # SURVEY.md sec. 8d's figure (every step re-reading its alpha window, the reference's access pattern)
        # over the same time is reported beside it as reference_pattern_gbs
        "roofline_cascade": {"bound": "hbm", "kernel": casc_kernel, "achieved": casc_min / casc_s / 1e9,
                             "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": casc_min / casc_s / 1e9 / HBM_PEAK_GBS,
                             "traffic": traffic, "traffic_source": tsrc, "algorithmic_bytes_per_launch": casc_min,
                             "table_readers": readers,
                             "reference_pattern_bytes_per_launch": casc_bytes, "reference_pattern_gbs": achieved,
                             "avg_launch_ms": casc_s * 1e3,
                             "note": "not HBM-bound: T = N+Nz-2 dependent stages per point (LDS/barrier latency)"},
        "invalid_outputs": bad,
        "phiphi_lookups_out_of_range": oob,
    }
    if "ws" in casc_kernel or gbs:   # the push on the matrix cores
        mf = scan.cascade_gb_flops_per_batch(N, Nz) * len(gbs) if gbs else scan.cascade_mfma_flops_per_point(N, Nz) * P
        out["roofline_cascade"]["mfma"] = {"flops_per_launch": mf, "achieved": mf / casc_s / 1e12,
                                           "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                                           "frac": mf / casc_s / 1e12 / FP64_PEAK_TFLOPS,
                                           "note": "v_mfma_f64_16x16x4f64 rank-4 pushes (scan.cascade_mfma_flops_per_point; "
                                                   "the gamma batch: scan.cascade_gb_flops_per_batch)"}
        # matrix-core counters of the cascade kernels (the profile's MFMA pass), summed over a step's launches
        mc = {}
        for kname, rec in pmc.get("kernels", {}).items():
            if "k_cascade" in kname:
                for c, v in rec.get("mfma_counters_per_launch", {}).items():
                    mc[c] = mc.get(c, 0.0) + v
        if mc:
            out["roofline_cascade"]["mfma"]["pmc_per_step"] = mc
            busy = mc.get("SQ_VALU_MFMA_BUSY_CYCLES")
            if busy:   # matrix-core busy cycles per v_mfma_f64_16x16x4f64 the push issues (2048 flops each)
                out["roofline_cascade"]["mfma"]["busy_cycles_per_mfma_pmc"] = busy / (
                    out["roofline_cascade"]["mfma"]["flops_per_launch"] / 2048.0)
    fl = pmc.get("k_alpha_fp64_flops_per_step")
    if fl and alpha_s >= casc_s:   # the dominant kernel: executed fp64 VALU flops (PMC counts) per second vs the fp64 vector peak
        ach = fl / alpha_s / 1e12
        out["roofline"] = {"bound": "valu", "kernel": alpha_kernel, "achieved": ach, "peak": FP64_PEAK_TFLOPS,
                           "unit": "TFLOP/s", "frac": ach / FP64_PEAK_TFLOPS,
                           "traffic": pmc.get("k_alpha_hbm_bytes_per_step"), "traffic_source": tsrc,
                           "flops": "executed fp64 VALU (SQ_INSTS_VALU_{ADD,MUL,TRANS}_F64 + 2 FMA) x 64 lanes, "
                                    "from the PMC pass; time = the kernel's HIP events in this run",
                           "note": "dominant kernel (alpha_table.share_of_step); fp64 vector-ALU bound "
                                   "(transcendental leaves), neither HBM nor MFMA"}
    else:   # the cascade dominates (C5's gamma batches), or no alpha counters for this binary
        out["roofline"] = dict(out["roofline_cascade"])
    if args.workload in ("c1", "c2") and rank == 0:
        out["single_propagation"] = single_point_latency(pts[0], max(20, args.steps))
        out["single_propagation"]["plan_ms_per_step"] = dt / args.steps * 1e3
    if rank == 0 and world == 1 and args.workload == "c4" and not args.no_secondary and not args.points:
        out["secondary_lines"] = secondary_lines(local)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(pts, args.cpu_seconds)
        if args.workload == "c1":
            out["cpu_baseline"]["c1_test_cpp"] = c1_cpu_lines(min(5.0, args.cpu_seconds / 3))
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

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
FLUX_RTOL = 1e-11              # the parity tests' flux bound vs the oracle in the matching mode (tests/cases.py)
NORTH_STAR_RTOL = 1e-9         # BASELINE.json north star: max relative flux error vs the CPU reference

# BASELINE config 2 (single propagation, N_E = 300; test.cpp:6-23 physics): C2a = the DSNB source with the resonance
# inside lE 4 -> 9, C2b = the power-law source on the constructor-default grid (tests/cases.py C2A / C2B)
C2_CASES = {
    "C2a": dict(mphi=3e3, g=0.03, mntot=0.1, si=2.5, norm=6.0, majorana=True, non_resonant=True, normal_ordering=True,
                N_bins_E=300, lEmin=4.0, lEmax=9.0, zmax=5.0, flav=2, phiphi=False, source_model=0),
    "C2b": dict(mphi=6e5, g=0.01, mntot=0.1, si=2.5, norm=6.0, majorana=True, non_resonant=True, normal_ordering=True,
                N_bins_E=300, lEmin=12.0, lEmax=17.0, zmax=5.0, flav=2, phiphi=False, source_model=1),
}


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
                    help="cascade kernel: auto = the library default (= mfma: the wavefront with the push on the fp64 "
                         "matrix cores, block-synchronous k_cascade_bs), wf = the bit-exact scalar cascade k_cascade")
    ap.add_argument("--rhs", type=int, default=0,
                    help="NUSI_OPT_CASCADE_RHS: 0 = the library default, 1 = one point per cascade workgroup, 2 = pairs "
                         "of points sharing a table, 3..16 = the gamma batch (k_cascade_bs_gamma)")
    ap.add_argument("--shared-order", action="store_true",
                    help="the opt-in fast table arithmetic, NUSI_OPT_REFERENCE_ORDER = 0 (this repository's dilogarithm "
                         "series and the batch-shared member Taylor coefficients; bit-exact to the oracle's default "
                         "mode).  Default: NUSI_OPT_REFERENCE_ORDER = 1, the library default -- the reference's own "
                         "arithmetic (GSL's dilogarithm algorithms on the reference's arguments; bit-exact to the "
                         "oracle's reference-order mode, DESIGN.md sec. 2)")
    ap.add_argument("--corner-mb", type=int, default=0,
                    help="NUSI_OPT_REFO_CORNER_MB (A/B): the reference order's member-corner block budget in MiB, "
                         "0 = the library's automatic choice")
    ap.add_argument("--reference-order", action="store_true", help="(the default; kept for old command lines)")
    ap.add_argument("--no-parity", action="store_true", help="skip the parity object (oracle fluxes of a sample)")
    ap.add_argument("--dry-run", action="store_true",
                    help="launch / rank / reduction plumbing only, no GPU work (gloo; CPU tests): prints the JSON "
                         "line with value null")
    ap.add_argument("--traffic-json", default="",
                    help="per-launch HBM bytes / fp64 VALU work from rocprofv3 --pmc passes (scripts/pmc_summary.py); "
                         "default: the committed profiles/pmc_traffic_<workload>.json, used only if its libnusi_sha256 matches the loaded library")
    args = ap.parse_args()
    if args.shared_order and args.reference_order:
        ap.error("--shared-order and --reference-order exclude each other")
    args.reference_order = not args.shared_order
    return args


def rank_points(args, rank, world):
    from nusiprop_amd import scan
    if args.workload == "c2":
        pts = [dict(C2_CASES["C2b"])]
        return pts * max(1, args.points or 1), ("C2: single propagation, N_E=300 -- the timed plan runs C2b (lE 12->17, "
                                                "power-law source, test.cpp physics); single_propagation and parity "
                                                "cover C2a (DSNB, resonance inside lE 4->9) and C2b")
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
    lo, hi, allp, desc = shard_of_scan(args, rank, world)
    return allp[lo:hi], desc


def global_scan(args, world):
    """The whole scan the `world` ranks share (C4, C4s, C5), and whether the per-GPU work is fixed as the GPU count
    grows ("weak") or the scan is ("strong"):
      c4 / c4s: the BASELINE config-4 grid (32 m_phi x 32 g) once per GPU, at gamma = 2.5 + 0.05 b for block b --
                one scan of 1024 N points, gamma slowest, so every GPU's shard is one 1024-point block (weak);
      c5:       BASELINE config 5, the 65 536-point (m_phi 64 x g 64 x gamma 16) scan, gamma fastest, partitioned
                over the GPUs (strong); --points P takes its first P points."""
    from nusiprop_amd import scan
    if args.workload in ("c4", "c4s"):
        grid = scan.c4_points if args.workload == "c4" else scan.c4s_points
        P = args.points or 1024
        allp = []
        for b in range(world):
            blk = grid(si=2.5 + 0.05 * b)
            while len(blk) < P:
                blk = blk + blk
            allp += blk[:P]
        return allp, "weak"
    allp = scan.c5_points()
    if args.points:
        allp = (allp * (1 + args.points // len(allp)))[:args.points]
    return allp, "strong"


def shard_of_scan(args, rank, world):
    """This rank's block [lo, hi) of global_scan: scan.shard_aligned, the function nusiprop_amd.dist.evolve_sharded
    partitions with (block ends on table-group boundaries: a gamma batch sharing a Stage-A table stays on one GPU)."""
    from nusiprop_amd import scan
    allp, _ = global_scan(args, world)
    lo, hi = scan.shard_aligned(allp, world, rank)
    if args.workload == "c4":
        desc = ("C4: (m_phi 32 x g 32) scan per GPU, N_E=300, lE 12->17, power-law source; rank r's block of the %d-point "
                "scan (gamma = 2.5 + 0.05 b per 1024-point block b, scan.shard_aligned)" % len(allp))
    elif args.workload == "c4s":
        desc = ("C4s (opt-in NUSI_OPT_SHIFT_REUSE=128): (m_phi 32 on the r^(-o/2) lattice, o = 0, 4, .., 124 below "
                "10^6.533 x g 32) scan per GPU, N_E=300, lE 12->17, power-law source; one base table set per g")
    else:
        desc = ("C5: rank r's block of the %d-point (m_phi 64 x g 64 x gamma 16) scan over %d GPU(s) (scan.shard_aligned: "
                "%d points here), N_E=300, power-law source; gamma batches of 16 share a table" % (len(allp), world, hi - lo))
    return lo, hi, allp, desc


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


def cpu_baseline(pts, budget_s, pp_tables=None, level=1):
    """_cpu_baseline in the oracle's arithmetic mode matching the timed tables (level 1: the reference's own, GSL's
    dilogarithm algorithms; 0: the shared-algorithm order)."""
    from oracle import oracle
    oracle.build()
    with oracle.reference_order(level):
        res = _cpu_baseline(pts, budget_s, pp_tables)
    res["arithmetic"] = "reference order (GSL algorithms, ora_gsl.c)" if level else "shared-algorithm order"
    return res


def _cpu_baseline(pts, budget_s, pp_tables=None):
    """The C oracle (test infrastructure, the reference's algorithm restated) on a bounded sample of the same
    workload: Stage A (tables) and Stage B (cascade) timed apart on one core for a quarter of the budget, then
    whole evolve()s on a thread pool over the host cores for the rest (ctypes releases the GIL, the oracle has
    no global state).  value = the pool's propagations/s.  With phi-phi tables (C3) one propagation on one core
    only: each pool worker would hold its own 400 MB copy of the tables, and one C3 propagation takes ~10 s."""
    import concurrent.futures as cf
    import threading
    from oracle import oracle
    oracle.build()
    threads, host = host_cores()
    if pp_tables is not None:
        o = _oracle(pts[-1])
        t0 = time.perf_counter()
        o.load_phiphi(*pp_tables)
        t1 = time.perf_counter()
        G, At, A = o.tables()
        t2 = time.perf_counter()
        o.cascade(G, At, A)
        t3 = time.perf_counter()
        return {"value": 1.0 / (t3 - t1), "unit": "propagations/s", "cores": 1, "kind": "port", "host": host,
                "s_per_prop": t3 - t1, "stage_a_s": t2 - t1, "stage_b_s": t3 - t2, "table_load_s": t1 - t0,
                "sample": "1 full propagation (the workload's strongest point, g = %.3g) of the single-threaded C "
                          "oracle on one core, phi-phi tables loaded beforehand (not timed)" % pts[-1]["g"],
                "cores_note": "one core; no pool (each worker would need its own 400 MB table copy)"}
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


def single_point_latency(pt, reps, refo=False):
    """One evolve() through the object API (nusi_create / nusi_evolve: host parameters in, tables and cascade
    on the GPU, fluxes copied to the host) -- the reference's own usage, calculate_flux::evolve() per object.
    Returns (timings, flavour fluxes [3, N] of the last evolve)."""
    import ctypes
    import numpy as np
    from nusiprop_amd import _lib
    L = _lib.load()
    p = dict(pt)
    src = p.pop("source_model")
    h = ctypes.c_void_p()
    _lib.check(L.nusi_create(ctypes.byref(_lib.make_params(source_model=src, **p)), ctypes.byref(h)))
    try:
        # (the object API's default is the reference order since round 6; the shared order is the opt-in)
        _lib.check(L.nusi_set_option(h, _lib.OPT_REFERENCE_ORDER, 1 if refo else 0))
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
    fla = np.array(out[:], dtype=np.float64).reshape(3, p["N_bins_E"])
    return {"median_ms": ts[len(ts) // 2] * 1e3, "min_ms": ts[0] * 1e3, "reps": reps, "props_per_s": 1e3 / (ts[len(ts) // 2] * 1e3),
            "path": "nusi_create + nusi_evolve + nusi_get_flux_fla (object API, host I/O and sync included)"}, fla


def rel_err(a, b, floor=1e-280):
    """max |a-b|/|b| over the entries with |b| > floor max|b|; inf unless a == 0 where b == 0 (tests/cases.py)."""
    import numpy as np
    a, b = np.asarray(a, dtype=np.float64), np.asarray(b, dtype=np.float64)
    zero = b == 0
    if np.any(a[zero] != 0):
        return float("inf")
    m = np.abs(b) > floor * (np.max(np.abs(b)) if b.size else 0.0)
    return float(np.max(np.abs(a[m] - b[m]) / np.abs(b[m]))) if np.any(m) else 0.0


def parity_indices(args, pts):
    """A deterministic sample of the workload for the parity object: the strongest-coupling column (g = max, where
    the closed forms' conditioning is worst) at every other m_phi, plus seeded picks; C3: its strongest point."""
    import numpy as np
    if args.workload == "c3":
        return [int(np.argmax([p["g"] for p in pts]))]
    n = 32 if args.workload in ("c4", "c4s") else 16
    gmax = max(p["g"] for p in pts)
    col = [i for i, p in enumerate(pts) if p["g"] == gmax]
    pick = col[::2][:n // 2]
    rng = np.random.default_rng(20250213)
    for i in rng.permutation(len(pts)):
        if len(pick) >= n:
            break
        if int(i) not in pick:
            pick.append(int(i))
    return sorted(pick)


ORDER_SPREAD = ("profiles/r5/reference_order_configs.json", "profiles/r5/reference_order_c4.json")


def order_floor(gpu_order):
    """The per-config floor of this run's fluxes against the reference's own arithmetic (the reference-order oracle):
    in the reference order the tables are bit-exact to it and the fluxes held to FLUX_RTOL; in the shared-algorithm
    order the two arithmetics' measured distance (the oracle in both modes on the CPU: tests/test_oracle_reference_order.py
    -> ORDER_SPREAD[0], the whole C4 grid scripts/reference_order_scan.py -> ORDER_SPREAD[1])."""
    fl = contraction_floor()
    if gpu_order == "reference":   # (tests/test_reference_order_gpu.py)
        out = {c: FLUX_RTOL for c in ("C1", "C2a", "C2b", "C3", "C4")}
    else:
        try:
            cf = json.load(open(os.path.join(ROOT, ORDER_SPREAD[0])))
            c4 = json.load(open(os.path.join(ROOT, ORDER_SPREAD[1])))
        except (OSError, ValueError):
            return None
        out = {"C1": cf["C1_N300"]["flux_max_rel"], "C2a": cf["C2a"]["flux_max_rel"], "C2b": cf["C2b"]["flux_max_rel"],
               "C3": cf["C3"]["flux_max_rel"], "C4": c4["flux_rel_default_vs_reference_order"]["max"]}
        out = {k: max(v, FLUX_RTOL) for k, v in out.items()}
        out["C4_points_above_1e-9"] = c4["flux_rel_default_vs_reference_order"]["points_above_1e-9"]
    # beyond GSL's algorithm, the reference's own binary (g++ -O3 on arm64: FMA contraction, Apple libm) is unpinned:
    # FMA contraction of the reference's expressions alone moves the reference-order fluxes by this much
    # (scripts/contraction_floor.py -> CONTRACTION_FLOOR)
    if fl:
        out["unpinned_beyond"] = fl
    return out


CONTRACTION_FLOOR = "profiles/r6/contraction_floor.json"


def contraction_floor():
    """{config: max relative flux change from FMA contraction alone} (the oracle's reference code and GSL built at
    -ffp-contract=fast against the parity oracle, reference order; scripts/contraction_floor.py)."""
    try:
        rec = json.load(open(os.path.join(ROOT, CONTRACTION_FLOOR)))["configs"]
    except (OSError, ValueError, KeyError):
        return None
    return {c.upper().replace("C2A", "C2a").replace("C2B", "C2b"): v["fc"]["max"] for c, v in rec.items()}


def parity(sel_pts, gpu_fla, gpu_order, phiphi_tables=None, label=""):
    """The GPU fluxes of `sel_pts` (flavour basis, from the timed run) against the C oracle's evolve() in both of
    its arithmetic modes: the shared-algorithm order the default tables are bit-exact to, and the reference's own
    operation order (NUSI_OPT_REFERENCE_ORDER's).  The oracle is the checker here, after the timed region."""
    import numpy as np
    from oracle import oracle
    oracle.build()
    t0 = time.perf_counter()
    res = {}
    for level, key in ((0, "vs_oracle_shared_order"), (1, "vs_oracle_reference_order")):
        _, fla = oracle.evolve_many(sel_pts, level=level, phiphi_tables=phiphi_tables)
        e = np.array([rel_err(gpu_fla[k], fla[k]) for k in range(len(sel_pts))])
        res[key] = {"max_rel": float(e.max()), "median_rel": float(np.median(e)),
                    "points_above_1e-11": int(np.sum(e > FLUX_RTOL)), "points_above_1e-9": int(np.sum(e > NORTH_STAR_RTOL)),
                    "worst": {"mphi": sel_pts[int(np.argmax(e))]["mphi"], "g": sel_pts[int(np.argmax(e))]["g"]}}
    match = "vs_oracle_reference_order" if gpu_order == "reference" else "vs_oracle_shared_order"
    res.update({
        "points": len(sel_pts), "sample": label, "gpu_table_order": gpu_order,
        "tolerance": {"flux_rtol_vs_matching_oracle": FLUX_RTOL, "north_star_rtol": NORTH_STAR_RTOL,
                      "within_flux_rtol_vs_matching_oracle": res[match]["max_rel"] <= FLUX_RTOL,
                      # the north star's bar (<= 1e-9 vs the CPU reference) against the reference-order oracle, whatever
                      # order this run's tables were built in
                      "within_north_star_vs_reference_order": res["vs_oracle_reference_order"]["max_rel"] <= NORTH_STAR_RTOL,
                      # per BASELINE config: how close this order's fluxes are to the reference's own arithmetic
                      "floor_vs_reference_order_per_config": order_floor(gpu_order),
                      "note": "this run's tables are bit-exact to the oracle's %s mode (tests/test_gpu_parity.py, "
                              "tests/test_reference_order_gpu.py); the fluxes differ from it by the cascade's summation "
                              "order only, held to %.0e. The other mode differs where the s-t interference closed forms "
                              "cancel (DESIGN.md sec. 2)" % ("reference-order" if gpu_order == "reference" else
                                                              "shared-algorithm", FLUX_RTOL)},
        "oracle_seconds": time.perf_counter() - t0})
    return res


def launch_ranks(args):
    """--gpus N > 1 without a launcher: start N rank processes with torch.distributed.run (one per GPU, RCCL
    rendezvous on 127.0.0.1) -- before anything here has touched the GPU -- and return their exit status.  A
    rank count that differs from --gpus is an error, never an N-GPU label on a different run."""
    if args.gpus is not None and args.gpus < 1:
        sys.exit("bench.py: --gpus must be >= 1")
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is not None:
        if args.gpus is not None and int(world_env) != args.gpus:
            sys.exit("bench.py: --gpus %d but WORLD_SIZE=%s ranks were launched" % (args.gpus, world_env))
        return None
    if args.gpus is None or args.gpus == 1:
        return None
    import subprocess
    # (--standalone: the rendezvous store binds a port the OS picks, no probe-then-bind race with other processes)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--standalone", "--local-addr", "127.0.0.1", "--nnodes=1",
           "--nproc-per-node", str(args.gpus), os.path.abspath(__file__)] + sys.argv[1:]
    print("bench.py: launching %d ranks: %s" % (args.gpus, " ".join(cmd)), file=sys.stderr, flush=True)
    return subprocess.call(cmd)


SECONDARY = (   # name, bench.py arguments, steps: BASELINE configs 5, 3 and 2, and C4 in the shared-algorithm order
    ("c5", ["--workload", "c5", "--no-cpu-baseline"], 10),
    ("c3", ["--workload", "c3", "--cpu-seconds", "10"], 3),
    ("c4_shared", ["--workload", "c4", "--shared-order", "--no-cpu-baseline"], 10),
    ("c2", ["--workload", "c2", "--cpu-seconds", "4"], 20),
)


def secondary_lines(local):
    """BASELINE configs 5, 3 and 2 and the C4 scan in the shared-algorithm order, measured beside the headline C4 line,
    each by a child bench.py process on the same GPU after the C4 timed region (so the driver's run records them
    too): props/s, stage times, kernels, parity, and (C3, C2) the oracle's CPU numbers."""
    import subprocess
    out = {}
    env = dict(os.environ, HIP_VISIBLE_DEVICES=os.environ.get("HIP_VISIBLE_DEVICES", str(local)))
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT", "GROUP_RANK",
              "ROLE_RANK", "TORCHELASTIC_RUN_ID"):
        env.pop(k, None)   # each child is a plain single-GPU run, not a rank of this job
    for name, extra, steps in SECONDARY:
        cmd = [sys.executable, os.path.abspath(__file__), "--steps", str(steps), "--warmup", "1", "--no-secondary"] + extra
        try:
            r = subprocess.run(cmd, capture_output=True, text=True, timeout=400, env=env)
            d = json.loads(r.stdout.strip().splitlines()[-1])
            out[name] = {k: d.get(k) for k in ("value", "unit", "ms_per_step", "steps", "stage_ms_per_step", "parity",
                                               "single_propagation")}
            out[name]["workload"] = d["config"]["workload"]
            out[name]["table_order"] = d["config"].get("table_order")
            out[name]["kernels"] = [d["config"]["alpha_kernel"], d["config"]["cascade_kernel"]]
            out[name]["roofline"] = {k: d["roofline"].get(k) for k in ("bound", "kernel", "achieved", "unit", "frac",
                                                                       "traffic", "critical_path")
                                     if k in d["roofline"]}
            if "cpu_baseline" in d:
                cb = d["cpu_baseline"]
                out[name]["cpu_baseline"] = {k: cb.get(k) for k in ("value", "unit", "cores", "kind", "sample",
                                                                    "s_per_prop", "single_core")}
        except Exception as e:   # a secondary line never fails the headline run
            out[name] = {"error": "%s: %s" % (type(e).__name__, e)}
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
    n_gpus = the ranks that ran and value null.  For the scan workloads every rank also forms its shard of the
    scan (shard_of_scan) and rank 0 checks the blocks: they cover every point exactly once, in order, and no
    group of points sharing a Stage-A table (a C5 gamma batch) is split across ranks."""
    import numpy as np
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
    shard = None
    if args.workload in ("c4", "c4s", "c5"):
        from nusiprop_amd import scan
        lo, hi, allp, _ = shard_of_scan(args, rank, world)
        blocks = torch.tensor([[lo, hi]], dtype=torch.int64)
        if dist is not None:
            got = [torch.zeros_like(blocks) for _ in range(world)]
            dist.all_gather(got, blocks)
            blocks = torch.cat(got)
        bl = [tuple(int(v) for v in b) for b in blocks.tolist()]
        seen = np.zeros(len(allp), dtype=np.int64)
        for a, b in bl:
            seen[a:b] += 1
        keys = [scan.table_key(p) for p in allp]
        split = sum(1 for a, _ in bl if 0 < a < len(allp) and keys[a] == keys[a - 1])
        shard = {"points": len(allp), "blocks": bl, "covered_once": bool(np.all(seen == 1)),
                 "in_order": all(bl[i][1] == bl[i + 1][0] for i in range(len(bl) - 1)), "table_groups_split": split,
                 "scaling": global_scan(args, world)[1]}
    if dist is not None:
        tt = torch.tensor([dt, 1.0], dtype=torch.float64)
        dist.all_reduce(tt[:1], op=dist.ReduceOp.MAX)
        one = torch.ones(1, dtype=torch.float64)
        dist.all_reduce(one, op=dist.ReduceOp.SUM)
        dt, ranks = float(tt[0]), int(one.item())
    if rank == 0:
        line = {"metric": METRIC, "value": None, "unit": "propagations/s", "n_gpus": world, "ranks_reporting": ranks,
                "steps": args.steps, "warmup": args.warmup, "ms_per_step": dt / max(args.steps, 1) * 1e3,
                "dry_run": True}
        if shard is not None:
            line["shard_check"] = shard
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def pmc_summary_path(workload, reference_order):
    """The committed PMC summary of a workload in one table arithmetic: profiles/pmc_traffic_<workload>.json for the
    reference order (the library default), ..._<workload>_shared.json for the opt-in shared order
    (scripts/gpu_profile_all.sh)."""
    return os.path.join(ROOT, "profiles", "pmc_traffic_%s%s.json" % (workload, "" if reference_order else "_shared"))


def load_pmc(path, lib_sha, order):
    """(summary, source, note): the PMC summary at `path` if it describes the loaded library (its libnusi_sha256) in
    the table arithmetic this run times (its table_order, "reference" / "shared"); otherwise an empty summary -- no
    traffic, no flops, no roofline from it -- and a note saying why.  Counters of another binary or of the other
    arithmetic are not this run's kernels (the shared-order line had been priced with the reference
    order's flops)."""
    if not path or not os.path.exists(path):
        return {}, None, None
    with open(path) as fh:
        pmc = json.load(fh)
    src = os.path.relpath(path, ROOT)
    if pmc.get("libnusi_sha256") != lib_sha:
        return {}, src, "%s was collected on libnusi.so %s, not the loaded %s: traffic / flops dropped" % (
            src, str(pmc.get("libnusi_sha256"))[:12], lib_sha[:12])
    if pmc.get("table_order") != order:
        return {}, src, "%s was collected in the %s table order, this run times the %s order: traffic / flops dropped" % (
            src, pmc.get("table_order"), order)
    return pmc, src, None


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
    if "WORLD_SIZE" in os.environ:   # under a launcher (torch.distributed.run): RCCL, even for one rank
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
    pp_tables, tdir = None, None
    if any(p.get("phiphi") for p in pts):
        import tempfile
        from nusiprop_amd.phiphi_tables import write_synthetic_tables
        tdir = tempfile.mkdtemp(prefix="nusi_phiphi_")
        pp_tables = write_synthetic_tables(tdir)          # the reference's geometry (1.6 GB of records)
        plan.load_phiphi(pp_tables[0], pp_tables[2])      # dims = NULL: {5000,100}, {1000,1000,100}
    try:
        return run(args, world, rank, local, dist, plan, pts, desc, pp_tables)
    finally:
        if tdir:
            import shutil
            shutil.rmtree(tdir, ignore_errors=True)


def run(args, world, rank, local, dist, plan, pts, desc, pp_tables):
    import torch
    from nusiprop_amd import _lib, scan
    P = len(pts)
    p0 = pts[0]
    arr = plan.params_array(pts)
    plan.set_cascade({"mfma": _lib.CASCADE_MFMA, "wf": _lib.CASCADE_WAVEFRONT, "auto": _lib.CASCADE_AUTO}[args.cascade])
    if args.workload == "c4s":
        plan.set_option(_lib.OPT_SHIFT_REUSE, 128)
    if args.rhs:
        plan.set_option(_lib.OPT_CASCADE_RHS, args.rhs)
    plan.set_option(_lib.OPT_REFERENCE_ORDER, 1 if args.reference_order else 0)   # (the library default is 1)
    if args.corner_mb:
        plan.set_option(_lib.OPT_REFO_CORNER_MB, args.corner_mb)
    order = "reference" if args.reference_order else "shared-algorithm"
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
    lib_sha = file_sha256(_lib.LIB_PATH)
    tj = args.traffic_json
    if not tj and not args.points:
        tj = pmc_summary_path(args.workload, args.reference_order)
    pmc, tsrc, pmc_note = load_pmc(tj, lib_sha, "reference" if args.reference_order else "shared")
    traffic = pmc.get("k_cascade_bytes_per_launch")
    achieved = casc_bytes / casc_s / 1e9
    # workgroups that read a table, and the bytes / matrix-core flops they must move / issue
    readers = P
    long_grid = Nz - 1 > 48   # step passes (k_cascade_bs beyond one pass)
    passes = "k_cascade_bs" in casc_kernel and long_grid
    casc_min = scan.cascade_min_bytes_per_point(N, Nz, passes=passes) * readers
    casc_mf = scan.cascade_mfma_flops_per_point(N, Nz) * P
    gbs = []
    if "k_cascade_bs" in casc_kernel:   # the block-synchronous kernels: the library's own grouping (scan.bs_groups)
        from collections import Counter
        sizes = Counter(scan.table_key(p) for p in pts).values()
        gamma_ok = "gamma" in casc_kernel or not any(c >= 3 for c in sizes)
        pairs_ok = "pairs" in casc_kernel or not any(c >= 2 for c in sizes)
        grp = scan.bs_groups(pts, args.rhs, gamma=gamma_ok, pairs=pairs_ok)
        gbs = [g for g in grp if g >= 3]
        one = scan.cascade_min_bytes_per_point(N, Nz, passes=passes)
        readers = len(grp)
        # a gamma batch reads its table once per pass plus its points' fluxes; a pair or a single point reads it
        # once (cascade_min_bytes_per_point holds one point's fluxes; a pair writes a second point's)
        casc_min = sum(scan.cascade_gb_bytes_per_batch(N, Nz) + 8 * 6 * N * g if g >= 3 else one + 8 * 6 * N * (g - 1)
                       for g in grp)
        casc_mf = sum(scan.cascade_gb_flops_per_batch(N, Nz) if g >= 3 else g * scan.cascade_mfma_flops_per_point(N, Nz)
                      for g in grp)
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
        "scaling": global_scan(args, world)[1] if args.workload in ("c4", "c4s", "c5") else "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (deterministic scan grid; power-law source)",
        "config": {"workload": desc, "N_E": N, "N_z": Nz, "points_per_gpu": P, "lEmin": p0["lEmin"],
                   "lEmax": p0["lEmax"], "parallelism": "independent points, %d GPU(s), no collective" % world,
                   "alpha_kernel": alpha_kernel, "cascade_kernel": casc_kernel, "cascade_kind": args.cascade,
                   "cascade_rhs": args.rhs or "auto",
                   "table_order": order + (" (NUSI_OPT_REFERENCE_ORDER = 1, the library default)" if args.reference_order
                                           else " (NUSI_OPT_REFERENCE_ORDER = 0, opt-in)"),
                   **({"refo_corner_mb": args.corner_mb} if args.corner_mb else {}),
                   "process_group": dist.get_backend() if dist is not None else None},
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
    if "ws" in casc_kernel or "bs" in casc_kernel or gbs:   # the push on the matrix cores
        mf = casc_mf
        out["roofline_cascade"]["mfma"] = {"flops_per_launch": mf, "achieved": mf / casc_s / 1e12,
                                           "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                                           "frac": mf / casc_s / 1e12 / FP64_PEAK_TFLOPS,
                                           "note": "v_mfma_f64_16x16x4f64 rank-4 pushes, summed over the launch's workgroups "
                                                   "as the library groups them (scan.bs_groups: gamma batches "
                                                   "scan.cascade_gb_flops_per_batch, pairs and single points "
                                                   "scan.cascade_mfma_flops_per_point each)"}
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
    elif alpha_s >= casc_s:   # the alpha table dominates, but no counters of this binary in this arithmetic
        out["roofline"] = {"bound": "valu", "kernel": alpha_kernel, "achieved": None, "peak": FP64_PEAK_TFLOPS,
                           "unit": "TFLOP/s", "frac": None, "traffic": None, "traffic_source": tsrc,
                           "note": "no executed-flop count for the dominant kernel: " + (
                               pmc_note or "no PMC summary of this workload (scripts/gpu_profile_all.sh)")}
    else:   # the cascade dominates (C5's gamma batches)
        out["roofline"] = dict(out["roofline_cascade"])
    if P == 1:   # a single propagation is latency-bound, not HBM- or VALU-bound: its critical path instead
        st = [m / max(ncalls, 1) for m in sum_ms]
        out["roofline"] = {
            "bound": "latency", "kernel": "critical path of one evolve()", "unit": "ms",
            "achieved": dt / args.steps * 1e3, "peak": None, "frac": None, "traffic": None,
            "critical_path": {
                "tables_ms": st[0] + st[1],
                "tables_note": "Gamma / alphaTilde (%s, side stream) beside the alpha kernels (%s): the later of the two "
                               "(stage events: gamma_alphatilde = the side stream's end, alpha = what alpha ran past it)"
                               % ("k_gamma_alphat", alpha_kernel),
                "cascade_ms": st[2], "cascade_dependent_stages": plan.T,
                "cascade_ns_per_stage": st[2] * 1e6 / plan.T,
                "launch_and_gaps_ms": dt / args.steps * 1e3 - sum(st)},
            "note": "one point fills a few dozen workgroups: the step is the Stage-A kernels' slowest lanes (GSL's "
                    "series, up to ~900 terms for |w| near 0.98) and the cascade's T dependent stages, not a bandwidth"}
    if dist is not None and args.workload in ("c4", "c4s", "c5"):
        # the scan's only data exchange, after the timed region: the fluxes of every rank's block gathered to rank 0
        # (nusiprop_amd.dist._gather_blocks, as evolve_sharded does; float64 tensors staged on the GPU, RCCL)
        from nusiprop_amd.dist import _gather_blocks
        torch.cuda.synchronize()
        barrier()
        tg = time.perf_counter()
        parts = _gather_blocks(fla.cpu().numpy(), P, (3, N), None)
        tg = time.perf_counter() - tg
        out["gather"] = {"seconds": tg, "bytes": 8 * 3 * N * len(global_scan(args, world)[0]),
                         "note": "flavour fluxes of all ranks to rank 0 (dist._gather_blocks), not in the timed region"}
        if rank == 0:
            out["gather"]["points_gathered"] = int(sum(len(x) for x in parts))
    if args.workload == "c1" and rank == 0:
        out["single_propagation"], _ = single_point_latency(pts[0], max(20, args.steps), args.reference_order)
        out["single_propagation"]["plan_ms_per_step"] = dt / args.steps * 1e3
    if args.workload == "c2" and rank == 0:   # both BASELINE config-2 cases through the object API
        out["single_propagation"], c2_fla = {}, {}
        for name, cp in C2_CASES.items():
            out["single_propagation"][name], c2_fla[name] = single_point_latency(cp, max(20, args.steps),
                                                                                args.reference_order)
        out["single_propagation"]["plan_ms_per_step_C2b"] = dt / args.steps * 1e3
        if not args.no_parity:
            out["parity"] = {name: parity([C2_CASES[name]], c2_fla[name][None], order, label=name + " (object API)")
                             for name in C2_CASES}
    elif rank == 0 and not args.no_parity:
        idx = parity_indices(args, pts)
        host_fla = fla.cpu().numpy()
        out["parity"] = parity([pts[i] for i in idx], host_fla[idx], order, phiphi_tables=pp_tables,
                               label="%d of the %d points: the g = max column at every other m_phi + seeded picks "
                                     "(parity_indices); fluxes of the last timed step" % (len(idx), P))
    if rank == 0 and world == 1 and args.workload == "c4" and not args.no_secondary and not args.points:
        out["secondary_lines"] = secondary_lines(local)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(pts, args.cpu_seconds, pp_tables, 1 if args.reference_order else 0)
        if args.workload == "c1":
            out["cpu_baseline"]["c1_test_cpp"] = c1_cpu_lines(min(5.0, args.cpu_seconds / 3))
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

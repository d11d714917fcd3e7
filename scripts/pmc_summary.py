"""Per-launch HBM traffic from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes.

FETCH_SIZE is scaled by the calibration factor measured in the same session
(scripts/calib/pmc_calib streams 2 GiB with 8-B/lane loads, the width of the
cascade's alpha-column loads): factor = bytes read / (FETCH_SIZE KB * 1024).
MI355X_MICROARCH.md (HBM) documents factor 2 for 16-B/lane loads on gfx950.

fp64 VALU work per launch (for the table kernel's VALU roofline) comes from an
optional fourth pass with SQ_INSTS_VALU_{ADD,MUL,FMA,TRANS}_F64: per-wave
instruction counts, x 64 lanes, FMA counted as 2 flops.

  python scripts/pmc_summary.py <fetch_dir> <write_dir> <calib_dir> [<valu_dir>] [--lib libnusi.so]
         [--order reference|shared] [--steps K] > traffic.json

--lib records the sha256 of the library the passes ran and --order the table arithmetic the profiled bench ran
(NUSI_OPT_REFERENCE_ORDER 1 / 0): bench.py drops traffic / flops taken from a summary whose hash or order differs
from the library it loads and the mode it times.  --steps is the number of evolve() calls each pass ran (warmup +
timed); without it the step count is the number of k_gamma_alphat dispatches (one per call, except under
NUSI_OPT_SHIFT_REUSE, which launches it for the direct and the base tables).
"""
import csv
import glob
import json
import sys
from collections import defaultdict


def per_kernel(d, counter):
    """{kernel name: [value per dispatch]}"""
    vals = defaultdict(list)
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            if row["Counter_Name"] == counter:
                vals[row["Kernel_Name"]].append(float(row["Counter_Value"]))
    return vals


STEPS = None   # --steps: evolve() calls per pass


def per_step(d, counter, name_part):
    """Sum over one step's launches of a kernel: every matching dispatch's value, divided by the number of steps the
    pass ran (--steps, else the dispatches of k_gamma_alphat).  (Grouping by grid size, as before round 5, counted
    the reference order's equal-sized member-corner chunks once.)  Returns (per-step value, launches per step)."""
    tot, n, steps = 0.0, 0, 0
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            if row["Counter_Name"] != counter:
                continue
            if "k_gamma_alphat" in row["Kernel_Name"]:
                steps += 1
            if name_part in row["Kernel_Name"]:
                tot += float(row["Counter_Value"])
                n += 1
    steps = STEPS if STEPS else max(steps, 1)
    return tot / steps, n // steps


def main():
    global STEPS
    argv = list(sys.argv[1:])
    lib = mfma_dir = order = None
    if "--order" in argv:
        k = argv.index("--order")
        order = argv[k + 1]
        assert order in ("reference", "shared"), order
        del argv[k:k + 2]
    if "--steps" in argv:
        k = argv.index("--steps")
        STEPS = int(argv[k + 1])
        del argv[k:k + 2]
    if "--lib" in argv:
        k = argv.index("--lib")
        lib = argv[k + 1]
        del argv[k:k + 2]
    if "--mfma" in argv:   # optional pass of matrix-core counters (whichever the box offered)
        k = argv.index("--mfma")
        mfma_dir = argv[k + 1]
        del argv[k:k + 2]
    sys.argv[1:] = argv
    fetch_dir, write_dir, calib_dir = sys.argv[1:4]
    calib_bytes = 2 << 30
    cal = per_kernel(calib_dir, "FETCH_SIZE")
    f64 = [v for k, v in cal.items() if "k_stream_b64" in k][0][0] * 1024.0
    f128 = [v for k, v in cal.items() if "k_stream_b128" in k][0][0] * 1024.0
    fac64, fac128 = calib_bytes / f64, calib_bytes / f128
    fetch, write = per_kernel(fetch_dir, "FETCH_SIZE"), per_kernel(write_dir, "WRITE_SIZE")
    out = {"calibration": {"bytes": calib_bytes, "fetch_factor_b64": fac64, "fetch_factor_b128": fac128}, "kernels": {}}
    for k in sorted(set(fetch) | set(write)):
        if "nusi::" not in k:
            continue
        fk = sum(fetch.get(k, [0])) / max(len(fetch.get(k, [])), 1)
        wk = sum(write.get(k, [0])) / max(len(write.get(k, [])), 1)
        out["kernels"][k] = {"FETCH_SIZE_KB_mean": fk, "WRITE_SIZE_KB_mean": wk, "launches": len(fetch.get(k, [])),
                             "hbm_bytes_per_launch": fk * 1024.0 * fac64 + wk * 1024.0}
    if len(sys.argv) > 4:
        ctr = {c: per_kernel(sys.argv[4], c) for c in
               ["SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_TRANS_F64"]}
        for k, rec in out["kernels"].items():
            mean = {c: (sum(v[k]) / len(v[k]) if v.get(k) else 0.0) for c, v in ctr.items()}
            rec["valu_f64_insts_per_launch"] = mean
            rec["fp64_flops_per_launch"] = 64.0 * (mean["SQ_INSTS_VALU_ADD_F64"] + mean["SQ_INSTS_VALU_MUL_F64"]
                                                    + 2.0 * mean["SQ_INSTS_VALU_FMA_F64"]
                                                    + mean["SQ_INSTS_VALU_TRANS_F64"])
    if mfma_dir:
        import os
        names = set()
        for f in glob.glob(mfma_dir + "/**/*counter_collection.csv", recursive=True):
            for row in csv.DictReader(open(f)):
                names.add(row["Counter_Name"])
        for c in sorted(names):
            vals = per_kernel(mfma_dir, c)
            for k, rec in out["kernels"].items():
                if vals.get(k):
                    rec.setdefault("mfma_counters_per_launch", {})[c] = sum(vals[k]) / len(vals[k])
        if not names and not os.path.isdir(mfma_dir):
            out["mfma_note"] = "no matrix-core pass"
    # the cascade stage of one step: the sum over its launches (C5 runs the multi-RHS kernel and, for a table's
    # odd point, the one-point kernel; grouped by kernel name and grid size like the alpha launches)
    fk, ng = per_step(fetch_dir, "FETCH_SIZE", "nusi::k_cascade")
    wk, _ = per_step(write_dir, "WRITE_SIZE", "nusi::k_cascade")
    if ng:
        out["k_cascade_launches_per_step"] = ng
        out["k_cascade_bytes_per_launch"] = fk * 1024.0 * fac64 + wk * 1024.0
    fk, ng = per_step(fetch_dir, "FETCH_SIZE", "nusi::k_alpha")   # tiles + the per-entry region
    wk, _ = per_step(write_dir, "WRITE_SIZE", "nusi::k_alpha")
    if ng:
        out["k_alpha_launches_per_step"] = ng
        out["k_alpha_hbm_bytes_per_step"] = fk * 1024.0 * fac64 + wk * 1024.0
        if len(sys.argv) > 4:
            add = per_step(sys.argv[4], "SQ_INSTS_VALU_ADD_F64", "nusi::k_alpha")[0]
            mul = per_step(sys.argv[4], "SQ_INSTS_VALU_MUL_F64", "nusi::k_alpha")[0]
            fma = per_step(sys.argv[4], "SQ_INSTS_VALU_FMA_F64", "nusi::k_alpha")[0]
            trn = per_step(sys.argv[4], "SQ_INSTS_VALU_TRANS_F64", "nusi::k_alpha")[0]
            out["k_alpha_fp64_flops_per_step"] = 64.0 * (add + mul + 2.0 * fma + trn)
    if order:
        out["table_order"] = order
    if STEPS:
        out["steps_per_pass"] = STEPS
    if lib:
        import hashlib
        with open(lib, "rb") as fh:
            out["libnusi_sha256"] = hashlib.sha256(fh.read()).hexdigest()
    json.dump(out, sys.stdout, indent=1)


if __name__ == "__main__":
    main()

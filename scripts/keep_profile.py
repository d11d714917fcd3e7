"""Copy what a GPU profile session left under gpurun_out/ into profiles/ (the tracked record):
  python scripts/keep_profile.py <profile session tag> <dest under profiles/> [<tests+bench session tag>]
Per workload: kernel_stats.csv (rocprofv3 --stats), pmc_traffic_summary.json (also copied to
profiles/pmc_traffic_<wl>.json, which bench.py reads), bench.json; from the other session pytest.log, smoke.log and
the default bench line."""
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    tag, dest = sys.argv[1], os.path.join(ROOT, "profiles", sys.argv[2])
    src = os.path.join(ROOT, "gpurun_out", tag, "prof")
    os.makedirs(dest, exist_ok=True)
    for wl in sorted(os.listdir(src)):
        d = os.path.join(src, wl)
        if not os.path.isdir(d) or not os.path.exists(os.path.join(d, "pmc_traffic_summary.json")):
            continue
        o = os.path.join(dest, wl)
        os.makedirs(o, exist_ok=True)
        shutil.copy(os.path.join(d, "kt", "kt_kernel_stats.csv"), os.path.join(o, "kernel_stats.csv"))
        shutil.copy(os.path.join(d, "pmc_traffic_summary.json"), o)
        shutil.copy(os.path.join(d, "pmc_traffic_summary.json"), os.path.join(ROOT, "profiles", "pmc_traffic_%s.json" % wl))
        shutil.copy(os.path.join(d, "bench.json"), o)
    for f in ("mfma_counters.txt",):
        if os.path.exists(os.path.join(src, f)):
            shutil.copy(os.path.join(src, f), dest)
    if len(sys.argv) > 3:
        s = os.path.join(ROOT, "gpurun_out", sys.argv[3])
        for f in ("pytest.log", "smoke.log"):
            if os.path.exists(os.path.join(s, f)):
                shutil.copy(os.path.join(s, f), dest)
        benches = sorted(f for f in os.listdir(s) if f.startswith("bench_") and f.endswith(".json"))
        if benches:
            shutil.copy(os.path.join(s, benches[-1]), os.path.join(dest, "bench_default.json"))
    print("kept", dest)


if __name__ == "__main__":
    main()

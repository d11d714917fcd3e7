"""Per-kernel SQ counter summary (mean per dispatch) from rocprofv3 --pmc pass directories."""
import csv, collections, glob, sys
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for d in sys.argv[1:]:
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        per = collections.defaultdict(float)
        for r in csv.DictReader(open(f)):
            per[(r["Kernel_Name"].split("(")[0], r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
        for (k, _, c), v in per.items():
            agg[k][c].append(v)
for k, cs in agg.items():
    if "rocclr" in k: continue
    print("==", k, "(%d dispatches)" % len(next(iter(cs.values()))))
    for c in sorted(cs):
        v = cs[c]; print("   %-26s %.4e" % (c, sum(v) / len(v)))
